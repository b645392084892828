// smj_host.hip -- the host-pointer half of the C ABI (include/smj.h): the
// device set (smj_init / smj_init_devices replace dpu_alloc, app.c:175,315,
// 422,638) and the entry points the app.c drop-in calls with host tables
// (smj_select / smj_sort / smj_merge / smj_join / smj_sort_merge_join).
//
// With one device every call stages its tables into device buffers that
// persist across calls (grow-only, per device of the set: a caller looping
// over smj_* does not re-allocate), runs the smj_dev_* pipeline and copies
// the result back.  With N devices, smj_sort_merge_join and smj_sort shard
// the work the way the reference spreads rows over NR_DPUS (app.c:155-218),
// but with one exchange instead of the host-mediated merge tree:
//
//   1. splitters: N - 1 weighted key quantiles of a host-side sample of both
//      tables (the WHERE clause applied), so device d owns key range d;
//   2. device d receives the contiguous input slice d of each table (one
//      H2D copy per table and device, all devices in parallel), selects and
//      stably partitions it by key range (smj_dev_partition);
//   3. exchange over xGMI: device d pulls range d from every device, in
//      source-device order -- equal keys keep their input order
//      (hipMemcpyPeerAsync; a plain device copy when two entries of the set
//      are the same physical GPU);
//   4. device d runs the fused select/sort/zip-join pipeline on its range
//      (smj_dev_sort_merge_join; tables over 1.6e8 rows are partitioned
//      further inside it);
//   5. the per-device joined rows are copied to the host result in device
//      order: key ranges ascend with d, so this is cpu_app.c's row order.
//
// One host thread per device of the set drives steps 2, 4 and 5 (the caller
// stays single-threaded, as app.c is).  Tables wider than 8 columns take the
// single-device index-sort path.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <utility>
#include <vector>

#include "smj.h"
#include "smj_internal.h"

using namespace smj;

#define HIP_TRY(x)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "smj: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_),     \
                    __FILE__, __LINE__);                                                   \
            return e_ == hipErrorOutOfMemory ? SMJ_ERR_NOMEM : SMJ_ERR_HIP;               \
        }                                                                                  \
    } while (0)

#define SMJ_TRY(x)                      \
    do {                                \
        int rc_ = (x);                  \
        if (rc_ != SMJ_OK) return rc_;  \
    } while (0)

namespace {
// device buffers of one entry of the device set (grow-only)
enum { B_IN0, B_IN1, B_PART0, B_PART1, B_RECV0, B_RECV1, B_OUT0, B_OUT1, B_J, B_SPL, B_N };

struct HostDev {
    int phys = -1;            // HIP device
    hipStream_t st = nullptr;
    hipStream_t cp = nullptr;  // staged H2D copies (overlapping the first pass)
    // exchange: one stream per source device, so the pulls from all sources
    // run at once (one xGMI link each) and join st through the events
    std::vector<hipStream_t> px;
    std::vector<hipEvent_t> pe;
    hipEvent_t in_ev[2] = {nullptr, nullptr};  // table x's slice has landed (cp -> st)
    // result D2H (d2h_result): per copy thread a stream, two pinned slots
    // and their events, made on the first large result
    std::vector<hipStream_t> ds;
    std::vector<hipEvent_t> de;
    std::vector<char *> dslot;
    void *b[B_N] = {};
    size_t c[B_N] = {};
};
std::vector<HostDev> g_devs;
int64_t g_shard_rows[64];  // rows (R + S) each device of the last sharded call received
int g_shard_n = 0;

int hgrow(HostDev &d, int i, size_t need) {
    need = std::max<size_t>(need, 64);
    if (need <= d.c[i]) return SMJ_OK;
    if (d.b[i]) HIP_TRY(dev_free(d.b[i]));
    d.b[i] = nullptr;
    d.c[i] = 0;
    HIP_TRY(dev_alloc(&d.b[i], need));
    d.c[i] = need;
    return SMJ_OK;
}

int need_init() {
    if (g_devs.empty()) return SMJ_ERR_NODEVICE;
    HIP_TRY(hipSetDevice(g_devs[0].phys));
    return SMJ_OK;
}

int check_block(const dpu_block_t *bl, const void *ptr) {
    if (!bl || bl->row_num < 0 || bl->col_num < 1) return SMJ_ERR_INVALID;
    if (bl->row_num > 0 && !ptr) return SMJ_ERR_INVALID;
    if (bl->col_num > SMJ_MAX_COLS) return SMJ_ERR_TOO_LARGE;  // row_num is an int: < SMJ_MAX_ROWS
    return SMJ_OK;
}

double ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// f(d) on every device of the set, one thread per device (inline for one);
// the first non-OK status wins
template <class F>
int on_devices(F f) {
    const int n = (int)g_devs.size();
    std::vector<int> rc(n, SMJ_OK);
    auto body = [&](int d) {
        if (hipSetDevice(g_devs[d].phys) != hipSuccess) {
            rc[d] = SMJ_ERR_HIP;
            return;
        }
        set_scratch_slot(n > 1 ? d : -1);
        rc[d] = f(d);
        set_scratch_slot(-1);
    };
    if (n == 1) {
        body(0);
    } else {
        std::vector<std::thread> th;
        for (int d = 0; d < n; d++) th.emplace_back(body, d);
        for (auto &t : th) t.join();
    }
    for (int d = 0; d < n; d++)
        if (rc[d] != SMJ_OK) return rc[d];
    return SMJ_OK;
}

// T = uint64 / double compare through the pipeline's order-preserving map
// (smj_kernels.hip key_fwd)
int64_t key_map_host(int64_t v, int ktype) {
    uint64_t u = (uint64_t)v;
    if (ktype == SMJ_KEY_INT64) return v;
    if (ktype == SMJ_KEY_UINT64) return (int64_t)(u ^ 0x8000000000000000ull);
    if (u == 0x8000000000000000ull) u = 0;  // -0.0
    return (int64_t)((u >> 63) ? (u ^ 0x7fffffffffffffffull) : u);
}

uint32_t map_mask(int key, int sel_col) { return (1u << key) | (1u << sel_col); }

// The caller free()s the result (app.c:759).  A large result is 2 MiB aligned
// and advised onto huge pages: its first touch -- the D2H copy -- then takes a
// few hundred page faults per GB instead of ~260 000 (a pageable D2H into a
// fresh 4 KiB-page buffer ran at 13-17 GB/s, tools/h2d_overlap.py).
void *result_alloc(size_t bytes) {
    if (bytes < ((size_t)64 << 20)) return malloc(std::max<size_t>(bytes, 1));
    void *p = nullptr;
    if (posix_memalign(&p, (size_t)2 << 20, bytes) != 0) return nullptr;
    madvise(p, bytes, MADV_HUGEPAGE);
    return p;
}
// Device -> host copy of a result into pageable (malloc'd) memory.  A plain
// hipMemcpy into pageable memory ran at 13-17 GB/s (tools/h2d_overlap.py:
// 35 ms for C3's 0.59 GB of joined rows): the runtime's single host thread
// copies each bounce buffer into the destination, first-touch page faults
// included.  Large results are cut into kD2HThreads contiguous parts; a
// thread per part pulls its part through two pinned slots on a stream of its
// own (DMA of chunk k + 1 while chunk k is copied into place), so the PCIe
// transfer and the host-side copies and page faults run in parallel.  The
// device's stream st must have produced src already (the caller synchronised).
constexpr int kD2HThreads = 8;
constexpr size_t kD2HSlot = (size_t)8 << 20;  // bytes per pinned slot (2 per thread: 128 MiB pinned per device)
constexpr size_t kD2HMin = (size_t)64 << 20;  // smaller results take one plain copy

int d2h_result(HostDev &hd, void *dst, const void *src, size_t bytes) {
    if (bytes == 0) return SMJ_OK;
    const char *mn = getenv("SMJ_D2H_MIN");  // tests: the threaded path at small sizes
    if (bytes < (mn ? (size_t)atoll(mn) : kD2HMin)) {
        HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, hd.st));
        HIP_TRY(hipStreamSynchronize(hd.st));
        return SMJ_OK;
    }
    if (hd.ds.empty()) {
        // created into locals and kept only once all exist: a failure part way
        // frees the partial set, so a later call never copies through a null
        // stream or slot
        std::vector<hipStream_t> ds(kD2HThreads, nullptr);
        std::vector<hipEvent_t> de(2 * kD2HThreads, nullptr);
        std::vector<char *> dslot(2 * kD2HThreads, nullptr);
        auto release = [&]() {
            for (auto x : ds)
                if (x) hipStreamDestroy(x);
            for (auto x : de)
                if (x) hipEventDestroy(x);
            for (auto x : dslot)
                if (x) hipHostFree(x);
        };
        hipError_t e = hipSuccess;
        for (int t = 0; t < kD2HThreads && e == hipSuccess; t++) e = hipStreamCreateWithFlags(&ds[t], hipStreamNonBlocking);
        for (int i = 0; i < 2 * kD2HThreads && e == hipSuccess; i++) {
            e = hipEventCreateWithFlags(&de[i], hipEventDisableTiming);
            if (e == hipSuccess) e = hipHostMalloc((void **)&dslot[i], kD2HSlot, hipHostMallocDefault);
        }
        if (e != hipSuccess) {
            fprintf(stderr, "smj: D2H staging setup failed: %s\n", hipGetErrorString(e));
            release();
            return e == hipErrorOutOfMemory ? SMJ_ERR_NOMEM : SMJ_ERR_HIP;
        }
        hd.ds = std::move(ds);
        hd.de = std::move(de);
        hd.dslot = std::move(dslot);
    }
    std::vector<int> rc(kD2HThreads, SMJ_OK);
    auto part = [&](int t) {
        if (hipSetDevice(hd.phys) != hipSuccess) {
            rc[t] = SMJ_ERR_HIP;
            return;
        }
        const size_t p0 = bytes * t / kD2HThreads / 8 * 8, p1 = t + 1 == kD2HThreads ? bytes : bytes * (t + 1) / kD2HThreads / 8 * 8;
        const size_t nch = (p1 - p0 + kD2HSlot - 1) / kD2HSlot;
        auto chunk = [&](size_t k, size_t &o, size_t &len) {
            o = p0 + k * kD2HSlot;
            len = std::min(kD2HSlot, p1 - o);
        };
        auto issue = [&](size_t k) -> hipError_t {
            size_t o, len;
            chunk(k, o, len);
            hipError_t e = hipMemcpyAsync(hd.dslot[2 * t + (k & 1)], (const char *)src + o, len, hipMemcpyDeviceToHost, hd.ds[t]);
            return e == hipSuccess ? hipEventRecord(hd.de[2 * t + (k & 1)], hd.ds[t]) : e;
        };
        if (nch && issue(0) != hipSuccess) {
            rc[t] = SMJ_ERR_HIP;
            return;
        }
        for (size_t k = 0; k < nch; k++) {
            // slot (k + 1) & 1 last held chunk k - 1, already copied out
            if (k + 1 < nch && issue(k + 1) != hipSuccess) {
                rc[t] = SMJ_ERR_HIP;
                return;
            }
            if (hipEventSynchronize(hd.de[2 * t + (k & 1)]) != hipSuccess) {
                rc[t] = SMJ_ERR_HIP;
                return;
            }
            size_t o, len;
            chunk(k, o, len);
            memcpy((char *)dst + o, hd.dslot[2 * t + (k & 1)], len);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < kD2HThreads; t++) th.emplace_back(part, t);
    for (auto &x : th) x.join();
    for (int t = 0; t < kD2HThreads; t++)
        if (rc[t] != SMJ_OK) return rc[t];
    return SMJ_OK;
}
}  // namespace

// ---------------------------------------------------------------------------
// lifetime
// ---------------------------------------------------------------------------
extern "C" int smj_init_devices(const int *device_ids, int n) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SMJ_ERR_NODEVICE;
    if (n < 1 || !device_ids) return SMJ_ERR_INVALID;
    if (!g_devs.empty()) smj_finalize();
    for (int d = 0; d < n; d++) {
        const int id = device_ids[d];
        if (id < 0 || id >= count) return SMJ_ERR_NODEVICE;
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, id));
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            fprintf(stderr, "smj: device %d is %s, this library is built for gfx950\n", id, prop.gcnArchName);
            return SMJ_ERR_NODEVICE;
        }
    }
    // peer access between distinct GPUs of the set (the exchange over xGMI)
    for (int a = 0; a < n; a++)
        for (int b = 0; b < n; b++) {
            const int pa = device_ids[a], pb = device_ids[b];
            if (pa == pb) continue;
            int ok = 0;
            if (hipDeviceCanAccessPeer(&ok, pa, pb) == hipSuccess && ok) {
                HIP_TRY(hipSetDevice(pa));
                const hipError_t e = hipDeviceEnablePeerAccess(pb, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_TRY(e);
                (void)hipGetLastError();  // clear an "already enabled" status
            }
        }
    g_devs.assign(n, HostDev{});
    for (int d = 0; d < n; d++) {
        g_devs[d].phys = device_ids[d];
        HIP_TRY(hipSetDevice(device_ids[d]));
        HIP_TRY(hipStreamCreateWithFlags(&g_devs[d].st, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&g_devs[d].cp, hipStreamNonBlocking));
        for (int x = 0; x < 2; x++) HIP_TRY(hipEventCreateWithFlags(&g_devs[d].in_ev[x], hipEventDisableTiming));
        if (n > 1) {
            g_devs[d].px.assign(n, nullptr);
            g_devs[d].pe.assign(n, nullptr);
            for (int q = 0; q < n; q++) {
                HIP_TRY(hipStreamCreateWithFlags(&g_devs[d].px[q], hipStreamNonBlocking));
                HIP_TRY(hipEventCreateWithFlags(&g_devs[d].pe[q], hipEventDisableTiming));
            }
        }
    }
    HIP_TRY(hipSetDevice(device_ids[0]));
    return n;
}

extern "C" int smj_init(int n_gpus) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SMJ_ERR_NODEVICE;
    const int n = (n_gpus <= 0 || n_gpus > count) ? count : n_gpus;
    std::vector<int> ids(n);
    for (int d = 0; d < n; d++) ids[d] = d;
    return smj_init_devices(ids.data(), n);
}

extern "C" int smj_device_count(void) { return (int)g_devs.size(); }

// Diagnostic: rows (R + S, after the WHERE clause) each device of the last
// sharded call received; returns the device count (at most `max` written).
extern "C" int smj_debug_shard_rows(int64_t *out, int max) {
    for (int d = 0; d < std::min(max, g_shard_n); d++) out[d] = g_shard_rows[d];
    return g_shard_n;
}

// Returns every device buffer the library holds (scratch sets, partition
// staging, the device set's staging buffers) once the work on them has
// drained; later calls allocate again.  The device set and its streams stay.
// Refused (SMJ_ERR_INVALID) while a smj_dev_sort_merge_join_begin job is open.
// Replaces the reference's per-phase dpu_free (app.c:307,402,503,761).
extern "C" int smj_trim(void) {
    if (open_jobs() > 0) return SMJ_ERR_INVALID;
    int cur = -1;
    const bool have_cur = hipGetDevice(&cur) == hipSuccess;
    for (auto &d : g_devs) {
        hipSetDevice(d.phys);
        HIP_TRY(hipDeviceSynchronize());
        for (int i = 0; i < B_N; i++) {
            dev_free(d.b[i]);
            d.b[i] = nullptr;
            d.c[i] = 0;
        }
    }
    if (have_cur) {
        hipSetDevice(cur);
        HIP_TRY(hipDeviceSynchronize());
    }
    api_free_all();
    if (have_cur) hipSetDevice(cur);
    return SMJ_OK;
}

extern "C" void smj_finalize(void) {
    for (auto &d : g_devs) {
        hipSetDevice(d.phys);
        for (int i = 0; i < B_N; i++) dev_free(d.b[i]);
        hipStreamDestroy(d.st);
        hipStreamDestroy(d.cp);
        for (auto e : d.in_ev) hipEventDestroy(e);
        for (auto q : d.px) hipStreamDestroy(q);
        for (auto e : d.pe) hipEventDestroy(e);
        for (auto q : d.ds) hipStreamDestroy(q);
        for (auto e : d.de) hipEventDestroy(e);
        for (auto p : d.dslot) hipHostFree(p);
    }
    g_devs.clear();
    api_free_all();
}

// ---------------------------------------------------------------------------
// single-device entry points (device 0 of the set)
// ---------------------------------------------------------------------------
extern "C" int smj_select(const dpu_block_t *bl, const T *in, T *out, int select_col, T select_val,
                          int *out_rows) {
    SMJ_TRY(need_init());
    SMJ_TRY(check_block(bl, in));
    if (!out_rows || (bl->row_num > 0 && !out) || select_col < 0 || select_col >= bl->col_num)
        return SMJ_ERR_INVALID;
    HostDev &hd = g_devs[0];
    const size_t bytes = (size_t)bl->row_num * bl->col_num * sizeof(T);
    SMJ_TRY(hgrow(hd, B_IN0, bytes));
    SMJ_TRY(hgrow(hd, B_OUT0, bytes));
    hipStream_t s = hd.st;
    HIP_TRY(hipMemcpyAsync(hd.b[B_IN0], in, bytes, hipMemcpyHostToDevice, s));
    int64_t m = 0;
    SMJ_TRY(smj_dev_select((T *)hd.b[B_IN0], bl->row_num, bl->col_num, select_col, select_val, (T *)hd.b[B_OUT0], &m,
                           s));
    HIP_TRY(hipMemcpyAsync(out, hd.b[B_OUT0], (size_t)m * bl->col_num * sizeof(T), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *out_rows = (int)m;
    return SMJ_OK;
}

extern "C" int smj_merge(const dpu_block_t *bl1, const T *a, const dpu_block_t *bl2, const T *b, int key_col,
                         T *out) {
    SMJ_TRY(need_init());
    SMJ_TRY(check_block(bl1, a));
    SMJ_TRY(check_block(bl2, b));
    if (bl1->col_num != bl2->col_num || key_col < 0 || key_col >= bl1->col_num) return SMJ_ERR_INVALID;
    const int cols = bl1->col_num;
    const int64_t na = bl1->row_num, nb = bl2->row_num;
    if (na + nb == 0) return SMJ_OK;
    if (!out) return SMJ_ERR_INVALID;
    HostDev &hd = g_devs[0];
    SMJ_TRY(hgrow(hd, B_IN0, (size_t)na * cols * 8));
    SMJ_TRY(hgrow(hd, B_IN1, (size_t)nb * cols * 8));
    SMJ_TRY(hgrow(hd, B_OUT0, (size_t)(na + nb) * cols * 8));
    hipStream_t s = hd.st;
    if (na) HIP_TRY(hipMemcpyAsync(hd.b[B_IN0], a, (size_t)na * cols * 8, hipMemcpyHostToDevice, s));
    if (nb) HIP_TRY(hipMemcpyAsync(hd.b[B_IN1], b, (size_t)nb * cols * 8, hipMemcpyHostToDevice, s));
    SMJ_TRY(smj_dev_merge((T *)hd.b[B_IN0], na, (T *)hd.b[B_IN1], nb, cols, key_col, (T *)hd.b[B_OUT0], s));
    HIP_TRY(hipMemcpyAsync(out, hd.b[B_OUT0], (size_t)(na + nb) * cols * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SMJ_OK;
}

extern "C" int smj_join(const dpu_block_t *r, const T *R, const dpu_block_t *s_, const T *S, int key1, int key2,
                        T **out, int64_t *out_rows) {
    SMJ_TRY(need_init());
    SMJ_TRY(check_block(r, R));
    SMJ_TRY(check_block(s_, S));
    if (!out || !out_rows || key1 < 0 || key1 >= r->col_num || key2 < 0 || key2 >= s_->col_num)
        return SMJ_ERR_INVALID;
    const int c1 = r->col_num, c2 = s_->col_num, tc = c1 + c2 - 1;
    const int64_t nr = r->row_num, ns = s_->row_num, cap = std::min(nr, ns);
    HostDev &hd = g_devs[0];
    SMJ_TRY(hgrow(hd, B_IN0, (size_t)nr * c1 * 8));
    SMJ_TRY(hgrow(hd, B_IN1, (size_t)ns * c2 * 8));
    SMJ_TRY(hgrow(hd, B_J, (size_t)cap * tc * 8));
    SMJ_TRY(hgrow(hd, B_SPL, 64 * sizeof(int64_t)));
    hipStream_t st = hd.st;
    if (nr) HIP_TRY(hipMemcpyAsync(hd.b[B_IN0], R, (size_t)nr * c1 * 8, hipMemcpyHostToDevice, st));
    if (ns) HIP_TRY(hipMemcpyAsync(hd.b[B_IN1], S, (size_t)ns * c2 * 8, hipMemcpyHostToDevice, st));
    int64_t j = 0;
    SMJ_TRY(smj_dev_join((T *)hd.b[B_IN0], nr, c1, (T *)hd.b[B_IN1], ns, c2, key1, key2, (T *)hd.b[B_J],
                         (int64_t *)hd.b[B_SPL], &j, st));
    T *res = (T *)result_alloc((size_t)j * tc * sizeof(T));
    if (!res) return SMJ_ERR_NOMEM;
    if (j && hipMemcpyAsync(res, hd.b[B_J], (size_t)j * tc * 8, hipMemcpyDeviceToHost, st) != hipSuccess) {
        free(res);
        return SMJ_ERR_HIP;
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
        free(res);
        return SMJ_ERR_HIP;
    }
    *out = res;
    *out_rows = j;
    return SMJ_OK;
}

// ---------------------------------------------------------------------------
// the sharded pipeline (N devices): select + stable sort (+ zip join)
// ---------------------------------------------------------------------------
namespace {
struct HTab {                 // one host table of a sharded call
    const int64_t *rows;
    int64_t n;
    int cols, sel_col, key;
    int64_t sel_map;          // the select value, mapped (T = uint64 / double)
};

// N - 1 splitters: weighted quantiles of a key sample of every table (a
// sample of table x stands for n_x / samples input rows; rows the WHERE
// clause drops are not samples).
std::vector<int64_t> host_splitters(const HTab *t, int ntab, int ktype, int parts) {
    constexpr int64_t kSamples = 8192;
    std::vector<std::pair<int64_t, double>> kw;
    double W = 0;
    for (int x = 0; x < ntab; x++) {
        const int64_t k = std::min(t[x].n, kSamples);
        if (k == 0) continue;
        const double w = (double)t[x].n / (double)k;
        for (int64_t j = 0; j < k; j++) {
            const int64_t r = k > 1 ? j * (t[x].n - 1) / (k - 1) : 0;
            const int64_t *row = t[x].rows + r * t[x].cols;
            if (key_map_host(row[t[x].sel_col], ktype) <= t[x].sel_map) continue;
            kw.emplace_back(key_map_host(row[t[x].key], ktype), w);
            W += w;
        }
    }
    std::sort(kw.begin(), kw.end());
    std::vector<int64_t> spl;
    double acc = 0;
    size_t i = 0;
    for (int p = 1; p < parts && !kw.empty(); p++) {
        const double target = W * (double)p / (double)parts;
        while (i + 1 < kw.size() && acc + kw[i].second < target) acc += kw[i++].second;
        if (spl.empty() || spl.back() < kw[i].first) spl.push_back(kw[i].first);
    }
    return spl;
}

// Partition boundaries for bucket(key) = #{bounds < key}: every splitter key
// u gets the single-key bucket (u - 1, u] (single[b] = 1), so that a heavy key
// can be cut between devices at an occurrence index (smj/dist.py
// bucket_bounds).  Key-only bounds when they would not
// fit the partition kernel's 64 buckets.
void shard_bounds(const std::vector<int64_t> &spl, std::vector<int64_t> &bounds, std::vector<char> &single) {
    bounds.clear();
    for (int64_t u : spl) {
        if (u > INT64_MIN && (bounds.empty() || bounds.back() < u - 1)) bounds.push_back(u - 1);
        bounds.push_back(u);
    }
    if ((int)bounds.size() > kMaxSplitters) bounds = spl;
    const int nb = (int)bounds.size() + 1;
    single.assign(nb, 0);
    for (int b = 0; b < nb; b++)
        single[b] = (b == 0 && !bounds.empty() && bounds[0] == INT64_MIN) ||
                    (b > 0 && b < nb - 1 && bounds[b] - bounds[b - 1] == 1);
}

// D - 1 cuts (bucket, occurrence) over the global bucket-ordered sequence,
// balancing R + S rows per device (smj/dist.py choose_cuts): rows of buckets
// < b go to the left, and of bucket b the occurrences < o; o != 0 only inside
// a single-key bucket, and the same o cuts R and S, so occurrence i of R and
// occurrence i of S -- a zip-join pair -- stay on one device.
std::vector<std::pair<int, int64_t>> shard_cuts(const std::vector<int64_t> &GR, const std::vector<int64_t> &GS,
                                                const std::vector<char> &single, int parts) {
    const int nb = (int)GR.size();
    std::vector<int64_t> tot(nb);
    int64_t total = 0;
    for (int b = 0; b < nb; b++) total += tot[b] = GR[b] + GS[b];
    std::vector<std::pair<int, int64_t>> cuts;
    std::pair<int, int64_t> prev{0, 0};
    int64_t acc = 0;
    int b = 0;
    for (int d = 1; d < parts; d++) {
        const double target = (double)total * d / parts;
        while (b < nb && (double)(acc + tot[b]) <= target) acc += tot[b++];
        std::pair<int, int64_t> cut;
        if (b == nb) {
            cut = {nb, 0};
        } else if (single[b]) {
            const double need = target - (double)acc;
            auto left = [&](int64_t o) { return (double)(std::min(o, GR[b]) + std::min(o, GS[b])); };
            int64_t lo = 0, hi = std::max(GR[b], GS[b]);
            while (lo < hi) {
                const int64_t mid = (lo + hi) / 2;
                if (left(mid) >= need) hi = mid; else lo = mid + 1;
            }
            if (lo > 0 && need - left(lo - 1) < left(lo) - need) lo--;
            cut = {b, lo};
        } else {  // a multi-key bucket moves whole: to the nearer side
            cut = target - (double)acc <= (double)(acc + tot[b]) - target ? std::make_pair(b, (int64_t)0)
                                                                        : std::make_pair(b + 1, (int64_t)0);
        }
        cut = std::max(cut, prev);
        cuts.push_back(cut);
        prev = cut;
    }
    return cuts;
}

// Row range [edge[d], edge[d + 1]) of one source's bucket-ordered slice goes
// to device d: cut (b, o) sits after the slice's buckets < b and, of bucket b,
// after its rows whose global occurrence (rows of bucket b on earlier sources
// + the local offset) is below o.
std::vector<int64_t> shard_edges(const std::vector<int64_t> &local, const std::vector<int64_t> &prefix,
                                 const std::vector<std::pair<int, int64_t>> &cuts) {
    const int nb = (int)local.size();
    std::vector<int64_t> before(nb + 1, 0);
    for (int b = 0; b < nb; b++) before[b + 1] = before[b] + local[b];
    std::vector<int64_t> e{0};
    for (const auto &c : cuts) {
        int64_t p = before[c.first];
        if (c.first < nb) p += std::min(std::max<int64_t>(c.second - prefix[c.first], 0), local[c.first]);
        e.push_back(p);
    }
    e.push_back(before[nb]);
    return e;
}

// ntab = 2: select -> sort -> zip join of R and S, *out / *out_rows the
// joined rows.  ntab = 1: select-free stable sort of one table, written back
// into sorted_back.  timing (may be NULL) in the reference's three buckets.
int sharded_run(int ktype, const HTab *tab, int ntab, int key2, T **out, int64_t *out_rows, int64_t *sorted_back,
                smj_timing_t *timing) {
    const int D = (int)g_devs.size();
    const double t0 = now_ms();
    std::vector<int64_t> bounds;
    std::vector<char> single;
    shard_bounds(host_splitters(tab, ntab, ktype, D), bounds, single);
    const int nspl = (int)bounds.size();
    const int NB = nspl + 1;  // partition buckets; cuts (bucket, occurrence) split them over the devices
    // counts[d][x][b]: rows of device d's slice of table x in bucket b
    std::vector<std::vector<std::vector<int64_t>>> counts(D, std::vector<std::vector<int64_t>>(2, std::vector<int64_t>(NB, 0)));
    std::vector<double> t_h2d(D, 0.0);
    auto slice = [&](int x, int d, int64_t &r0, int64_t &r1) {
        r0 = tab[x].n * d / D;
        r1 = tab[x].n * (d + 1) / D;
    };
    // 2. H2D of the slices on the copy stream; the key map, select and stable
    //    bucket partition of table x start as soon as its slice has landed (so
    //    R's partition overlaps S's copy)
    SMJ_TRY(on_devices([&](int d) -> int {
        HostDev &hd = g_devs[d];
        SMJ_TRY(hgrow(hd, B_SPL, 64 * sizeof(int64_t)));
        if (nspl) HIP_TRY(hipMemcpyAsync(hd.b[B_SPL], bounds.data(), sizeof(int64_t) * nspl, hipMemcpyHostToDevice, hd.st));
        for (int x = 0; x < ntab; x++) {
            int64_t r0, r1;
            slice(x, d, r0, r1);
            const size_t bytes = (size_t)(r1 - r0) * tab[x].cols * 8;
            SMJ_TRY(hgrow(hd, B_IN0 + x, bytes));
            SMJ_TRY(hgrow(hd, B_PART0 + x, bytes));
            if (bytes) HIP_TRY(hipMemcpyAsync(hd.b[B_IN0 + x], tab[x].rows + r0 * tab[x].cols, bytes, hipMemcpyHostToDevice, hd.cp));
            HIP_TRY(hipEventRecord(hd.in_ev[x], hd.cp));
        }
        for (int x = 0; x < ntab; x++) {
            int64_t r0, r1;
            slice(x, d, r0, r1);
            if (x == ntab - 1) {  // the CPU-GPU bucket ends when the last slice has landed
                HIP_TRY(hipEventSynchronize(hd.in_ev[x]));
                t_h2d[d] = now_ms();
            }
            if (r1 == r0) continue;
            HIP_TRY(hipStreamWaitEvent(hd.st, hd.in_ev[x], 0));
            if (ktype != SMJ_KEY_INT64)
                HIP_TRY(launch_key_map((const int64_t *)hd.b[B_IN0 + x], (int64_t *)hd.b[B_IN0 + x], r1 - r0,
                                       tab[x].cols, map_mask(tab[x].key, tab[x].sel_col), ktype, 0, hd.st));
            SMJ_TRY(smj_dev_partition((const T *)hd.b[B_IN0 + x], r1 - r0, tab[x].cols, ntab > 1 ? 1 : 0,
                                      tab[x].sel_col, tab[x].sel_map, tab[x].key, (const T *)hd.b[B_SPL], nspl,
                                      (T *)hd.b[B_PART0 + x], counts[d][x].data(), hd.st));
        }
        return SMJ_OK;
    }));
    const double t_h2d_end = *std::max_element(t_h2d.begin(), t_h2d.end());
    // 3. the cuts over the global counts; edges[s][x][d]: device d takes rows
    //    [edges[d], edges[d + 1]) of source s's partitioned slice of table x
    std::vector<int64_t> G[2] = {std::vector<int64_t>(NB, 0), std::vector<int64_t>(NB, 0)};
    for (int d = 0; d < D; d++)
        for (int x = 0; x < ntab; x++)
            for (int b = 0; b < NB; b++) G[x][b] += counts[d][x][b];
    const auto cuts = shard_cuts(G[0], G[1], single, D);
    std::vector<std::vector<std::vector<int64_t>>> edges(D, std::vector<std::vector<int64_t>>(2));
    for (int x = 0; x < ntab; x++) {
        std::vector<int64_t> prefix(NB, 0);
        for (int s = 0; s < D; s++) {
            edges[s][x] = shard_edges(counts[s][x], prefix, cuts);
            for (int b = 0; b < NB; b++) prefix[b] += counts[s][x][b];
        }
    }
    // 4. device d pulls its range from every source at once (one stream per
    //    source: the xGMI links run in parallel), placed in source order so
    //    that equal keys keep their input order; then the pipeline
    std::vector<int64_t> J(D, 0), M(D, 0);
    const int tc = ntab > 1 ? tab[0].cols + tab[1].cols - 1 : 1;
    g_shard_n = std::min(D, 64);
    SMJ_TRY(on_devices([&](int d) -> int {
        HostDev &hd = g_devs[d];
        int64_t rows[2] = {0, 0};
        for (int x = 0; x < ntab; x++) {
            for (int s = 0; s < D; s++) rows[x] += edges[s][x][d + 1] - edges[s][x][d];
            SMJ_TRY(hgrow(hd, B_RECV0 + x, (size_t)rows[x] * tab[x].cols * 8));
            SMJ_TRY(hgrow(hd, B_OUT0 + x, (size_t)rows[x] * tab[x].cols * 8));
        }
        if (d < 64) g_shard_rows[d] = rows[0] + (ntab > 1 ? rows[1] : 0);
        int64_t at[2] = {0, 0};
        for (int s = 0; s < D; s++) {
            hipStream_t q = D > 1 ? hd.px[s] : hd.st;
            for (int x = 0; x < ntab; x++) {
                const int64_t c = edges[s][x][d + 1] - edges[s][x][d];
                if (c == 0) continue;
                const size_t W = (size_t)tab[x].cols * 8;
                char *dst = (char *)hd.b[B_RECV0 + x] + at[x] * W;
                const char *src = (const char *)g_devs[s].b[B_PART0 + x] + edges[s][x][d] * W;
                if (g_devs[s].phys == hd.phys)
                    HIP_TRY(hipMemcpyAsync(dst, src, c * W, hipMemcpyDeviceToDevice, q));
                else
                    HIP_TRY(hipMemcpyPeerAsync(dst, hd.phys, src, g_devs[s].phys, c * W, q));
                at[x] += c;
            }
            if (D > 1) {
                HIP_TRY(hipEventRecord(hd.pe[s], q));
                HIP_TRY(hipStreamWaitEvent(hd.st, hd.pe[s], 0));
            }
        }
        if (ntab == 1) {
            if (rows[0]) {
                SMJ_TRY(smj_dev_select_sort((const T *)hd.b[B_RECV0], rows[0], tab[0].cols, 0, 0, 0, tab[0].key, 0,
                                            (T *)hd.b[B_OUT0], &M[d], hd.st));
                if (ktype != SMJ_KEY_INT64)
                    HIP_TRY(launch_key_map((const int64_t *)hd.b[B_OUT0], (int64_t *)hd.b[B_OUT0], M[d], tab[0].cols,
                                           map_mask(tab[0].key, tab[0].key), ktype, 1, hd.st));
            }
            HIP_TRY(hipStreamSynchronize(hd.st));
            return SMJ_OK;
        }
        SMJ_TRY(hgrow(hd, B_J, (size_t)std::max<int64_t>(1, std::min(rows[0], rows[1])) * tc * 8));
        if (rows[0] && rows[1]) {
            int64_t h[3] = {0, 0, 0};
            SMJ_TRY(smj_dev_sort_merge_join((const T *)hd.b[B_RECV0], rows[0], tab[0].cols, 0, 0, 0, tab[0].key,
                                            (const T *)hd.b[B_RECV1], rows[1], tab[1].cols, 0, 0, 0, tab[1].key,
                                            (T *)hd.b[B_OUT0], (T *)hd.b[B_OUT1], (T *)hd.b[B_J], h, hd.st));
            J[d] = h[2];
            if (ktype != SMJ_KEY_INT64 && J[d]) {  // map the key / select columns of the joined rows back
                uint32_t mO = map_mask(tab[0].key, tab[0].sel_col);
                const int sc2 = tab[1].sel_col, k2 = tab[1].key;
                if (sc2 != k2) mO |= 1u << (tab[0].cols + (sc2 < k2 ? sc2 : sc2 - 1));
                HIP_TRY(launch_key_map((const int64_t *)hd.b[B_J], (int64_t *)hd.b[B_J], J[d], tc, mO, ktype, 1, hd.st));
            }
        }
        HIP_TRY(hipStreamSynchronize(hd.st));
        return SMJ_OK;
    }));
    const double t_gpu_end = now_ms();
    // 5. results to the host, in device (= key range) order
    std::vector<int64_t> at(D + 1, 0);
    T *res = nullptr;
    if (ntab > 1) {
        for (int d = 0; d < D; d++) at[d + 1] = at[d] + J[d];
        res = (T *)result_alloc((size_t)at[D] * tc * sizeof(T));
        if (!res) return SMJ_ERR_NOMEM;
    } else {
        for (int d = 0; d < D; d++) at[d + 1] = at[d] + M[d];
    }
    const int rc = on_devices([&](int d) -> int {
        HostDev &hd = g_devs[d];
        const int64_t n = ntab > 1 ? J[d] : M[d];
        if (n == 0) return SMJ_OK;
        const size_t W = (size_t)(ntab > 1 ? tc : tab[0].cols) * 8;
        void *dst = ntab > 1 ? (void *)((char *)res + at[d] * W) : (void *)((char *)sorted_back + at[d] * W);
        return d2h_result(hd, dst, hd.b[ntab > 1 ? B_J : B_OUT0], n * W);
    });
    if (rc != SMJ_OK) {
        free(res);
        return rc;
    }
    if (timing) {
        timing->cpu_gpu_ms = t_h2d_end - t0;
        timing->gpu_ms = t_gpu_end - t_h2d_end;
        timing->gpu_cpu_ms = now_ms() - t_gpu_end;
    }
    if (ntab > 1) {
        *out = res;
        *out_rows = at[D];
    }
    return SMJ_OK;
}
}  // namespace

extern "C" int smj_sort(const dpu_block_t *bl, T *rows, int key_col) {
    SMJ_TRY(need_init());
    SMJ_TRY(check_block(bl, rows));
    if (key_col < 0 || key_col >= bl->col_num) return SMJ_ERR_INVALID;
    if (bl->row_num < 2) return SMJ_OK;
    if (g_devs.size() > 1 && bl->col_num <= 8) {
        const HTab t{rows, bl->row_num, bl->col_num, key_col, key_col, INT64_MIN};
        return sharded_run(SMJ_KEY_INT64, &t, 1, 0, nullptr, nullptr, rows, nullptr);
    }
    HostDev &hd = g_devs[0];
    const size_t bytes = (size_t)bl->row_num * bl->col_num * sizeof(T);
    SMJ_TRY(hgrow(hd, B_IN0, bytes));
    SMJ_TRY(hgrow(hd, B_OUT0, bytes));
    hipStream_t s = hd.st;
    HIP_TRY(hipMemcpyAsync(hd.b[B_IN0], rows, bytes, hipMemcpyHostToDevice, s));
    int64_t m = 0;
    SMJ_TRY(smj_dev_select_sort((T *)hd.b[B_IN0], bl->row_num, bl->col_num, 0, 0, 0, key_col, 0, (T *)hd.b[B_OUT0],
                                &m, s));
    HIP_TRY(hipMemcpyAsync(rows, hd.b[B_OUT0], bytes, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SMJ_OK;
}

extern "C" int smj_sort_merge_join(const dpu_block_t *r, const T *R, const dpu_block_t *s_, const T *S,
                                   int select_col1, T select_val1, int select_col2, T select_val2, int key1,
                                   int key2, T **out, int64_t *out_rows, smj_timing_t *timing) {
    return smj_sort_merge_join_typed(SMJ_KEY_INT64, r, R, s_, S, select_col1, (uint64_t)select_val1, select_col2,
                                     (uint64_t)select_val2, key1, key2, (void **)out, out_rows, timing);
}

extern "C" int smj_sort_merge_join_typed(int key_type, const dpu_block_t *r, const void *R, const dpu_block_t *s_,
                                         const void *S, int select_col1, uint64_t sel_bits1, int select_col2,
                                         uint64_t sel_bits2, int key1, int key2, void **out, int64_t *out_rows,
                                         smj_timing_t *timing) {
    SMJ_TRY(need_init());
    SMJ_TRY(check_block(r, (const T *)R));
    SMJ_TRY(check_block(s_, (const T *)S));
    if (!out || !out_rows) return SMJ_ERR_INVALID;
    if (key_type != SMJ_KEY_INT64 && key_type != SMJ_KEY_UINT64 && key_type != SMJ_KEY_DOUBLE) return SMJ_ERR_INVALID;
    const int c1 = r->col_num, c2 = s_->col_num, tc = c1 + c2 - 1;
    if (key1 < 0 || key1 >= c1 || key2 < 0 || key2 >= c2 || select_col1 < 0 || select_col1 >= c1 ||
        select_col2 < 0 || select_col2 >= c2)
        return SMJ_ERR_INVALID;
    const int64_t nr = r->row_num, ns = s_->row_num;
    if (g_devs.size() > 1 && c1 <= 8 && c2 <= 8) {
        const HTab t[2] = {{(const int64_t *)R, nr, c1, select_col1, key1, key_map_host((int64_t)sel_bits1, key_type)},
                           {(const int64_t *)S, ns, c2, select_col2, key2, key_map_host((int64_t)sel_bits2, key_type)}};
        return sharded_run(key_type, t, 2, key2, (T **)out, out_rows, nullptr, timing);
    }
    HostDev &hd = g_devs[0];
    hipStream_t st = hd.st;
    hipEvent_t ev[3];
    for (auto &e : ev) HIP_TRY(hipEventCreate(&e));
    struct EvFree {
        hipEvent_t *e;
        ~EvFree() {
            for (int i = 0; i < 3; i++) hipEventDestroy(e[i]);
        }
    } evf{ev};
    SMJ_TRY(hgrow(hd, B_IN0, (size_t)nr * c1 * 8));
    SMJ_TRY(hgrow(hd, B_IN1, (size_t)ns * c2 * 8));
    SMJ_TRY(hgrow(hd, B_OUT0, (size_t)nr * c1 * 8));
    SMJ_TRY(hgrow(hd, B_OUT1, (size_t)ns * c2 * 8));
    SMJ_TRY(hgrow(hd, B_J, (size_t)std::max<int64_t>(1, std::min(nr, ns)) * tc * 8));
    HIP_TRY(hipEventRecord(ev[0], st));
    int64_t rows[3] = {0, 0, 0};
    // staged: the tables cross PCIe in chunks while part_a already runs on the
    // landed ones (SMJ_STAGED=0: one copy per table, then the pipeline)
    static const bool staged_on = !getenv("SMJ_STAGED") || atoi(getenv("SMJ_STAGED")) != 0;
    int rc = SMJ_ERR_UNSUPPORTED;
    if (staged_on && key_type == SMJ_KEY_INT64) {
        HIP_TRY(hipStreamWaitEvent(hd.cp, ev[0], 0));
        rc = msd_staged_sort_merge_join((const int64_t *)R, nr, c1, select_col1, (int64_t)sel_bits1, key1,
                                        (const int64_t *)S, ns, c2, select_col2, (int64_t)sel_bits2, key2,
                                        (int64_t *)hd.b[B_IN0], (int64_t *)hd.b[B_IN1], (int64_t *)hd.b[B_OUT0],
                                        (int64_t *)hd.b[B_OUT1], (int64_t *)hd.b[B_J], rows, st, hd.cp, ev[1]);
        if (rc != SMJ_OK && rc != SMJ_ERR_UNSUPPORTED) return rc;
    }
    if (rc == SMJ_ERR_UNSUPPORTED) {
        if (nr) HIP_TRY(hipMemcpyAsync(hd.b[B_IN0], R, (size_t)nr * c1 * 8, hipMemcpyHostToDevice, st));
        if (ns) HIP_TRY(hipMemcpyAsync(hd.b[B_IN1], S, (size_t)ns * c2 * 8, hipMemcpyHostToDevice, st));
        HIP_TRY(hipEventRecord(ev[1], st));
        SMJ_TRY(smj_dev_sort_merge_join_typed(key_type, hd.b[B_IN0], nr, c1, 1, select_col1, sel_bits1, key1,
                                              hd.b[B_IN1], ns, c2, 1, select_col2, sel_bits2, key2, hd.b[B_OUT0],
                                              hd.b[B_OUT1], hd.b[B_J], rows, st));
    }
    const int64_t j = rows[2];
    HIP_TRY(hipEventRecord(ev[2], st));
    HIP_TRY(hipEventSynchronize(ev[2]));
    const double t2 = now_ms();
    T *res = (T *)result_alloc((size_t)j * tc * sizeof(T));
    if (!res) return SMJ_ERR_NOMEM;
    const int rc2 = d2h_result(hd, res, hd.b[B_J], (size_t)j * tc * 8);
    if (rc2 != SMJ_OK) {
        free(res);
        return rc2;
    }
    if (timing) {
        timing->cpu_gpu_ms = ev_ms(ev[0], ev[1]);
        timing->gpu_ms = ev_ms(ev[1], ev[2]);
        timing->gpu_cpu_ms = now_ms() - t2;
    }
    *out = res;
    *out_rows = j;
    return SMJ_OK;
}
