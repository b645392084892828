// smj_api.hip -- the C-ABI of libsmj_hip.so (declared in include/smj.h).
//
// Host orchestration of the hot-path kernels: per-device scratch, the
// select+sort plan, pass scheduling, the merge-path join, and the
// host-pointer entry points that replace the reference's DPU calls
// (app.c: dpu_alloc/dpu_load/dpu_push_xfer/dpu_launch/dpu_free).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <map>
#include <unordered_map>
#include <memory>
#include <new>
#include <mutex>
#include <string>
#include <vector>

#include "smj.h"
#include "smj_internal.h"

using namespace smj;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
extern "C" const char *smj_strerror(int code) {
    switch (code) {
    case SMJ_OK: return "ok";
    case SMJ_ERR_INVALID: return "invalid argument";
    case SMJ_ERR_HIP: return "HIP runtime error";
    case SMJ_ERR_NOMEM: return "out of memory";
    case SMJ_ERR_NODEVICE: return "no usable gfx950 device";
    case SMJ_ERR_TOO_LARGE: return "table too large (rows >= 2^31 or cols > 1024)";
    case SMJ_ERR_TIMEOUT: return "look-back wait timed out in a kernel";
    case SMJ_ERR_UNSUPPORTED: return "unsupported";
    default: return "unknown error";
    }
}

extern "C" const char *smj_version(void) { return "smj-mi355x 0.1 (gfx950, radix10 onesweep, merge-path join)"; }

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

// ---------------------------------------------------------------------------
// profiling: hipEvents around every launch, on the launch's stream
// ---------------------------------------------------------------------------
namespace {
struct ProfRec {
    const char *name;
    hipEvent_t a, b;
    double bytes;
    int dev;  // the device the events were created on (the pool they return to)
};
bool g_prof_on = false;
std::vector<ProfRec> g_prof;
std::map<int, std::vector<hipEvent_t>> g_event_pool;  // per device: an event records only on its own device's streams
std::mutex g_mu;  // scratch maps and profiler records (the host API drives devices from worker threads)
thread_local int t_slot = -1;  // smj::set_scratch_slot
thread_local int t_msd_var = 0;  // msd_large: the MsdScratch set of the part in flight (0 / 1)

hipEvent_t take_event(int dev) {
    std::vector<hipEvent_t> &pool = g_event_pool[dev];
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;  // on the calling thread's current device = dev
    return e;
}

struct ProfScope {
    ProfRec rec{};
    hipStream_t s;
    bool on;
    ProfScope(const char *name, double bytes, hipStream_t st) : s(st), on(g_prof_on) {
        if (!on) return;
        rec.name = name;
        rec.bytes = bytes;
        if (hipGetDevice(&rec.dev) != hipSuccess) {
            on = false;
            return;
        }
        {
            std::lock_guard<std::mutex> lk(g_mu);
            rec.a = take_event(rec.dev);
            rec.b = take_event(rec.dev);
        }
        if (rec.a && hipEventRecord(rec.a, s) != hipSuccess) on = false;
    }
    ~ProfScope() {
        if (!on || !rec.a || !rec.b) return;
        if (hipEventRecord(rec.b, s) != hipSuccess) return;  // a missing record is dropped, never misread
        std::lock_guard<std::mutex> lk(g_mu);
        g_prof.push_back(rec);
    }
};
}  // namespace

extern "C" void smj_prof_enable(int on) { g_prof_on = on != 0; }

// Diagnostic only (not part of smj.h): chunk_scatter phase cycles collected
// under SMJ_DEBUG_PASS bit 3; out[0..6] cycles per phase, out[7] tiles.
extern "C" int smj_debug_phase_cycles(unsigned long long *out16) {
    hipDeviceSynchronize();
    return read_phase_cycles(out16) == hipSuccess ? SMJ_OK : SMJ_ERR_HIP;
}

// Diagnostic only (not part of smj.h): msd_final phase cycles collected under
// SMJ_DEBUG_MSD=1 (24 words): out[k] cycles of staged-final phase k summed
// over workgroups, out[9] groups, out[10..15] its sort / issue sub-phases,
// out[16..21] part_b phases, out[23] part_b tiles.
extern "C" int smj_debug_msd_phases(unsigned long long *out24) {
    hipDeviceSynchronize();
    return read_msd_phases(out24) == hipSuccess ? SMJ_OK : SMJ_ERR_HIP;
}

static std::string prof_json() {
    struct Agg { long launches = 0; double ms = 0, bytes = 0; };
    std::map<std::string, Agg> agg;
    for (auto &r : g_prof) {
        hipEventSynchronize(r.b);
        float ms = 0;
        hipEventElapsedTime(&ms, r.a, r.b);
        Agg &a = agg[r.name];
        a.launches++;
        a.ms += ms;
        a.bytes += r.bytes;
    }
    std::string out = "{";
    bool first = true;
    for (auto &kv : agg) {
        char tmp[256];
        snprintf(tmp, sizeof tmp, "%s\"%s\": {\"launches\": %ld, \"ms\": %.6f, \"bytes\": %.0f}",
                 first ? "" : ", ", kv.first.c_str(), kv.second.launches, kv.second.ms, kv.second.bytes);
        out += tmp;
        first = false;
    }
    return out + "}";
}

// Returns SMJ_OK after filling buf (and resetting the records), or the
// buffer size needed (records kept) when buf is NULL / too small.
extern "C" int smj_prof_report(char *buf, size_t buflen) {
    std::lock_guard<std::mutex> lk(g_mu);
    const std::string out = prof_json();
    if (!buf || buflen < out.size() + 1) return (int)out.size() + 1;
    memcpy(buf, out.c_str(), out.size() + 1);
    for (auto &r : g_prof) {
        g_event_pool[r.dev].push_back(r.a);
        g_event_pool[r.dev].push_back(r.b);
    }
    g_prof.clear();
    return SMJ_OK;
}

// ---------------------------------------------------------------------------
// per-device scratch (grow-only)
// ---------------------------------------------------------------------------
namespace {
struct DevScratch {
    int dev = -1;
    void *tmp = nullptr;  size_t tmp_bytes = 0;     // ping-pong rows
    void *status = nullptr; size_t status_bytes = 0; // pass chunk tables / join look-back words
    uint32_t *segsum = nullptr;                      // kScanSegs * kRadix
    int64_t *trash = nullptr;                        // kSortThreads * 16 int64 write sink
    void *apart = nullptr; size_t apart_bytes = 0;   // merge-path partition
    uint32_t *hist = nullptr;                        // kNumPos * kRadix
    SortPlan *plan = nullptr;                        // device
    Counters *ctr = nullptr;                         // device, 8 slots
    int64_t *dcount = nullptr;                       // device scratch int64 x 256
    SortPlan *h_plan = nullptr;                      // pinned
    int64_t *h_small = nullptr;                      // pinned, 256 int64
    void *rst = nullptr; size_t c_rst = 0;           // smj_dev_partition_regions: look-back words
    int64_t *rwords = nullptr;                       // its region words (128) + flags (u32 x 4)
};
std::map<int, DevScratch> g_scratch;

// Scratch is per device, or per slot when a host worker thread set one: the
// multi-device host API may run several pipelines on one physical device
// (virtual devices, smj_init_devices) and they must not share buffers.
int scratch_key(int *dev) {
    if (hipGetDevice(dev) != hipSuccess) return -1;
    return t_slot >= 0 ? (1 << 16) + t_slot : *dev;
}

// pinned host twin of grow() (staging of small device <-> host lists: a
// pageable copy runs through the runtime's bounce buffer and blocks)
int grow_host(void **p, size_t *cap, size_t need) {
    if (need <= *cap) return SMJ_OK;
    if (*p) HIP_TRY(hipHostFree(*p));
    *p = nullptr;
    *cap = 0;
    size_t n = std::max(need, (size_t)1 << 20);
    HIP_TRY(hipHostMalloc(p, n, hipHostMallocDefault));
    *cap = n;
    return SMJ_OK;
}

// smj_debug_fail_front: the next grow() of this thread fails with
// SMJ_ERR_NOMEM (the partitioned mode's no-room path)
thread_local bool t_fail_grow = false;

int grow(void **p, size_t *cap, size_t need) {
    if (t_fail_grow) {
        t_fail_grow = false;
        return SMJ_ERR_NOMEM;
    }
    if (need <= *cap) return SMJ_OK;
    if (*p) HIP_TRY(dev_free(*p));
    *p = nullptr;
    *cap = 0;
    size_t n = std::max(need, (size_t)1 << 20);
    HIP_TRY(dev_alloc(p, n));
    *cap = n;
    return SMJ_OK;
}

int scratch(DevScratch **out) {
    int dev = 0;
    const int key = scratch_key(&dev);
    if (key < 0) return SMJ_ERR_HIP;
    std::lock_guard<std::mutex> lk(g_mu);
    DevScratch &s = g_scratch[key];
    if (s.dev < 0) {
        HIP_TRY(dev_alloc(&s.hist, sizeof(uint32_t) * kNumPos * kRadix));
        HIP_TRY(dev_alloc(&s.plan, sizeof(SortPlan)));
        HIP_TRY(dev_alloc(&s.ctr, sizeof(Counters) * 8));
        HIP_TRY(hipMemset(s.ctr, 0, sizeof(Counters) * 8));
        HIP_TRY(dev_alloc(&s.dcount, sizeof(int64_t) * 256));
        HIP_TRY(dev_alloc(&s.segsum, sizeof(uint32_t) * kScanSegs * kRadix));
        HIP_TRY(dev_alloc(&s.trash, sizeof(int64_t) * kSortThreads * 16));
        HIP_TRY(hipHostMalloc(&s.h_plan, sizeof(SortPlan), hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&s.h_small, sizeof(int64_t) * 256, hipHostMallocDefault));
        s.dev = dev;  // only once every buffer exists
    }
    *out = &s;
    return SMJ_OK;
}

int check_table(int64_t n, int cols, int col_a, int col_b) {
    if (n < 0 || cols < 1 || col_a < 0 || col_a >= cols || col_b < 0 || col_b >= cols)
        return SMJ_ERR_INVALID;
    if (cols > SMJ_MAX_COLS || n >= SMJ_MAX_ROWS) return SMJ_ERR_TOO_LARGE;
    return SMJ_OK;
}

// Row kernels are instantiated for 1..8 columns; wider tables take the
// index-sort path ((key, row id) pairs through the same kernels, then row
// gathers) wherever an entry point offers it, else SMJ_ERR_UNSUPPORTED.
constexpr int kDirectCols = 8;
int direct_only(int cols) { return cols > kDirectCols ? SMJ_ERR_UNSUPPORTED : SMJ_OK; }

// wide-row forms of the standalone select / merge / join (index-sort path, below)
int idx_select(const T *in, int64_t n, int cols, int sel_col, T sel_val, T *out, int64_t *out_rows, hipStream_t s);
int idx_merge(const T *a, int64_t na, const T *b, int64_t nb, int cols, int key_col, T *out, hipStream_t s);
int idx_join(const T *R, int64_t nr, int c1, const T *S, int64_t ns, int c2, int key1, int key2, T *out,
             int64_t *d_out_rows, int64_t *h_out_rows, hipStream_t s);
}  // namespace

// One scatter pass (chunk_hist -> chunk_scan -> chunk_scatter).  rows_out:
// rows the pass writes (for the profiler's algorithmic byte count).
static int run_pass(DevScratch *sc, const PassSpec &ps, const uint32_t *base, Counters *ctr, bool have_table,
                    int64_t rows_out, hipStream_t s) {
    static const char *names[3][3] = {{"radix_hist", "radix_scan", "radix_scatter"},
                                      {"select_hist", "select_scan", "select_scatter"},
                                      {"partition_hist", "partition_scan", "partition_scatter"}};
    const int k = ps.kind == DIGIT_RADIX ? 0 : ps.kind == DIGIT_ZERO ? 1 : 2;
    const double rowb = 8.0 * ps.cols;
    const_cast<PassSpec &>(ps).trash = sc->trash;
    const size_t tbytes = (size_t)pass_chunks(ps) * pass_radix(ps) * sizeof(uint32_t);
    SMJ_TRY(grow(&sc->status, &sc->status_bytes, tbytes));
    uint32_t *table = (uint32_t *)sc->status;
    if (!have_table) {
        ProfScope p1(names[k][0], rowb * ps.nsrc, s);
        HIP_TRY(launch_chunk_hist(ps, table, s));
    }
    {
        ProfScope p2(names[k][1], 0, s);
        HIP_TRY(launch_chunk_scan(ps, table, sc->segsum, base, s));
    }
    ProfScope p3(names[k][2], rowb * (ps.nsrc + rows_out), s);
    HIP_TRY(launch_chunk_scatter(ps, table, ctr, s));
    return SMJ_OK;
}

// ---------------------------------------------------------------------------
// select + sort
// ---------------------------------------------------------------------------
static int lsd_select_sort(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val,
                           int key_col, uint64_t key_base, T *out, int64_t *out_rows, hipStream_t s) {
    SMJ_TRY(check_table(n, cols, use_select ? sel_col : 0, key_col));
    SMJ_TRY(direct_only(cols));
    if (!out_rows) return SMJ_ERR_INVALID;
    *out_rows = 0;
    if (n == 0) return SMJ_OK;
    if (!in || !out || in == out) return SMJ_ERR_INVALID;
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    const double rowb = 8.0 * cols;

    HIP_TRY(hipMemsetAsync(sc->hist, 0, sizeof(uint32_t) * kNumPos * kRadix, s));
    HIP_TRY(hipMemsetAsync(&sc->ctr[0], 0, sizeof(Counters), s));
    // chunk table of the first pass (digit 0), filled by hist_radix
    SMJ_TRY(grow(&sc->status, &sc->status_bytes, (size_t)((n + chunk_rows(cols) - 1) / chunk_rows(cols)) * kRadix * 4));
    {
        ProfScope ps("hist_radix", rowb * n, s);
        HIP_TRY(launch_hist_radix(in, n, cols, use_select, sel_col, sel_val, key_col, key_base, sc->hist,
                                  (uint32_t *)sc->status, s));
    }
    {
        ProfScope ps("plan", 0, s);
        HIP_TRY(launch_plan(sc->hist, sc->plan, s));
    }
    HIP_TRY(hipMemcpyAsync(sc->h_plan, sc->plan, sizeof(SortPlan), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const SortPlan plan = *sc->h_plan;
    const int64_t m = plan.m;
    if (m == 0) return SMJ_OK;
    const int P = plan.npasses;
    if (P > 1) SMJ_TRY(grow(&sc->tmp, &sc->tmp_bytes, (size_t)m * cols * 8));
    const T *src = in;
    for (int k = 0; k < P; k++) {
        T *dst = ((P - 1 - k) % 2 == 0) ? out : (T *)sc->tmp;
        PassSpec ps{};
        ps.src = src;
        ps.nsrc = k == 0 ? n : m;
        ps.dst = dst;
        ps.cols = cols;
        ps.use_select = k == 0 ? use_select : 0;
        ps.sel_col = sel_col;
        ps.key_col = key_col;
        ps.sel_val = sel_val;
        ps.kind = DIGIT_RADIX;
        ps.key_base = key_base;
        ps.shift = plan.pos[k] * kRadixBits;
        // pass 0 on digit 0 reuses the chunk counts hist_radix already wrote
        SMJ_TRY(run_pass(sc, ps, sc->hist + plan.pos[k] * kRadix, &sc->ctr[0], k == 0 && plan.pos[0] == 0, m, s));
        src = dst;
    }
    *out_rows = m;
    return SMJ_OK;
}

extern "C" int smj_dev_select_sort_lsd(const T *in, int64_t n_rows, int col_num, int use_select, int select_col,
                                       T select_val, int key_col, uint64_t key_base, T *out, int64_t *out_rows,
                                       void *stream) {
    return lsd_select_sort(in, n_rows, col_num, use_select, select_col, select_val, key_col, key_base, out,
                           out_rows, (hipStream_t)stream);
}

extern "C" int smj_dev_select(const T *in, int64_t n, int cols, int sel_col, T sel_val, T *out,
                              int64_t *out_rows, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    SMJ_TRY(check_table(n, cols, sel_col, 0));
    if (!out_rows) return SMJ_ERR_INVALID;
    *out_rows = 0;
    if (n == 0) return SMJ_OK;
    if (!in || !out || in == out) return SMJ_ERR_INVALID;
    if (cols > kDirectCols) return idx_select(in, n, cols, sel_col, sel_val, out, out_rows, s);
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    HIP_TRY(hipMemsetAsync(&sc->ctr[1], 0, sizeof(Counters), s));
    PassSpec ps{};
    ps.src = in;
    ps.nsrc = n;
    ps.dst = out;
    ps.cols = cols;
    ps.use_select = 1;
    ps.sel_col = sel_col;
    ps.sel_val = sel_val;
    ps.kind = DIGIT_ZERO;
    SMJ_TRY(run_pass(sc, ps, nullptr, &sc->ctr[1], false, n, s));
    Counters c;
    HIP_TRY(hipMemcpyAsync(&c, &sc->ctr[1], sizeof(Counters), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *out_rows = c.count;
    return SMJ_OK;
}

// ---------------------------------------------------------------------------
// merge and join
// ---------------------------------------------------------------------------
extern "C" int smj_dev_merge(const T *a, int64_t na, const T *b, int64_t nb, int cols, int key_col, T *out,
                             void *stream) {
    hipStream_t s = (hipStream_t)stream;
    SMJ_TRY(check_table(na, cols, key_col, key_col));
    SMJ_TRY(check_table(nb, cols, key_col, key_col));
    if (na + nb == 0) return SMJ_OK;
    if (!out || (na && !a) || (nb && !b)) return SMJ_ERR_INVALID;
    if (cols > kDirectCols) return idx_merge(a, na, b, nb, cols, key_col, out, s);
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    const int64_t ntiles = (na + nb + kJoinTile - 1) / kJoinTile;
    SMJ_TRY(grow(&sc->apart, &sc->apart_bytes, (size_t)(ntiles + 1) * sizeof(int64_t)));
    {
        ProfScope ps("merge_partition", 0, s);
        HIP_TRY(launch_merge_partition(a, na, cols, key_col, b, nb, cols, key_col, (int64_t *)sc->apart, nullptr,
                                       ntiles, kJoinTile, s));
    }
    ProfScope ps("merge_tiles", 2.0 * 8 * cols * (na + nb), s);
    HIP_TRY(launch_merge_tiles(a, na, b, nb, cols, key_col, (const int64_t *)sc->apart, ntiles, out, s));
    return SMJ_OK;
}

extern "C" int smj_dev_join(const T *R, int64_t nr, int c1, const T *S, int64_t ns, int c2, int key1, int key2,
                            T *out, int64_t *d_out_rows, int64_t *h_out_rows, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    SMJ_TRY(check_table(nr, c1, key1, key1));
    SMJ_TRY(check_table(ns, c2, key2, key2));
    if (!d_out_rows) return SMJ_ERR_INVALID;
    if ((c1 > kDirectCols || c2 > kDirectCols) && nr > 0 && ns > 0) {
        if (!R || !S || !out) return SMJ_ERR_INVALID;
        return idx_join(R, nr, c1, S, ns, c2, key1, key2, out, d_out_rows, h_out_rows, s);
    }
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    if (nr == 0 || ns == 0) {
        HIP_TRY(hipMemsetAsync(d_out_rows, 0, sizeof(int64_t), s));
    } else {
        if (!R || !S || !out) return SMJ_ERR_INVALID;
        const int jt = join_tile_size(c1, c2);
        const int64_t ntiles = (nr + ns + jt - 1) / jt;
        const int tc = c1 + c2 - 1;
        // apart (ntiles+1) | run_start (ntiles) | offs (ntiles u32) | counts (ntiles u32); slots (nr rows)
        SMJ_TRY(grow(&sc->apart, &sc->apart_bytes, (size_t)(3 * ntiles + 2) * sizeof(int64_t)));
        SMJ_TRY(grow(&sc->tmp, &sc->tmp_bytes, (size_t)nr * tc * sizeof(int64_t)));
        int64_t *apart = (int64_t *)sc->apart;
        int64_t *run_start = apart + ntiles + 1;
        uint32_t *offs = (uint32_t *)(run_start + ntiles);
        uint32_t *counts = offs + ntiles;
        int64_t *slots = (int64_t *)sc->tmp;
        {
            ProfScope ps("join_partition", 0, s);
            HIP_TRY(launch_merge_partition(R, nr, c1, key1, S, ns, c2, key2, apart, run_start, ntiles, jt, s));
        }
        {
            ProfScope ps("join_tiles", 8.0 * (c1 * nr + c2 * ns), s);
            HIP_TRY(launch_join(R, nr, c1, key1, S, ns, c2, key2, apart, run_start, ntiles, slots, counts, offs,
                                out, d_out_rows, 0, s));
        }
        {
            ProfScope ps("join_scan", 0, s);
            HIP_TRY(launch_join(R, nr, c1, key1, S, ns, c2, key2, apart, run_start, ntiles, slots, counts, offs,
                                out, d_out_rows, 1, s));
        }
        ProfScope ps("join_compact", 0, s);
        HIP_TRY(launch_join(R, nr, c1, key1, S, ns, c2, key2, apart, run_start, ntiles, slots, counts, offs, out,
                            d_out_rows, 2, s));
    }
    if (h_out_rows) {
        HIP_TRY(hipMemcpyAsync(sc->h_small, d_out_rows, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        *h_out_rows = sc->h_small[0];
    }
    return SMJ_OK;
}

// ---------------------------------------------------------------------------
// MSD sample-sort pipeline (smj_msd.hip): select + stable sort
// of one or two tables and, for two, their zip join, in one pass structure
// ---------------------------------------------------------------------------
namespace {
struct MsdTabScratch {
    void *tempA = nullptr, *tempB = nullptr, *offsA = nullptr, *tmm = nullptr, *list = nullptr,
         *tinfo = nullptr, *offsB = nullptr, *seg = nullptr, *bk = nullptr, *fb = nullptr, *fb2 = nullptr;
    size_t c_tempA = 0, c_tempB = 0, c_offsA = 0, c_tmm = 0, c_list = 0, c_tinfo = 0, c_offsB = 0, c_seg = 0,
           c_bk = 0, c_fb = 0, c_fb2 = 0;
};
struct MsdScratch {
    int dev = -1;
    MsdTabScratch t[2];
    int64_t *spl = nullptr, *samp = nullptr;
    MsdGroup *groups = nullptr;
    uint32_t *gpart = nullptr;  // group_sum partials
    uint32_t *cpart = nullptr;  // count_scan chunk sums
    uint32_t *counts = nullptr, *offs = nullptr, *single_list = nullptr, *big_list = nullptr, *ngrp = nullptr,
             *wide_list = nullptr, *radix_list = nullptr;
    MsdPlan *plan = nullptr, *h_plan = nullptr;
    void *slots = nullptr;
    size_t c_slots = 0;
    void *work = nullptr;
    size_t c_work = 0;
    void *jb = nullptr;  // batched fallback: join rows of the oversized groups
    size_t c_jb = 0;
    void *cwork = nullptr;  // msd_compact_big work list ({dense group, chunk})
    size_t c_cwork = 0;
    int64_t n_cwork = 0;
    int64_t *d_tmp = nullptr;
    int64_t *lspl = nullptr;    // partitioned mode: the part splitters (device)
    int64_t *h_samp = nullptr;  // partitioned mode: the sampled keys (pinned)
    void *giant = nullptr, *gmap = nullptr, *gh = nullptr;  // msd_giant_*: groups, job map, job counts
    size_t c_giant = 0, c_gmap = 0, c_gh = 0;
    void *pick = nullptr, *h_pick = nullptr;  // msd_fallback: the listed groups (device, pinned host)
    size_t c_pick = 0, c_hpick = 0;
    void *h_work = nullptr;                   // msd_fallback: pinned work lists
    size_t c_hwork = 0;
    void *pst[2] = {nullptr, nullptr};  // partitioned mode: the one-pass partition's part regions per table
    size_t c_pst[2] = {0, 0};
    void *p1st = nullptr;               // its look-back words
    size_t c_p1st = 0;
    int64_t *p1d = nullptr;             // device [2][kP1Words]: oc[128], tot[64], flags[4] (u32 x 8) per table
    int64_t *p1h = nullptr;             // pinned twin
    int64_t *heavy = nullptr;           // [kBucketsA][kHeavyMax] heavy keys per bucket (msd_heavy_kernel)
    uint32_t *nheavy = nullptr;         // [kBucketsA] their count
    MsdSeg *seg = nullptr;              // [kBucketsA] segmented pass-B digits (msd_bases_kernel)
    MsdSegFind *segf = nullptr;         // [kBucketsA] their intervals (msd_runs_seg_kernel)
    uint32_t *p1c = nullptr;            // chunked partition: device [2][kP1cWords]: rows per (chunk, part), flags
    uint32_t *h_p1c = nullptr;          // pinned twin
    void *p1desc[2] = {nullptr, nullptr};  // its parts' part_a tile descriptors per table
    size_t c_p1desc[2] = {0, 0};
};
constexpr int kP1Words = 128 + 64 + 4;
constexpr int kP1cWords = 1024 * 64 + 64;  // [chunk][64] rows, then flags
std::map<int, MsdScratch> g_msd;
int64_t g_msd_stats[4] = {0, 0, 0, 0};  // last pipeline: single-key groups, LSD-fallback groups, m_R, m_S
int64_t g_msd_groups[4] = {0, 0, 0, 0};  // last pipeline: dense groups, radix-tier, wide-tier, in-LDS LSD groups
int64_t g_msd_bigdev = 0;                // last pipeline: oversized multi-key groups sorted on the device
int64_t g_msd_packb = 0;                 // last pipeline: pass-B rows packed (MsdPlan::packB)
int64_t g_msd_wstage = 0;                // last pipeline: groups the wide-span staged kernel took (MsdPlan::nwst)
int64_t g_msd_segb = 0;                  // last pipeline: buckets with a segmented pass-B digit (MsdPlan::nsegb)
struct PbLast {  // last pipeline call's part_b launches (smj_debug_part_b_time)
    MsdPartBParams p;
    int cols;
    int64_t maxB;
};
PbLast g_pb_last[2];
int g_pb_ntab = 0;
MsdFinalParams g_fin_last{};  // last pipeline call's final launch (smj_debug_final_time)

// polls of msd_group_kernel's look-back before it gives up (smj_debug_spin_limit)
uint32_t g_spin_limit = kMsdSpinLimit;

MsdBgLimits msd_bg_limits() {  // read per call: a test may change them between calls
    MsdBgLimits r{kBgMaxRows, kBgSeg};
    if (const char *e = getenv("SMJ_BG_MAX_ROWS")) r.max_rows = (uint32_t)std::max(1, atoi(e));
    if (const char *e = getenv("SMJ_BG_SEG")) r.seg = (uint32_t)std::max(1, atoi(e) / kGroupCap) * kGroupCap;
    return r;
}

int msd_scratch(MsdScratch **out) {
    int dev = 0;
    const int base = scratch_key(&dev);
    if (base < 0) return SMJ_ERR_HIP;
    const int key = base + (t_msd_var << 20);
    std::lock_guard<std::mutex> lk(g_mu);
    MsdScratch &m = g_msd[key];
    if (m.dev < 0) {
        HIP_TRY(dev_alloc(&m.spl, sizeof(int64_t) * (kSplA + 1)));
        HIP_TRY(dev_alloc(&m.samp, sizeof(int64_t) * kSampScratch));
        HIP_TRY(dev_alloc(&m.groups, sizeof(MsdGroup) * kSlots));
        HIP_TRY(dev_alloc(&m.gpart, sizeof(uint32_t) * 2 * kBucketsA * kGroupSlices * kRadB));
        HIP_TRY(dev_alloc(&m.ngrp, sizeof(uint32_t) * kOffsA));
        HIP_TRY(dev_alloc(&m.cpart, sizeof(uint32_t) * 256));
        HIP_TRY(dev_alloc(&m.counts, sizeof(uint32_t) * kSlots));
        HIP_TRY(dev_alloc(&m.offs, sizeof(uint32_t) * kSlots));
        HIP_TRY(dev_alloc(&m.single_list, sizeof(uint32_t) * kSlots));
        HIP_TRY(dev_alloc(&m.big_list, sizeof(uint32_t) * kSlots));
        HIP_TRY(dev_alloc(&m.wide_list, sizeof(uint32_t) * kSlots));
        HIP_TRY(dev_alloc(&m.radix_list, sizeof(uint32_t) * kSlots));
        HIP_TRY(dev_alloc(&m.plan, sizeof(MsdPlan)));
        HIP_TRY(dev_alloc(&m.d_tmp, sizeof(int64_t) * 8));
        HIP_TRY(dev_alloc(&m.lspl, sizeof(int64_t) * 64));
        HIP_TRY(dev_alloc(&m.p1d, sizeof(int64_t) * 2 * kP1Words));
        HIP_TRY(hipHostMalloc(&m.p1h, sizeof(int64_t) * 2 * kP1Words, hipHostMallocDefault));
        HIP_TRY(dev_alloc(&m.p1c, sizeof(uint32_t) * 2 * kP1cWords));
        HIP_TRY(dev_alloc(&m.heavy, sizeof(int64_t) * kBucketsA * kHeavyMax));
        HIP_TRY(dev_alloc(&m.nheavy, sizeof(uint32_t) * kBucketsA));
        HIP_TRY(dev_alloc(&m.seg, sizeof(MsdSeg) * kBucketsA));
        HIP_TRY(dev_alloc(&m.segf, sizeof(MsdSegFind) * kBucketsA));
        HIP_TRY(hipHostMalloc(&m.h_p1c, sizeof(uint32_t) * 2 * kP1cWords, hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&m.h_plan, sizeof(MsdPlan), hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&m.h_samp, sizeof(int64_t) * (2 * kSampleMax + 64), hipHostMallocDefault));
        m.dev = dev;  // only once every buffer exists (a failed call retries the allocation)
    }
    *out = &m;
    return SMJ_OK;
}

std::map<int, std::array<hipStream_t, 2>> g_part_streams;  // msd_large's part streams per scratch key
int g_fail_front = -1;  // smj_debug_fail_front: msd_large's front of this part fails for want of scratch
int g_seq_from = -1;    // the part from which the last partitioned call ran its parts in turn (-1: none)

void msd_free_one(MsdScratch &m) {  // also a set whose creation failed half-way (dev still -1)
    if (m.dev >= 0) hipSetDevice(m.dev);
    for (auto &t : m.t)
        for (void *p : {t.tempA, t.tempB, t.offsA, t.tmm, t.list, t.tinfo, t.offsB, t.seg, t.bk, t.fb, t.fb2})
            dev_free(p);
    for (void *p : {(void *)m.spl, (void *)m.samp, (void *)m.groups, (void *)m.gpart, (void *)m.cpart, (void *)m.ngrp, (void *)m.counts, (void *)m.offs, (void *)m.single_list,
                    (void *)m.big_list, (void *)m.wide_list, (void *)m.radix_list, (void *)m.plan, m.slots, m.work, m.jb, m.cwork, (void *)m.d_tmp,
                    (void *)m.lspl, m.giant, m.gmap, m.gh, m.pst[0], m.pst[1], m.p1st, (void *)m.p1d, m.pick,
                    (void *)m.p1c, m.p1desc[0], m.p1desc[1], (void *)m.heavy, (void *)m.nheavy, (void *)m.seg, (void *)m.segf})
        dev_free(p);
    hipHostFree(m.p1h);
    hipHostFree(m.h_p1c);
    hipHostFree(m.h_pick);
    hipHostFree(m.h_work);
    hipHostFree(m.h_plan);
    hipHostFree(m.h_samp);
    m = MsdScratch{};
}

void msd_free_all() {
    for (auto &kv : g_part_streams)
        for (hipStream_t st : kv.second) hipStreamDestroy(st);
    g_part_streams.clear();
    for (auto &kv : g_msd) msd_free_one(kv.second);
    g_msd.clear();
}

// Releases this thread's scratch set `var` on the current device (nothing of
// it may be in flight): the partitioned mode's second set when it could not
// all be had.
void msd_release_var(int var) {
    int dev = 0;
    const int base = scratch_key(&dev);
    if (base < 0) return;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_msd.find(base + (var << 20));
    if (it == g_msd.end()) return;
    msd_free_one(it->second);
    g_msd.erase(it);
    hipSetDevice(dev);
}

struct MsdIn {            // one input table of the pipeline
    const T *src;
    int64_t n;
    int cols, use_sel, sel_col, key;
    T sel_val;
    T *out;               // sorted selected rows
    const uint64_t *desc = nullptr;  // a chunked part (msd_part1c): its pass-A tiles' rows in src (MsdPartAParams::desc)
    int64_t ntiles = 0;
    int pk = 0;                      // packed input (MsdTable::pk): one word per row, cols == 2, no select
    int64_t pkk = 0, pkp = 0;
};

// Records the index of the last profiling record (to patch its byte count
// once the row counts are known).
size_t prof_last() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_prof.empty() ? (size_t)-1 : g_prof.size() - 1;
}
void prof_set_bytes(size_t i, double bytes) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_prof_on && i < g_prof.size()) g_prof[i].bytes = bytes;
}

// Oversized groups after the main pass: single-key ones stream through
// msd_single_kernel; multi-key ones (and groups whose key range does not fit
// the LDS sort word) are gathered into one buffer per table, sorted by one
// LSD sort and joined by one zip join (a fixed number of launches however
// many such groups there are: Zipf tables have thousands).
int msd_fallback(MsdScratch *ms, const MsdIn *in, int ntab, int join, const MsdFinalParams &fp, int64_t *out_j,
                 hipStream_t s, bool *redo_compact) {
    const MsdPlan &pl = *ms->h_plan;
    *redo_compact = false;
    if (pl.nsingle == 0 && pl.nbig == 0) return SMJ_OK;
    // only the listed groups come to the host (picked on the device, pinned
    // staging): the dense group array is ~10 MB per 1.5e8-row part
    const uint32_t nl = pl.nsingle + pl.nbig;
    SMJ_TRY(grow(&ms->pick, &ms->c_pick, (size_t)nl * sizeof(MsdGroup)));
    SMJ_TRY(grow_host(&ms->h_pick, &ms->c_hpick, (size_t)nl * (sizeof(MsdGroup) + 4)));
    HIP_TRY(launch_msd_pick_groups(ms->groups, ms->single_list, ms->big_list, pl.nsingle, pl.nbig,
                                   (MsdGroup *)ms->pick, s));
    MsdGroup *picked = (MsdGroup *)ms->h_pick;
    uint32_t *slots_h = (uint32_t *)(picked + nl);
    HIP_TRY(hipMemcpyAsync(picked, ms->pick, sizeof(MsdGroup) * nl, hipMemcpyDeviceToHost, s));
    if (pl.nsingle) HIP_TRY(hipMemcpyAsync(slots_h, ms->single_list, 4 * pl.nsingle, hipMemcpyDeviceToHost, s));
    if (pl.nbig) HIP_TRY(hipMemcpyAsync(slots_h + pl.nsingle, ms->big_list, 4 * pl.nbig, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // list entry i: dense slot slots_h[i], record picked[i] (singles first, then the oversized groups)
    struct Listed {
        uint32_t slot;
        const MsdGroup *g;
    };
    std::vector<Listed> singles(pl.nsingle), bigs(pl.nbig);
    for (uint32_t i = 0; i < nl; i++) (i < pl.nsingle ? singles[i] : bigs[i - pl.nsingle]) = Listed{slots_h[i], picked + i};
    // pinned work lists, packed back to back (their H2D copies need no sync)
    size_t hw_at = 0;
    auto hw_take = [&](size_t bytes) -> int {
        hw_at = (hw_at + 15) & ~(size_t)15;
        const size_t need = hw_at + bytes;
        if (need > ms->c_hwork) return SMJ_ERR_HIP;  // sized above: never
        return SMJ_OK;
    };
    {
        size_t bound = 0;  // every list below, with its alignment
        for (uint32_t i = 0; i < nl; i++) {
            const MsdGroup &g = picked[i];
            const uint32_t rows = std::max(g.nR, ntab > 1 ? g.nS : 0u);
            bound += (rows / kGroupCap + 2) * sizeof(uint2) + (rows / kCompactChunk + 2) * sizeof(uint2);
        }
        SMJ_TRY(grow_host(&ms->h_work, &ms->c_hwork, bound + 64));
    }
    if (pl.nsingle) {
        SMJ_TRY(hw_take(0));
        uint2 *work = (uint2 *)((char *)ms->h_work + hw_at);
        size_t nw = 0;
        for (const Listed &e : singles) {
            const MsdGroup &g = *e.g;
            const uint32_t rows = std::max(g.nR, ntab > 1 ? g.nS : 0u);
            if (g.pad[0] == 1) {  // a heavy key's sub-bucket: run by run, kSingleRunRows a work item
                for (uint32_t c = 0; c * kSingleRunRows < rows; c++) work[nw++] = make_uint2(e.slot, kSingleRuns | c);
                continue;
            }
            for (uint32_t c = 0; c * (uint32_t)kGroupCap < rows; c++) work[nw++] = make_uint2(e.slot, c);
        }
        hw_at += nw * sizeof(uint2);
        SMJ_TRY(grow(&ms->work, &ms->c_work, nw * sizeof(uint2)));
        HIP_TRY(hipMemcpyAsync(ms->work, work, nw * sizeof(uint2), hipMemcpyHostToDevice, s));
        double b = 0;  // rows read + written once, join rows min(nR, nS) (single key: all pair up)
        for (const Listed &e : singles) {
            const MsdGroup &g = *e.g;
            b += 2.0 * 8.0 * ((double)g.nR * in[0].cols + (ntab > 1 ? (double)g.nS * in[1].cols : 0.0));
            if (join) b += 8.0 * (in[0].cols + in[1].cols - 1) * (double)std::min(g.nR, g.nS);
        }
        ProfScope ps("msd_single", b, s);
        HIP_TRY(launch_msd_single(fp, (const uint2 *)ms->work, (int64_t)nw, s));
    }
    // oversized multi-key groups of a small key span are sorted (and joined)
    // on the device (msd_big_stage_kernel, msd_giant_*; 2-column tables),
    // launched here where the plan shows some; the rest on the host path below
    const bool two = in[0].cols == 2 && (ntab == 1 || in[1].cols == 2);
    if (pl.nbig && two) {
        // the job split's buffers (msd_giant_*), sized from this call's
        // oversized groups: a group over bg_max rows per table becomes
        // ceil(rows / seg) jobs with 2 x kStageRange residual counts each
        const MsdBgLimits bl = msd_bg_limits();
        int64_t ngiant = 0, njobs = 0;
        for (const Listed &e : bigs) {
            const MsdGroup &g = *e.g;
            const uint32_t m = std::max(g.nR, ntab > 1 ? g.nS : 0u);
            if (std::max(g.nR, g.nS) > bl.max_rows) {
                ngiant++;
                njobs += (m + bl.seg - 1) / bl.seg;
            }
        }
        SMJ_TRY(grow(&ms->giant, &ms->c_giant, (size_t)(ngiant + 1) * sizeof(uint4)));
        SMJ_TRY(grow(&ms->gmap, &ms->c_gmap, (size_t)(njobs + 1) * 4));
        SMJ_TRY(grow(&ms->gh, &ms->c_gh, (size_t)(njobs + 1) * 2 * kStageRange * 4));
        MsdFinalParams fb = fp;
        if (fp.pk_mode == 3) {  // packed pass-B rows: the unpacked copy of the oversized groups
            for (int x = 0; x < ntab; x++) fb.tab[x].tempB = fp.shadow[x];
            fb.pk_mode = -1;
        }
        fb.giant = (uint4 *)ms->giant;
        fb.gmap = (uint32_t *)ms->gmap;
        fb.gh = (uint32_t *)ms->gh;
        {
            ProfScope ps("msd_big_dev", 0, s);
            HIP_TRY(launch_msd_big(fb, s));
        }
        if (g_prof_on) {
            // algorithmic bytes of the device tiers: every row of
            // the groups they sort read and written once, plus the join rows
            // they write (the groups' counts, read back: profiling steps only)
            const size_t pi = prof_last();
            std::vector<uint32_t> cnt(std::max<uint32_t>(pl.ngroups, 1));
            HIP_TRY(hipMemcpyAsync(cnt.data(), ms->counts, 4 * (size_t)pl.ngroups, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            const int tcb = join ? in[0].cols + in[1].cols - 1 : 0;
            double b = 0;
            for (const Listed &e : bigs) {
                const MsdGroup &g = *e.g;
                if (!msd_big_on_device(g.span, g.kt[0], g.kt[1])) continue;
                b += 2.0 * 8.0 * ((double)g.nR * in[0].cols + (ntab > 1 ? (double)g.nS * in[1].cols : 0.0));
                b += 8.0 * tcb * (double)cnt[e.slot];
            }
            prof_set_bytes(pi, b);
        }
    }
    std::vector<Listed> host_bigs;
    for (const Listed &e : bigs) {
        const MsdGroup &g = *e.g;
        if (!(two && msd_big_on_device(g.span, g.kt[0], g.kt[1]))) host_bigs.push_back(e);
    }
    if (getenv("SMJ_DEBUG_BIG")) {  // size distribution of the oversized multi-key groups (rows, log2 bins)
        int64_t hist[2][33] = {}, rows[2][33] = {};
        for (const Listed &e : bigs) {
            const MsdGroup &g = *e.g;
            const uint32_t m = std::max(g.nR, g.nS);
            const int b = 31 - __builtin_clz(std::max(m, 1u)), d = g.span <= (uint32_t)kStageRange ? 0 : 1;
            hist[d][b]++;
            rows[d][b] += (int64_t)g.nR + g.nS;
        }
        for (int d = 0; d < 2; d++)
            for (int b = 0; b < 33; b++)
                if (hist[d][b])
                    fprintf(stderr, "smj big groups span%s4096 rows 2^%d: %lld groups, %lld rows\n", d ? ">" : "<=", b,
                            (long long)hist[d][b], (long long)rows[d][b]);
        int shown = 0;  // and the first few: bucket, sub-buckets, rows, key interval
        for (const Listed &e : bigs) {
            const MsdGroup &g = *e.g;
            if (shown++ >= 12) break;
            fprintf(stderr, "smj big group a=%u b=[%u,%u) nR=%u nS=%u base=%lld span=%u\n", g.a, g.b0, g.b1, g.nR, g.nS,
                    (long long)g.base, g.span);
            if (shown <= 3) {  // its bucket's digit
                MsdBucket bk;
                MsdSeg sg;
                hipMemcpy(&bk, (const MsdBucket *)ms->t[0].bk + g.a, sizeof bk, hipMemcpyDeviceToHost);
                hipMemcpy(&sg, ms->seg + g.a, sizeof sg, hipMemcpyDeviceToHost);
                fprintf(stderr, "  bucket lo=%lld L=%u one_key=%#x scale=%llu s32=%u maxspan=%u\n", (long long)bk.lo, bk.L,
                        bk.one_key, (unsigned long long)bk.scale, bk.s32, bk.maxspan);
                if (bk.one_key & kBucketSeg)
                    for (uint32_t k = 0; k < sg.nseg; k++)
                        fprintf(stderr, "  seg %u st=%lld s32=%u db=%u dn=%u sh=%u ms=%u (hi %lld)\n", k, (long long)sg.st[k],
                                sg.s32[k], seg_db(sg.pk[k]), seg_dn(sg.pk[k]), seg_sh(sg.pk[k]), sg.ms[k], (long long)sg.hi);
            }
        }
    }
    if (!host_bigs.empty()) {
        // all remaining oversized multi-key groups at once: gather (in key
        // order) -> one stable sort per table -> copy back to each group's
        // output rows; with join, one zip join of the two sorted buffers split
        // per group
        constexpr uint32_t kSeg = 4096;  // rows per copy-back work item
        std::sort(host_bigs.begin(), host_bigs.end(), [](const Listed &a, const Listed &b) { return a.slot < b.slot; });  // dense group index = key order (the list is filled by atomics)
        std::vector<uint4> gw[2], cw[2], bw;
        int64_t tot[2] = {0, 0};
        for (const Listed &e : host_bigs) {
            const uint32_t slot = e.slot;
            const MsdGroup &g = *e.g;
            const uint32_t nx[2] = {g.nR, ntab > 1 ? g.nS : 0u};
            const uint32_t ox[2] = {g.outR, g.outS};
            bw.push_back(make_uint4(slot, (uint32_t)tot[0], nx[0], nx[1]));
            for (int x = 0; x < ntab; x++) {
                for (uint32_t v = 0; v < nx[x]; v += kGroupCap)
                    gw[x].push_back(make_uint4(slot, v, (uint32_t)(tot[x] + v), 0));
                for (uint32_t v = 0; v < nx[x]; v += kSeg)
                    cw[x].push_back(make_uint4((uint32_t)(tot[x] + v), ox[x] + v, std::min(kSeg, nx[x] - v), 0));
                tot[x] += nx[x];
            }
        }
        if (tot[0] >= (int64_t)UINT32_MAX || tot[1] >= (int64_t)UINT32_MAX) return SMJ_ERR_TOO_LARGE;
        std::vector<uint4> all;
        size_t at[5];
        for (int i = 0; i < 5; i++) {
            const std::vector<uint4> &v = i < 2 ? gw[i] : i < 4 ? cw[i - 2] : bw;
            at[i] = all.size();
            all.insert(all.end(), v.begin(), v.end());
        }
        SMJ_TRY(grow(&ms->work, &ms->c_work, all.size() * sizeof(uint4)));
        const uint4 *dw = (const uint4 *)ms->work;
        HIP_TRY(hipMemcpyAsync(ms->work, all.data(), all.size() * sizeof(uint4), hipMemcpyHostToDevice, s));
        for (int x = 0; x < ntab; x++) {
            if (tot[x] == 0) continue;
            MsdTabScratch &ts = ms->t[x];
            SMJ_TRY(grow(&ts.fb, &ts.c_fb, (size_t)tot[x] * in[x].cols * 8));
            SMJ_TRY(grow(&ts.fb2, &ts.c_fb2, (size_t)tot[x] * in[x].cols * 8));
            {
                ProfScope ps("msd_big", 16.0 * in[x].cols * tot[x], s);
                MsdTab tbx = fp.tab[x];  // packed pass-B rows: the unpacked copy (oversized groups)
                if (fp.pk_mode == 3) tbx.tempB = fp.shadow[x];
                HIP_TRY(launch_msd_gather_list(tbx, ms->groups, dw + at[x], (int64_t)gw[x].size(),
                                               (int64_t *)ts.fb, s));
            }
            int64_t m = 0;
            SMJ_TRY(lsd_select_sort((const T *)ts.fb, tot[x], in[x].cols, 0, 0, 0, in[x].key, 0, (T *)ts.fb2, &m, s));
            if (m != tot[x]) return SMJ_ERR_HIP;
            ProfScope ps("msd_big", 16.0 * in[x].cols * tot[x], s);
            HIP_TRY(launch_msd_seg_copy((const int64_t *)ts.fb2, in[x].out, dw + at[2 + x], (int64_t)cw[x].size(),
                                        in[x].cols, s));
        }
        if (join) {
            const int tc = in[0].cols + in[1].cols - 1;
            SMJ_TRY(grow(&ms->jb, &ms->c_jb, (size_t)std::max<int64_t>(1, std::min(tot[0], tot[1])) * tc * 8));
            SMJ_TRY(smj_dev_join((const T *)ms->t[0].fb2, tot[0], in[0].cols, (const T *)ms->t[1].fb2, tot[1],
                                 in[1].cols, in[0].key, in[1].key, (T *)ms->jb, ms->d_tmp, nullptr, s));
            ProfScope ps("msd_big", 0, s);
            HIP_TRY(launch_msd_big_split((const int64_t *)ms->jb, ms->d_tmp, tc, (const int64_t *)ms->t[0].fb2,
                                         in[0].cols, in[0].key, dw + at[4], (int64_t)bw.size(), ms->groups,
                                         (int64_t *)ms->slots, ms->counts, s));
        }
        HIP_TRY(hipStreamSynchronize(s));  // the work list is host-owned
    }
    if (join) {  // the oversized groups' join rows are packed in chunks (msd_compact_big_kernel)
        SMJ_TRY(hw_take(0));
        uint2 *cw = (uint2 *)((char *)ms->h_work + hw_at);
        size_t nc = 0;
        for (const std::vector<Listed> *l : {&singles, &bigs})
            for (const Listed &e : *l) {
                const uint32_t m = std::min(e.g->nR, e.g->nS);
                if (m > (uint32_t)kGroupCap)
                    for (uint32_t c = 0; c * kCompactChunk < m; c++) cw[nc++] = make_uint2(e.slot, c);
            }
        hw_at += nc * sizeof(uint2);
        ms->n_cwork = (int64_t)nc;
        if (nc) {
            SMJ_TRY(grow(&ms->cwork, &ms->c_cwork, nc * sizeof(uint2)));
            HIP_TRY(hipMemcpyAsync(ms->cwork, cw, nc * sizeof(uint2), hipMemcpyHostToDevice, s));
        }
    }
    (void)out_j;
    *redo_compact = join != 0;
    return SMJ_OK;
}

// The pipeline.  h_rows[x] gets the selected row count of table x and, with
// join, h_rows[2] the joined row count.  One stream synchronisation at the
// end (plus one more round when oversized groups need the fallback).
// Staged host input (the host-pointer path): table x's
// rows are copied from host[x] into in[x].src in chunks on the copy stream,
// and part_a runs on each chunk's tiles as soon as it has landed, while the
// next chunk is in flight.  The splitter sample is gathered on the host.
struct MsdStage {
    const int64_t *host[2];
    hipStream_t copy;
    int64_t chunk_rows;  // a multiple of every pass-A tile
    hipEvent_t landed;   // recorded on the copy stream after the last chunk
};

// the samples msd_sample_gather_kernel would take, read from the host tables
void host_sample(const MsdIn *in, const MsdStage &stg, int ntab, int64_t *samp) {
    constexpr int kRun = 16, kClusters = kSampleMax / kRun;
    for (int b = 0; b < kSampleGatherBlocksH; b++) samp[2 * kSampleMax + b] = 0;
    for (int x = 0; x < 2; x++)
        for (int64_t j = 0; j < kSampleMax; j++) {
            int64_t k = INT64_MAX;
            if (x < ntab && in[x].n > 0 && j < std::min<int64_t>(in[x].n, kSampleMax)) {
                const int64_t n = in[x].n;
                const int64_t r = n <= kSampleMax ? j : std::min(n - 1, ((2 * (j / kRun) + 1) * n) / (2 * kClusters) + j % kRun);
                const int64_t *row = stg.host[x] + r * in[x].cols;
                if (!in[x].use_sel || row[in[x].sel_col] > in[x].sel_val) {
                    k = row[in[x].key];
                    samp[2 * kSampleMax + (x * kSampleMax + j) / 256]++;
                }
            }
            samp[x * kSampleMax + j] = k;
        }
}

// Combined final groups (<= kStRows rows of both tables together, the staged
// final kernel) for 2-column tables of skewed sizes (or one table): a group
// then fills with the larger table's rows instead of stopping at kGroupCap of
// them.  Balanced tables keep <= kGroupCap rows per table (the staged kernel's
// per-table layout: C3 msd_final 1.59 vs 1.70 ms combined; C5 11.6 -> 9.1 ms
// combined, profiles/r03/r03s).  SMJ_ST_COMBINED=0 / 1 forces either (A/B).
int msd_combined(const MsdIn *in, int ntab) {
    static const int force = [] {
        const char *e = getenv("SMJ_ST_COMBINED");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    for (int x = 0; x < ntab; x++)
        if (in[x].cols != 2) return 0;
    if (force >= 0) return force;
    if (ntab < 2) return 1;
    const int64_t lo = std::min(in[0].n, in[1].n), hi = std::max(in[0].n, in[1].n);
    return 2 * hi > 3 * lo ? 1 : 0;  // over 1.5 : 1
}

// The pipeline in two phases: msd_front launches sample .. final (no host
// wait), msd_back the count scan + compact, reads the plan back and runs the
// fallback tiers.  msd_large overlaps part p's back (its host round trips)
// with part p + 1's front on another stream and scratch set.
struct MsdCtx {
    MsdScratch *ms = nullptr;
    MsdFinalParams fp{};
    const MsdIn *in = nullptr;
    int ntab = 0, join = 0, tc = 1;
    size_t pa[2] = {(size_t)-1, (size_t)-1}, pb[2] = {(size_t)-1, (size_t)-1}, pf = (size_t)-1;
    bool pa_fused = false;
};

thread_local bool t_job_open = false;  // smj_dev_sort_merge_join_begin's job, until its _end
std::atomic<int> g_open_jobs{0};       // begun jobs of every thread (smj_trim refuses while one is open)

int msd_front(const MsdIn *in, int ntab, int join, int key2, hipStream_t s, const MsdStage *stg, MsdCtx *cx) {
    if (t_job_open) return SMJ_ERR_INVALID;  // a begun job owns this thread's scratch until its _end
    for (int x = 0; x < ntab; x++)  // internal callers too: a bad column index would fault on the device
        SMJ_TRY(check_table(in[x].n, in[x].cols, in[x].use_sel ? in[x].sel_col : 0, in[x].key));
    if (join && (ntab != 2 || key2 != in[1].key)) return SMJ_ERR_INVALID;
    for (int x = 0; x < ntab; x++)  // packed input: two columns, no select, contiguous (read by the sampler and part_a)
        if (in[x].pk && (in[x].cols != 2 || in[x].use_sel || in[x].desc || stg)) return SMJ_ERR_INVALID;
    MsdScratch *ms;
    SMJ_TRY(msd_scratch(&ms));
    // packed pass-B rows (MsdPlan::packB; decided on the device from the data)
    int pack_mode = msd_packb_mode();  // 0 off, 1 unskewed tables, 2 forced (tests)
    for (int x = 0; x < ntab; x++) pack_mode = in[x].cols == 2 ? pack_mode : 0;
    const bool pack_ok = pack_mode != 0;
    int T_[2] = {1, 1}, TB_[2] = {1, 1};  // pass-A / pass-B tile rows
    int64_t tilesA[2] = {0, 0}, maxB[2] = {0, 0};
    for (int x = 0; x < ntab; x++) {
        const MsdIn &t = in[x];
        MsdTabScratch &ts = ms->t[x];
        T_[x] = msd_tile_a(t.cols);
        TB_[x] = msd_tile_b(t.cols);
        tilesA[x] = t.desc ? t.ntiles : (t.n + T_[x] - 1) / T_[x];
        maxB[x] = (t.n + TB_[x] - 1) / TB_[x] + kBucketsA;  // every bucket adds <= 1 partial pass-B tile
        const size_t W = (size_t)t.cols * 8;
        // (with packed pass-B rows tempA is also the unpacked shadow of tempB: >= its rows)
        SMJ_TRY(grow(&ts.tempA, &ts.c_tempA,
                     (size_t)std::max<int64_t>({(int64_t)1, t.n, tilesA[x] * T_[x], pack_ok ? maxB[x] * TB_[x] : 0}) * W));
        SMJ_TRY(grow(&ts.tempB, &ts.c_tempB, (size_t)maxB[x] * TB_[x] * W));
        SMJ_TRY(grow(&ts.offsA, &ts.c_offsA, std::max<int64_t>(1, tilesA[x]) * kOffsARow * 4));
        SMJ_TRY(grow(&ts.tmm, &ts.c_tmm, std::max<int64_t>(1, tilesA[x]) * 16));
        SMJ_TRY(grow(&ts.list, &ts.c_list, std::max<int64_t>(1, std::min<int64_t>(tilesA[x] * kBucketsA, t.n)) * 8));
        SMJ_TRY(grow(&ts.tinfo, &ts.c_tinfo, (size_t)maxB[x] * 8));
        SMJ_TRY(grow(&ts.offsB, &ts.c_offsB, (size_t)maxB[x] * kOffsB * sizeof(uint16_t)));
        SMJ_TRY(grow(&ts.seg, &ts.c_seg, 2 * kMsdSegs * kOffsA * 4 + kMsdSegs * 4 * 16 + 2 * kOffsA * 4));
        SMJ_TRY(grow(&ts.bk, &ts.c_bk, kOffsA * sizeof(MsdBucket)));
    }
    const int tc = ntab > 1 ? in[0].cols + in[1].cols - 1 : 1;
    if (join) SMJ_TRY(grow(&ms->slots, &ms->c_slots, std::max<size_t>(1, in[0].n) * tc * 8));
    HIP_TRY(hipMemsetAsync(ms->plan, 0, sizeof(MsdPlan), s));
    auto segL = [&](int x) { return (uint32_t *)ms->t[x].seg; };
    auto segC = [&](int x) { return (uint32_t *)ms->t[x].seg + kMsdSegs * kOffsA; };
    auto segMM = [&](int x) { return (int64_t *)((uint32_t *)ms->t[x].seg + 2 * kMsdSegs * kOffsA); };
    auto segT = [&](int x, int c) {  // bucket totals (rows, runs), after the min / max partials
        return (uint32_t *)(segMM(x) + 2 * kMsdSegs * 4) + c * kOffsA;
    };
    {
        MsdSampleParams sp{};
        for (int x = 0; x < ntab; x++)
        {
            sp.tab[x] = MsdTable{in[x].src, in[x].n, in[x].cols, in[x].key, in[x].use_sel, in[x].sel_col, in[x].sel_val,
                                 in[x].desc, in[x].ntiles, T_[x]};
            sp.tab[x].pk = in[x].pk;
            sp.tab[x].pkk = in[x].pkk;
            sp.tab[x].pkp = in[x].pkp;
        }
        sp.ntab = ntab;
        sp.spl = ms->spl;
        sp.samp = ms->samp;
        sp.plan = ms->plan;
        ProfScope ps("msd_sample", 0, s);
        if (stg) {
            host_sample(in, *stg, ntab, ms->h_samp);
            HIP_TRY(hipMemcpyAsync(ms->samp, ms->h_samp, sizeof(int64_t) * (2 * kSampleMax + kSampleGatherBlocksH),
                                   hipMemcpyHostToDevice, s));
            HIP_TRY(launch_msd_sample_select(sp, s));
        } else {
            HIP_TRY(launch_msd_sample(sp, s));
        }
    }

    size_t pa[2] = {(size_t)-1, (size_t)-1};
    std::vector<hipEvent_t> chunk_ev;  // staged input: one event per landed chunk
    struct EvRelease {
        std::vector<hipEvent_t> &v;
        ~EvRelease() {
            for (auto e : v) hipEventDestroy(e);
        }
    } ev_release{chunk_ev};
    MsdPartAParams pp[2];
    for (int x = 0; x < ntab; x++) {
        pp[x] = MsdPartAParams{in[x].src, in[x].n, in[x].use_sel, in[x].sel_col, in[x].key, 0, in[x].sel_val, ms->spl,
                               (int64_t *)ms->t[x].tempA, (uint32_t *)ms->t[x].offsA, (int64_t *)ms->t[x].tmm,
                               in[x].desc, in[x].ntiles};
        pp[x].pk = in[x].pk;
        pp[x].pkk = in[x].pkk;
        pp[x].pkp = in[x].pkp;
        pp[x].nopack = pack_ok ? &ms->plan->nopack : nullptr;
    }
    if (stg && (in[0].desc || (ntab > 1 && in[1].desc))) return SMJ_ERR_INVALID;  // (staged input is contiguous)
    // both tables in one launch when nothing is staged and the widths agree (no tail between them)
    const bool pa_fused = !stg && ntab == 2 && in[0].cols == in[1].cols;
    if (pa_fused) {
        ProfScope ps("msd_part_a", 0, s);
        HIP_TRY(launch_msd_part_a2(pp[0], pp[1], in[0].cols, s));
    }
    for (int x = 0; x < ntab && !pa_fused; x++) {
        const MsdPartAParams &p = pp[x];
        if (stg) {  // copy chunk c on the copy stream; part_a of chunk c once it has landed
            const int64_t W = (int64_t)in[x].cols * 8, ch = stg->chunk_rows;
            for (int64_t r0 = 0; r0 < in[x].n; r0 += ch) {
                const int64_t r1 = std::min(in[x].n, r0 + ch);
                HIP_TRY(hipMemcpyAsync((char *)in[x].src + r0 * W, (const char *)stg->host[x] + r0 * W, (r1 - r0) * W,
                                       hipMemcpyHostToDevice, stg->copy));
                hipEvent_t e;
                HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                chunk_ev.push_back(e);
                HIP_TRY(hipEventRecord(e, stg->copy));
                if (x == ntab - 1 && r1 == in[x].n && stg->landed) HIP_TRY(hipEventRecord(stg->landed, stg->copy));
                HIP_TRY(hipStreamWaitEvent(s, e, 0));
                ProfScope ps("msd_part_a", 0, s);
                HIP_TRY(launch_msd_part_a_tiles(p, in[x].cols, r0 / T_[x], (r1 + T_[x] - 1) / T_[x], s));
            }
        } else {
            ProfScope ps("msd_part_a", 0, s);
            HIP_TRY(launch_msd_part_a(p, in[x].cols, s));
        }
        pa[x] = prof_last();
    }
    if (pa_fused) pa[0] = prof_last();
    {
        ProfScope ps("msd_runs", 0, s);
        MsdRunsArgs ra{};
        for (int x = 0; x < ntab; x++) {
            ra.offs[x] = (const uint32_t *)ms->t[x].offsA;
            ra.ntiles[x] = tilesA[x];
            ra.segL[x] = segL(x);
            ra.segC[x] = segC(x);
            ra.tmm[x] = (const int64_t *)ms->t[x].tmm;
            ra.segmm[x] = segMM(x);
            ra.T[x] = T_[x];
            ra.TB[x] = TB_[x];
            ra.bk[x] = (const MsdBucket *)ms->t[x].bk;
            ra.list[x] = (uint2 *)ms->t[x].list;
            ra.tinfo[x] = (uint2 *)ms->t[x].tinfo;
        }
        ra.ntab = ntab;
        // the segmented digit's sample scan (clustered keys; SMJ_SEG=0: the linear digit everywhere)
        const bool seg_on = !(getenv("SMJ_SEG") && atoi(getenv("SMJ_SEG")) == 0);
        if (seg_on) {
            ra.seg_samp = ms->samp;
            ra.seg_spl = ms->spl;
            ra.seg_plan = ms->plan;
            ra.segf = ms->segf;
        }
        HIP_TRY(launch_msd_runs_seg(ra, s));
        uint32_t *sa[4], *ta[4];
        for (int x = 0; x < ntab; x++) {
            sa[2 * x] = segL(x);
            sa[2 * x + 1] = segC(x);
            ta[2 * x] = segT(x, 0);
            ta[2 * x + 1] = segT(x, 1);
        }
        HIP_TRY(launch_msd_seg_scan(sa, ta, 2 * ntab, s));
        // heavy keys per bucket (a skewed sample only; SMJ_HEAVY=0 turns it off)
        const bool heavy_on = !(getenv("SMJ_HEAVY") && atoi(getenv("SMJ_HEAVY")) == 0) && in[0].cols <= kDirectCols &&
                              (ntab < 2 || in[1].cols <= kDirectCols);
        if (heavy_on) {
            MsdHeavyParams hp{};
            for (int x = 0; x < ntab; x++) {
                hp.tempA[x] = (const int64_t *)ms->t[x].tempA;
                hp.offs[x] = (const uint32_t *)ms->t[x].offsA;
                hp.ntiles[x] = tilesA[x];
                hp.tile[x] = T_[x];
                hp.cols[x] = in[x].cols;
                hp.key[x] = in[x].key;
                hp.totL[x] = segT(x, 0);
            }
            hp.spl = ms->spl;
            hp.ntab = ntab;
            hp.heavy = ms->heavy;
            hp.nheavy = ms->nheavy;
            hp.plan = ms->plan;
            ProfScope ps("msd_heavy", 0, s);
            HIP_TRY(launch_msd_heavy(hp, s));
        }
        MsdBasesParams bp{};
        bp.nheavy = heavy_on ? ms->nheavy : nullptr;
        for (int x = 0; x < ntab; x++) {
            bp.totL[x] = segT(x, 0);
            bp.totC[x] = segT(x, 1);
            bp.segmm[x] = segMM(x);
            bp.ntiles[x] = tilesA[x];
            bp.tile[x] = TB_[x];
            bp.bk[x] = (MsdBucket *)ms->t[x].bk;
        }
        bp.ntab = ntab;
        bp.full_radix = getenv("SMJ_PASSB_FULL") && atoi(getenv("SMJ_PASSB_FULL")) == 1;
        bp.combined = msd_combined(in, ntab);
        bp.spl = ms->spl;
        bp.plan = ms->plan;
        bp.pack_ok = pack_mode;
        bp.segf = seg_on ? ms->segf : nullptr;
        bp.seg = ms->seg;
        HIP_TRY(launch_msd_bases(bp, s));
        HIP_TRY(launch_msd_runs_apply(ra, s));
    }
    size_t pb[2] = {(size_t)-1, (size_t)-1};
    for (int x = 0; x < ntab; x++) {
        MsdPartBParams p{(const int64_t *)ms->t[x].tempA, (int64_t *)ms->t[x].tempB, (const uint2 *)ms->t[x].list,
                         (const uint2 *)ms->t[x].tinfo, (const MsdBucket *)ms->t[x].bk, ms->plan,
                         (uint16_t *)ms->t[x].offsB, in[x].key, x};
        p.heavy = ms->heavy;
        p.seg = ms->seg;
        {
            ProfScope ps("msd_part_b", 0, s);
            HIP_TRY(launch_msd_part_b(p, in[x].cols, maxB[x], s, pack_ok));
        }
        if (t_slot < 0) {  // diagnostics of the calling thread's last pipeline (not the host API's workers)
            g_pb_last[x] = PbLast{p, in[x].cols, maxB[x]};
            g_pb_ntab = ntab;
        }
        pb[x] = prof_last();
    }
    {
        MsdGroupParams gp{};
        for (int x = 0; x < ntab; x++) {
            gp.offs[x] = (const uint16_t *)ms->t[x].offsB;
            gp.bk[x] = (const MsdBucket *)ms->t[x].bk;
            gp.tile[x] = TB_[x];
        }
        gp.ntab = ntab;
        gp.combined = msd_combined(in, ntab);
        gp.part = ms->gpart;
        gp.ngrp = ms->ngrp;
        gp.groups = ms->groups;
        gp.counts = ms->counts;
        gp.plan = ms->plan;
        gp.single_list = ms->single_list;
        gp.big_list = ms->big_list;
        gp.spin_limit = g_spin_limit;
        gp.heavy = ms->heavy;
        gp.seg = ms->seg;
        ProfScope ps("msd_group", 0, s);
        HIP_TRY(launch_msd_group(gp, s));
    }
    MsdFinalParams fp{};
    for (int x = 0; x < ntab; x++)
        fp.tab[x] = MsdTab{(const int64_t *)ms->t[x].tempB, (const uint16_t *)ms->t[x].offsB,
                           (const MsdBucket *)ms->t[x].bk, in[x].out, TB_[x], in[x].cols, in[x].key, x,
                           maxB[x] * TB_[x]};
    fp.groups = ms->groups;
    fp.slots = (int64_t *)ms->slots;
    fp.counts = ms->counts;
    fp.plan = ms->plan;
    fp.big_list = ms->big_list;
    fp.single_list = ms->single_list;
    fp.wide_list = ms->wide_list;
    fp.radix_list = ms->radix_list;
    fp.giant = nullptr;  // the job split's buffers: sized and set by msd_fallback
    fp.gmap = nullptr;
    fp.gh = nullptr;
    const MsdBgLimits bl = msd_bg_limits();
    fp.bg_max = bl.max_rows;
    fp.bg_seg = bl.seg;
    fp.ntab = ntab;
    fp.join = join;
    fp.combined = msd_combined(in, ntab);
    fp.key2 = key2;
    for (int x = 0; x < ntab; x++) fp.shadow[x] = pack_ok ? (int64_t *)ms->t[x].tempA : nullptr;
    if (t_slot < 0) g_fin_last = fp;
    {
        ProfScope ps("msd_final", 0, s);
        HIP_TRY(launch_msd_final(fp, s));
    }
    cx->ms = ms;
    cx->fp = fp;
    cx->in = in;
    cx->ntab = ntab;
    cx->join = join;
    cx->tc = tc;
    cx->pf = prof_last();
    for (int x = 0; x < 2; x++) {
        cx->pa[x] = pa[x];
        cx->pb[x] = pb[x];
    }
    cx->pa_fused = pa_fused;
    return SMJ_OK;
}

int msd_back(MsdCtx &cx, T *out_j, int64_t *h_rows, hipStream_t s) {
    MsdScratch *ms = cx.ms;
    const MsdIn *in = cx.in;
    const int ntab = cx.ntab, join = cx.join, tc = cx.tc;
    const MsdFinalParams &fp = cx.fp;
    const size_t pf = cx.pf;
    const size_t *pa = cx.pa, *pb = cx.pb;
    const bool pa_fused = cx.pa_fused;
    auto compact = [&](int after_fallback) -> int {
        {
            ProfScope ps("msd_count_scan", 0, s);
            HIP_TRY(launch_msd_count_scan(ms->counts, ms->cpart, ms->offs, ms->plan, s));
        }
        ProfScope ps("msd_compact", 0, s);
        HIP_TRY(launch_msd_compact((const int64_t *)ms->slots, ms->groups, ms->counts, ms->offs, ms->plan, tc, out_j,
                                   after_fallback, s));
        if (after_fallback)
            HIP_TRY(launch_msd_compact_big((const int64_t *)ms->slots, ms->groups, ms->counts, ms->offs,
                                           (const uint2 *)ms->cwork, ms->n_cwork, tc, out_j, s));
        return SMJ_OK;
    };
    size_t pc = (size_t)-1;
    if (join) {  // speculative: a no-op when the plan turns out to have oversized groups
        SMJ_TRY(compact(0));
        pc = prof_last();
    }
    HIP_TRY(hipMemcpyAsync(ms->h_plan, ms->plan, sizeof(MsdPlan), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (ms->h_plan->err) {  // every kernel after msd_group returned at entry (msd_plan_failed)
        const uint32_t e = ms->h_plan->err;
        fprintf(stderr, "smj: pipeline %s (err 0x%x)\n",
                (e & 1u) ? "look-back wait timed out" : (e & 2u) ? "run metadata inconsistent (SMJ_BOUNDS check)"
                                                             : "group plan inconsistent",
                e);
        return (e & 1u) ? SMJ_ERR_TIMEOUT : SMJ_ERR_HIP;
    }
    if (t_slot < 0) {
        g_msd_stats[0] = ms->h_plan->nsingle;
        g_msd_stats[1] = ms->h_plan->nbig;
        g_msd_stats[2] = ms->h_plan->m[0];
        g_msd_stats[3] = ms->h_plan->m[1];
        g_msd_groups[0] = ms->h_plan->ngroups;
        g_msd_groups[1] = ms->h_plan->nradix;
        g_msd_groups[2] = ms->h_plan->nwide;
        g_msd_bigdev = ms->h_plan->nbigdev;
        g_msd_groups[3] = ms->h_plan->nlsd;
        g_msd_packb = ms->h_plan->packB;
        g_msd_wstage = ms->h_plan->nwst;
        g_msd_segb = ms->h_plan->nsegb;
    }
    bool redo = false;
    // 2-column tables: the groups the staged kernel did not sort (wide groups
    // with 64-bit payloads, the radix / 64-bit tiers' hand-overs) -- launched
    // only when the plan shows some; the speculative compact was then a no-op
    // (msd_compact_kernel) and runs again below
    const bool two = fp.tab[0].cols == 2 && (ntab == 1 || fp.tab[1].cols == 2);
    const bool tiers = two && (ms->h_plan->nwst || ms->h_plan->nradix);
    size_t pt = (size_t)-1;
    if (tiers) {
        {
            ProfScope ps("msd_final_tiers", 0, s);
            HIP_TRY(launch_msd_final_tiers(fp, s));
        }
        pt = prof_last();
        // the 64-bit tier lists a group whose keys span over 48 bits as
        // oversized (final_group: plan->nbig, big_list) for the fallback
        // below, which must see the plan as the tiers left it (far outliers
        // next to dense keys: a wide sub-bucket's group handed down the tiers)
        HIP_TRY(hipMemcpyAsync(ms->h_plan, ms->plan, sizeof(MsdPlan), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (ms->h_plan->err) {
            fprintf(stderr, "smj: pipeline group plan inconsistent in the final tiers (err 0x%x)\n", ms->h_plan->err);
            return SMJ_ERR_HIP;
        }
        if (t_slot < 0) g_msd_stats[1] = ms->h_plan->nbig;
    }
    ms->n_cwork = 0;  // (msd_fallback lists the oversized groups' join chunks, if any)
    MsdFinalParams ff = fp;  // packed pass-B rows: the single-key tier reads the words (pk_mode 3), the
                             // others read the shadow, which the unpack kernel fills for the oversized groups
    ff.pk_mode = ms->h_plan->packB ? 3 : -1;
    if (ms->h_plan->packB && ms->h_plan->nbig) HIP_TRY(launch_msd_unpack_groups(fp, s));
    SMJ_TRY(msd_fallback(ms, in, ntab, join, ff, out_j, s, &redo));
    redo = redo || (tiers && join);
    if (redo) {
        SMJ_TRY(compact(1));
        pc = prof_last();
    }
    if (redo || ms->h_plan->nbig || tiers) {  // joined (after the redo), the device big-group count, the tiers' counts
        HIP_TRY(hipMemcpyAsync(ms->h_plan, ms->plan, sizeof(MsdPlan), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (ms->h_plan->err) {  // a tier handed a group over its capacity (a bug: err bit 2)
            fprintf(stderr, "smj: pipeline group plan inconsistent after the final tiers (err 0x%x)\n", ms->h_plan->err);
            return SMJ_ERR_HIP;
        }
        if (t_slot < 0) {
            g_msd_bigdev = ms->h_plan->nbigdev;
            g_msd_groups[1] = ms->h_plan->nradix;
            g_msd_groups[2] = ms->h_plan->nwide;
            g_msd_wstage = ms->h_plan->nwst;
        }
    }
    const MsdPlan &pl = *ms->h_plan;
    double pa_bytes = 0.0;
    for (int x = 0; x < ntab; x++) {
        const double W = 8.0 * in[x].cols;
        pa_bytes += W * ((double)in[x].n + pl.m[x]);
        if (!pa_fused) prof_set_bytes(pa[x], W * ((double)in[x].n + pl.m[x]));
        prof_set_bytes(pb[x], W * 2.0 * pl.m[x]);
        h_rows[x] = pl.m[x];
    }
    if (pa_fused) prof_set_bytes(pa[0], pa_bytes);
    const double Jb = join ? 8.0 * tc * (double)pl.joined : 0.0;
    double fb = Jb;
    for (int x = 0; x < ntab; x++) fb += 2.0 * 8.0 * in[x].cols * pl.m[x];
    if (pt != (size_t)-1 && pl.ngroups) {  // the tiers' share of the rows, by their groups (wide groups: all of C3-wide's)
        const double share = std::min(1.0, (double)(pl.nwst + pl.nradix) / (double)pl.ngroups);
        prof_set_bytes(pt, fb * share);
        fb -= fb * share;
    }
    prof_set_bytes(pf, fb);
    prof_set_bytes(pc, 2.0 * Jb);
    if (join) h_rows[2] = pl.joined;
    return SMJ_OK;
}

int msd_run(const MsdIn *in, int ntab, int join, int key2, T *out_j, int64_t *h_rows, hipStream_t s,
            const MsdStage *stg = nullptr) {
    MsdCtx cx;
    SMJ_TRY(msd_front(in, ntab, join, key2, s, stg, &cx));
    return msd_back(cx, out_j, h_rows, s);
}

int msd_check(const T *src, int64_t n, int cols, int use_sel, int sel_col, int key, const T *out) {
    SMJ_TRY(check_table(n, cols, use_sel ? sel_col : 0, key));
    if (n > 0 && (!src || !out || src == out)) return SMJ_ERR_INVALID;
    return SMJ_OK;
}

// ---------------------------------------------------------------------------
// Partitioned mode (tables over kMsdSingleMax rows; BASELINE C4 / C5 on one
// GPU).  One MSD pipeline call has 256 x 2048 sub-buckets of <= 1024 rows per
// table, i.e. room for ~4e8 rows of well-spread keys; larger tables are first
// range-partitioned on the key into P parts of <= kMsdPartRows rows per table
// (smj_dev_partition: the WHERE clause + a stable bucket scatter, one read and
// one write), and each part runs the pipeline in place.  Parts are disjoint,
// ascending key ranges and sort + zip join are per-key operations, so part p's
// sorted rows belong exactly where the partition put them (the exclusive
// prefix of the part counts) and its joined rows follow part p - 1's: the
// concatenation is cpu_app.c's result.  Splitters are weighted quantiles of a
// key sample of both tables (a key never spans two parts).
// ---------------------------------------------------------------------------
constexpr int64_t kMsdSingleMax = 160000000;  // rows per table of one pipeline call (<= 256 pass-B tiles per bucket)
// Target rows per part of the larger table.  Smaller parts mean fewer pass-B
// tiles per bucket, i.e. fewer and longer runs per final group (msd_final
// 17.6 -> 16.0 ms at C4 with 14 parts instead of 7), against a fixed cost per
// part that the skewed tables' fallback tiers make larger (host round
// trips, oversized groups).  Same-box sweeps (profiles/r04/r04ze): C4 (equal
// sizes) 7 parts 61.2-62.2 ms, 14: 58.3-60.4, 20: 58.8, 28: 59.4-59.7; C5
// (1:10 sizes, Zipf) 7 parts 43.0-43.5, 10: 42.8, 14: 45.0.
constexpr int64_t kMsdPartRows = 50000000;         // tables of similar size
constexpr int64_t kMsdPartRowsSkewed = 100000000;  // one table over 1.5x the other (msd_combined's test)

int g_force_parts = 0;  // smj_debug_force_parts: the partitioned mode at any size (tests)

int64_t msd_large_parts(const MsdIn *in, int ntab) {
    if (g_force_parts > 0) return std::min(64, g_force_parts);
    int64_t mx = 0;
    for (int x = 0; x < ntab; x++) mx = std::max(mx, in[x].n);
    static const int64_t rows = [] {  // SMJ_PART_ROWS: A/B of the part size
        const char *e = getenv("SMJ_PART_ROWS");
        const int64_t v = e ? (int64_t)atof(e) : 0;
        return v >= 1000000 && v <= kMsdSingleMax ? v : 0;
    }();
    int64_t lo = in[0].n, hi = in[0].n;
    for (int x = 1; x < ntab; x++) {
        lo = std::min(lo, in[x].n);
        hi = std::max(hi, in[x].n);
    }
    const int64_t per = rows ? rows : (ntab > 1 && 2 * hi > 3 * lo) ? kMsdPartRowsSkewed : kMsdPartRows;
    return std::min<int64_t>(64, (mx + per - 1) / per);
}

// The one-pass partition (msd_part1_kernel) for tables of up to 8 columns;
// SMJ_PART1=0 keeps the counting partition (A/B runs).
bool msd_part1_on(const MsdIn *in, int ntab) {
    static const bool on = [] {
        const char *e = getenv("SMJ_PART1");
        return !(e && e[0] == '0');
    }();
    for (int x = 0; x < ntab; x++)
        if (in[x].cols > kDirectCols) return false;
    return on;
}

// The one-pass partition's regions (~1.3x each table) stay allocated between
// calls (a C4 step would otherwise pay hipFree + hipMalloc of ~20 GB); they are
// released when they cannot all be had -- before the counting partition runs
// -- and by smj_finalize.
void msd_part1_release(MsdScratch *ms) {
    for (int x = 0; x < 2; x++) {
        if (ms->pst[x]) dev_free(ms->pst[x]);
        ms->pst[x] = nullptr;
        ms->c_pst[x] = 0;
    }
    if (ms->p1st) dev_free(ms->p1st);
    ms->p1st = nullptr;
    ms->c_p1st = 0;
    for (int x = 0; x < 2; x++) {
        if (ms->p1desc[x]) dev_free(ms->p1desc[x]);
        ms->p1desc[x] = nullptr;
        ms->c_p1desc[x] = 0;
    }
}

// The chunked one-pass partition (msd_part1c_kernel, no look-back; SMJ_PART1C=0
// keeps the look-back partition).  Chunk g of G takes K consecutive tiles; part
// b's sub-region per chunk holds the chunk's estimated share of it (the key
// sample's fraction f of the chunk's rows), plus 8 standard deviations of the
// sample's estimate of f and 8 of the chunk's own binomial count, plus a tile.
// *staged = false when a sub-region overflowed (input clustered by key; the
// caller then runs the look-back partition).  On success part b of table x
// is the rows at the descriptors (*desc)[x][b] (ntl[x][b] tiles of part_a's
// tile rows) into ms->pst[x]; cnt[x][b] its rows.
int msd_part1c(MsdScratch *ms, const MsdIn *in, int ntab, const std::vector<int64_t> &spl, std::vector<int64_t> *cnt,
               std::vector<const uint64_t *> *desc, std::vector<int64_t> *ntl, bool *staged, hipStream_t s) {
    static const bool on = [] {
        const char *e = getenv("SMJ_PART1C");
        return !(e && e[0] == '0');
    }();
    *staged = false;
    if (!on) return SMJ_OK;
    const int nspl = (int)spl.size(), nb = nspl + 1;
    int G[2] = {0, 0};
    int64_t K[2] = {0, 0};
    std::vector<int64_t> dbase[2];
    for (int x = 0; x < ntab; x++) {
        cnt[x].assign(nb, 0);
        ntl[x].assign(nb, 0);
        desc[x].assign(nb, nullptr);
        if (in[x].n == 0) continue;
        const int64_t tile = p1_tile(in[x].cols), nt = (in[x].n + tile - 1) / tile, Ta = msd_tile_a(in[x].cols);
        const int gmax = msd_part1c_grid(in[x].cols);
        if (gmax < 1) return SMJ_OK;
        K[x] = (nt + gmax - 1) / gmax;
        G[x] = (int)((nt + K[x] - 1) / K[x]);
        const double R = (double)(K[x] * tile);  // rows per chunk (the last one fewer)
        const int64_t m = std::min<int64_t>(in[x].n, kSampleMax);
        std::vector<int64_t> sc(nb, 0);
        for (int64_t j = 0; j < m; j++) {
            const int64_t k = ms->h_samp[x * kSampleMax + j];
            if (k == INT64_MAX) continue;
            sc[std::lower_bound(spl.begin(), spl.end(), k) - spl.begin()]++;
        }
        const char *cs = getenv("SMJ_PART1_CAP");  // tests: scaled-down sub-regions force the fallback
        const double scale = cs ? atof(cs) : 1.0;
        P1cWords w{};
        P1cDesc d{};
        dbase[x].assign(nb + 1, 0);
        int64_t at = 0;
        for (int b = 0; b < nb; b++) {
            const double f = (double)sc[b] / (double)m;
            const double est = f * R + 8.0 * R * std::sqrt(f * (1.0 - f) / (double)m + 1.0 / ((double)m * m)) +
                               8.0 * std::sqrt(R * f * (1.0 - f) + 1.0);
            const int64_t cap = std::min<int64_t>((int64_t)R, (int64_t)(est * scale) + (scale < 1.0 ? 0 : tile));
            w.v[b] = d.st[b] = at;
            w.v[64 + b] = d.cap[b] = cap;
            at += (int64_t)G[x] * cap;
            d.dbase[b] = dbase[x][b];
            dbase[x][b + 1] = dbase[x][b] + (int64_t)G[x] * ((cap + Ta - 1) / Ta);
        }
        for (int b = 0; b < nspl; b++) w.v[128 + b] = spl[b];
        if (grow(&ms->pst[x], &ms->c_pst[x], (size_t)std::max<int64_t>(1, at) * in[x].cols * sizeof(T)) != SMJ_OK ||
            grow(&ms->p1desc[x], &ms->c_p1desc[x], (size_t)std::max<int64_t>(1, dbase[x][nb]) * 8) != SMJ_OK) {
            (void)hipGetLastError();
            msd_part1_release(ms);
            return SMJ_OK;  // the counting partition (with all of it free) or the look-back one runs
        }
        uint32_t *c = ms->p1c + (size_t)x * kP1cWords;
        HIP_TRY(hipMemsetAsync(c + 1024 * 64, 0, 64 * sizeof(uint32_t), s));
        MsdPart1cParams p{};
        p.src = in[x].src;
        p.n = in[x].n;
        p.use_sel = in[x].use_sel;
        p.sel_col = in[x].sel_col;
        p.key_col = in[x].key;
        p.nspl = nspl;
        p.sel_val = in[x].sel_val;
        p.dst = (int64_t *)ms->pst[x];
        p.cnt = c;
        p.flags = c + 1024 * 64;
        p.ntiles = nt;
        p.chunk = K[x];
        {
            ProfScope ps("partition_1pass", 16.0 * in[x].cols * in[x].n, s);
            HIP_TRY(launch_msd_part1c(p, w, in[x].cols, G[x], s));
        }
        HIP_TRY(launch_p1c_desc(c, G[x], nb, (int)Ta, d, (uint64_t *)ms->p1desc[x], s));
    }
    for (int x = 0; x < ntab; x++) {
        if (in[x].n == 0) continue;
        const size_t off = (size_t)x * kP1cWords;
        HIP_TRY(hipMemcpyAsync(ms->h_p1c + off, ms->p1c + off, sizeof(uint32_t) * (size_t)G[x] * 64, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(ms->h_p1c + off + 1024 * 64, ms->p1c + off + 1024 * 64, sizeof(uint32_t) * 4,
                               hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    for (int x = 0; x < ntab; x++) {
        if (in[x].n == 0) continue;
        const uint32_t *h = ms->h_p1c + (size_t)x * kP1cWords;
        if (h[1024 * 64 + 1]) {
            if (getenv("SMJ_DEBUG_PART1")) fprintf(stderr, "smj: chunked partition overflowed a sub-region\n");
            return SMJ_OK;  // *staged = false
        }
        const int64_t Ta = msd_tile_a(in[x].cols);
        for (int g = 0; g < G[x]; g++)
            for (int b = 0; b < nb; b++) {
                const int64_t c = h[(size_t)g * 64 + b];
                cnt[x][b] += c;
                ntl[x][b] += (c + Ta - 1) / Ta;
            }
        for (int b = 0; b < nb; b++) desc[x][b] = (const uint64_t *)ms->p1desc[x] + dbase[x][b];
    }
    *staged = true;
    return SMJ_OK;
}

// Region capacities from the key sample (ms->h_samp: table x's sampled keys at
// [x * kSampleMax, + min(n, kSampleMax)), INT64_MAX for a row the select
// drops): part b's estimated rows plus 8 binomial standard deviations plus a
// tile, capped at the table's rows.  *staged = false when a region overflowed
// (the caller then runs the counting partition instead); cnt / roff: rows per
// part and region starts.
int msd_part1(MsdScratch *ms, const MsdIn *in, int ntab, const std::vector<int64_t> &spl, std::vector<int64_t> *cnt,
              std::vector<int64_t> *roff, bool *staged, hipStream_t s) {
    const int nspl = (int)spl.size(), nb = nspl + 1;
    *staged = false;
    int64_t nt[2] = {0, 0};
    for (int x = 0; x < ntab; x++) {
        cnt[x].assign(nb, 0);
        roff[x].assign(nb + 1, 0);
        if (in[x].n == 0) continue;
        const int64_t m = std::min<int64_t>(in[x].n, kSampleMax);
        std::vector<int64_t> sc(nb, 0);
        for (int64_t j = 0; j < m; j++) {
            const int64_t k = ms->h_samp[x * kSampleMax + j];
            if (k == INT64_MAX) continue;
            sc[std::lower_bound(spl.begin(), spl.end(), k) - spl.begin()]++;
        }
        const double w = (double)in[x].n / (double)m;
        const int64_t tile = p1_tile(in[x].cols);
        const char *cs = getenv("SMJ_PART1_CAP");  // tests: scaled-down regions force the fallback
        const double scale = cs ? atof(cs) : 1.0;
        int64_t *oc = ms->p1h + x * kP1Words;
        for (int b = 0; b < nb; b++) {
            const double f = (double)sc[b] / (double)m;
            const double sd = w * std::sqrt((double)m * f * (1.0 - f) + 1.0);
            const int64_t cap =
                std::min<int64_t>(in[x].n, (int64_t)(((double)sc[b] * w + 8.0 * sd) * scale) + (scale < 1.0 ? 0 : tile));
            oc[b] = roff[x][b];
            oc[64 + b] = cap;
            roff[x][b + 1] = roff[x][b] + cap;
        }
        // the regions need ~1.3x the table on top of the in-place partition's
        // memory: if the device cannot hold them, the counting partition runs
        if (grow(&ms->pst[x], &ms->c_pst[x], (size_t)roff[x][nb] * in[x].cols * sizeof(T)) != SMJ_OK) {
            (void)hipGetLastError();
            if (getenv("SMJ_DEBUG_PART1")) fprintf(stderr, "smj: one-pass partition regions not allocated (%zu B)\n",
                                                    (size_t)roff[x][nb] * in[x].cols * sizeof(T));
            msd_part1_release(ms);  // the counting partition runs with all of it free
            return SMJ_OK;          // *staged = false
        }
        nt[x] = (in[x].n + tile - 1) / tile;
    }
    if (grow(&ms->p1st, &ms->c_p1st, (size_t)std::max(nt[0], nt[1]) * nb * 8) != SMJ_OK) {
        (void)hipGetLastError();
        msd_part1_release(ms);
        return SMJ_OK;
    }
    for (int x = 0; x < ntab; x++) {
        if (in[x].n == 0) continue;
        int64_t *d = ms->p1d + x * kP1Words;
        // oc from the pinned twin; tot and flags zeroed (one copy: the twin's zeros)
        int64_t *h = ms->p1h + x * kP1Words;
        for (int i = 128; i < kP1Words; i++) h[i] = 0;
        HIP_TRY(hipMemcpyAsync(d, h, sizeof(int64_t) * kP1Words, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemsetAsync(ms->p1st, 0, (size_t)nt[x] * nb * 8, s));
        MsdPart1Params p{};
        p.src = in[x].src;
        p.n = in[x].n;
        p.use_sel = in[x].use_sel;
        p.sel_col = in[x].sel_col;
        p.key_col = in[x].key;
        p.nspl = nspl;
        p.sel_val = in[x].sel_val;
        p.spl = ms->lspl;
        p.oc = d;
        p.dst = (int64_t *)ms->pst[x];
        p.status = (unsigned long long *)ms->p1st;
        p.tot = (long long *)(d + 128);
        p.flags = (uint32_t *)(d + 192);
        p.ntiles = nt[x];
        ProfScope ps("partition_1pass", 16.0 * in[x].cols * in[x].n, s);
        HIP_TRY(launch_msd_part1(p, in[x].cols, s));
    }
    HIP_TRY(hipMemcpyAsync(ms->p1h, ms->p1d, sizeof(int64_t) * 2 * kP1Words, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    bool over = false;
    for (int x = 0; x < ntab; x++) {
        if (in[x].n == 0) continue;
        const int64_t *h = ms->p1h + x * kP1Words;
        const uint32_t *fl = (const uint32_t *)(h + 192);
        if (fl[2]) return SMJ_ERR_TIMEOUT;
        over |= fl[1] != 0;
        for (int b = 0; b < nb; b++) cnt[x][b] = h[128 + b];
    }
    if (over && getenv("SMJ_DEBUG_PART1")) fprintf(stderr, "smj: one-pass partition overflowed a region\n");
    *staged = !over;
    return SMJ_OK;
}

// LSD radix sort of (key, weight) pairs by key, 8-bit digits, skipping the
// digits every key shares: ~8k samples in tens of microseconds where
// std::sort took ~0.3 ms of idle GPU per partitioned call (SMJ_DEBUG_HOST)
void radix_sort_keys(std::vector<std::pair<int64_t, double>> &v) {
    const size_t n = v.size();
    if (n < 2) return;
    std::vector<std::pair<int64_t, double>> tmp(n);
    auto ukey = [](int64_t k) { return (uint64_t)k ^ (1ull << 63); };  // signed order as unsigned
    uint64_t all_or = 0, all_and = ~0ull;
    for (const auto &e : v) {
        all_or |= ukey(e.first);
        all_and &= ukey(e.first);
    }
    const uint64_t varying = all_or ^ all_and;
    for (int sh = 0; sh < 64; sh += 8) {
        if (((varying >> sh) & 0xffu) == 0) continue;
        size_t c[257] = {0};
        for (const auto &e : v) c[((ukey(e.first) >> sh) & 0xffu) + 1]++;
        for (int d = 0; d < 256; d++) c[d + 1] += c[d];
        for (const auto &e : v) tmp[c[(ukey(e.first) >> sh) & 0xffu]++] = e;
        v.swap(tmp);
    }
}

// SMJ_PART_OVERLAP=0: the parts strictly in turn on the caller's stream (A/B)
bool msd_overlap_on() {
    static const bool on = [] {
        const char *e = getenv("SMJ_PART_OVERLAP");
        return !(e && e[0] == '0');
    }();
    return on;
}

// the partitioned mode's two part streams per scratch key (non-blocking: no
// implicit ordering with the legacy default stream)
int part_streams(hipStream_t out[2]) {
    int dev = 0;
    const int key = scratch_key(&dev);
    if (key < 0) return SMJ_ERR_HIP;
    std::lock_guard<std::mutex> lk(g_mu);
    auto &m = g_part_streams;
    auto it = m.find(key);
    if (it == m.end()) {
        std::array<hipStream_t, 2> a{};
        for (auto &x : a) HIP_TRY(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        it = m.emplace(key, a).first;
    }
    out[0] = it->second[0];
    out[1] = it->second[1];
    return SMJ_OK;
}

// SMJ_DEBUG_HOST=1: the partitioned mode's host timeline per call (us since
// entry at each phase, and the host time since the previous call returned)
struct HostMarks {
    using clk = std::chrono::steady_clock;
    bool on = getenv("SMJ_DEBUG_HOST") != nullptr;
    clk::time_point t0 = clk::now();
    std::string log;
    static clk::time_point &last_exit() {
        static clk::time_point t = clk::time_point{};
        return t;
    }
    void mark(const char *what) {
        if (!on) return;
        char b[96];
        snprintf(b, sizeof b, " %s %.0f", what, std::chrono::duration<double, std::micro>(clk::now() - t0).count());
        log += b;
    }
    ~HostMarks() {
        if (!on) return;
        mark("exit");
        const double gap = last_exit() == clk::time_point{} ? 0.0
                                                             : std::chrono::duration<double, std::micro>(t0 - last_exit()).count();
        fprintf(stderr, "smj host: since last call %.0f us |%s\n", gap, log.c_str());
        last_exit() = clk::now();
    }
};

int msd_large(const MsdIn *in, int ntab, int join, int key2, T *out_j, int64_t *h_rows, hipStream_t s) {
    HostMarks hm;
    MsdScratch *ms;
    SMJ_TRY(msd_scratch(&ms));
    const int64_t P = msd_large_parts(in, ntab);
    // 1. a sample of the selected keys of every table (msd_sample_gather_kernel)
    {
        MsdSampleParams sp{};
        for (int x = 0; x < ntab; x++)
            sp.tab[x] = MsdTable{in[x].src, in[x].n, in[x].cols, in[x].key, in[x].use_sel, in[x].sel_col, in[x].sel_val};
        sp.ntab = ntab;
        sp.spl = ms->spl;
        sp.samp = ms->samp;
        ProfScope ps("msd_part_sample", 0, s);
        HIP_TRY(launch_msd_sample_gather(sp, s));
    }
    HIP_TRY(hipMemcpyAsync(ms->h_samp, ms->samp, sizeof(int64_t) * (2 * kSampleMax + kSampleGatherBlocksH),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    hm.mark("sample");
    // 2. P - 1 splitters: weighted quantiles (a sample of table x stands for
    // n_x / (its sample count) input rows; dropped rows are not samples)
    std::vector<std::pair<int64_t, double>> kw;
    double W = 0;
    for (int x = 0; x < ntab; x++) {
        const int64_t cnt = std::min<int64_t>(in[x].n, kSampleMax);
        if (cnt == 0) continue;
        const double w = (double)in[x].n / (double)cnt;
        for (int64_t j = 0; j < cnt; j++) {
            const int64_t k = ms->h_samp[x * kSampleMax + j];
            if (k == INT64_MAX) continue;  // a row the select drops
            kw.emplace_back(k, w);
            W += w;
        }
    }
    radix_sort_keys(kw);  // by key (the order among equal keys does not change which key a quantile picks)
    std::vector<int64_t> spl;
    {
        double acc = 0;
        size_t i = 0;
        for (int64_t p = 1; p < P && !kw.empty(); p++) {
            const double target = W * (double)p / (double)P;
            while (i + 1 < kw.size() && acc + kw[i].second < target) acc += kw[i++].second;
            const int64_t k = kw[i].first;  // bucket(key) = #{splitters < key}: key k closes part p - 1
            if (spl.empty() || spl.back() < k) spl.push_back(k);
        }
    }
    const int nspl = (int)spl.size();
    hm.mark("splitters");
    if (nspl) HIP_TRY(hipMemcpyAsync(ms->lspl, spl.data(), sizeof(int64_t) * nspl, hipMemcpyHostToDevice, s));
    // 3. select + stable partition of every table: in one pass into part
    // regions sized from the sample (msd_part1_kernel; each part is then sorted
    // from its region to its place in the output), or -- when a region would
    // overflow, or SMJ_PART1=0 -- counted, then scattered straight into the
    // output buffer (smj_dev_partition; the parts are then sorted in place)
    std::vector<int64_t> cnt[2], off[2], roff[2], ntl[2];
    std::vector<const uint64_t *> desc[2];
    bool staged = false, chunked = false;
    if (msd_part1_on(in, ntab)) {
        SMJ_TRY(msd_part1c(ms, in, ntab, spl, cnt, desc, ntl, &chunked, s));
        if (!chunked) SMJ_TRY(msd_part1(ms, in, ntab, spl, cnt, roff, &staged, s));
    }
    hm.mark("partition");
    if (getenv("SMJ_DEBUG_PART1")) {
        fprintf(stderr, "smj: partitioned mode: %lld x %lld rows, %d parts (%zu weighted samples), %s; splitters", (long long)in[0].n,
                (long long)(ntab > 1 ? in[1].n : 0), nspl + 1, kw.size(),
                chunked ? "chunked one-pass" : staged ? "one-pass regions" : "counting partition");
        for (int64_t k : spl) fprintf(stderr, " %lld", (long long)k);
        fprintf(stderr, "\n");
    }
    for (int x = 0; x < ntab; x++) {
        if (!staged && !chunked) {
            cnt[x].assign(nspl + 1, 0);
            if (in[x].n)
                SMJ_TRY(smj_dev_partition(in[x].src, in[x].n, in[x].cols, in[x].use_sel, in[x].sel_col,
                                          in[x].sel_val, in[x].key, ms->lspl, nspl, in[x].out, cnt[x].data(), s));
        }
        off[x].assign(nspl + 2, 0);
        for (int p = 0; p <= nspl; p++) off[x][p + 1] = off[x][p] + cnt[x][p];
        h_rows[x] = off[x][nspl + 1];
    }
    // 4. the pipeline per part, in place
    int64_t J = 0;
    const int tc = ntab > 1 ? in[0].cols + in[1].cols - 1 : 1;
    std::vector<MsdIn> parts(2 * (size_t)(nspl + 1));
    std::vector<int> nps(nspl + 1, 0);
    bool all_joined = join != 0;  // every part has rows of both tables
    for (int p = 0; p <= nspl; p++) {
        MsdIn *part = &parts[2 * (size_t)p];
        int &np = nps[p];
        for (int x = 0; x < ntab; x++) {
            if (cnt[x][p] == 0) continue;
            T *base = in[x].out + off[x][p] * in[x].cols;
            if (chunked) {  // the part's tiles through its descriptors into the staging buffer
                part[np++] = MsdIn{(const T *)ms->pst[x], cnt[x][p], in[x].cols, 0, 0, in[x].key, 0, base, desc[x][p],
                                   ntl[x][p]};
                continue;
            }
            const T *src = staged ? (const T *)ms->pst[x] + roff[x][p] * in[x].cols : base;
            part[np++] = MsdIn{src, cnt[x][p], in[x].cols, 0, 0, in[x].key, 0, base};
        }
        all_joined &= np == 2;
    }
    if (all_joined && !g_prof_on && msd_overlap_on()) {
        // part p's back phase (its host round trips: plan, fallback lists)
        // overlaps part p + 1's front phase, which runs on the other stream
        // with the other scratch set (part p - 1's, whose back has returned).
        // Profiling steps run the parts in turn: their per-kernel times stay
        // those of a kernel alone on the GPU.
        hipStream_t ps[2];
        SMJ_TRY(part_streams(ps));
        hipEvent_t fe[2] = {nullptr, nullptr};  // front p launched: front p + 1 starts behind it
        struct Guard {  // on any exit: no part still in flight, scratch set 0 current
            hipStream_t *ps;
            hipEvent_t *fe;
            ~Guard() {
                hipStreamSynchronize(ps[0]);
                hipStreamSynchronize(ps[1]);
                for (int i = 0; i < 2; i++)
                    if (fe[i]) hipEventDestroy(fe[i]);
                t_msd_var = 0;
            }
        } guard{ps, fe};
        for (int i = 0; i < 2; i++) HIP_TRY(hipEventCreateWithFlags(&fe[i], hipEventDisableTiming));
        hipEvent_t ready;
        HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        const hipError_t er = hipEventRecord(ready, s);  // the partition's output on s
        for (int i = 0; i < 2 && er == hipSuccess; i++) HIP_TRY(hipStreamWaitEvent(ps[i], ready, 0));
        hipEventDestroy(ready);
        HIP_TRY(er);
        std::vector<MsdCtx> cx(nspl + 1);
        // SMJ_PART_CHAIN=1: front p + 1 waits for front p's kernels, so that it
        // shares the GPU with part p's back phase rather than with front p
        static const bool chain = getenv("SMJ_PART_CHAIN") && getenv("SMJ_PART_CHAIN")[0] == '1';
        auto front = [&](int p) -> int {
            t_msd_var = p & 1;
            if (p == g_fail_front) t_fail_grow = true;  // (a test: this part's scratch "cannot be had")
            if (p > 0 && chain) HIP_TRY(hipStreamWaitEvent(ps[p & 1], fe[(p - 1) & 1], 0));
            SMJ_TRY(msd_front(&parts[2 * (size_t)p], 2, 1, key2, ps[p & 1], nullptr, &cx[p]));
            HIP_TRY(hipEventRecord(fe[p & 1], ps[p & 1]));
            return SMJ_OK;
        };
        SMJ_TRY(front(0));
        hm.mark("f0");
        // seq: the second scratch set could not be allocated (its front
        // returned SMJ_ERR_NOMEM before the part was fully launched): the part
        // whose back is due still finishes on its own set, set 1 is released,
        // and the remaining parts run one after another on set 0 -- the memory
        // the sequential path needs
        bool seq = false;
        for (int p = 0; p <= nspl; p++) {
            int64_t rows[3] = {0, 0, 0};
            if (seq) {
                t_msd_var = 0;
                SMJ_TRY(msd_run(&parts[2 * (size_t)p], 2, 1, key2, out_j + J * tc, rows, ps[0]));
                J += rows[2];
                continue;
            }
            if (p < nspl) {
                const int rc = front(p + 1);
                t_fail_grow = false;
                if (rc == SMJ_ERR_NOMEM) {
                    seq = true;
                    g_seq_from = p + 1;
                } else {
                    SMJ_TRY(rc);
                }
            }
            t_msd_var = p & 1;
            SMJ_TRY(msd_back(cx[p], out_j + J * tc, rows, ps[p & 1]));
            J += rows[2];
            hm.mark("b");
            if (seq) {
                HIP_TRY(hipStreamSynchronize(ps[0]));
                HIP_TRY(hipStreamSynchronize(ps[1]));
                t_msd_var = 0;
                msd_release_var(1);
                if (getenv("SMJ_DEBUG_PART1"))
                    fprintf(stderr, "smj: partitioned mode: no room for a second scratch set; parts %d.. in turn\n", p + 1);
            }
        }
        h_rows[2] = J;
        return SMJ_OK;
    }
    for (int p = 0; p <= nspl; p++) {
        MsdIn *part = &parts[2 * (size_t)p];
        const int np = nps[p];
        int64_t rows[3] = {0, 0, 0};
        if (np == 2 && join) {
            SMJ_TRY(msd_run(part, 2, 1, key2, out_j + J * tc, rows, s));
            J += rows[2];
        } else {
            for (int i = 0; i < np; i++) SMJ_TRY(msd_run(&part[i], 1, 0, 0, nullptr, rows, s));
        }
    }
    if (join) h_rows[2] = J;
    return SMJ_OK;
}

// the pipeline, partitioned when a table exceeds one call's capacity
int msd_any(const MsdIn *in, int ntab, int join, int key2, T *out_j, int64_t *h_rows, hipStream_t s) {
    bool large = g_force_parts > 0;
    for (int x = 0; x < ntab; x++) large |= in[x].n > kMsdSingleMax;
    return large ? msd_large(in, ntab, join, key2, out_j, h_rows, s) : msd_run(in, ntab, join, key2, out_j, h_rows, s);
}

// ---------------------------------------------------------------------------
// Index-sort path (col_num > 8 -- cpu_app.c's load_csv
// takes any column count, :46-79, and join_in_cpu emits c1 + c2 - 1 of them,
// :204-266).  The pipeline runs on 16-B (key, row id) pairs -- the 2-column
// kernels whatever the width -- and whole rows are gathered once by id at
// the end; joined rows are gathered from (key, R id, S id) triples.  Stable
// order is preserved (ids ascend within a key).  For T = uint64 / double the
// pair kernel compares keys and select values through the order-preserving
// map, and the gathered rows are the input rows bit for bit.
// ---------------------------------------------------------------------------
struct IdxScratch {
    int dev = -1;
    void *pr[2] = {nullptr, nullptr}, *ps[2] = {nullptr, nullptr}, *jp = nullptr;
    size_t cpr[2] = {0, 0}, cps[2] = {0, 0}, cjp = 0;
};
std::map<int, IdxScratch> g_idx;

int idx_scratch(IdxScratch **out) {
    int dev = 0;
    const int key = scratch_key(&dev);
    if (key < 0) return SMJ_ERR_HIP;
    std::lock_guard<std::mutex> lk(g_mu);
    *out = &g_idx[key];
    (*out)->dev = dev;
    return SMJ_OK;
}

void idx_free_all() {
    for (auto &kv : g_idx) {
        if (kv.second.dev < 0) continue;
        hipSetDevice(kv.second.dev);
        for (void *q : {kv.second.pr[0], kv.second.pr[1], kv.second.ps[0], kv.second.ps[1], kv.second.jp}) dev_free(q);
    }
    g_idx.clear();
}

// pairs of table x into ix->pr[x] (sel_val already mapped for ktype != 0)
int idx_pairs(IdxScratch *ix, int x, const MsdIn &t, int ktype, int64_t row0, hipStream_t s) {
    const size_t b = (size_t)std::max<int64_t>(1, t.n) * 16;
    SMJ_TRY(grow(&ix->pr[x], &ix->cpr[x], b));
    SMJ_TRY(grow(&ix->ps[x], &ix->cps[x], b));
    ProfScope ps("idx_pairs", 8.0 * t.cols * t.n + 16.0 * t.n, s);
    HIP_TRY(launch_row_pairs(t.src, t.n, t.cols, t.key, t.use_sel, t.sel_col, t.sel_val, ktype, row0,
                             (int64_t *)ix->pr[x], s));
    return SMJ_OK;
}

int msd_indexed(const MsdIn *in, int ntab, int join, int key2, int ktype, T *out_j, int64_t *h_rows, hipStream_t s) {
    IdxScratch *ix;
    SMJ_TRY(idx_scratch(&ix));
    MsdIn pin[2];
    for (int x = 0; x < ntab; x++) {
        SMJ_TRY(idx_pairs(ix, x, in[x], ktype, 0, s));
        pin[x] = MsdIn{(const T *)ix->pr[x], in[x].n, 2, 1, 1, 0, (T)-1, (T *)ix->ps[x]};  // key 0, keep id > -1
    }
    int64_t rows[3] = {0, 0, 0};
    if (join) {
        SMJ_TRY(grow(&ix->jp, &ix->cjp, (size_t)std::max<int64_t>(1, std::min(in[0].n, in[1].n)) * 24));
        SMJ_TRY(msd_any(pin, 2, 1, 0, (T *)ix->jp, rows, s));
    } else {
        SMJ_TRY(msd_any(pin, ntab, 0, 0, nullptr, rows, s));
    }
    for (int x = 0; x < ntab; x++) {
        h_rows[x] = rows[x];
        ProfScope ps("idx_gather", 2.0 * 8.0 * in[x].cols * rows[x], s);
        HIP_TRY(launch_gather_rows(in[x].src, in[x].n, nullptr, in[x].cols, (const int64_t *)ix->ps[x], 2, 1, rows[x],
                                   in[x].out, s));
    }
    if (join) {
        h_rows[2] = rows[2];
        const int tc = in[0].cols + in[1].cols - 1;
        ProfScope ps("idx_join_gather", 8.0 * (2 * tc + 3) * rows[2], s);
        HIP_TRY(launch_join_gather(in[0].src, in[0].cols, in[1].src, in[1].cols, key2, (const int64_t *)ix->jp,
                                   rows[2], out_j, s));
    }
    return SMJ_OK;
}

int idx_select(const T *in, int64_t n, int cols, int sel_col, T sel_val, T *out, int64_t *out_rows, hipStream_t s) {
    IdxScratch *ix;
    SMJ_TRY(idx_scratch(&ix));
    SMJ_TRY(idx_pairs(ix, 0, MsdIn{in, n, cols, 1, sel_col, 0, sel_val, out}, SMJ_KEY_INT64, 0, s));
    int64_t m = 0;
    SMJ_TRY(smj_dev_select((const T *)ix->pr[0], n, 2, 1, (T)-1, (T *)ix->ps[0], &m, s));
    HIP_TRY(launch_gather_rows(in, n, nullptr, cols, (const int64_t *)ix->ps[0], 2, 1, m, out, s));
    *out_rows = m;
    return SMJ_OK;
}

int idx_merge(const T *a, int64_t na, const T *b, int64_t nb, int cols, int key_col, T *out, hipStream_t s) {
    IdxScratch *ix;
    SMJ_TRY(idx_scratch(&ix));
    SMJ_TRY(idx_pairs(ix, 0, MsdIn{a, na, cols, 0, 0, key_col, 0, out}, SMJ_KEY_INT64, 0, s));
    SMJ_TRY(idx_pairs(ix, 1, MsdIn{b, nb, cols, 0, 0, key_col, 0, out}, SMJ_KEY_INT64, na, s));
    SMJ_TRY(grow(&ix->jp, &ix->cjp, (size_t)(na + nb) * 16));
    SMJ_TRY(smj_dev_merge((const T *)ix->pr[0], na, (const T *)ix->pr[1], nb, 2, 0, (T *)ix->jp, s));
    HIP_TRY(launch_gather_rows(a, na, b, cols, (const int64_t *)ix->jp, 2, 1, na + nb, out, s));
    return SMJ_OK;
}

int idx_join(const T *R, int64_t nr, int c1, const T *S, int64_t ns, int c2, int key1, int key2, T *out,
             int64_t *d_out_rows, int64_t *h_out_rows, hipStream_t s) {
    IdxScratch *ix;
    SMJ_TRY(idx_scratch(&ix));
    SMJ_TRY(idx_pairs(ix, 0, MsdIn{R, nr, c1, 0, 0, key1, 0, out}, SMJ_KEY_INT64, 0, s));
    SMJ_TRY(idx_pairs(ix, 1, MsdIn{S, ns, c2, 0, 0, key2, 0, out}, SMJ_KEY_INT64, 0, s));
    SMJ_TRY(grow(&ix->jp, &ix->cjp, (size_t)std::min(nr, ns) * 24));
    int64_t J = 0;
    SMJ_TRY(smj_dev_join((const T *)ix->pr[0], nr, 2, (const T *)ix->pr[1], ns, 2, 0, 0, (T *)ix->jp, d_out_rows, &J, s));
    HIP_TRY(launch_join_gather(R, c1, S, c2, key2, (const int64_t *)ix->jp, J, out, s));
    if (h_out_rows) {
        HIP_TRY(hipStreamSynchronize(s));
        *h_out_rows = J;
    }
    return SMJ_OK;
}
}  // namespace

// Diagnostic only (not part of smj.h): re-run the last pipeline call's part_b
// launches `reps` times with ablation bits `dbg` (smj_msd.hip, part_b) and
// return the average ms per round over both tables.  Overwrites tempB / offsB.
extern "C" int smj_debug_part_b_time(int dbg, int reps, float *ms) {
    if (g_pb_ntab == 0 || reps <= 0 || !ms) return SMJ_ERR_INVALID;
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    HIP_TRY(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++)
        for (int x = 0; x < g_pb_ntab; x++) {
            MsdPartBParams p = g_pb_last[x].p;
            p.dbg = dbg;
            HIP_TRY(launch_msd_part_b(p, g_pb_last[x].cols, g_pb_last[x].maxB, 0));
        }
    HIP_TRY(hipEventRecord(b, 0));
    HIP_TRY(hipEventSynchronize(b));
    HIP_TRY(hipEventElapsedTime(ms, a, b));
    *ms /= (float)reps;
    hipEventDestroy(a);
    hipEventDestroy(b);
    return SMJ_OK;
}

// Diagnostic only (not part of smj.h): re-run the last pipeline call's final
// launches `reps` times with ablation bits `dbg` (smj_msd.hip launch_msd_final)
// and return the average ms.  Rewrites the same outputs.
extern "C" int smj_debug_final_time(int dbg, int reps, float *ms) {
    if (!g_fin_last.groups || reps <= 0 || !ms) return SMJ_ERR_INVALID;
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    HIP_TRY(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++) {
        MsdFinalParams p = g_fin_last;
        p.dbg = dbg;
        HIP_TRY(launch_msd_final(p, 0));
    }
    HIP_TRY(hipEventRecord(b, 0));
    HIP_TRY(hipEventSynchronize(b));
    HIP_TRY(hipEventElapsedTime(ms, a, b));
    *ms /= (float)reps;
    hipEventDestroy(a);
    hipEventDestroy(b);
    return SMJ_OK;
}

// Diagnostic only (not part of smj.h): msd_big_stage_kernel cycles per
// oversized-group size class and per phase (SMJ_STAMPS build, SMJ_DEBUG_BIG=1;
// tools/big_times.py); resets them.
extern "C" int smj_debug_big_times(unsigned long long *out72) {
    hipDeviceSynchronize();
    return read_big_times(out72) == hipSuccess ? SMJ_OK : SMJ_ERR_HIP;
}

// Diagnostic: final-stage group counts of the last MSD pipeline (smj.h).
extern "C" void smj_debug_msd_groups(int64_t *out3) {
    for (int i = 0; i < 3; i++) out3[i] = g_msd_groups[i];
}

extern "C" void smj_debug_msd_tiers(int64_t *out4) {
    for (int i = 0; i < 4; i++) out4[i] = g_msd_groups[i];
}

// Diagnostic only (not part of smj.h): oversized multi-key groups of the last
// pipeline call that msd_big_stage_kernel sorted (the rest: host fallback)
extern "C" int64_t smj_debug_msd_bigdev(void) { return g_msd_bigdev; }
// Diagnostic only: 1 if the last pipeline call packed its pass-B rows
extern "C" int64_t smj_debug_msd_packb(void) { return g_msd_packb; }
// Diagnostic only: groups of the last pipeline call that the wide-span staged
// kernel took (msd_final_wstage_kernel: key spans over kStageRange)
extern "C" int64_t smj_debug_msd_wstage(void) { return g_msd_wstage; }
// Diagnostic only: pass-A buckets of the last pipeline call given a segmented
// pass-B digit (MsdSeg: keys in dense intervals with wide gaps between)
extern "C" int64_t smj_debug_msd_segmented(void) { return g_msd_segb; }
// Diagnostic only: the wide-span staged kernel hands a group to the radix tier
// when a bin holds more than `rows` rows (-1: the built-in SMJ_ST_MAXRUN; 0:
// every group -- the tests' way to the hand-over path)
extern "C" void smj_debug_wide_maxrun(int rows) { g_wide_maxrun = rows; }

extern "C" void smj_debug_msd_stats(int64_t *out4) {
    for (int i = 0; i < 4; i++) out4[i] = g_msd_stats[i];
}

static int smj_dev_select_sort_impl(const T *in, int64_t n_rows, int col_num, int use_select, int select_col,
                                   T select_val, int key_col, uint64_t key_base, T *out, int64_t *out_rows,
                                   void *stream) {
    (void)key_base;  // the MSD pipeline derives its digits from the data
    if (!out_rows) return SMJ_ERR_INVALID;
    *out_rows = 0;
    SMJ_TRY(msd_check(in, n_rows, col_num, use_select, select_col, key_col, out));
    if (n_rows == 0) return SMJ_OK;
    MsdIn t{in, n_rows, col_num, use_select, select_col, key_col, select_val, out};
    int64_t rows[3] = {0, 0, 0};
    if (col_num > kDirectCols)
        SMJ_TRY(msd_indexed(&t, 1, 0, 0, SMJ_KEY_INT64, nullptr, rows, (hipStream_t)stream));
    else
        SMJ_TRY(msd_any(&t, 1, 0, 0, nullptr, rows, (hipStream_t)stream));
    *out_rows = rows[0];
    return SMJ_OK;
}


extern "C" int smj_dev_select_sort(const T *in, int64_t n_rows, int col_num, int use_select, int select_col,
                                   T select_val, int key_col, uint64_t key_base, T *out, int64_t *out_rows,
                                   void *stream) {
    const int rc = smj_dev_select_sort_impl(in, n_rows, col_num, use_select, select_col, select_val, key_col, key_base, out, out_rows, stream);
    if (rc == SMJ_OK) trim_if_over_limit();
    return rc;
}

static int smj_dev_sort_merge_join_impl(const T *R, int64_t nr, int c1, int use_sel1, int sel_col1, T sel_val1,
                                       int key1, const T *S, int64_t ns, int c2, int use_sel2, int sel_col2,
                                       T sel_val2, int key2, T *R_sorted, T *S_sorted, T *out, int64_t *h_rows,
                                       void *stream) {
    if (!h_rows) return SMJ_ERR_INVALID;
    h_rows[0] = h_rows[1] = h_rows[2] = 0;
    SMJ_TRY(msd_check(R, nr, c1, use_sel1, sel_col1, key1, R_sorted));
    SMJ_TRY(msd_check(S, ns, c2, use_sel2, sel_col2, key2, S_sorted));
    if (nr > 0 && ns > 0 && !out) return SMJ_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    if (nr == 0 || ns == 0) {  // nothing to join: sort what there is
        if (nr) SMJ_TRY(smj_dev_select_sort(R, nr, c1, use_sel1, sel_col1, sel_val1, key1, 0, R_sorted, &h_rows[0], s));
        if (ns) SMJ_TRY(smj_dev_select_sort(S, ns, c2, use_sel2, sel_col2, sel_val2, key2, 0, S_sorted, &h_rows[1], s));
        return SMJ_OK;
    }
    const MsdIn t[2] = {{R, nr, c1, use_sel1, sel_col1, key1, sel_val1, R_sorted},
                        {S, ns, c2, use_sel2, sel_col2, key2, sel_val2, S_sorted}};
    if (c1 > kDirectCols || c2 > kDirectCols) return msd_indexed(t, 2, 1, key2, SMJ_KEY_INT64, out, h_rows, s);
    return msd_any(t, 2, 1, key2, out, h_rows, s);
}


extern "C" int smj_dev_sort_merge_join(const T *R, int64_t nr, int c1, int use_sel1, int sel_col1, T sel_val1,
                                       int key1, const T *S, int64_t ns, int c2, int use_sel2, int sel_col2,
                                       T sel_val2, int key2, T *R_sorted, T *S_sorted, T *out, int64_t *h_rows,
                                       void *stream) {
    const int rc = smj_dev_sort_merge_join_impl(R, nr, c1, use_sel1, sel_col1, sel_val1, key1, S, ns, c2, use_sel2, sel_col2, sel_val2, key2, R_sorted, S_sorted, out, h_rows, stream);
    if (rc == SMJ_OK) trim_if_over_limit();
    return rc;
}

// The fused call in two halves (smj.h): _begin launches the pipeline up to
// its final kernel and returns; _end runs the count scan and compaction into
// out, reads the plan back and runs the fallback tiers.  Between them the
// caller's host thread is free -- the multi-GPU driver posts the next stage's
// transfers there -- but must not start another pipeline call (the job owns
// the thread's scratch).  Shapes the split does not cover (partitioned
// sizes, wide rows, an empty table) run whole inside _end.
struct SmjJob {
    MsdIn in[2];
    MsdCtx cx;
    hipStream_t s = nullptr;
    bool whole = false;
    const T *R = nullptr, *S = nullptr;
    int64_t nr = 0, ns = 0;
    int c1 = 0, c2 = 0, use_sel1 = 0, sel_col1 = 0, key1 = 0, use_sel2 = 0, sel_col2 = 0, key2 = 0;
    T sel_val1 = 0, sel_val2 = 0;
    T *R_sorted = nullptr, *S_sorted = nullptr;
};
thread_local SmjJob *t_job = nullptr;  // the thread's job between _begin and _end

extern "C" int smj_dev_sort_merge_join_begin(const T *R, int64_t nr, int c1, int use_sel1, int sel_col1, T sel_val1,
                                             int key1, const T *S, int64_t ns, int c2, int use_sel2, int sel_col2,
                                             T sel_val2, int key2, T *R_sorted, T *S_sorted, void *stream,
                                             void **job) {
    if (!job) return SMJ_ERR_INVALID;
    *job = nullptr;
    if (t_job) return SMJ_ERR_INVALID;  // an earlier _begin has not been ended
    SMJ_TRY(msd_check(R, nr, c1, use_sel1, sel_col1, key1, R_sorted));
    SMJ_TRY(msd_check(S, ns, c2, use_sel2, sel_col2, key2, S_sorted));
    SmjJob *j = new (std::nothrow) SmjJob;
    if (!j) return SMJ_ERR_NOMEM;
    *j = SmjJob{};
    j->s = (hipStream_t)stream;
    j->R = R, j->S = S, j->nr = nr, j->ns = ns, j->c1 = c1, j->c2 = c2;
    j->use_sel1 = use_sel1, j->sel_col1 = sel_col1, j->sel_val1 = sel_val1, j->key1 = key1;
    j->use_sel2 = use_sel2, j->sel_col2 = sel_col2, j->sel_val2 = sel_val2, j->key2 = key2;
    j->R_sorted = R_sorted, j->S_sorted = S_sorted;
    j->whole = nr == 0 || ns == 0 || c1 > kDirectCols || c2 > kDirectCols || g_force_parts > 0 ||
               nr > kMsdSingleMax || ns > kMsdSingleMax;
    if (!j->whole) {
        j->in[0] = MsdIn{R, nr, c1, use_sel1, sel_col1, key1, sel_val1, R_sorted};
        j->in[1] = MsdIn{S, ns, c2, use_sel2, sel_col2, key2, sel_val2, S_sorted};
        const int rc = msd_front(j->in, 2, 1, key2, j->s, nullptr, &j->cx);
        if (rc != SMJ_OK) {
            delete j;
            return rc;
        }
    }
    t_job = j;
    t_job_open = true;
    g_open_jobs++;
    *job = j;
    return SMJ_OK;
}

// smj_dev_sort_merge_join_begin for 2-column tables of which either may be
// packed (pkX: one word per row, smj_dev_partition_regions_pk's format with
// bases kbX / obX), no select -- the multi-GPU driver's received stages.
// Packed tables over kMsdSingleMax rows are SMJ_ERR_UNSUPPORTED (the caller
// unpacks them first: smj_dev_unpack_rows).
extern "C" int smj_dev_sort_merge_join_begin_pk(const int64_t *R, int64_t nr, int key1, int pk1, int64_t kb1, int64_t ob1,
                                                const int64_t *S, int64_t ns, int key2, int pk2, int64_t kb2,
                                                int64_t ob2, T *R_sorted, T *S_sorted, void *stream, void **job) {
    if (!job) return SMJ_ERR_INVALID;
    *job = nullptr;
    if (!pk1 && !pk2)
        return smj_dev_sort_merge_join_begin(R, nr, 2, 0, 0, 0, key1, S, ns, 2, 0, 0, 0, key2, R_sorted, S_sorted, stream,
                                             job);
    if (t_job) return SMJ_ERR_INVALID;
    SMJ_TRY(msd_check(R, nr, 2, 0, 0, key1, R_sorted));
    SMJ_TRY(msd_check(S, ns, 2, 0, 0, key2, S_sorted));
    if (nr == 0 || ns == 0 || nr > kMsdSingleMax || ns > kMsdSingleMax || g_force_parts > 0)
        return SMJ_ERR_UNSUPPORTED;
    SmjJob *j = new (std::nothrow) SmjJob;
    if (!j) return SMJ_ERR_NOMEM;
    *j = SmjJob{};
    j->s = (hipStream_t)stream;
    j->R = R, j->S = S, j->nr = nr, j->ns = ns, j->c1 = 2, j->c2 = 2, j->key1 = key1, j->key2 = key2;
    j->R_sorted = R_sorted, j->S_sorted = S_sorted;
    j->whole = false;
    j->in[0] = MsdIn{R, nr, 2, 0, 0, key1, 0, R_sorted};
    j->in[1] = MsdIn{S, ns, 2, 0, 0, key2, 0, S_sorted};
    j->in[0].pk = pk1, j->in[0].pkk = kb1, j->in[0].pkp = ob1;
    j->in[1].pk = pk2, j->in[1].pkk = kb2, j->in[1].pkp = ob2;
    const int rc = msd_front(j->in, 2, 1, key2, j->s, nullptr, &j->cx);
    if (rc != SMJ_OK) {
        delete j;
        return rc;
    }
    t_job = j;
    t_job_open = true;
    g_open_jobs++;
    *job = j;
    return SMJ_OK;
}

static int smj_dev_sort_merge_join_end_impl(void *job, T *out, int64_t *h_rows) {
    SmjJob *j = (SmjJob *)job;
    if (!j || j != t_job || !h_rows) return SMJ_ERR_INVALID;
    t_job = nullptr;
    t_job_open = false;
    g_open_jobs--;
    std::unique_ptr<SmjJob> own(j);
    h_rows[0] = h_rows[1] = h_rows[2] = 0;
    if (j->whole)
        return smj_dev_sort_merge_join(j->R, j->nr, j->c1, j->use_sel1, j->sel_col1, j->sel_val1, j->key1, j->S,
                                       j->ns, j->c2, j->use_sel2, j->sel_col2, j->sel_val2, j->key2, j->R_sorted,
                                       j->S_sorted, out, h_rows, j->s);
    if (!out) {  // the launched half still has to drain before its scratch is reused
        hipStreamSynchronize(j->s);
        return SMJ_ERR_INVALID;
    }
    return msd_back(j->cx, out, h_rows, j->s);
}


extern "C" int smj_dev_sort_merge_join_end(void *job, T *out, int64_t *h_rows) {
    const int rc = smj_dev_sort_merge_join_end_impl(job, out, h_rows);
    if (rc == SMJ_OK) trim_if_over_limit();
    return rc;
}

// The host-pointer path with staged input (smj_host.hip): R and S are
// copied from the host in chunks overlapping part_a.  SMJ_ERR_UNSUPPORTED
// where the plain path must be used instead (wide rows, partitioned sizes,
// an empty table).
int smj::msd_staged_sort_merge_join(const int64_t *hR, int64_t nr, int c1, int sc1, int64_t sv1, int key1,
                                    const int64_t *hS, int64_t ns, int c2, int sc2, int64_t sv2, int key2, int64_t *dR,
                                    int64_t *dS, int64_t *dRs, int64_t *dSs, int64_t *dJ, int64_t *h_rows,
                                    hipStream_t s, hipStream_t copy, hipEvent_t landed) {
    const int64_t lcm = 4 * 5 * 3 * 7 * 8192;  // every pass-A tile (msd_tile: 512 x {16, 8, 5, 4, 3, 2} rows) divides it
    const int64_t chunk = lcm * std::max<int64_t>(1, (int64_t)(1 << 22) / lcm);
    // tables that fit one chunk gain nothing from staging (one copy each is
    // faster: tools/h2d_overlap.py, 1e6 rows 0.96 vs 1.36 ms)
    if (c1 > kDirectCols || c2 > kDirectCols || nr == 0 || ns == 0 || nr > kMsdSingleMax || ns > kMsdSingleMax ||
        g_force_parts > 0 || std::max(nr, ns) <= chunk)
        return SMJ_ERR_UNSUPPORTED;
    SMJ_TRY(check_table(nr, c1, sc1, key1));
    SMJ_TRY(check_table(ns, c2, sc2, key2));
    const MsdIn t[2] = {{dR, nr, c1, 1, sc1, key1, sv1, dRs}, {dS, ns, c2, 1, sc2, key2, sv2, dSs}};
    const MsdStage stg{{hR, hS}, copy, chunk, landed};
    return msd_run(t, 2, 1, key2, dJ, h_rows, s, &stg);
}

// Diagnostic only (not part of smj.h): run every pipeline call in the
// partitioned mode with `parts` parts (0 = automatic: tables over 1.6e8 rows).
extern "C" void smj_debug_force_parts(int parts) { g_force_parts = parts > 0 ? parts : 0; }

// Diagnostic only (not part of smj.h): in the partitioned mode's overlapped
// order, the front phase of part `part` fails as if its scratch set could not
// be allocated (-1: never); returns the part from which the previous
// partitioned call ran its parts one at a time on one set (-1: it did not).
extern "C" int smj_debug_fail_front(int part) {
    const int r = g_seq_from;
    g_fail_front = part;
    g_seq_from = -1;
    return r;
}

extern "C" void smj_debug_spin_limit(int64_t polls) {
    g_spin_limit = polls < 0 ? kMsdSpinLimit : (uint32_t)std::min<int64_t>(polls, UINT32_MAX);
}

// ---------------------------------------------------------------------------
// T = UINT64 / DOUBLE (common.h:3-9): the int64 pipeline
// on an order-preserving image of the key and select columns
// (launch_key_map), the select value mapped alike, and the same columns of
// the outputs mapped back.  NaN keys are outside the contract (the
// reference's comparisons give no order for them); -0.0 compares equal to
// +0.0 as in the reference and comes back as +0.0 in key / select columns.
// ---------------------------------------------------------------------------
namespace {
struct TypedScratch {
    int dev = -1;
    void *r = nullptr, *s = nullptr;
    size_t cr = 0, cs = 0;
};
std::map<int, TypedScratch> g_typed;

void typed_free_all() {
    for (auto &kv : g_typed) {
        if (kv.second.dev < 0) continue;
        hipSetDevice(kv.second.dev);
        dev_free(kv.second.r);
        dev_free(kv.second.s);
    }
    g_typed.clear();
}

int64_t key_fwd_host(uint64_t u, int ktype) {
    if (ktype == SMJ_KEY_UINT64) return (int64_t)(u ^ 0x8000000000000000ull);
    if (u == 0x8000000000000000ull) u = 0;  // -0.0
    return (int64_t)((u >> 63) ? (u ^ 0x7fffffffffffffffull) : u);
}
uint32_t cols_mask(int key, int use_sel, int sel_col) { return (1u << key) | (use_sel ? 1u << sel_col : 0u); }
}  // namespace

static int smj_dev_sort_merge_join_typed_impl(int key_type, const void *R, int64_t nr, int c1, int use_sel1,
                                             int sel_col1, uint64_t sel_bits1, int key1, const void *S, int64_t ns,
                                             int c2, int use_sel2, int sel_col2, uint64_t sel_bits2, int key2,
                                             void *R_sorted, void *S_sorted, void *out, int64_t *h_rows,
                                             void *stream) {
    if (key_type == SMJ_KEY_INT64)
        return smj_dev_sort_merge_join((const T *)R, nr, c1, use_sel1, sel_col1, (T)sel_bits1, key1, (const T *)S, ns,
                                       c2, use_sel2, sel_col2, (T)sel_bits2, key2, (T *)R_sorted, (T *)S_sorted,
                                       (T *)out, h_rows, stream);
    if (key_type != SMJ_KEY_UINT64 && key_type != SMJ_KEY_DOUBLE) return SMJ_ERR_INVALID;
    if (!h_rows) return SMJ_ERR_INVALID;
    SMJ_TRY(msd_check((const T *)R, nr, c1, use_sel1, sel_col1, key1, (const T *)R_sorted));
    SMJ_TRY(msd_check((const T *)S, ns, c2, use_sel2, sel_col2, key2, (const T *)S_sorted));
    hipStream_t st = (hipStream_t)stream;
    if (c1 > kDirectCols || c2 > kDirectCols) {  // index sort: the map is applied inside the pair kernel
        if (nr > 0 && ns > 0 && !out) return SMJ_ERR_INVALID;
        h_rows[0] = h_rows[1] = h_rows[2] = 0;
        MsdIn t[2] = {{(const T *)R, nr, c1, use_sel1, sel_col1, key1, key_fwd_host(sel_bits1, key_type), (T *)R_sorted},
                      {(const T *)S, ns, c2, use_sel2, sel_col2, key2, key_fwd_host(sel_bits2, key_type), (T *)S_sorted}};
        if (nr > 0 && ns > 0) {
            SMJ_TRY(msd_indexed(t, 2, 1, key2, key_type, (T *)out, h_rows, st));
        } else {
            int64_t rows[3] = {0, 0, 0};
            for (int x = 0; x < 2; x++)
                if (t[x].n) {
                    SMJ_TRY(msd_indexed(&t[x], 1, 0, 0, key_type, nullptr, rows, st));
                    h_rows[x] = rows[0];
                }
        }
        HIP_TRY(hipStreamSynchronize(st));
        return SMJ_OK;
    }
    int dev = 0;
    const int key = scratch_key(&dev);
    if (key < 0) return SMJ_ERR_HIP;
    TypedScratch *tsp;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        tsp = &g_typed[key];
        tsp->dev = dev;
    }
    TypedScratch &ts = *tsp;
    SMJ_TRY(grow(&ts.r, &ts.cr, std::max<size_t>(1, (size_t)nr * c1 * 8)));
    SMJ_TRY(grow(&ts.s, &ts.cs, std::max<size_t>(1, (size_t)ns * c2 * 8)));
    const uint32_t mR = cols_mask(key1, use_sel1, sel_col1), mS = cols_mask(key2, use_sel2, sel_col2);
    HIP_TRY(launch_key_map((const int64_t *)R, (int64_t *)ts.r, nr, c1, mR, key_type, 0, st));
    HIP_TRY(launch_key_map((const int64_t *)S, (int64_t *)ts.s, ns, c2, mS, key_type, 0, st));
    SMJ_TRY(smj_dev_sort_merge_join((const T *)ts.r, nr, c1, use_sel1, sel_col1, key_fwd_host(sel_bits1, key_type),
                                    key1, (const T *)ts.s, ns, c2, use_sel2, sel_col2,
                                    key_fwd_host(sel_bits2, key_type), key2, (T *)R_sorted, (T *)S_sorted, (T *)out,
                                    h_rows, stream));
    HIP_TRY(launch_key_map((const int64_t *)R_sorted, (int64_t *)R_sorted, h_rows[0], c1, mR, key_type, 1, st));
    HIP_TRY(launch_key_map((const int64_t *)S_sorted, (int64_t *)S_sorted, h_rows[1], c2, mS, key_type, 1, st));
    if (h_rows[2] > 0) {  // join rows: R's columns, then S's without key2
        uint32_t mO = mR;
        if (use_sel2 && sel_col2 != key2) mO |= 1u << (c1 + (sel_col2 < key2 ? sel_col2 : sel_col2 - 1));
        HIP_TRY(launch_key_map((const int64_t *)out, (int64_t *)out, h_rows[2], c1 + c2 - 1, mO, key_type, 1, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    return SMJ_OK;
}


extern "C" int smj_dev_sort_merge_join_typed(int key_type, const void *R, int64_t nr, int c1, int use_sel1,
                                             int sel_col1, uint64_t sel_bits1, int key1, const void *S, int64_t ns,
                                             int c2, int use_sel2, int sel_col2, uint64_t sel_bits2, int key2,
                                             void *R_sorted, void *S_sorted, void *out, int64_t *h_rows,
                                             void *stream) {
    const int rc = smj_dev_sort_merge_join_typed_impl(key_type, R, nr, c1, use_sel1, sel_col1, sel_bits1, key1, S, ns, c2, use_sel2, sel_col2, sel_bits2, key2, R_sorted, S_sorted, out, h_rows, stream);
    if (rc == SMJ_OK) trim_if_over_limit();
    return rc;
}

// ---------------------------------------------------------------------------
// multi-GPU range partition
// ---------------------------------------------------------------------------
extern "C" int smj_dev_partition_count(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val,
                                       int key_col, const T *d_splitters, int n_split, int64_t *h_counts,
                                       T *h_minmax, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    SMJ_TRY(check_table(n, cols, use_select ? sel_col : 0, key_col));
    SMJ_TRY(direct_only(cols));
    if (n_split < 0 || n_split > kMaxSplitters || !h_counts || !h_minmax) return SMJ_ERR_INVALID;
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    int64_t spl[kMaxSplitters];
    if (n_split) {
        if (!d_splitters) return SMJ_ERR_INVALID;
        HIP_TRY(hipMemcpyAsync(spl, d_splitters, sizeof(int64_t) * n_split, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    constexpr int kNB = 1 << kBucketBits;
    unsigned long long *gcount = (unsigned long long *)sc->dcount;
    long long *gminmax = (long long *)(sc->dcount + kNB);
    HIP_TRY(hipMemsetAsync(gcount, 0, sizeof(int64_t) * kNB, s));
    const long long init[2] = {INT64_MAX, INT64_MIN};
    HIP_TRY(hipMemcpyAsync(gminmax, init, sizeof init, hipMemcpyHostToDevice, s));
    if (n > 0) {
        ProfScope ps("partition_count", 8.0 * cols * n, s);
        HIP_TRY(launch_hist_bucket(in, n, cols, use_select, sel_col, sel_val, key_col, spl, n_split, gcount,
                                   gminmax, s));
    }
    HIP_TRY(hipMemcpyAsync(sc->h_small, sc->dcount, sizeof(int64_t) * (kNB + 2), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int b = 0; b <= n_split; b++) h_counts[b] = sc->h_small[b];
    h_minmax[0] = sc->h_small[kNB];
    h_minmax[1] = sc->h_small[kNB + 1];
    return SMJ_OK;
}

extern "C" int smj_dev_partition_scatter(const T *in, int64_t n, int cols, int use_select, int sel_col,
                                         T sel_val, int key_col, const T *d_splitters, int n_split,
                                         const int64_t *h_counts, T *out, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    SMJ_TRY(check_table(n, cols, use_select ? sel_col : 0, key_col));
    SMJ_TRY(direct_only(cols));
    if (n_split < 0 || n_split > kMaxSplitters || !h_counts || !out || in == out) return SMJ_ERR_INVALID;
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    if (n == 0) return SMJ_OK;
    int64_t spl[kMaxSplitters];
    if (n_split) {
        HIP_TRY(hipMemcpyAsync(spl, d_splitters, sizeof(int64_t) * n_split, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    // global bucket starts -> device (one tiny copy)
    uint32_t *h_base = (uint32_t *)sc->h_small;
    int64_t run = 0, total = 0;
    for (int b = 0; b < (1 << kBucketBits); b++) {
        h_base[b] = (uint32_t)run;
        if (b <= n_split) run += h_counts[b];
    }
    total = run;
    if (total >= SMJ_MAX_ROWS) return SMJ_ERR_TOO_LARGE;
    uint32_t *d_base = (uint32_t *)(sc->dcount);
    HIP_TRY(hipMemcpyAsync(d_base, h_base, sizeof(uint32_t) * (1 << kBucketBits), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(&sc->ctr[3], 0, sizeof(Counters), s));
    PassSpec ps{};
    ps.src = in;
    ps.nsrc = n;
    ps.dst = out;
    ps.cols = cols;
    ps.use_select = use_select;
    ps.sel_col = sel_col;
    ps.key_col = key_col;
    ps.sel_val = sel_val;
    ps.kind = DIGIT_BUCKET;
    ps.spl = spl;
    ps.nspl = n_split;
    SMJ_TRY(run_pass(sc, ps, d_base, &sc->ctr[3], false, total, s));
    // the pinned staging buffer is reused by the next call: wait for the copy
    HIP_TRY(hipStreamSynchronize(s));
    return SMJ_OK;
}

// One-call partition (the multi-GPU hot path): chunk_hist -> bases on the
// device -> chunk_scatter; the bucket counts come back with the rows, so no
// separate counting pass reads the table.
extern "C" int smj_dev_partition(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val,
                                 int key_col, const T *d_splitters, int n_split, T *out, int64_t *h_counts,
                                 void *stream) {
    hipStream_t s = (hipStream_t)stream;
    SMJ_TRY(check_table(n, cols, use_select ? sel_col : 0, key_col));
    SMJ_TRY(direct_only(cols));
    if (n_split < 0 || n_split > kMaxSplitters || !h_counts) return SMJ_ERR_INVALID;
    for (int b = 0; b <= n_split; b++) h_counts[b] = 0;
    if (n == 0) return SMJ_OK;
    if (!out || in == out || (n_split && !d_splitters)) return SMJ_ERR_INVALID;
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    int64_t spl[kMaxSplitters];
    if (n_split) {
        HIP_TRY(hipMemcpyAsync(spl, d_splitters, sizeof(int64_t) * n_split, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    PassSpec ps{};
    ps.src = in;
    ps.nsrc = n;
    ps.dst = out;
    ps.cols = cols;
    ps.use_select = use_select;
    ps.sel_col = sel_col;
    ps.key_col = key_col;
    ps.sel_val = sel_val;
    ps.kind = DIGIT_BUCKET;
    ps.spl = spl;
    ps.nspl = n_split;
    ps.trash = sc->trash;
    SMJ_TRY(grow(&sc->status, &sc->status_bytes, (size_t)pass_chunks(ps) * pass_radix(ps) * sizeof(uint32_t)));
    uint32_t *table = (uint32_t *)sc->status;
    uint32_t *d_base = (uint32_t *)sc->dcount;                                // [64] u32
    unsigned long long *d_cnt = (unsigned long long *)(sc->dcount + 64);      // [64] u64
    const double rowb = 8.0 * cols;
    {
        ProfScope p1("partition_hist", rowb * n, s);
        HIP_TRY(launch_chunk_hist(ps, table, s));
    }
    {
        ProfScope p2("partition_scan", 0, s);
        HIP_TRY(launch_chunk_scan_dev(ps, table, sc->segsum, d_base, d_cnt, s));
    }
    HIP_TRY(hipMemsetAsync(&sc->ctr[3], 0, sizeof(Counters), s));
    {
        ProfScope p3("partition_scatter", rowb * 2 * n, s);  // bytes assume every row selected
        HIP_TRY(launch_chunk_scatter(ps, table, &sc->ctr[3], s));
    }
    HIP_TRY(hipMemcpyAsync(sc->h_small, d_cnt, sizeof(int64_t) * (n_split + 1), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int b = 0; b <= n_split; b++) h_counts[b] = sc->h_small[b];
    return SMJ_OK;
}

// the plan / apply split (smj.h): host splitters, device counts, no stream sync
namespace {
int partition_spec(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val, int key_col,
                   const T *h_spl, int n_split, PassSpec &ps) {
    SMJ_TRY(check_table(n, cols, use_select ? sel_col : 0, key_col));
    SMJ_TRY(direct_only(cols));
    if (n_split < 0 || n_split > kMaxSplitters || (n_split && !h_spl)) return SMJ_ERR_INVALID;
    for (int i = 1; i < n_split; i++)
        if (h_spl[i] < h_spl[i - 1]) return SMJ_ERR_INVALID;  // the bucket search needs sorted splitters
    ps = PassSpec{};
    ps.src = in;
    ps.nsrc = n;
    ps.cols = cols;
    ps.use_select = use_select;
    ps.sel_col = sel_col;
    ps.key_col = key_col;
    ps.sel_val = sel_val;
    ps.kind = DIGIT_BUCKET;
    ps.spl = h_spl;
    ps.nspl = n_split;
    return SMJ_OK;
}
}  // namespace

extern "C" size_t smj_partition_plan_bytes(int64_t n, int cols, int n_split) {
    if (n < 0 || cols < 1 || cols > kDirectCols || n_split < 0 || n_split > kMaxSplitters) return 0;
    PassSpec ps{};
    ps.nsrc = std::max<int64_t>(n, 1);
    ps.cols = cols;
    ps.kind = DIGIT_BUCKET;
    ps.nspl = n_split;
    return (size_t)pass_chunks(ps) * pass_radix(ps) * sizeof(uint32_t);
}

extern "C" int smj_dev_partition_plan(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val,
                                      int key_col, const T *h_spl, int n_split, void *d_plan, int64_t *d_counts,
                                      void *stream) {
    hipStream_t s = (hipStream_t)stream;
    PassSpec ps;
    SMJ_TRY(partition_spec(in, n, cols, use_select, sel_col, sel_val, key_col, h_spl, n_split, ps));
    if (!d_counts || (n && (!in || !d_plan))) return SMJ_ERR_INVALID;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(d_counts, 0, sizeof(int64_t) * (n_split + 1), s));
        return SMJ_OK;
    }
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    ps.trash = sc->trash;
    uint32_t *table = (uint32_t *)d_plan;
    uint32_t *d_base = (uint32_t *)sc->dcount;                            // [64] u32
    unsigned long long *d_cnt = (unsigned long long *)(sc->dcount + 64);  // [64] u64
    {
        ProfScope p1("partition_hist", 8.0 * cols * n, s);
        HIP_TRY(launch_chunk_hist(ps, table, s));
    }
    {
        ProfScope p2("partition_scan", 0, s);
        HIP_TRY(launch_chunk_scan_dev(ps, table, sc->segsum, d_base, d_cnt, s));
    }
    HIP_TRY(hipMemcpyAsync(d_counts, d_cnt, sizeof(int64_t) * (n_split + 1), hipMemcpyDeviceToDevice, s));
    return SMJ_OK;
}

static int partition_regions_impl(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val, int key_col,
                                  const T *h_spl, int n_split, const int64_t *h_region, T *out, int64_t *d_counts,
                                  int pk, int64_t pkk, int64_t pkp, void *stream);

extern "C" int smj_dev_partition_regions(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val,
                                         int key_col, const T *h_spl, int n_split, const int64_t *h_region, T *out,
                                         int64_t *d_counts, void *stream) {
    return partition_regions_impl(in, n, cols, use_select, sel_col, sel_val, key_col, h_spl, n_split, h_region, out,
                                  d_counts, 0, 0, 0, stream);
}

extern "C" int smj_dev_partition_regions_pk(const T *in, int64_t n, int use_select, int sel_col, T sel_val, int key_col,
                                            const T *h_spl, int n_split, const int64_t *h_region, int64_t *out,
                                            int64_t *d_counts, int64_t key_base, int64_t other_base, void *stream) {
    return partition_regions_impl(in, n, 2, use_select, sel_col, sel_val, key_col, h_spl, n_split, h_region, out,
                                  d_counts, 1, key_base, other_base, stream);
}

static int partition_regions_impl(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val, int key_col,
                                  const T *h_spl, int n_split, const int64_t *h_region, T *out, int64_t *d_counts,
                                  int pk, int64_t pkk, int64_t pkp, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    PassSpec ps;
    SMJ_TRY(partition_spec(in, n, cols, use_select, sel_col, sel_val, key_col, h_spl, n_split, ps));
    if (!d_counts || !h_region) return SMJ_ERR_INVALID;
    const int nb = n_split + 1;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(d_counts, 0, sizeof(int64_t) * (nb + 1), s));
        return SMJ_OK;
    }
    if (!in || !out || in == out) return SMJ_ERR_INVALID;
    // region starts / capacities and the splitters travel as kernel arguments
    // (stream-ordered: no host staging buffer a second call could overwrite)
    P1Words w{};
    for (int b = 0; b < nb; b++) {
        if (h_region[b] < 0 || h_region[nb + b] < 0 || (b && h_region[b] < h_region[b - 1] + h_region[nb + b - 1]))
            return SMJ_ERR_INVALID;  // regions ascending and disjoint (the caller sized out for them)
        w.v[b] = h_region[b];
        w.v[64 + b] = h_region[nb + b];
    }
    for (int i = 0; i < n_split; i++) w.v[128 + i] = h_spl[i];
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    if (!sc->rwords) HIP_TRY(dev_alloc(&sc->rwords, sizeof(int64_t) * (192 + 2)));
    const int64_t tile = p1_tile(cols), nt = (n + tile - 1) / tile;
    SMJ_TRY(grow(&sc->rst, &sc->c_rst, (size_t)nt * nb * 8));
    uint32_t *flags = (uint32_t *)(sc->rwords + 192);
    HIP_TRY(launch_p1_words(w, sc->rwords, flags, s));
    HIP_TRY(hipMemsetAsync(sc->rst, 0, (size_t)nt * nb * 8, s));
    HIP_TRY(hipMemsetAsync(d_counts, 0, sizeof(int64_t) * nb, s));
    MsdPart1Params p{};
    p.src = in;
    p.n = n;
    p.use_sel = use_select;
    p.sel_col = sel_col;
    p.key_col = key_col;
    p.nspl = n_split;
    p.sel_val = sel_val;
    p.spl = sc->rwords + 128;
    p.oc = sc->rwords;
    p.dst = out;
    p.status = (unsigned long long *)sc->rst;
    p.tot = (long long *)d_counts;
    p.flags = flags;
    p.ntiles = nt;
    p.pk = pk;
    p.pkk = pkk;
    p.pkp = pkp;
    {
        ProfScope ps1("partition_1pass", (pk ? 8.0 + 8.0 * cols : 16.0 * cols) * n, s);
        HIP_TRY(launch_msd_part1(p, cols, s));
    }
    HIP_TRY(launch_p1_finish(flags, d_counts + nb, s));
    return SMJ_OK;
}

extern "C" int smj_dev_partition_apply(const T *in, int64_t n, int cols, int use_select, int sel_col, T sel_val,
                                       int key_col, const T *h_spl, int n_split, const void *d_plan, T *out,
                                       void *stream) {
    hipStream_t s = (hipStream_t)stream;
    PassSpec ps;
    SMJ_TRY(partition_spec(in, n, cols, use_select, sel_col, sel_val, key_col, h_spl, n_split, ps));
    if (n == 0) return SMJ_OK;
    if (!in || !out || in == out || !d_plan) return SMJ_ERR_INVALID;
    DevScratch *sc;
    SMJ_TRY(scratch(&sc));
    ps.dst = out;
    ps.trash = sc->trash;
    HIP_TRY(hipMemsetAsync(&sc->ctr[3], 0, sizeof(Counters), s));
    ProfScope p3("partition_scatter", 8.0 * cols * 2 * n, s);  // bytes assume every row selected
    HIP_TRY(launch_chunk_scatter(ps, (uint32_t *)d_plan, &sc->ctr[3], s));
    return SMJ_OK;
}

// ---------------------------------------------------------------------------
// synthetic data
// ---------------------------------------------------------------------------
extern "C" int smj_dev_gen_uniform(T *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t key_range,
                                   void *stream) {
    if (rows < 0 || (rows && !out) || key_range == 0) return SMJ_ERR_INVALID;
    if (rows == 0) return SMJ_OK;
    HIP_TRY(launch_gen_uniform(out, row0, rows, seed, key_range, (hipStream_t)stream));
    return SMJ_OK;
}

extern "C" double smj_zipf_zeta(int64_t n, double theta) {
    // exact sum for the head, Euler-Maclaurin for the tail (n up to 1e10)
    const int64_t H = std::min<int64_t>(n, 1000000);
    double z = 0;
    for (int64_t i = H; i >= 1; i--) z += pow((double)i, -theta);
    if (n > H) {
        const double a = (double)H, b = (double)n, s = 1.0 - theta;
        z += (pow(b, s) - pow(a, s)) / s + 0.5 * (pow(b, -theta) - pow(a, -theta)) -
             theta / 12.0 * (pow(b, -theta - 1) - pow(a, -theta - 1));
    }
    return z;
}

extern "C" int smj_dev_gen_zipf(T *out, int64_t row0, int64_t rows, uint64_t seed, int64_t domain, double theta,
                                double zeta_n, void *stream) {
    if (rows < 0 || (rows && !out) || domain < 2 || !(theta > 0 && theta < 1)) return SMJ_ERR_INVALID;
    if (rows == 0) return SMJ_OK;
    HIP_TRY(launch_gen_zipf(out, row0, rows, seed, domain, theta, zeta_n, (hipStream_t)stream));
    return SMJ_OK;
}

extern "C" int smj_dev_gen_wide(T *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t plant_seed,
                                int64_t plant_rows, void *stream) {
    if (rows < 0 || (rows && !out) || plant_rows < 0 || row0 < 0) return SMJ_ERR_INVALID;
    if (rows == 0) return SMJ_OK;
    HIP_TRY(launch_gen_wide(out, row0, rows, seed, plant_seed, plant_rows, (hipStream_t)stream));
    return SMJ_OK;
}

extern "C" int smj_dev_digest(const T *rows, int64_t n_rows, int col_num, int64_t pos0, uint64_t *d_digest,
                              void *stream) {
    if (n_rows < 0 || (n_rows && !rows) || !d_digest || col_num < 1 || col_num > SMJ_MAX_COLS || pos0 < 0)
        return SMJ_ERR_INVALID;
    HIP_TRY(launch_digest(rows, n_rows, col_num, pos0, d_digest, (hipStream_t)stream));
    return SMJ_OK;
}

extern "C" int smj_dev_dist_sample(const T *R, int64_t nR, int colsR, int keyR, const T *S, int64_t nS, int colsS,
                                   int keyS, int samples, int64_t *d_buf, void *stream) {
    if (nR < 0 || nS < 0 || (nR && !R) || (nS && !S) || !d_buf || samples < 1 || samples > (1 << 20) ||
        colsR < 1 || colsS < 1 || keyR < 0 || keyR >= colsR || keyS < 0 || keyS >= colsS)
        return SMJ_ERR_INVALID;
    DistSampleArgs a{};
    a.t[0] = R;
    a.t[1] = S;
    a.n[0] = nR;
    a.n[1] = nS;
    a.cols[0] = colsR;
    a.cols[1] = colsS;
    a.key[0] = keyR;
    a.key[1] = keyS;
    a.samples = samples;
    a.buf = d_buf;
    HIP_TRY(launch_dist_sample(a, (hipStream_t)stream));
    return SMJ_OK;
}

extern "C" int smj_dev_dist_splitters(const int64_t *d_all, int world, int64_t stride, int parts, const int32_t *q20,
                                      int64_t *d_out, void *stream) {
    if (!d_all || !d_out || world < 1 || stride <= kDistHdr || parts < 1 || parts > kDistMaxParts)
        return SMJ_ERR_INVALID;
    DistSelectArgs a{};
    a.all = d_all;
    a.stride = stride;
    a.world = world;
    a.parts = parts;
    a.use_q = q20 ? 1 : 0;
    for (int i = 0; q20 && i < parts - 1; i++) {
        if (q20[i] < 0 || q20[i] > (1 << 20)) return SMJ_ERR_INVALID;
        a.q20[i] = q20[i];
    }
    a.out = d_out;
    HIP_TRY(launch_dist_select(a, (hipStream_t)stream));
    return SMJ_OK;
}

extern "C" int smj_dev_unpack_rows(const int64_t *d_packed, int64_t n, int key_col, int64_t key_base,
                                   int64_t other_base, int64_t *d_out, void *stream) {
    if (n < 0 || (n && (!d_packed || !d_out)) || key_col < 0 || key_col > 1) return SMJ_ERR_INVALID;
    HIP_TRY(launch_unpack_rows(d_packed, n, key_col, key_base, other_base, d_out, (hipStream_t)stream));
    return SMJ_OK;
}

// ---------------------------------------------------------------------------
// device memory account (smj_scratch_bytes, smj_set_scratch_limit, smj_trim)
// ---------------------------------------------------------------------------
namespace {
std::mutex g_alloc_mu;
std::unordered_map<void *, size_t> g_alloc;
int64_t g_held = 0;
int64_t g_scratch_limit = -1;  // bytes; -1 = none (SMJ_SCRATCH_LIMIT)
bool g_limit_read = false;
}  // namespace

hipError_t smj::dev_alloc_raw(void **p, size_t n) {
    const hipError_t e = hipMalloc(p, n);
    if (e == hipSuccess && *p) {
        std::lock_guard<std::mutex> lk(g_alloc_mu);
        g_alloc[*p] = n;
        g_held += (int64_t)n;
    }
    return e;
}

hipError_t smj::dev_free(void *p) {
    if (!p) return hipSuccess;
    {
        std::lock_guard<std::mutex> lk(g_alloc_mu);
        auto it = g_alloc.find(p);
        if (it != g_alloc.end()) {
            g_held -= (int64_t)it->second;
            g_alloc.erase(it);
        }
    }
    return hipFree(p);
}

int64_t smj::dev_held_bytes() {
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    return g_held;
}

extern "C" int64_t smj_scratch_bytes(void) { return dev_held_bytes(); }

extern "C" void smj_set_scratch_limit(int64_t bytes) {
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    g_scratch_limit = bytes < 0 ? -1 : bytes;
    g_limit_read = true;
}

int smj::open_jobs() { return g_open_jobs.load(); }

void smj::trim_if_over_limit() {
    int64_t lim, held;
    {
        std::lock_guard<std::mutex> lk(g_alloc_mu);
        if (!g_limit_read) {
            const char *e = getenv("SMJ_SCRATCH_LIMIT");
            g_scratch_limit = e ? atoll(e) : -1;
            g_limit_read = true;
        }
        lim = g_scratch_limit;
        held = g_held;
    }
    if (lim >= 0 && held > lim && g_open_jobs.load() == 0) smj_trim();
}

// ---------------------------------------------------------------------------
// release of every library-owned buffer (smj_finalize, smj_host.hip)
// ---------------------------------------------------------------------------
void smj::api_free_all() {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto &kv : g_scratch) {
        DevScratch &s = kv.second;
        if (s.dev < 0) continue;
        hipSetDevice(s.dev);
        for (void *q : {s.tmp, s.status, s.apart, (void *)s.hist, (void *)s.plan, (void *)s.ctr, (void *)s.dcount,
                        (void *)s.segsum, (void *)s.trash, s.rst, (void *)s.rwords})
            dev_free(q);
        hipHostFree(s.h_plan);
        hipHostFree(s.h_small);
    }
    g_scratch.clear();
    msd_free_all();
    idx_free_all();
    typed_free_all();
    for (auto &kv : g_event_pool)
        for (auto e : kv.second) hipEventDestroy(e);
    g_event_pool.clear();
}

void smj::set_scratch_slot(int slot) { t_slot = slot; }
