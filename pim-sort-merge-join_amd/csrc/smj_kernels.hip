// smj_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the sort-merge-join
// hot path.  Row layout: row-major int64 tables (include/common.h), any column
// count 1..8, key / select columns chosen at run time.
//
// Reference map (the DPU kernels these replace; /root/reference/sort-merge-join):
//   hist_radix_kernel + onesweep_kernel  <- select.c (:63-194) fused with
//       sort_dpu.c (:189-328) and the merge tree (merge_dpu.c :55-223, app.c
//       :412-547): a stable LSD radix sort whose first pass also applies the
//       WHERE predicate (cpu_app.c select_in_cpu :81-112 + insertion_sort_in_cpu
//       :172-202 semantics: stable, signed ascending).
//   merge_partition_kernel + join_tile_kernel <- join.c (:58-266) + host
//       splitters (app.c :585-633): merge-path partitioned 1:1 zip join
//       (cpu_app.c join_in_cpu :204-266 semantics).
//   merge_tile_kernel <- merge_dpu.c (:55-223): stable merge-path merge.
//
// Everything here is HBM-bandwidth-bound integer work: no MFMA.  See DESIGN.md
// for the roofline and per-kernel algorithmic bytes.
#include "smj_internal.h"
#include "smj_device.h"

#include <math.h>

#include <stdlib.h>

#include <algorithm>

namespace smj {

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
// lower_bound / upper_bound over an LDS key array
__device__ __forceinline__ int lds_lower_bound(const int64_t *a, int n, int64_t k) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int lds_upper_bound(const int64_t *a, int n, int64_t k) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] <= k) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------
// digit functors
// ---------------------------------------------------------------------------
struct RadixDigit {   // digit of the biased key relative to a base: ((key ^ 2^63) - base) >> shift
    uint64_t kbase;   // base ^ 2^63, so that the digit is (key - kbase) >> shift (mod 2^64)
    int shift;
    __device__ __forceinline__ uint32_t operator()(int64_t key) const {
        return (uint32_t)(((uint64_t)key - kbase) >> shift);
    }
};
struct ZeroDigit {    // select-only compaction: one bin
    __device__ __forceinline__ uint32_t operator()(int64_t) const { return 0; }
};
struct BucketDigit {  // multi-GPU range partition: #splitters < key
    int64_t spl[kMaxSplitters];
    int nspl;
    __device__ __forceinline__ uint32_t operator()(int64_t key) const {
        uint32_t b = 0;  // unused entries are INT64_MAX (make_bucket): never < key
#pragma unroll
        for (int i = 0; i < kMaxSplitters; i++) b += spl[i] < key ? 1u : 0u;
        return b;
    }
};
// A digit functor as the pass kernels evaluate it.  BucketDigit's splitters
// are staged in LDS (padded to 64 with INT64_MAX) and searched branch-free in
// 6 probes instead of 63 64-bit compares per key.
static_assert(kMaxSplitters == 63, "the staged bucket search assumes 2^6 - 1 splitters");
template <class DigitF>
struct DigitLds {
    static constexpr int N = 1;
    __device__ static void stage(const DigitF &, int64_t *, int) {}
    __device__ static uint32_t eval(const DigitF &f, const int64_t *, int64_t key) { return f(key); }
};
template <>
struct DigitLds<BucketDigit> {
    static constexpr int N = 64;
    __device__ static void stage(const BucketDigit &f, int64_t *sp, int tid) {
        if (tid < 64) sp[tid] = tid < kMaxSplitters ? f.spl[tid] : INT64_MAX;
    }
    __device__ static uint32_t eval(const BucketDigit &, const int64_t *sp, int64_t key) {
        uint32_t b = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1) b += sp[b + step - 1] < key ? step : 0u;
        return b;
    }
};

// ---------------------------------------------------------------------------
// one radix / bucket / compaction pass = chunk_hist -> chunk_scan -> chunk_scatter
//
// A pass is cut into chunks of kChunkTiles tiles.  chunk_hist counts each
// chunk's digits (the WHERE predicate of pass 0 applied), chunk_scan turns
// the [chunk][digit] table into exclusive global offsets in place, and
// chunk_scatter moves every chunk with one workgroup that walks its tiles in
// order, carrying running digit offsets in LDS.  No workgroup ever waits on
// another: on MI355X a cross-XCD status round trip under full streaming load
// costs microseconds, which made a decoupled look-back the bottleneck.
// ---------------------------------------------------------------------------
template <class DigitF>
struct PassParams {
    const int64_t *src;
    int64_t *dst;
    int64_t nsrc;
    int64_t sel_val;
    int use_select, sel_col, key_col, dbg;  // dbg bit 3: phase stamps (SMJ_DEBUG_PASS), 0 in production
    DigitF digit;
    uint32_t *table;  // [nchunks][RADIX]: counts (chunk_hist) -> exclusive offsets (chunk_scan)
    Counters *ctr;
    int64_t *trash;   // kSortThreads * 16 int64 scratch: dummy / empty-tile stores
};

template <int COLS, int DBITS>
struct PassLds {
    static constexpr int RADIX = 1 << DBITS;
    static constexpr int TILE = sort_tile_rows(COLS);
    static constexpr int ROW_BYTES = TILE * COLS * 8;
    static constexpr int CNT_BYTES = kSortWaves * RADIX * 4;
    static constexpr int A = ROW_BYTES > CNT_BYTES ? ROW_BYTES : CNT_BYTES;
    static constexpr int R16 = ((RADIX * 4 + 15) / 16) * 16;
    static constexpr int OFF_DIG = A;              // u16 digit of every staged row (slot order)
    static constexpr int OFF_BIN = OFF_DIG + ((TILE * 2 + 15) / 16) * 16;  // u32 tile-local digit starts
    static constexpr int OFF_ADJ = OFF_BIN + R16;  // i32 global - local offset per digit
    static constexpr int OFF_RUN = OFF_ADJ + R16;  // i32 running global offset per digit
    static constexpr int OFF_MISC = OFF_RUN + R16;
    static constexpr int OFF_PH = OFF_MISC + 128;  // u64[16] phase stamps (SMJ_DEBUG_PASS bit 3)
    static constexpr int BYTES = OFF_PH + 128;
};

// Rows past `end` are loaded from row end-1 instead (and masked out by the
// caller): no branches around the loads, so the compiler can count them in
// s_waitcnt vmcnt(N) instead of draining every outstanding store (vmcnt(0)).
template <int COLS, int ITEMS>
__device__ __forceinline__ void load_tile(const int64_t *__restrict__ src, int64_t end, int64_t row0,
                                          int64_t (&rows)[ITEMS][COLS]) {
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const int64_t r = min(row0 + it * 64, end - 1);
        load_row<COLS>(src + r * COLS, rows[it]);
    }
}

// ---- chunk_hist: digit counts of every chunk ------------------------------
template <int COLS, int DBITS, class DigitF>
__global__ __launch_bounds__(512) void chunk_hist_kernel(const PassParams<DigitF> p) {
    constexpr int RADIX = 1 << DBITS;
    constexpr uint32_t MASK = RADIX - 1;
    constexpr int64_t CH = chunk_rows(COLS);
    constexpr int U = 8;
    __shared__ uint32_t sh[RADIX];
    __shared__ int64_t s_dspl[DigitLds<DigitF>::N];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < RADIX; i += 512) sh[i] = 0;
    DigitLds<DigitF>::stage(p.digit, s_dspl, tid);
    __syncthreads();
    const int64_t begin = (int64_t)blockIdx.x * CH;
    const int64_t end = min(begin + CH, p.nsrc);
    for (int64_t r0 = begin; r0 < end; r0 += 512 * U) {
        int64_t key[U], sv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t r = min(r0 + u * 512 + tid, end - 1);  // clamped: no branches around loads
            key[u] = p.src[r * COLS + p.key_col];
            sv[u] = p.src[r * COLS + p.sel_col];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t r = r0 + u * 512 + tid;
            const bool ok = r < end && (!p.use_select || sv[u] > p.sel_val);
            const uint64_t act = __ballot(ok);
            if (act == 0) continue;
            const uint32_t d = DigitLds<DigitF>::eval(p.digit, s_dspl, key[u]) & MASK;
            const int leader = __ffsll((unsigned long long)act) - 1;
            const uint32_t dl = __shfl(d, leader, 64);
            if (__ballot(ok && d == dl) == act) {
                if (lane == leader) atomicAdd(&sh[dl], (uint32_t)__popcll(act));
            } else if (ok) {
                atomicAdd(&sh[d], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < RADIX; i += 512) p.table[(size_t)blockIdx.x * RADIX + i] = sh[i];
}

// ---- chunk_scan: table[c][d] <- base[d] + sum_{c' < c} table[c'][d] ---------
// grid (ceil(radix/64), kScanSegs) x 256 threads; lane = digit, the chunks of
// a segment are split into 4 contiguous runs, one per wave.
__device__ __forceinline__ void scan_seg_range(int64_t nchunks, int64_t &c0, int64_t &c1) {
    const int64_t L = (nchunks + kScanSegs - 1) / kScanSegs;
    c0 = min((int64_t)blockIdx.y * L, nchunks);
    c1 = min(c0 + L, nchunks);
    const int64_t L4 = (c1 - c0 + 3) / 4;
    const int w = threadIdx.x >> 6;
    const int64_t s0 = min(c0 + w * L4, c1);
    c1 = min(s0 + L4, c1);
    c0 = s0;
}

__global__ __launch_bounds__(256) void chunk_scan_seg_kernel(const uint32_t *__restrict__ table, int64_t nchunks,
                                                             int radix, uint32_t *__restrict__ segsum) {
    __shared__ uint32_t part[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int bin = blockIdx.x * 64 + lane;
    int64_t c0, c1;
    scan_seg_range(nchunks, c0, c1);
    uint32_t sum = 0;
    if (bin < radix) {
#pragma unroll 8
        for (int64_t c = c0; c < c1; c++) sum += table[c * radix + bin];
    }
    part[w][lane] = sum;
    __syncthreads();
    if (w == 0 && bin < radix)
        segsum[(size_t)blockIdx.y * radix + bin] = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
}

__global__ __launch_bounds__(256) void chunk_scan_apply_kernel(uint32_t *__restrict__ table, int64_t nchunks,
                                                               int radix, const uint32_t *__restrict__ segsum,
                                                               const uint32_t *__restrict__ base) {
    __shared__ uint32_t part[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int bin = blockIdx.x * 64 + lane;
    int64_t c0, c1;
    scan_seg_range(nchunks, c0, c1);
    uint32_t sum = 0;
    if (bin < radix) {
#pragma unroll 8
        for (int64_t c = c0; c < c1; c++) sum += table[c * radix + bin];
    }
    part[w][lane] = sum;
    __syncthreads();
    if (bin >= radix) return;
    uint32_t off = base ? base[bin] : 0u;
    for (int s = 0; s < (int)blockIdx.y; s++) off += segsum[(size_t)s * radix + bin];
    for (int v = 0; v < w; v++) off += part[v][lane];
#pragma unroll 8
    for (int64_t c = c0; c < c1; c++) {
        const uint32_t x = table[c * radix + bin];
        table[c * radix + bin] = off;
        off += x;
    }
}

// Bases of a pass whose digit totals are not known on the host (the
// multi-GPU partition): totals = sum of the scan segments, bases = their
// exclusive prefix in digit order.  One wave, lane = digit (radix <= 64).
__global__ __launch_bounds__(64) void digit_base_kernel(const uint32_t *__restrict__ segsum, int radix,
                                                        uint32_t *__restrict__ base,
                                                        unsigned long long *__restrict__ counts) {
    const int lane = threadIdx.x;
    uint32_t tot = 0;
    if (lane < radix)
        for (int sg = 0; sg < kScanSegs; sg++) tot += segsum[(size_t)sg * radix + lane];
    const uint32_t incl = wave_incl_scan(tot, lane);
    if (lane < radix) {
        base[lane] = incl - tot;
        counts[lane] = tot;
    }
}

// ---- chunk_scatter: stable scatter of one chunk per workgroup ---------------
// Tiles of the chunk are taken in order; the next tile's rows are loaded into
// registers while the current one is ranked and scattered.  Per tile:
//   rank     stable digit ranks: DBITS ballots per 64-row item find the lanes
//            with the same digit (one v_bitop3 per ballot half folds each bit
//            into the peer mask); per-wave running counters in LDS order the
//            items of a wave; a cross-wave prefix orders the waves;
//   stage    rows (and their digits, u16) are written to LDS in digit order
//            (block scan of the digit totals gives each digit's local start);
//   scatter  consecutive LDS rows of one digit leave as one contiguous run at
//            the digit's running global offset.
// Every wave zeroes only its own counter row, so no barrier separates the
// zeroing from the ranking.  Row offsets inside a chunk are 32-bit.
// Diagnostic phase stamps (SMJ_DEBUG_PASS bit 3): cycles between the
// barriers of chunk_scatter, summed over workgroups (thread 0's view).
__device__ unsigned long long g_phase_cycles[16];
#define SMJ_STAMP(k)                                                       \
    if (p.dbg & 8) {                                                       \
        if (tid == 0) {                                                    \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
            s_ph[k] += t_ - s_ph[15];                                      \
            s_ph[15] = t_;                                                 \
        }                                                                  \
    }

template <int COLS, int DBITS, class DigitF>
__global__ __launch_bounds__(kSortThreads, 4) void chunk_scatter_kernel(const PassParams<DigitF> p) {
    using L = PassLds<COLS, DBITS>;
    constexpr int RADIX = L::RADIX;
    constexpr int ITEMS = sort_items(COLS);
    constexpr uint32_t TILE = L::TILE;
    constexpr int64_t CH = chunk_rows(COLS);
    constexpr uint32_t MASK = RADIX - 1;
    constexpr int BPT = RADIX > kSortThreads ? RADIX / kSortThreads : 1;  // digits d = tid + j*kSortThreads

    __shared__ __attribute__((aligned(16))) unsigned char smem[L::BYTES];
    __shared__ int64_t s_dspl[DigitLds<DigitF>::N];
    int64_t *s_rows = reinterpret_cast<int64_t *>(smem);          // staging tile (after ranking)
    uint32_t *s_wcnt = reinterpret_cast<uint32_t *>(smem);        // [wave][digit] counters (ranking)
    uint16_t *s_dig = reinterpret_cast<uint16_t *>(smem + L::OFF_DIG);
    uint32_t *s_binstart = reinterpret_cast<uint32_t *>(smem + L::OFF_BIN);
    int32_t *s_adj = reinterpret_cast<int32_t *>(smem + L::OFF_ADJ);
    int32_t *s_run = reinterpret_cast<int32_t *>(smem + L::OFF_RUN);
    uint32_t *s_misc = reinterpret_cast<uint32_t *>(smem + L::OFF_MISC);
    unsigned long long *s_ph = reinterpret_cast<unsigned long long *>(smem + L::OFF_PH);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t begin = (int64_t)blockIdx.x * CH;
    const uint32_t clen = (uint32_t)min(CH, p.nsrc - begin);  // rows of this chunk (>= 1)
    const int64_t *src = p.src + begin * COLS;
    const uint32_t lane_row = (uint32_t)wave * (ITEMS * 64) + lane;
    uint32_t *wc = s_wcnt + wave * RADIX;

#pragma unroll
    for (int j = 0; j < BPT; j++) {
        const int d = tid + j * kSortThreads;
        if (d < RADIX) s_run[d] = (int32_t)p.table[(size_t)blockIdx.x * RADIX + d];
    }
    zero_counters<RADIX>(wc, lane);
    DigitLds<DigitF>::stage(p.digit, s_dspl, tid);
    int64_t rows[ITEMS][COLS];
#pragma unroll
    for (int it = 0; it < ITEMS; it++) load_row<COLS>(src + (int64_t)min(lane_row + it * 64, clen - 1) * COLS, rows[it]);
    // ITEMS dummy stores behind the first loads: the loop is then always
    // entered with (loads, then ITEMS stores) in flight, exactly as from its
    // back edge, so hipcc's vmcnt waits for the rows skip the stores
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        int64_t z[COLS];
#pragma unroll
        for (int c = 0; c < COLS; c++) z[c] = 0;
        store_row<COLS>(p.trash + ((size_t)it * kSortThreads + tid) * COLS, z);
    }
    uint32_t chunk_total = 0;
    if ((p.dbg & 8) && tid == 0) {
        for (int k = 0; k < 15; k++) s_ph[k] = 0;
        s_ph[15] = __builtin_amdgcn_s_memtime();
    }
    __syncthreads();  // s_run published

    for (uint32_t tile0 = 0;;) {
        SMJ_STAMP(0);
        // ---- digits (select predicate fused into pass 0)
        const uint32_t row0 = tile0 + lane_row;
        uint32_t dig[ITEMS];
        uint32_t vmask = 0;
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {  // branch-free: every term is computed
            const bool inb = row0 + it * 64 < clen;
            const bool pass = !p.use_select | (pick<COLS>(rows[it], p.sel_col) > p.sel_val);
            const bool v = inb & pass;
            dig[it] = v ? (DigitLds<DigitF>::eval(p.digit, s_dspl, pick<COLS>(rows[it], p.key_col)) & MASK) : 0u;
            vmask |= v ? (1u << it) : 0u;
        }
        // ---- stable rank within the tile; dig[it] becomes (rank << 16) | digit
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const bool v = (vmask >> it) & 1u;
            const uint64_t act = __ballot(v);
            uint32_t plo = (uint32_t)act, phi = (uint32_t)(act >> 32);
            const uint32_t dd = dig[it];
#pragma unroll
            for (int b = 0; b < DBITS; b++) {
                const uint32_t sb = (uint32_t)((int32_t)(dd << (31 - b)) >> 31);  // ~0 iff bit b
                const uint64_t bb = __ballot(sb != 0u);
                plo = peer_fold(plo, (uint32_t)bb, sb);
                phi = peer_fold(phi, (uint32_t)(bb >> 32), sb);
            }
            if (v) {
                const uint32_t base = wc[dd];
                // lanes below this one with the same digit (mbcnt), and the last of them
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, base));
                const uint64_t peers = ((uint64_t)phi << 32) | plo;
                if ((peers >> lane) == 1ull) wc[dd] = base + (uint32_t)__popcll(peers);
                dig[it] = dd | (rank << 16);
            }
        }
        __syncthreads();  // B2
        SMJ_STAMP(1);

        // ---- per-digit totals, cross-wave exclusive prefix in place
        uint32_t tot[BPT], incl[BPT];
#pragma unroll
        for (int j = 0; j < BPT; j++) {
            const int d = tid + j * kSortThreads;
            uint32_t run = 0;
            if (d < RADIX) {
#pragma unroll
                for (int w = 0; w < kSortWaves; w++) {
                    const uint32_t c = s_wcnt[w * RADIX + d];
                    s_wcnt[w * RADIX + d] = run;
                    run += c;
                }
            }
            tot[j] = run;
            incl[j] = wave_incl_scan(run, lane);
            if (lane == 63) s_misc[4 + j * kSortWaves + wave] = incl[j];
        }
        __syncthreads();  // B3
        SMJ_STAMP(2);
        // ---- block exclusive scan of the totals in digit order -> local starts
        uint32_t run = 0;
#pragma unroll
        for (int j = 0; j < BPT; j++) {
            uint32_t before = 0, all = 0;
#pragma unroll
            for (int w = 0; w < kSortWaves; w++) {
                const uint32_t x = s_misc[4 + j * kSortWaves + w];
                before += (w < wave) ? x : 0u;
                all += x;
            }
            const int d = tid + j * kSortThreads;
            if (d < RADIX) s_binstart[d] = run + before + incl[j] - tot[j];
            run += all;
        }
        const uint32_t tile_total = run;
        chunk_total += tile_total;
        __syncthreads();  // B4
        SMJ_STAMP(3);

        // ---- tile-local slots: dig[it] becomes (digit << 16) | slot
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const uint32_t d = dig[it] & 0xffffu;
            const uint32_t slot = s_binstart[d] + wc[d] + (dig[it] >> 16);
            dig[it] = (d << 16) | slot;
        }
        const uint32_t next0 = tile0 + TILE;
        __syncthreads();  // B5: counters dead, the region becomes the staging tile
        SMJ_STAMP(4);
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            if ((vmask >> it) & 1u) {
                const uint32_t slot = dig[it] & 0xffffu;
                store_row<COLS>(s_rows + (size_t)slot * COLS, rows[it]);
                s_dig[slot] = (uint16_t)(dig[it] >> 16);
            }
        }
        // the rows are staged: their registers now take the next tile's rows,
        // in flight while this tile is scattered (after the last tile: an
        // L2-hot reload of this one -- unconditional, so vmcnt stays exact)
        {
            const uint32_t nrow0 = (next0 < clen ? next0 : tile0) + lane_row;
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                load_row<COLS>(src + (int64_t)min(nrow0 + it * 64, clen - 1) * COLS, rows[it]);
        }
#pragma unroll
        for (int j = 0; j < BPT; j++) {
            const int d = tid + j * kSortThreads;
            if (d < RADIX) {
                const int32_t r = s_run[d];
                s_adj[d] = r - (int32_t)s_binstart[d];
                s_run[d] = r + (int32_t)tot[j];
            }
        }
        __syncthreads();  // B6
        SMJ_STAMP(5);

        // ---- scatter: consecutive LDS rows of one digit -> consecutive HBM rows
        // exactly ITEMS unconditional stores per thread (a static count keeps
        // the compiler's vmcnt waits for the prefetch exact): slots past
        // tile_total rewrite the last row with its own value; an empty tile
        // writes its (garbage) slots to the trash buffer
        {
            const bool any = tile_total > 0;
            uint32_t slot[ITEMS], d[ITEMS];
#pragma unroll
            for (int it = 0; it < ITEMS; it++) {
                slot[it] = any ? min((uint32_t)(tid + it * kSortThreads), tile_total - 1u) : 0u;
                d[it] = s_dig[slot[it]];
            }
#pragma unroll
            for (int it = 0; it < ITEMS; it++) {
                int64_t r[COLS];
                load_row<COLS>(s_rows + (size_t)slot[it] * COLS, r);
                const int64_t g = (int64_t)s_adj[d[it]] + (int64_t)slot[it];
                int64_t *q = any ? p.dst + g * COLS : p.trash + ((size_t)it * kSortThreads + tid) * COLS;
                store_row<COLS>(q, r);
            }
        }
        SMJ_STAMP(6);
        if ((p.dbg & 8) && tid == 0) s_ph[7]++;
        if (next0 >= clen) break;
        __syncthreads();  // B0: staging tile read before it becomes counters again
        zero_counters<RADIX>(wc, lane);
        tile0 = next0;
    }
    if (tid == 0 && chunk_total) atomicAdd(&p.ctr->count, chunk_total);
    if ((p.dbg & 8) && tid == 0)
        for (int k = 0; k < 8; k++) atomicAdd(&g_phase_cycles[k], s_ph[k]);
}

// ---------------------------------------------------------------------------
// histogram (upsweep) of all digit positions of the selected rows
// ---------------------------------------------------------------------------
// Histograms of every digit position of the selected rows, chunk by chunk
// (the chunks of the first radix pass): the digit-0 counts of each chunk are
// also written to table0[chunk][*], so the first pass needs no chunk_hist of
// its own when digit 0 is not trivial (the usual case).
template <int COLS>
__global__ __launch_bounds__(512) void hist_radix_kernel(const int64_t *__restrict__ src, int64_t n,
                                                         int use_select, int sel_col, int64_t sel_val,
                                                         int key_col, uint64_t base,
                                                         uint32_t *__restrict__ ghist,
                                                         uint32_t *__restrict__ table0) {
    __shared__ uint32_t sh[kNumPos * kRadix];
    __shared__ uint32_t sh0[kRadix];  // this block's digit-0 totals over its chunks
    constexpr int64_t CH = chunk_rows(COLS);
    constexpr int U = 8;
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < kNumPos * kRadix; i += 512) sh[i] = 0;
    for (int i = tid; i < kRadix; i += 512) sh0[i] = 0;
    __syncthreads();
    const int64_t nchunks = (n + CH - 1) / CH;
    for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
        const int64_t begin = chunk * CH, end = min(begin + CH, n);
        for (int64_t r0 = begin; r0 < end; r0 += 512 * U) {
            int64_t key[U], sv[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int64_t r = min(r0 + u * 512 + tid, end - 1);  // clamped: no branches around loads
                key[u] = src[r * COLS + key_col];
                sv[u] = src[r * COLS + sel_col];
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int64_t r = r0 + u * 512 + tid;
                const bool ok = r < end && (!use_select || sv[u] > sel_val);
                const uint64_t act = __ballot(ok);
                if (act == 0) continue;
                const int leader = __ffsll((unsigned long long)act) - 1;
                const uint64_t x = biased(key[u]) - base;
#pragma unroll
                for (int ps = 0; ps < kNumPos; ps++) {
                    const uint32_t d = (uint32_t)(x >> (ps * kRadixBits)) & (kRadix - 1);
                    const uint32_t dl = __shfl(d, leader, 64);
                    const uint64_t same = __ballot(ok && d == dl);
                    if (same == act) {
                        if (lane == leader) atomicAdd(&sh[ps * kRadix + dl], (uint32_t)__popcll(act));
                    } else if (ok) {
                        atomicAdd(&sh[ps * kRadix + d], 1u);
                    }
                }
            }
        }
        __syncthreads();
        for (int i = tid; i < kRadix; i += 512) {
            const uint32_t c = sh[i];
            table0[chunk * kRadix + i] = c;
            sh0[i] += c;
            sh[i] = 0;
        }
        __syncthreads();
    }
    for (int i = tid; i < kNumPos * kRadix; i += 512) {
        const uint32_t c = i < kRadix ? sh0[i] : sh[i];
        if (c) atomicAdd(&ghist[i], c);
    }
}

// ---------------------------------------------------------------------------
// plan: selected row count, non-trivial digit positions, in-place exclusive
// scan of their histograms.  One workgroup of 1024 threads (= kRadix).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t block_sum_1024(uint32_t v, uint32_t *scratch) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) s += scratch[w];
    return s;
}
__device__ __forceinline__ uint32_t block_max_1024(uint32_t v, uint32_t *scratch) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor(v, o, 64));
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) s = max(s, scratch[w]);
    return s;
}
__device__ __forceinline__ uint32_t block_excl_scan_1024(uint32_t v, uint32_t *scratch) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t incl = wave_incl_scan(v, lane);
    __syncthreads();
    if (lane == 63) scratch[wave] = incl;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) off += (w < wave) ? scratch[w] : 0u;
    return off + incl - v;
}

__global__ __launch_bounds__(1024) void plan_kernel(uint32_t *ghist, SortPlan *plan) {
    static_assert(kRadix <= 1024, "plan_kernel: one thread per digit");
    __shared__ uint32_t scratch[16];
    __shared__ int s_np;
    __shared__ int s_pos[8];
    const int tid = threadIdx.x;
    const bool mine = tid < kRadix;
    const uint32_t m = block_sum_1024(mine ? ghist[tid] : 0u, scratch);
    if (tid == 0) s_np = 0;
    __syncthreads();
    for (int ps = 0; ps < kNumPos; ps++) {
        const uint32_t mx = block_max_1024(mine ? ghist[ps * kRadix + tid] : 0u, scratch);
        if (tid == 0 && m > 0 && mx < m && s_np < 8) s_pos[s_np++] = ps;
        __syncthreads();
    }
    if (tid == 0 && s_np == 0) { s_pos[0] = 0; s_np = 1; }  // still one pass: it compacts
    __syncthreads();
    const int np = s_np;
    for (int k = 0; k < np; k++) {
        uint32_t *h = ghist + s_pos[k] * kRadix;
        const uint32_t e = block_excl_scan_1024(mine ? h[tid] : 0u, scratch);
        if (mine) h[tid] = e;
    }
    if (tid == 0) {
        plan->m = m;
        plan->npasses = np;
        for (int k = 0; k < 8; k++) plan->pos[k] = k < np ? s_pos[k] : -1;
    }
}

// ---------------------------------------------------------------------------
// multi-GPU partition: per-bucket counts + min/max of selected keys
// ---------------------------------------------------------------------------
template <int COLS>
__global__ __launch_bounds__(512) void hist_bucket_kernel(const int64_t *__restrict__ src, int64_t n,
                                                          int use_select, int sel_col, int64_t sel_val,
                                                          int key_col, const BucketDigit dg,
                                                          unsigned long long *gcount,
                                                          long long *gminmax) {
    __shared__ uint32_t sh[1 << kBucketBits];
    __shared__ long long smin[8], smax[8];
    __shared__ int64_t s_dspl[DigitLds<BucketDigit>::N];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < (1 << kBucketBits)) sh[tid] = 0;
    DigitLds<BucketDigit>::stage(dg, s_dspl, tid);
    __syncthreads();
    long long mn = INT64_MAX, mx = INT64_MIN;
    for (int64_t r = (int64_t)blockIdx.x * 512 + tid; r < n; r += (int64_t)gridDim.x * 512) {
        const int64_t key = src[r * COLS + key_col];
        const bool ok = !use_select || src[r * COLS + sel_col] > sel_val;
        if (ok) {
            atomicAdd(&sh[DigitLds<BucketDigit>::eval(dg, s_dspl, key)], 1u);
            mn = min(mn, (long long)key);
            mx = max(mx, (long long)key);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (long long)__shfl_xor(mn, o, 64));
        mx = max(mx, (long long)__shfl_xor(mx, o, 64));
    }
    if (lane == 0) { smin[wave] = mn; smax[wave] = mx; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 8; w++) { mn = min(mn, smin[w]); mx = max(mx, smax[w]); }
        if (mn != INT64_MAX) {
            atomicMin(&gminmax[0], mn);
            atomicMax(&gminmax[1], mx);
        }
    }
    if (tid < (1 << kBucketBits) && sh[tid]) atomicAdd(&gcount[tid], (unsigned long long)sh[tid]);
}

// ---------------------------------------------------------------------------
// merge path: a_t = #rows of A among the first min(t*kJoinTile, na+nb) rows
// of the stable merge (A first on equal keys); one thread per diagonal,
// binary search.  With run_start != nullptr the thread also finds the first
// A row carrying A[a_t].key (the join needs the start of the key run that a
// tile begins in): gallop backwards, then bisect -- one probe when keys are
// distinct, O(log run) under skew.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void merge_partition_kernel(const int64_t *__restrict__ a, int64_t na, int ca,
                                                              int ka, const int64_t *__restrict__ b, int64_t nb,
                                                              int cb, int kb, int64_t *apart, int64_t *run_start,
                                                              int64_t ntiles, int tile) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    const int64_t d = min(t * (int64_t)tile, na + nb);
    int64_t lo = max((int64_t)0, d - nb), hi = min(d, na);
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        // A[mid] precedes B[d-1-mid] iff A.key <= B.key  -> take more of A
        if (a[mid * ca + ka] <= b[(d - 1 - mid) * cb + kb]) lo = mid + 1; else hi = mid;
    }
    apart[t] = lo;
    if (!run_start || t == ntiles) return;
    int64_t first = lo;
    if (lo < na && lo > 0) {
        const int64_t k = a[lo * ca + ka];
        if (a[(lo - 1) * ca + ka] == k) {
            int64_t h = lo - 1, l = -1, step = 1;  // a[h] == k; first equal lies in (l, h]
            while (true) {
                const int64_t c = h - step;
                if (c < 0) { l = -1; break; }
                if (a[c * ca + ka] != k) { l = c; break; }
                h = c;
                step <<= 1;
            }
            int64_t x = l + 1;
            while (x < h) {
                const int64_t mid = (x + h) >> 1;
                if (a[mid * ca + ka] == k) h = mid; else x = mid + 1;
            }
            first = x;
        }
    }
    run_start[t] = first;
}

// ---------------------------------------------------------------------------
// join: one merge-path tile per workgroup (kJoinTile merged elements of R
// and S, R first on equal keys).  For an R row i with key k:
//   lbS(k) = first S row with key k   (merge path: S[<b0] < k <= S[>=b1], so
//            lbS = b0 + #S-piece rows merged before i)
//   lbR(k) = first R row with key k   (local, or galloped for the tile's first key)
//   occ = i - lbR(k);  partner p = lbS(k) + occ;  match iff S[p].key == k
// i.e. exactly cpu_app.c's zip (:211-227): the occ-th R occurrence of k pairs
// with the occ-th S occurrence.  Every thread walks kJoinPer consecutive
// merged elements.  Matches of tile t are written, in R order, to rows
// [a0_t, a0_t + cnt_t) of a slot buffer (a tile holds at most a1_t - a0_t
// matches) and counted; join_scan + join_compact then pack the slots.  No
// workgroup waits on another.
// ---------------------------------------------------------------------------
struct JoinParams {
    const int64_t *R;
    const int64_t *S;
    const int64_t *apart;
    const int64_t *run_start;  // first R row with the key of R[apart[t]]
    int64_t *slots;      // [nr][c1 + c2 - 1]
    uint32_t *counts;    // [ntiles]
    int64_t nr, ns, ntiles;
    int c1, key1, c2, key2;
    int jt;              // merged elements per tile (join_tile_size)
};

// Both pieces of a tile are staged in LDS as whole rows: one read of R and S
// whose loads are all in flight together (kJoinLoads unrolled, clamped, no
// branches around them).  The matches are then listed in LDS in output order
// and the slot rows leave as consecutive 8-B words, every lane of a store
// instruction on the next address.  LDS: 64 KiB of rows + 16 KiB of match list
// = 80 KiB, so two workgroups share a CU (one loads while the other walks).
constexpr int kJoinLdsWords = 8192;                       // 64 KiB
constexpr int kJoinLoads = kJoinLdsWords / kJoinThreads;  // 16 words per thread
constexpr uint32_t kMatchFar = 0xFFFFFu;  // list entry: (R row << 20) | (partner - b0), or this escape

// first row of a strided LDS piece whose word `col` is >= k
__device__ __forceinline__ int lds_lower_bound_rows(const int64_t *a, int stride, int col, int n, int64_t k) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid * stride + col] < k) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kJoinThreads) void join_tile_kernel(const JoinParams p) {
    __shared__ __attribute__((aligned(16))) int64_t s_rows[kJoinLdsWords];
    __shared__ uint32_t s_match[kJoinLdsWords / 2];  // first holds the wave sums of the count scan
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t tile = blockIdx.x;
    const int64_t L = p.nr + p.ns;
    const int64_t d0 = tile * p.jt, d1 = min(d0 + p.jt, L);
    const int64_t a0 = p.apart[tile], a1 = p.apart[tile + 1];
    const int64_t b0 = d0 - a0, b1 = d1 - a1;
    const int nR = (int)(a1 - a0), nS = (int)(b1 - b0), nM = nR + nS;
    const int c1 = p.c1, c2 = p.c2, k1 = p.key1, k2 = p.key2;
    const int sbase = nR * c1;            // S piece starts here in s_rows
    const int nwords = sbase + nS * c2;   // >= 1: a tile is never empty
    {
        const int64_t *rs = p.R + a0 * c1;
        const int64_t *ss = p.S + b0 * c2;
        int64_t v[kJoinLoads];
#pragma unroll
        for (int u = 0; u < kJoinLoads; u++) {
            const int j = min(tid + u * kJoinThreads, nwords - 1);
            v[u] = j < sbase ? rs[j] : ss[j - sbase];
        }
#pragma unroll
        for (int u = 0; u < kJoinLoads; u++) {
            const int j = tid + u * kJoinThreads;
            if (j < nwords) s_rows[j] = v[u];
        }
    }
    const int64_t lbr0 = p.run_start[tile];
    __syncthreads();

    // this thread's merged elements [m0, m1): merge-path split inside the tile
    const int per = p.jt / kJoinThreads;
    const int m0 = min(tid * per, nM), m1 = min(m0 + per, nM);
    int ai, bi;
    {
        int lo = max(0, m0 - nS), hi = min(m0, nR);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_rows[mid * c1 + k1] <= s_rows[sbase + (m0 - 1 - mid) * c2 + k2]) lo = mid + 1; else hi = mid;
        }
        ai = lo;
        bi = m0 - lo;
    }
    int64_t lbr = 0, prev = 0;
    bool have_prev = false;
    uint32_t mmask = 0;
    uint32_t ment[kJoinPer];  // list entry of the q-th element if it matched
#pragma unroll
    for (int q = 0; q < kJoinPer; q++) {
        ment[q] = 0;
        if (m0 + q < m1) {
            const int64_t rkey = ai < nR ? s_rows[ai * c1 + k1] : 0;
            const bool takeR = ai < nR && (bi >= nS || rkey <= s_rows[sbase + bi * c2 + k2]);
            if (takeR) {
                if (!have_prev || rkey != prev) {
                    if (have_prev) {
                        lbr = a0 + ai;  // a new run starts here
                    } else {        // first R row of this thread: find the run start
                        const int lo = lds_lower_bound_rows(s_rows, c1, k1, ai, rkey);
                        lbr = lo == 0 ? lbr0 : a0 + lo;
                    }
                    prev = rkey;
                    have_prev = true;
                }
                // S rows merged before this R row are exactly those with a smaller key
                const int64_t pidx = b0 + bi + (a0 + ai - lbr);
                if (pidx < p.ns) {
                    const int64_t skey = pidx < b1 ? s_rows[sbase + (int)(pidx - b0) * c2 + k2]
                                                   : p.S[pidx * c2 + k2];
                    if (skey == rkey) {
                        const int64_t rel = pidx - b0;
                        ment[q] = ((uint32_t)ai << 20) | (rel < (int64_t)kMatchFar ? (uint32_t)rel : kMatchFar);
                        mmask |= 1u << q;
                    }
                }
                ai++;
            } else {
                bi++;
            }
        }
    }
    // block exclusive scan of the match counts -> this thread's list offset
    const uint32_t cnt = __popc(mmask);
    const uint32_t incl = wave_incl_scan(cnt, lane);
    if (lane == 63) s_match[wave] = incl;
    __syncthreads();
    uint32_t off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kJoinThreads / 64; w++) {
        const uint32_t x = s_match[w];
        off += (w < wave) ? x : 0u;
        total += x;
    }
    off += incl - cnt;
    __syncthreads();  // wave sums read before the list overwrites them
#pragma unroll
    for (int q = 0; q < kJoinPer; q++)
        if ((mmask >> q) & 1u) s_match[off + __popc(mmask & ((1u << q) - 1u))] = ment[q];
    if (tid == 0) p.counts[tile] = total;
    __syncthreads();

    // slot rows [a0, a0 + total): word w = (row o, column c), c < c1 from R,
    // then the S columns without key2
    const int tc = c1 + c2 - 1;
    const uint32_t W = total * (uint32_t)tc;  // <= 4096 * 15 < 2^16: the reciprocal below is exact
    const uint32_t magic = tc > 1 ? (uint32_t)((0x100000000ull + tc - 1) / tc) : 0u;
    int64_t *dst = p.slots + a0 * tc;
    for (uint32_t w = tid; w < W; w += kJoinThreads) {
        const uint32_t o = tc > 1 ? __umulhi(w, magic) : w;
        const int c = (int)(w - o * (uint32_t)tc);
        const uint32_t m = s_match[o];
        const int r = (int)(m >> 20);
        int64_t val;
        if (c < c1) {
            val = s_rows[r * c1 + c];
        } else {
            const int j = c - c1;
            const int sc = j + (j >= k2 ? 1 : 0);
            int64_t part;
            if ((m & kMatchFar) != kMatchFar) {
                part = b0 + (m & kMatchFar);
            } else {  // partner far past the tile (long duplicate runs): recompute it
                const int64_t k = s_rows[r * c1 + k1];
                const int lbs = lds_lower_bound_rows(s_rows + sbase, c2, k2, nS, k);
                const int lo = lds_lower_bound_rows(s_rows, c1, k1, r, k);
                const int64_t lr = lo == 0 ? lbr0 : a0 + lo;
                part = b0 + lbs + (a0 + r - lr);
            }
            val = part < b1 ? s_rows[sbase + (int)(part - b0) * c2 + sc] : p.S[part * c2 + sc];
        }
        dst[w] = val;
    }
}

// exclusive scan of the per-tile match counts (one workgroup of 1024): rounds
// of 16 Ki counts staged through LDS (coalesced in and out), 16 per thread.
// Writes the joined row count to *out_rows.
__global__ __launch_bounds__(1024) void join_scan_kernel(const uint32_t *__restrict__ counts, int64_t ntiles,
                                                         uint32_t *__restrict__ offs, int64_t *out_rows) {
    constexpr int PER = 16, ROUND = 1024 * PER;
    __shared__ uint32_t s_c[ROUND];
    __shared__ uint32_t s_w[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t carry = 0;
    for (int64_t base = 0; base < ntiles; base += ROUND) {
        const int64_t n = min((int64_t)ROUND, ntiles - base);
        for (int i = tid; i < ROUND; i += 1024) s_c[i] = i < n ? counts[base + i] : 0u;
        __syncthreads();
        uint32_t v[PER], sum = 0;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            v[k] = s_c[tid * PER + k];
            sum += v[k];
        }
        const uint32_t incl = wave_incl_scan(sum, lane);
        if (lane == 63) s_w[wave] = incl;
        __syncthreads();
        uint32_t run = carry + incl - sum, all = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) {
            run += (w < wave) ? s_w[w] : 0u;
            all += s_w[w];
        }
#pragma unroll
        for (int k = 0; k < PER; k++) {
            s_c[tid * PER + k] = run;
            run += v[k];
        }
        __syncthreads();
        for (int i = tid; i < n; i += 1024) offs[base + i] = s_c[i];
        carry += all;
        __syncthreads();
    }
    if (tid == 0) *out_rows = (int64_t)carry;
}

// pack the slots: tile t's cnt_t rows at slot row a0_t -> output row offs_t
__global__ __launch_bounds__(256) void join_compact_kernel(const int64_t *__restrict__ slots,
                                                           const int64_t *__restrict__ apart,
                                                           const uint32_t *__restrict__ counts,
                                                           const uint32_t *__restrict__ offs, int tc,
                                                           int64_t *__restrict__ out) {
    const int64_t t = blockIdx.x;
    const int64_t n = (int64_t)counts[t] * tc;
    const int64_t *src = slots + apart[t] * tc;
    int64_t *dst = out + (int64_t)offs[t] * tc;
    for (int64_t i = threadIdx.x; i < n; i += 256) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// stable merge of two sorted runs (merge_dpu.c replacement)
// ---------------------------------------------------------------------------
template <int COLS>
__global__ __launch_bounds__(kJoinThreads) void merge_tile_kernel(const int64_t *__restrict__ a, int64_t na,
                                                                  const int64_t *__restrict__ b, int64_t nb,
                                                                  int key_col, const int64_t *apart,
                                                                  int64_t *__restrict__ out) {
    __shared__ int64_t s_keys[kJoinTile];
    const int tid = threadIdx.x;
    const int64_t tile = blockIdx.x;
    const int64_t d0 = tile * kJoinTile, d1 = min(d0 + kJoinTile, na + nb);
    const int64_t a0 = apart[tile], a1 = apart[tile + 1];
    const int64_t b0 = d0 - a0, b1 = d1 - a1;
    const int nA = (int)(a1 - a0), nB = (int)(b1 - b0);
    for (int j = tid; j < nA + nB; j += kJoinThreads)
        s_keys[j] = j < nA ? a[(a0 + j) * COLS + key_col] : b[(b0 + j - nA) * COLS + key_col];
    __syncthreads();
    for (int j = tid; j < nA + nB; j += kJoinThreads) {
        int64_t r[COLS];
        int64_t dst;
        if (j < nA) {
            dst = d0 + j + lds_lower_bound(s_keys + nA, nB, s_keys[j]);
            load_row<COLS>(a + (a0 + j) * COLS, r);
        } else {
            const int jj = j - nA;
            dst = d0 + jj + lds_upper_bound(s_keys, nA, s_keys[j]);
            load_row<COLS>(b + (b0 + jj) * COLS, r);
        }
        store_row<COLS>(out + dst * COLS, r);
    }
}

// ---------------------------------------------------------------------------
// synthetic tables: splitmix64, payload = global row index
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void gen_uniform_kernel(int64_t *out, int64_t row0, int64_t rows, uint64_t seed,
                                   uint64_t key_range) {
    const uint64_t salt = seed * 0xD1B54A32D192ED03ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t g = (uint64_t)(row0 + i);
        const uint64_t h = splitmix64(g + salt);
        i64x2 v;
        v.x = (long long)(1 + __umul64hi(h, key_range));
        v.y = (long long)g;
        reinterpret_cast<i64x2 *>(out)[i] = v;
    }
}

// C3-wide: full-range signed keys; with plant_rows > 0 a third
// of the rows take the key of a random row of the plant_seed table (smj.h)
__global__ void gen_wide_kernel(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t plant_seed,
                                uint64_t plant_rows) {
    const uint64_t salt = seed * 0xD1B54A32D192ED03ull, psalt = plant_seed * 0xD1B54A32D192ED03ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t g = (uint64_t)(row0 + i);
        uint64_t key = splitmix64(g + salt);
        if (plant_rows) {
            const uint64_t d = splitmix64(key ^ 0x2545F4914F6CDD1Dull);
            if (__umul64hi(d, 3ull) == 0) key = splitmix64(__umul64hi(splitmix64(d), plant_rows) + psalt);
        }
        i64x2 v;
        v.x = (long long)key;
        v.y = (long long)g;
        reinterpret_cast<i64x2 *>(out)[i] = v;
    }
}

__global__ void gen_zipf_kernel(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, int64_t n,
                                double theta, double zetan) {
    const uint64_t salt = seed * 0xD1B54A32D192ED03ull;
    const double alpha = 1.0 / (1.0 - theta);
    const double zeta2 = 1.0 + pow(0.5, theta);
    const double eta = (1.0 - pow(2.0 / (double)n, 1.0 - theta)) / (1.0 - zeta2 / zetan);
    const uint64_t A = 2654435761ull;  // odd prime, coprime with any 2^a 5^b domain
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t g = (uint64_t)(row0 + i);
        const double u = (double)(splitmix64(g + salt) >> 11) * 0x1.0p-53;
        const double uz = u * zetan;
        int64_t rank;  // 1-based
        if (uz < 1.0) rank = 1;
        else if (uz < zeta2) rank = 2;
        else rank = 1 + (int64_t)((double)n * pow(eta * u - eta + 1.0, alpha));
        rank = rank < 1 ? 1 : (rank > n ? n : rank);
        const uint64_t key = (uint64_t)(((unsigned __int128)(uint64_t)(rank - 1) * A + 12345u) %
                                        (unsigned __int128)(uint64_t)n);
        i64x2 v;
        v.x = (long long)(key + 1);
        v.y = (long long)g;
        reinterpret_cast<i64x2 *>(out)[i] = v;
    }
}

// ---------------------------------------------------------------------------
// order-sensitive table digest (smj_dev_digest): sum over rows of a hash of
// (global position, every cell), mod 2^64.  Sums of slices at their global
// positions add up to the digest of the whole, so per-rank digests of a
// distributed result can be checked against one single-GPU call.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t digest_row(uint64_t pos, const int64_t *r, int cols) {
    uint64_t h = splitmix64(pos ^ 0x5851F42D4C957F2Dull);
    for (int c = 0; c < cols; c++) h = splitmix64(h + (uint64_t)r[c]);
    return h;
}

__global__ __launch_bounds__(256) void digest_kernel(const int64_t *__restrict__ rows, int64_t n, int cols,
                                                     int64_t pos0, unsigned long long *out) {
    uint64_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        acc += digest_row((uint64_t)(pos0 + i), rows + i * cols, cols);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    __shared__ uint64_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(part[0] + part[1] + part[2] + part[3]));
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------

hipError_t launch_digest(const int64_t *rows, int64_t n, int cols, int64_t pos0, uint64_t *out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(uint64_t), s);
    if (e != hipSuccess || n <= 0) return e;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(n, 256), 4096));
    hipLaunchKernelGGL(digest_kernel, dim3(grid), dim3(256), 0, s, rows, n, cols, pos0, (unsigned long long *)out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// distributed splitters (smj/dist.py choose_splitters)
// ---------------------------------------------------------------------------
// Sample: thread j < 2 samples -> buf[kDistHdr + j]: the key of row
// jj (n - 1) / (c - 1) of table x (c = min(samples, n) rows, exact int64: the
// evenly spaced rows of dist.sample_index), R's c0 samples then S's c1, then
// INT64_MAX pads; thread 0 writes the header [c0 + c1, c0, c1, nR, nS].
__global__ __launch_bounds__(256) void dist_sample_kernel(const DistSampleArgs a) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= 2LL * a.samples) return;
    const int64_t c0 = min((int64_t)a.samples, a.n[0]), c1 = min((int64_t)a.samples, a.n[1]);
    if (j == 0) {
        a.buf[0] = c0 + c1;
        a.buf[1] = c0;
        a.buf[2] = c1;
        a.buf[3] = a.n[0];
        a.buf[4] = a.n[1];
    }
    int64_t v = INT64_MAX;
    if (j < c0 + c1) {
        const int x = j < c0 ? 0 : 1;
        const int64_t jj = x ? j - c0 : j, c = x ? c1 : c0, n = a.n[x];
        const int64_t r = jj * (n - 1) / max(c - 1, (int64_t)1);
        v = a.t[x][r * a.cols[x] + a.key[x]];
    }
    a.buf[kDistHdr + j] = v;
}

// Select: the gathered samples of every rank (world rows of `stride` words:
// header + cap keys), L = the sum of the ranks' valid counts; splitter q =
// the key at sorted position max(0, (q + 1) L / parts - 1), or max(0, q20[q]
// L / 2^20 - 1) with stage fractions -- the value at a sorted position does
// not depend on how ties break, so each key's rank under (key, index) (a
// permutation), counted against all N = world cap keys, picks them: block b
// ranks keys [32 b, 32 b + 32); lane & 31 picks the key, 2 wave + (lane >> 5)
// one of 32 slices of every rank's row to count against.  out[parts - 1] = L
// (L = 0: every splitter 0).  grid ceil(N / 32) x 1024.
constexpr int kDsKeys = 32, kDsSlices = 32;
__global__ __launch_bounds__(1024) void dist_select_kernel(const DistSelectArgs a) {
    __shared__ uint32_t s_rank[kDsSlices][kDsKeys];
    __shared__ int64_t s_pos[kDistMaxParts];
    __shared__ int64_t s_L;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t cap = a.stride - kDistHdr, N = (int64_t)a.world * cap;
    if (tid == 0) {
        int64_t L = 0;
        for (int r = 0; r < a.world; r++) L += a.all[(int64_t)r * a.stride];
        s_L = L;
    }
    __syncthreads();
    const int64_t L = s_L;
    if (tid < a.parts - 1) {
        const int64_t q = a.use_q ? (int64_t)a.q20[tid] * L / (1 << 20) : (int64_t)(tid + 1) * L / a.parts;
        s_pos[tid] = max(q - 1, (int64_t)0);
    }
    const int li = lane & 31, slice = 2 * w + (lane >> 5);
    const int64_t i = (int64_t)blockIdx.x * kDsKeys + li;
    const int64_t ir = i / max(cap, (int64_t)1), ij = i - ir * cap;
    const int64_t my = i < N ? a.all[ir * a.stride + kDistHdr + ij] : INT64_MAX;
    const int64_t j0 = slice * cap / kDsSlices, j1 = (slice + 1) * cap / kDsSlices;
    uint32_t rk = 0;
    for (int r = 0; r < a.world; r++) {
        const int64_t *row = a.all + (int64_t)r * a.stride + kDistHdr;
        const int64_t base = (int64_t)r * cap;
#pragma unroll 8
        for (int64_t j = j0; j < j1; j++) {
            const int64_t o = row[j];
            rk += (o < my || (o == my && base + j < i)) ? 1u : 0u;
        }
    }
    s_rank[slice][li] = rk;
    __syncthreads();
    if (tid < kDsKeys && i < N && L > 0) {
        uint32_t rank = 0;
#pragma unroll
        for (int q = 0; q < kDsSlices; q++) rank += s_rank[q][tid];
        for (int q = 0; q < a.parts - 1; q++)
            if (s_pos[q] == (int64_t)rank) a.out[q] = my;
    }
    if (blockIdx.x == 0) {
        if (tid == 0) a.out[a.parts - 1] = L;
        if (L == 0 && tid < a.parts - 1) a.out[tid] = 0;
    }
}

hipError_t launch_dist_sample(const DistSampleArgs &a, hipStream_t s) {
    const int n = 2 * a.samples;
    hipLaunchKernelGGL(dist_sample_kernel, dim3((unsigned)blocks_for(n, 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_dist_select(const DistSelectArgs &a, hipStream_t s) {
    const int64_t N = (int64_t)a.world * (a.stride - kDistHdr);
    hipLaunchKernelGGL(dist_select_kernel, dim3((unsigned)std::max<int64_t>(1, blocks_for(N, kDsKeys))), dim3(1024), 0, s,
                       a);
    return hipGetLastError();
}

// Ablation switches for profiling builds of the bench tools only (unset in
// production): SMJ_DEBUG_PASS bit0 = no look-back, bit1 = no HBM stores,
// bit2 = no LDS staging / scatter; SMJ_DEBUG_JOIN bit0 = no look-back.
static int debug_bits(const char *name) {
    const char *v = getenv(name);
    return v ? atoi(v) : 0;
}

static BucketDigit make_bucket(const int64_t *spl, int nspl) {
    BucketDigit d{};
    for (int i = 0; i < kMaxSplitters; i++) d.spl[i] = i < nspl ? spl[i] : INT64_MAX;
    d.nspl = nspl;
    return d;
}

hipError_t launch_hist_radix(const int64_t *src, int64_t n, int cols, int use_select, int sel_col,
                             int64_t sel_val, int key_col, uint64_t key_base, uint32_t *ghist, uint32_t *table0,
                             hipStream_t s) {
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(n, chunk_rows(cols)), 1024));
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((hist_radix_kernel<C>), dim3(grid), dim3(512), 0, s, src, n,
                                             use_select, sel_col, sel_val, key_col, key_base, ghist, table0));
    return hipGetLastError();
}

hipError_t launch_plan(uint32_t *ghist, SortPlan *plan, hipStream_t s) {
    hipLaunchKernelGGL(plan_kernel, dim3(1), dim3(1024), 0, s, ghist, plan);
    return hipGetLastError();
}

hipError_t launch_hist_bucket(const int64_t *src, int64_t n, int cols, int use_select, int sel_col,
                              int64_t sel_val, int key_col, const int64_t *spl, int nspl,
                              unsigned long long *gcount, long long *gminmax, hipStream_t s) {
    const BucketDigit dg = make_bucket(spl, nspl);
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(n, 2048), 1024));
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((hist_bucket_kernel<C>), dim3(grid), dim3(512), 0, s, src, n,
                                             use_select, sel_col, sel_val, key_col, dg, gcount, gminmax));
    return hipGetLastError();
}

int pass_radix(const PassSpec &ps) {
    return ps.kind == DIGIT_RADIX ? kRadix : ps.kind == DIGIT_BUCKET ? (1 << kBucketBits) : 1;
}

int64_t pass_chunks(const PassSpec &ps) { return (ps.nsrc + chunk_rows(ps.cols) - 1) / chunk_rows(ps.cols); }

// dispatch a pass kernel over (cols, digit kind)
#define SMJ_PASS_DISPATCH(KERNEL, BLOCK)                                                                   \
    do {                                                                                                   \
        const unsigned grid = (unsigned)pass_chunks(ps);                                                   \
        const int dbg = debug_bits("SMJ_DEBUG_PASS");                                                      \
        if (ps.kind == DIGIT_RADIX) {                                                                      \
            PassParams<RadixDigit> p{ps.src, ps.dst, ps.nsrc, ps.sel_val, ps.use_select, ps.sel_col,        \
                                     ps.key_col, dbg, RadixDigit{ps.key_base ^ 0x8000000000000000ull, ps.shift}, table, ctr,       \
                                     ps.trash};                                                            \
            SMJ_COLS_SWITCH(ps.cols, hipLaunchKernelGGL((KERNEL<C, kRadixBits, RadixDigit>), dim3(grid),    \
                                                        dim3(BLOCK), 0, s, p));                           \
        } else if (ps.kind == DIGIT_BUCKET) {                                                              \
            PassParams<BucketDigit> p{ps.src, ps.dst, ps.nsrc, ps.sel_val, ps.use_select, ps.sel_col,       \
                                      ps.key_col, dbg, make_bucket(ps.spl, ps.nspl), table, ctr, ps.trash}; \
            SMJ_COLS_SWITCH(ps.cols, hipLaunchKernelGGL((KERNEL<C, kBucketBits, BucketDigit>), dim3(grid),  \
                                                        dim3(BLOCK), 0, s, p));                           \
        } else {                                                                                           \
            PassParams<ZeroDigit> p{ps.src, ps.dst, ps.nsrc, ps.sel_val, ps.use_select, ps.sel_col,         \
                                    ps.key_col, dbg, ZeroDigit{}, table, ctr, ps.trash};                   \
            SMJ_COLS_SWITCH(ps.cols, hipLaunchKernelGGL((KERNEL<C, 0, ZeroDigit>), dim3(grid), dim3(BLOCK), \
                                                        0, s, p));                                         \
        }                                                                                                  \
    } while (0)

hipError_t launch_chunk_hist(const PassSpec &ps, uint32_t *table, hipStream_t s) {
    Counters *ctr = nullptr;
    SMJ_PASS_DISPATCH(chunk_hist_kernel, 512);
    return hipGetLastError();
}

hipError_t launch_chunk_scan(const PassSpec &ps, uint32_t *table, uint32_t *segsum, const uint32_t *base,
                             hipStream_t s) {
    const int radix = pass_radix(ps);
    const int64_t nch = pass_chunks(ps);
    const dim3 grid((radix + 63) / 64, kScanSegs);
    hipLaunchKernelGGL(chunk_scan_seg_kernel, grid, dim3(256), 0, s, table, nch, radix, segsum);
    hipLaunchKernelGGL(chunk_scan_apply_kernel, grid, dim3(256), 0, s, table, nch, radix, segsum, base);
    return hipGetLastError();
}

hipError_t launch_chunk_scan_dev(const PassSpec &ps, uint32_t *table, uint32_t *segsum, uint32_t *base,
                                 unsigned long long *counts, hipStream_t s) {
    const int radix = pass_radix(ps);
    if (radix > 64) return hipErrorInvalidValue;
    const int64_t nch = pass_chunks(ps);
    const dim3 grid((radix + 63) / 64, kScanSegs);
    hipLaunchKernelGGL(chunk_scan_seg_kernel, grid, dim3(256), 0, s, table, nch, radix, segsum);
    hipLaunchKernelGGL(digit_base_kernel, dim3(1), dim3(64), 0, s, segsum, radix, base, counts);
    hipLaunchKernelGGL(chunk_scan_apply_kernel, grid, dim3(256), 0, s, table, nch, radix, segsum, base);
    return hipGetLastError();
}

hipError_t launch_chunk_scatter(const PassSpec &ps, uint32_t *table, Counters *ctr, hipStream_t s) {
    SMJ_PASS_DISPATCH(chunk_scatter_kernel, kSortThreads);
    return hipGetLastError();
}

hipError_t launch_merge_partition(const int64_t *a, int64_t na, int ca, int ka, const int64_t *b,
                                  int64_t nb, int cb, int kb, int64_t *apart, int64_t *run_start, int64_t ntiles,
                                  int tile, hipStream_t s) {
    hipLaunchKernelGGL(merge_partition_kernel, dim3(blocks_for(ntiles + 1, 256)), dim3(256), 0, s, a, na, ca, ka, b,
                       nb, cb, kb, apart, run_start, ntiles, tile);
    return hipGetLastError();
}

hipError_t launch_join(const int64_t *R, int64_t nr, int c1, int key1, const int64_t *S, int64_t ns, int c2,
                       int key2, const int64_t *apart, const int64_t *run_start, int64_t ntiles, int64_t *slots,
                       uint32_t *counts, uint32_t *offs, int64_t *out, int64_t *out_rows, int phase,
                       hipStream_t s) {
    if (phase == 0) {
        JoinParams p{R, S, apart, run_start, slots, counts, nr, ns, ntiles, c1, key1, c2, key2, join_tile_size(c1, c2)};
        hipLaunchKernelGGL(join_tile_kernel, dim3((unsigned)ntiles), dim3(kJoinThreads), 0, s, p);
    } else if (phase == 1) {
        hipLaunchKernelGGL(join_scan_kernel, dim3(1), dim3(1024), 0, s, counts, ntiles, offs, out_rows);
    } else {
        hipLaunchKernelGGL(join_compact_kernel, dim3((unsigned)ntiles), dim3(256), 0, s, slots, apart, counts, offs,
                           c1 + c2 - 1, out);
    }
    return hipGetLastError();
}

hipError_t launch_count_scan(const uint32_t *counts, int64_t n, uint32_t *offs, int64_t *total, hipStream_t s) {
    hipLaunchKernelGGL(join_scan_kernel, dim3(1), dim3(1024), 0, s, counts, n, offs, total);
    return hipGetLastError();
}

hipError_t launch_merge_tiles(const int64_t *a, int64_t na, const int64_t *b, int64_t nb, int cols,
                              int key_col, const int64_t *apart, int64_t ntiles, int64_t *out,
                              hipStream_t s) {
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((merge_tile_kernel<C>), dim3((unsigned)ntiles),
                                             dim3(kJoinThreads), 0, s, a, na, b, nb, key_col, apart, out));
    return hipGetLastError();
}

// diagnostic: read and clear the chunk_scatter phase cycle sums
hipError_t read_phase_cycles(unsigned long long *out16) {
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_phase_cycles), sizeof(unsigned long long) * 16);
    if (e != hipSuccess) return e;
    static const unsigned long long zero[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), zero, sizeof(zero));
}

// ---------------------------------------------------------------------------
// T = UINT64 / DOUBLE (common.h): order-preserving maps onto int64, so the
// int64 pipeline sorts, selects and joins in T's order.  uint64: x ^ 2^63
// (an involution).  double: bits u (-0.0 folded onto +0.0, which compare
// equal), negative values with their 63 low bits flipped.  key_map_kernel
// applies the map (or its inverse) to the columns in colmask of every row.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t key_fwd(int64_t v, int ktype) {
    uint64_t u = (uint64_t)v;
    if (ktype == 1) return (int64_t)(u ^ 0x8000000000000000ull);
    if (u == 0x8000000000000000ull) u = 0;  // -0.0
    return (int64_t)((u >> 63) ? (u ^ 0x7fffffffffffffffull) : u);
}
__device__ __forceinline__ int64_t key_inv(int64_t k, int ktype) {
    if (ktype == 1) return (int64_t)((uint64_t)k ^ 0x8000000000000000ull);
    return k < 0 ? (int64_t)((uint64_t)k ^ 0x7fffffffffffffffull) : k;
}

__global__ __launch_bounds__(256) void key_map_kernel(const int64_t *src, int64_t *dst, int64_t cells,
                                                      int cols, uint32_t colmask, int ktype, int inverse) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells; i += stride) {
        int64_t v = src[i];
        if ((colmask >> (int)(i % cols)) & 1u) v = inverse ? key_inv(v, ktype) : key_fwd(v, ktype);
        dst[i] = v;
    }
}

hipError_t launch_key_map(const int64_t *src, int64_t *dst, int64_t rows, int cols, uint32_t colmask, int ktype,
                          int inverse, hipStream_t s) {
    const int64_t cells = rows * cols;
    if (cells <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(cells, 256), 16384));
    hipLaunchKernelGGL(key_map_kernel, dim3(grid), dim3(256), 0, s, src, dst, cells, cols, colmask, ktype, inverse);
    return hipGetLastError();
}

hipError_t launch_gen_uniform(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t key_range,
                              hipStream_t s) {
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(rows, 256), 8192));
    hipLaunchKernelGGL(gen_uniform_kernel, dim3(grid), dim3(256), 0, s, out, row0, rows, seed, key_range);
    return hipGetLastError();
}

hipError_t launch_gen_wide(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t plant_seed,
                           int64_t plant_rows, hipStream_t s) {
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(rows, 256), 8192));
    hipLaunchKernelGGL(gen_wide_kernel, dim3(grid), dim3(256), 0, s, out, row0, rows, seed, plant_seed,
                       (uint64_t)plant_rows);
    return hipGetLastError();
}

hipError_t launch_gen_zipf(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, int64_t domain,
                           double theta, double zeta_n, hipStream_t s) {
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(rows, 256), 8192));
    hipLaunchKernelGGL(gen_zipf_kernel, dim3(grid), dim3(256), 0, s, out, row0, rows, seed, domain, theta,
                       zeta_n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// index-sort path for wide rows (col_num > 8, any T):
// the pipeline runs on 16-B (key, row id) pairs and whole rows are gathered
// once at the end, so a row of any width moves twice instead of six times
// ---------------------------------------------------------------------------
// pair r = (map(key), row0 + r), or (map(key), -1) when the WHERE predicate
// (map(row[sel_col]) > sel_val, sel_val already mapped) drops the row: the
// pipeline then selects on payload > -1.  ktype: 0 int64, 1 uint64, 2 double.
__global__ __launch_bounds__(256) void row_pairs_kernel(const int64_t *__restrict__ src, int64_t n, int cols,
                                                        int key, int use_sel, int sel_col, int64_t sel_val,
                                                        int ktype, int64_t row0, i64x2 *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) {
        const int64_t *row = src + r * cols;
        int64_t k = row[key];
        bool keep = true;
        if (use_sel) {
            int64_t v = row[sel_col];
            if (ktype) v = key_fwd(v, ktype);
            keep = v > sel_val;
        }
        if (ktype) k = key_fwd(k, ktype);
        i64x2 pr;
        pr.x = k;
        pr.y = keep ? row0 + r : -1;
        out[r] = pr;
    }
}

// dst row i = source row id(i) whole (id = ids[i * id_stride + id_col]); ids
// below n0 name rows of src0, the others rows id - n0 of src1.  One thread
// per output word: reads run along a source row, writes are coalesced.
__global__ __launch_bounds__(256) void gather_rows_kernel(const int64_t *__restrict__ src0, int64_t n0,
                                                          const int64_t *__restrict__ src1, int cols,
                                                          const int64_t *__restrict__ ids, int id_stride, int id_col,
                                                          int64_t m, uint32_t magic, int64_t *__restrict__ dst) {
    constexpr int64_t kRowsPerBlock = 128;
    for (int64_t b = blockIdx.x; b * kRowsPerBlock < m; b += gridDim.x) {
        const int64_t r0 = b * kRowsPerBlock, rows = min(kRowsPerBlock, m - r0);
        const uint32_t words = (uint32_t)(rows * cols);
        for (uint32_t w = threadIdx.x; w < words; w += 256) {
            const uint32_t i = cols > 1 ? __umulhi(w, magic) : w, c = w - i * (uint32_t)cols;
            const int64_t id = ids[(r0 + i) * id_stride + id_col];
            const int64_t *s = id < n0 ? src0 + id * cols : src1 + (id - n0) * cols;
            dst[(r0 + i) * cols + c] = s[c];
        }
    }
}

// joined row j = R row jp[j].y (c1 words) then S row jp[j].z without key2;
// jp rows are (key, R row id, S row id).  One thread per output word.
__global__ __launch_bounds__(256) void join_gather_kernel(const int64_t *__restrict__ R, int c1,
                                                          const int64_t *__restrict__ S, int c2, int key2,
                                                          const int64_t *__restrict__ jp, int64_t J, uint32_t magic,
                                                          int64_t *__restrict__ out) {
    constexpr int64_t kRowsPerBlock = 128;
    const int tc = c1 + c2 - 1;
    for (int64_t b = blockIdx.x; b * kRowsPerBlock < J; b += gridDim.x) {
        const int64_t r0 = b * kRowsPerBlock, rows = min(kRowsPerBlock, J - r0);
        const uint32_t words = (uint32_t)(rows * tc);
        for (uint32_t w = threadIdx.x; w < words; w += 256) {
            const uint32_t i = tc > 1 ? __umulhi(w, magic) : w;
            const int c = (int)(w - i * (uint32_t)tc);
            const int64_t *t = jp + (r0 + i) * 3;
            int64_t v;
            if (c < c1) {
                v = R[t[1] * c1 + c];
            } else {
                const int j = c - c1;
                v = S[t[2] * c2 + j + (j >= key2 ? 1 : 0)];
            }
            out[(r0 + i) * tc + c] = v;
        }
    }
}

// floor(w / d) as __umulhi(w, magic): exact while w * (magic * d - 2^32) < 2^32,
// i.e. for w < 128 * d with d <= 2^11 (one block's words)
static uint32_t div_magic(int d) { return d > 1 ? (uint32_t)((0x100000000ull + d - 1) / d) : 0u; }

hipError_t launch_row_pairs(const int64_t *src, int64_t n, int cols, int key, int use_sel, int sel_col,
                            int64_t sel_val, int ktype, int64_t row0, int64_t *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(n, 256), 16384));
    hipLaunchKernelGGL(row_pairs_kernel, dim3(grid), dim3(256), 0, s, src, n, cols, key, use_sel, sel_col, sel_val,
                       ktype, row0, reinterpret_cast<i64x2 *>(out));
    return hipGetLastError();
}

hipError_t launch_gather_rows(const int64_t *src0, int64_t n0, const int64_t *src1, int cols, const int64_t *ids,
                              int id_stride, int id_col, int64_t m, int64_t *dst, hipStream_t s) {
    if (m <= 0) return hipSuccess;
    if (cols > 1024) return hipErrorInvalidValue;  // 128 rows x cols words per block: div_magic stays exact
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(m, 128), 16384));
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid), dim3(256), 0, s, src0, n0, src1, cols, ids, id_stride, id_col,
                       m, div_magic(cols), dst);
    return hipGetLastError();
}

hipError_t launch_join_gather(const int64_t *R, int c1, const int64_t *S, int c2, int key2, const int64_t *jp,
                              int64_t J, int64_t *out, hipStream_t s) {
    if (J <= 0) return hipSuccess;
    if (c1 + c2 - 1 > 2047) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks_for(J, 128), 16384));
    hipLaunchKernelGGL(join_gather_kernel, dim3(grid), dim3(256), 0, s, R, c1, S, c2, key2, jp, J,
                       div_magic(c1 + c2 - 1), out);
    return hipGetLastError();
}

}  // namespace smj
