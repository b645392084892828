// smj_msd.hip -- the MSD sample-sort pipeline of the sort-merge-join hot path
// (gfx950).  Replaces, in one pipeline over both tables,
//   select.c (:63-194)                  -> the WHERE predicate of part_a
//   sort_dpu.c (:189-328) + merge tree   -> part_a, part_b, final (LDS sort)
//     (merge_dpu.c :55-223, app.c :412-547)
//   join.c (:58-266) + splitters          -> final (zip join in LDS)
//     (app.c :585-633)
// with cpu_app.c's semantics (select_in_cpu :81-112, stable signed
// insertion_sort_in_cpu :172-202, 1:1 zip join_in_cpu :204-266).
//
// Data flow per table:
//   sample    one workgroup sorts <= 16 Ki sampled keys of R and S (bitonic,
//             LDS) and keeps 255 splitters; pass-A bucket of a key =
//             #{splitters < key} (+ 1 for a key the sample repeats: a heavy
//             key gets a bucket to itself): 256 buckets.
//   part_a    every tile of T rows (64 KiB) is select-filtered and stably
//             partitioned by bucket IN ITS OWN REGION of tempA: one read, one
//             fully coalesced write.  offsA[tile][bucket] = tile-local starts.
//   runs      per bucket, the non-empty (tile, bucket) runs are listed in
//             tile order (= input order) with their bucket-virtual start; a
//             pass-B tile is every T consecutive rows of a bucket.
//   part_b    a pass-B tile gathers its rows through the run list (runs of
//             ~T/128 rows), and partitions them stably by 9 more key bits
//             (floor((key - lo) * 512 / interval) of the bucket), again in its own region of
//             tempB.  offsB[tile][sub-bucket] = tile-local starts.
//   group     per bucket, consecutive sub-buckets are packed greedily into
//             groups of <= kGroupCap rows per table; a key never spans groups.
//   final     per group: gather R and S keys (one contiguous range per pass-B
//             tile of the bucket), stable LSD radix sort of (key residual,
//             index) in LDS, write sorted R and S to their final rows, and the
//             zip join of the group into join slots (group row offset).
//   compact   exclusive scan of the per-group match counts (groups are in key
//             order) and packing of the slots into the output.
// Oversized groups: single-key groups stream through msd_single_kernel (no
// sort needed); multi-key ones fall back to the LSD path on the host side.
#include "smj_internal.h"
#include "smj_device.h"

// Phase stamps (tools/msd_phases.py) are compiled in only with -DSMJ_STAMPS=1
// (they hold registers); at run time they also need SMJ_DEBUG_MSD=1.
#ifndef SMJ_BOUNDS
#define SMJ_BOUNDS 0  // debug builds: run metadata checked before the gathers it drives (plan->err bit 1)
#endif
#ifndef SMJ_STAMPS
#define SMJ_STAMPS 0
#endif

#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>

namespace smj {

// ---------------------------------------------------------------------------
// block helpers (kMsdThreads = 512 threads = 8 waves)
// ---------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_wsum, uint32_t *total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t incl = wave_incl_scan(v, lane);
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const uint32_t x = s_wsum[w];
        before += (w < wave) ? x : 0u;
        all += x;
    }
    *total = all;
    __syncthreads();  // s_wsum reusable on return
    return before + incl - v;
}

// block_excl_scan without the trailing barrier (s_wsum must not be rewritten
// before every thread has read it: callers separate uses by a barrier)
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan_nb(uint32_t v, uint32_t *s_wsum, uint32_t *total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t incl = wave_incl_scan(v, lane);
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const uint32_t x = s_wsum[w];
        before += (w < wave) ? x : 0u;
        all += x;
    }
    *total = all;
    return before + incl - v;
}

template <int NW>
__device__ __forceinline__ void block_minmax(int64_t &mn, int64_t &mx, int64_t *s_mm) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o, 64));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o, 64));
    }
    if (lane == 0) {
        s_mm[wave] = mn;
        s_mm[NW + wave] = mx;
    }
    __syncthreads();
    // the NW wave partials through lanes [0, NW) and one more wave reduction
    // (reading all of them per thread kept 4 NW VGPRs live: spills at NW = 16)
    static_assert(NW <= 64, "one partial per lane");
    mn = lane < NW ? s_mm[lane] : INT64_MAX;
    mx = lane < NW ? s_mm[NW + lane] : INT64_MIN;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o, 64));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o, 64));
    }
    __syncthreads();
}

// Stable ranks of the rows of a tile by a DBITS-bit digit.  Rows are ordered
// wave-major, then item, then lane.  dig[it] holds the digit of valid rows
// (vmask bit it); wc is this wave's zeroed counter row.  On return dig[it] =
// digit | (rank among this wave's earlier rows of that digit) << 16, and wc
// holds the wave's per-digit counts.  Peers with the same digit are found
// with DBITS ballots, each folded into the peer mask by one v_bitop3 per half.
template <int ITEMS, int DBITS>
__device__ __forceinline__ void wave_rank(uint32_t (&dig)[ITEMS], uint32_t vmask, uint32_t *wc, int lane) {
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
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, base));
            const uint64_t peers = ((uint64_t)phi << 32) | plo;
            if ((peers >> lane) == 1ull) wc[dd] = base + (uint32_t)__popcll(peers);
            dig[it] = dd | (rank << 16);
        }
    }
}

// threadIdx.x as a value the compiler may not hoist out of the group loop:
// per-lane addresses are recomputed where used instead of living (spilled)
// across the whole loop
__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// wave_rank over u16 counters (a wave ranks at most 64 * ITEMS rows)
template <int ITEMS, int DBITS>
__device__ __forceinline__ void wave_rank16(uint32_t (&dig)[ITEMS], uint32_t vmask, uint16_t *wc, int lane) {
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const bool v = (vmask >> it) & 1u;
        const uint64_t act = __ballot(v);
        uint32_t plo = (uint32_t)act, phi = (uint32_t)(act >> 32);
        const uint32_t dd = dig[it];
#pragma unroll
        for (int b = 0; b < DBITS; b++) {
            const uint32_t sb = (uint32_t)((int32_t)(dd << (31 - b)) >> 31);
            const uint64_t bb = __ballot(sb != 0u);
            plo = peer_fold(plo, (uint32_t)bb, sb);
            phi = peer_fold(phi, (uint32_t)(bb >> 32), sb);
        }
        if (v) {
            const uint32_t base = wc[dd];
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, base));
            const uint64_t peers = ((uint64_t)phi << 32) | plo;
            if ((peers >> lane) == 1ull) wc[dd] = (uint16_t)(base + (uint32_t)__popcll(peers));
            dig[it] = dd | (rank << 16);
        }
    }
}

// Per-digit cross-wave exclusive prefixes (in place in s_wcnt[wave][digit])
// and tile-local exclusive digit starts s_bin[0..RADIX] (s_bin[RADIX] = the
// tile's row count).  Thread t owns digits [t * DPT, t * DPT + DPT).  Ends
// with a barrier.
template <int RADIX, int NT = kMsdThreads>
__device__ __forceinline__ uint32_t tile_digit_starts(uint32_t *s_wcnt, uint32_t *s_bin, uint32_t *s_wsum) {
    constexpr int DPT = RADIX > NT ? RADIX / NT : 1, NW = NT / 64;
    const int tid = threadIdx.x;
    uint32_t tot[DPT], sum = 0;
#pragma unroll
    for (int j = 0; j < DPT; j++) {
        const int d = tid * DPT + j;
        uint32_t t = 0;
        if (d < RADIX) {
#pragma unroll
            for (int w = 0; w < NW; w++) {
                const uint32_t c = s_wcnt[w * RADIX + d];
                s_wcnt[w * RADIX + d] = t;
                t += c;
            }
        }
        tot[j] = t;
        sum += t;
    }
    uint32_t all;
    uint32_t ex = block_excl_scan<NW>(sum, s_wsum, &all);
#pragma unroll
    for (int j = 0; j < DPT; j++) {
        const int d = tid * DPT + j;
        if (d < RADIX) s_bin[d] = ex;
        ex += tot[j];
    }
    if (tid == 0) s_bin[RADIX] = all;
    __syncthreads();
    return all;
}

// wave-uniform copy (SGPR) of a value loaded through a vector load
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// packed rows (MsdTable::pk, MsdPart1Params::pk): word = (int32 key - base_k)
// | (int32 other - base_p) << 32, differences mod 2^64
__device__ __forceinline__ int64_t pk_key(int64_t w, int64_t bk) {
    return (int64_t)((uint64_t)bk + (uint64_t)(int64_t)(int32_t)(uint32_t)w);
}
__device__ __forceinline__ int64_t pk_other(int64_t w, int64_t bp) {
    return (int64_t)((uint64_t)bp + (uint64_t)(int64_t)(int32_t)(uint32_t)((uint64_t)w >> 32));
}
// the packed word of (key, other), and whether both differences fit int32
__device__ __forceinline__ int64_t pk_pack(int64_t key, int64_t other, int64_t bk, int64_t bp, bool &fits) {
    const int64_t dk = (int64_t)((uint64_t)key - (uint64_t)bk), dp = (int64_t)((uint64_t)other - (uint64_t)bp);
    fits = dk == (int64_t)(int32_t)dk && dp == (int64_t)(int32_t)dp;
    return (int64_t)(((uint64_t)(uint32_t)dk) | ((uint64_t)(uint32_t)dp << 32));
}

// pass-A bucket of a key: pos = #{splitters < key}, or pos + 1 when the key
// equals spl[pos] == spl[pos + 1] (a repeated splitter: a heavy key gets
// bucket pos + 1 to itself; no other key maps there)
__device__ __forceinline__ uint32_t bucket_a(const int64_t *s_spl, int64_t k) {
    int pos = 0;
#pragma unroll
    for (int step = kBucketsA / 2; step >= 1; step >>= 1)
        pos += (s_spl[pos + step - 1] < k) ? step : 0;  // index <= kSplA - 1
    const int q = pos + 1 < kSplA ? pos : kSplA - 2;
    const bool rep = pos + 1 < kSplA && s_spl[q] == k && s_spl[q + 1] == k;
    return (uint32_t)pos + (rep ? 1u : 0u);
}


// ---------------------------------------------------------------------------
// sample -> splitters
// ---------------------------------------------------------------------------
// Splitters in two launches.  Gather: sample j of table x (clusters of 16
// consecutive rows spread evenly over the table: 16x fewer distinct pages,
// i.e. TLB walks, than single rows) -> samp[x * kSampleMax + j], INT64_MAX
// for a row the select drops or a missing row; per-block valid counts at
// samp[kSampleN + block].  grid kSampleN / 256 x 256.
constexpr int kSampleN = 2 * kSampleMax, kSampleGatherBlocks = kSampleN / 256;
static_assert(kSampleGatherBlocks <= 64, "one wave sums the gather blocks' valid counts");
__global__ __launch_bounds__(256) void msd_sample_gather_kernel(const MsdSampleParams p) {
    __shared__ uint32_t s_c[4];
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int x = j >= kSampleMax ? 1 : 0, jj = j - x * kSampleMax;
    const MsdTable &t = p.tab[x];
    int64_t k = INT64_MAX;
    uint32_t valid = 0;
    if (x < p.ntab && t.n > 0 && jj < min(t.n, (int64_t)kSampleMax)) {
        constexpr int kSampleRun = 16, kClusters = kSampleMax / kSampleRun;
        int64_t r = t.n <= kSampleMax
                        ? jj
                        : min(t.n - 1, ((2 * (int64_t)(jj / kSampleRun) + 1) * t.n) / (2 * kClusters) +
                                           jj % kSampleRun);
        bool dup = false;
        if (t.desc) {  // a chunked part: row r of tile r / tile (clamped to the tile's rows) -- any row of it samples
            const uint64_t d = t.desc[min(t.ntiles - 1, r / t.tile)];
            const int64_t rows = (int64_t)(d & 0xffffu);
            // a clamped sample after its cluster's first repeats the row before
            // it: dropped, so that the sample's repeated keys (plan->skew, the
            // heavy-key gate) are repeated keys of the table, not of the clamp
            dup = r % t.tile >= rows && jj % kSampleRun != 0;
            r = (int64_t)(d >> 16) + min(r % t.tile, rows - 1);
        }
        int64_t sv, kv;
        if (t.pk) {  // packed input (no select)
            kv = pk_key(t.src[r], t.pkk);
            sv = kv;
        } else {
            const int64_t *row = t.src + r * t.cols;
            sv = row[t.use_sel ? t.sel_col : t.key_col];
            kv = row[t.key_col];
        }
        if (!dup && (!t.use_sel || sv > t.sel_val)) {
            k = kv;
            valid = 1;
        }
    }
    p.samp[j] = k;
    uint32_t c = valid;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) p.samp[kSampleN + blockIdx.x] = s_c[0] + s_c[1] + s_c[2] + s_c[3];
}

// Select: splitter i = the sample of sorted position at(i) = min(M - 1,
// (i + 1) M / (kSplA + 1)) (M valid samples; the dropped ones hold INT64_MAX
// and sort behind every valid key).  Sample i's position is its rank under
// (key, index) -- a permutation -- counted against all kSampleN samples in
// LDS: block b ranks samples [32 b, 32 b + 32); lane & 31 picks the sample,
// and 2 wave + (lane >> 5) one of 32 slices of kSampleN / 32 samples to
// count against (two LDS words per wave read: broadcast).
// grid kSampleN / 32 x 1024.
constexpr int kSelSamples = 32, kSelSlices = 32;
__global__ __launch_bounds__(1024) void msd_sample_select_kernel(const MsdSampleParams p) {
    __shared__ int64_t s_key[kSampleN];
    __shared__ uint32_t s_rank[kSelSlices][kSelSamples];
    __shared__ uint32_t s_eq[kSelSlices][kSelSamples];
    __shared__ uint32_t s_m;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    {
        const int4 *src = reinterpret_cast<const int4 *>(p.samp);
        int4 *dst = reinterpret_cast<int4 *>(s_key);
#pragma unroll
        for (int i = 0; i < kSampleN / 2 / 1024; i++) dst[tid + i * 1024] = src[tid + i * 1024];
    }
    if (tid < 64) {
        uint32_t m = tid < kSampleGatherBlocks ? (uint32_t)p.samp[kSampleN + tid] : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o, 64);
        if (tid == 0) s_m = m;
    }
    __syncthreads();
    const uint32_t M = s_m;
    const int li = lane & 31, i = blockIdx.x * kSelSamples + li, part = 2 * w + (lane >> 5);
    const int64_t my = s_key[i];
    uint32_t r = 0, eq = 0;
    constexpr int SL = kSampleN / kSelSlices;
    const int j0 = part * SL;
#pragma unroll 8
    for (int j = j0; j < j0 + SL; j++) {
        const int64_t o = s_key[j];
        r += (o < my || (o == my && j < i)) ? 1u : 0u;
        eq += (o == my) ? 1u : 0u;  // itself included
    }
    s_rank[part][li] = r;
    s_eq[part][li] = eq;
    __syncthreads();
    if (tid < kSelSamples) {
        uint32_t rank = 0, e = 0;
#pragma unroll
        for (int q = 0; q < kSelSlices; q++) {
            rank += s_rank[q][tid];
            e += s_eq[q][tid];
        }
        const int64_t key = s_key[blockIdx.x * kSelSamples + tid];
        // skew signal: sampled keys some other sample repeats (uniform keys
        // over a range >> the sample: ~0 of them; Zipf: thousands)
        const uint64_t rep = __ballot(e > 1u && key != INT64_MAX && rank < M);
        if (tid == 0 && rep && p.plan) atomicAdd(&p.plan->skew, (uint32_t)__popcll(rep));
        if (rank < M) p.samp[kSortedOff + rank] = key;  // key order (msd_bases_kernel's segmented digit)
        if (M > 0 && rank < M)
            for (int q = 0; q < kSplA; q++)
                if (min(M - 1, (uint32_t)(((uint64_t)(q + 1) * M) / (kSplA + 1))) == rank) p.spl[q] = key;
    }
    if (M == 0 && blockIdx.x == 0 && tid < kSplA) p.spl[tid] = INT64_MAX;
}

// ---------------------------------------------------------------------------
// part_a: select + stable tile-local partition by pass-A bucket
// ---------------------------------------------------------------------------
#ifndef SMJ_PA_NTLOAD
#define SMJ_PA_NTLOAD 0  // A/B switch: part_a's input rows through nontemporal loads
#endif
#ifndef SMJ_PB_NTLOAD
#define SMJ_PB_NTLOAD 0  // A/B switch: the pipelined part_b's gathers through nontemporal loads
#endif
template <int COLS>
__global__ __launch_bounds__(pa_threads(COLS), pa_waves_per_eu(COLS)) void msd_part_a_kernel(
    const MsdPartA2 q) {
    const unsigned bid = blockIdx.x;
    // one launch may cover both tables (the same column count): blocks past
    // q.tiles0 take table 1's tiles
    const bool second = bid >= q.tiles0;
    const MsdPartAParams &p = second ? q.t[1] : q.t[0];
    const unsigned bx = bid - (second ? q.tiles0 : 0u);
    constexpr int ITEMS = pa_items(COLS), T = msd_tile_a(COLS), RADIX = kBucketsA;
    constexpr int NT = pa_threads(COLS), NW = NT / 64;
    constexpr int ROWB = T * COLS * 8, CNTB = NW * RADIX * 4;
    constexpr int UB = ROWB > CNTB ? ROWB : CNTB;
    __shared__ __attribute__((aligned(16))) unsigned char s_u[UB];
    __shared__ int64_t s_spl[kSplA + 1];
    __shared__ uint32_t s_bin[RADIX + 1];
    __shared__ uint32_t s_wsum[NW];
    __shared__ int64_t s_mm[2 * NW];
    int64_t *s_rows = reinterpret_cast<int64_t *>(s_u);
    uint32_t *s_wcnt = reinterpret_cast<uint32_t *>(s_u);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t t = (int64_t)p.tile0 + bx, row0 = t * T;
    int64_t rs = row0;  // first input row of the tile (a chunked part: its descriptor)
    int nrows;
    if (p.desc) {
        const uint64_t d = p.desc[t];
        rs = (int64_t)(d >> 16);
        nrows = (int)(d & 0xffffu);
    } else {
        nrows = (int)min((int64_t)T, p.n - row0);
    }
    uint32_t *wc = s_wcnt + wave * RADIX;
    if (tid < kSplA) s_spl[tid] = p.spl[tid];
    zero_counters<RADIX>(wc, lane);
    const int lrow0 = wave * ITEMS * 64 + lane;
    int64_t rows[ITEMS][COLS];
    bool packed = false;
    if constexpr (COLS == 2) packed = p.pk != 0;  // block-uniform
    if (packed) {  // one word per row (MsdPartAParams::pk): both columns rebuilt here
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const int64_t w = p.src[rs + min(lrow0 + it * 64, nrows - 1)];
            const int64_t k = pk_key(w, p.pkk), o = pk_other(w, p.pkp);
            rows[it][0] = p.key_col ? o : k;
            rows[it][COLS - 1] = p.key_col ? k : o;
        }
    } else {
#pragma unroll
        for (int it = 0; it < ITEMS; it++)
            if (SMJ_PA_NTLOAD) load_row_nt<COLS>(p.src + (rs + min(lrow0 + it * 64, nrows - 1)) * COLS, rows[it]);
            else load_row<COLS>(p.src + (rs + min(lrow0 + it * 64, nrows - 1)) * COLS, rows[it]);
    }
    __syncthreads();  // splitters

    uint32_t dig[ITEMS];
    uint32_t vmask = 0;
    int64_t mn = INT64_MAX, mx = INT64_MIN;
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const bool inb = lrow0 + it * 64 < nrows;
        const bool pass = !p.use_sel | (pick<COLS>(rows[it], p.sel_col) > p.sel_val);
        const bool v = inb & pass;
        const int64_t k = pick<COLS>(rows[it], p.key_col);
        dig[it] = v ? bucket_a(s_spl, k) : 0u;
        vmask |= v ? (1u << it) : 0u;
        mn = v ? min(mn, k) : mn;
        mx = v ? max(mx, k) : mx;
    }
    wave_rank<ITEMS, kBitsA>(dig, vmask, wc, lane);
    __syncthreads();
    const uint32_t total = tile_digit_starts<RADIX, NT>(s_wcnt, s_bin, s_wsum);
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t d = dig[it] & 0xffffu;
        dig[it] = s_bin[d] + wc[d] + (dig[it] >> 16);
    }
    block_minmax<NW>(mn, mx, s_mm);  // its barriers also retire the counters
#pragma unroll
    for (int it = 0; it < ITEMS; it++)
        if ((vmask >> it) & 1u) store_row<COLS>(s_rows + (size_t)dig[it] * COLS, rows[it]);
    // (after the staging stores: off the loads -> ranks chain)
    if constexpr (COLS == 2) {
        if (p.nopack) {  // packed pass-B rows need the other column in int32 (MsdPlan::packB)
            bool bad = false;
#pragma unroll
            for (int it = 0; it < ITEMS; it++) {
                const int64_t o = rows[it][1 - p.key_col];
                bad = bad || (((vmask >> it) & 1u) && (int64_t)(int32_t)o != o);
            }
            const uint64_t bm = __ballot(bad);
            if (bm && lane == __builtin_ctzll(bm)) atomicOr(p.nopack, 1u);
        }
    }
    static_assert(RADIX < kOffsARow, "the offsA row holds the starts and the count");
    for (int i = tid; i <= RADIX; i += NT) p.offs[t * kOffsARow + i] = s_bin[i];  // s_bin[RADIX] = the tile's selected rows
    if (tid == 0) {
        p.tmm[2 * t] = mn;
        p.tmm[2 * t + 1] = mx;
    }
    __syncthreads();
    if (total > 0) {
        int64_t *dst = p.out + row0 * COLS;
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const uint32_t s = min((uint32_t)(tid + it * NT), total - 1u);
            int64_t r[COLS];
            load_row<COLS>(s_rows + (size_t)s * COLS, r);
            store_row<COLS>(dst + (size_t)s * COLS, r);
        }
    }
}

// ---------------------------------------------------------------------------
// part1: the partitioned mode's range partition in ONE pass (no counting pass)
// ---------------------------------------------------------------------------
// Every tile (T rows, taken in ticket order) is select-filtered, ranked by its
// part (#{splitters < key}, <= 64 parts) and staged in LDS like part_a; its
// part counts go out as an aggregate status word per part, and wave 0 looks
// back over the predecessors' words (64 lanes = up to 64 / nb predecessors x
// nb parts per round trip) until each part meets an inclusive prefix: the
// decoupled look-back, with ~T / nb rows per part per tile and <= 64 parts it
// costs one status word per (tile, part).  Part b's rows go to its own region
// [oc[b], oc[b] + oc[64 + b]) of the staging buffer, at the exclusive prefix:
// stable (tile order = input order) and contiguous.  The region capacities
// come from the key sample (smj_api.hip msd_large); a part whose rows exceed
// its region sets flags[1] and the host falls back to the counting partition.
// Status word: bits 63..62 = 1 aggregate, 2 inclusive prefix; 61..0 the value.
// The look-back never waits on a later ticket, so the grid always drains; a
// wait over 2^24 polls (a bug) sets flags[2].
constexpr uint64_t kP1Agg = 1ull << 62, kP1Inc = 2ull << 62, kP1Val = (1ull << 62) - 1;
#ifndef SMJ_P1_ABL
#define SMJ_P1_ABL 0
#endif

template <int COLS>
__global__ __launch_bounds__(kMsdThreads, p1_waves_per_eu(COLS)) void msd_part1_kernel(const MsdPart1Params p) {
    constexpr int ITEMS = p1_items(COLS), T = p1_tile(COLS), RADIX = 64;
    constexpr int ROWB = T * COLS * 8, CNTB = kMsdWaves * RADIX * 4;
    constexpr int UB = ROWB > CNTB ? ROWB : CNTB;
    __shared__ __attribute__((aligned(16))) unsigned char s_u[UB];
    __shared__ uint8_t s_pd[T];        // part of each staged row
    __shared__ int64_t s_spl[RADIX];
    __shared__ uint32_t s_bin[RADIX + 1];
    __shared__ uint32_t s_wsum[kMsdWaves];
    __shared__ unsigned long long s_acc[RADIX];
    __shared__ int64_t s_gb[RADIX];    // global row of part b's first row in this tile, minus its tile-local start
    __shared__ uint32_t s_ok[RADIX];   // part b's rows fit its region
    __shared__ uint32_t s_t;
    int64_t *s_rows = reinterpret_cast<int64_t *>(s_u);
    uint32_t *s_wcnt = reinterpret_cast<uint32_t *>(s_u);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nb = p.nspl + 1;
    if (tid == 0) s_t = atomicAdd(&p.flags[0], 1u);
    if (tid < RADIX) {
        s_spl[tid] = tid < p.nspl ? p.spl[tid] : INT64_MAX;
        s_acc[tid] = 0;
    }
    uint32_t *wc = s_wcnt + wave * RADIX;
    zero_counters<RADIX>(wc, lane);
    __syncthreads();
    const int64_t t = s_t;
    const int64_t row0 = t * T;
    const int nrows = (int)min((int64_t)T, p.n - row0);
    const int lrow0 = wave * ITEMS * 64 + lane;
    int64_t rows[ITEMS][COLS];
#pragma unroll
    for (int it = 0; it < ITEMS; it++) load_row<COLS>(p.src + (row0 + min(lrow0 + it * 64, nrows - 1)) * COLS, rows[it]);
    uint32_t dig[ITEMS];
    uint32_t vmask = 0;
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const bool inb = lrow0 + it * 64 < nrows;
        const bool pass = !p.use_sel | (pick<COLS>(rows[it], p.sel_col) > p.sel_val);
        const bool v = inb & pass;
        const int64_t k = pick<COLS>(rows[it], p.key_col);
        uint32_t b = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1) b += s_spl[b + step - 1] < k ? step : 0u;
        dig[it] = v ? b : 0u;
        vmask |= v ? (1u << it) : 0u;
    }
    wave_rank<ITEMS, 6>(dig, vmask, wc, lane);
    __syncthreads();
    const uint32_t total = tile_digit_starts<RADIX>(s_wcnt, s_bin, s_wsum);
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t d = dig[it] & 0xffffu;
        dig[it] = (d << 16) | (s_bin[d] + wc[d] + (dig[it] >> 16));  // part << 16 | staging slot
    }
    __syncthreads();  // counters read out: the region becomes the staging tile
    // waves 1..7 stage their rows while wave 0 looks back (then stages its own)
    if (wave == 0) {
        const uint32_t cnt = lane < nb ? s_bin[lane + 1] - s_bin[lane] : 0u;
        unsigned long long *st = p.status + t * nb;
        if (t > 0 && !SMJ_P1_ABL) {  // (SMJ_P1_ABL: timing ablation, no look-back -- tile t at t x its share of the region)
            if (lane < nb) atomicExch(&st[lane], kP1Agg | cnt);
            // (one predecessor per lane with all its part words -- 64 tiles per
            // round trip -- was slower: C4 partition 19.4 vs 14.4 ms, its 7x
            // more uncached status loads per round; profiles/r03/r03w_ab_c4.txt)
            const int J = max(1, 64 / nb);  // predecessors per round
            const int j = lane / nb, b = lane - j * nb;
            const bool lv = lane < J * nb;
            bool done = false;
            uint32_t spins = 0;
            for (int64_t tt = t - 1;; tt -= J) {
                const bool act = lv && !done;
                uint64_t s = 0;
                if (act) {
                    const int64_t tj = tt - j;
                    if (tj < 0) {
                        s = kP1Inc;  // before the first tile: prefix 0
                    } else {
                        for (;;) {
                            s = __hip_atomic_load(&p.status[tj * nb + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (s >> 62) break;
                            if (++spins > (1u << 24)) {
                                atomicOr(&p.flags[2], 1u);
                                s = kP1Inc;
                                break;
                            }
                            __builtin_amdgcn_s_sleep(1);
                        }
                    }
                }
                const uint64_t im = __ballot(act && (s >> 62) == 2u);
                int jinc = J;  // this part's nearest predecessor with an inclusive prefix
                for (int q = 0; q < J; q++)
                    if ((im >> (q * nb + b)) & 1ull) {
                        jinc = q;
                        break;
                    }
                if (act && j <= jinc) atomicAdd(&s_acc[b], (unsigned long long)(s & kP1Val));
                done = done || jinc < J;
                if (__ballot(lv && !done) == 0ull) break;
            }
        }
        if (SMJ_P1_ABL && lane < nb) {  // distinct rows per tile (its share of the region), clamped into it
            const uint64_t cap = (uint64_t)p.oc[64 + lane], per = cap / (uint64_t)p.ntiles;
            s_acc[lane] = min((uint64_t)t * per, cap - min(cap, (uint64_t)cnt));
        }
        if (lane < nb) {
            const uint64_t ex = s_acc[lane];
            atomicExch(&st[lane], kP1Inc | (ex + cnt));
            const bool ok = ex + cnt <= (uint64_t)p.oc[64 + lane];
            if (!ok) atomicOr(&p.flags[1], 1u);
            s_ok[lane] = ok ? 1u : 0u;
            s_gb[lane] = p.oc[lane] + (int64_t)ex - (int64_t)s_bin[lane];
            if (t == p.ntiles - 1) p.tot[lane] = (long long)(ex + cnt);
        }
    }
#pragma unroll
    for (int it = 0; it < ITEMS; it++)
        if ((vmask >> it) & 1u) {
            const uint32_t slot = dig[it] & 0xffffu;
            store_row<COLS>(s_rows + (size_t)slot * COLS, rows[it]);
            s_pd[slot] = (uint8_t)(dig[it] >> 16);
        }
    __syncthreads();  // staging tile, prefixes and region checks published
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t slot = (uint32_t)(tid + it * kMsdThreads);
        if (slot < total) {
            // (searching the part starts instead of keeping s_pd: C4 partition
            // +0.5-0.9 ms, profiles/r03/r03ze_ab_c4.txt)
            const uint32_t b = s_pd[slot];
            if (s_ok[b]) {
                int64_t r[COLS];
                load_row<COLS>(s_rows + (size_t)slot * COLS, r);
                bool pk = false;
                if constexpr (COLS == 2) pk = p.pk != 0;  // block-uniform
                if (pk) {  // one word per row (MsdPart1Params::pk)
                    bool fits;
                    const int64_t w = pk_pack(p.key_col ? r[COLS - 1] : r[0], p.key_col ? r[0] : r[COLS - 1], p.pkk,
                                              p.pkp, fits);
                    if (!fits) atomicOr(&p.flags[3], 1u);
                    p.dst[s_gb[b] + (int64_t)slot] = w;
                } else {
                    store_row<COLS>(p.dst + (s_gb[b] + (int64_t)slot) * COLS, r);
                }
            }
        }
    }
}

// packed rows -> 2-column rows (smj_dev_unpack_rows): one row per thread, 16-B stores
__global__ __launch_bounds__(256) void unpack_rows_kernel(const int64_t *__restrict__ in, int64_t n, int key_col,
                                                          int64_t pkk, int64_t pkp, int64_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t w = in[i], k = pk_key(w, pkk), o = pk_other(w, pkp);
        i64x2 r;
        r.x = key_col ? o : k;
        r.y = key_col ? k : o;
        reinterpret_cast<i64x2 *>(out)[i] = r;
    }
}

hipError_t launch_unpack_rows(const int64_t *packed, int64_t n, int key_col, int64_t pkk, int64_t pkp, int64_t *out,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<int64_t>(8192, (n + 255) / 256);
    hipLaunchKernelGGL(unpack_rows_kernel, dim3(grid), dim3(256), 0, s, packed, n, key_col, pkk, pkp, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// part1c: the chunked one-pass partition (no look-back; smj_internal.h)
// ---------------------------------------------------------------------------
// The look-back of msd_part1_kernel costs ~1.9 ms per 1e9-row table
// (tools/p1_probe.py: 7.2 ms with it, 5.3 ms for the same kernel writing each
// tile at a fixed share of its region without it).  Here no tile waits on
// another: workgroup g walks its own chunk of consecutive tiles in order and
// keeps a running cursor per part, so its rows of part b land contiguous and
// in input order in its sub-region; a part is the chunks' sub-regions in g
// order.  The next tile's rows are loaded while the current one is ranked,
// staged and stored.  Sub-regions are sized from the key sample (their
// per-chunk share plus 8 sigma plus a tile); an overflow only sets flags[1]
// (the caller then runs the look-back partition).
#ifndef SMJ_P1C_PF
#define SMJ_P1C_PF 0  // A/B switch: the next tile's rows loaded while this one is placed (+32 VGPRs: spills at 128)
#endif
template <int COLS>
__global__ __launch_bounds__(kMsdThreads, p1_waves_per_eu(COLS)) void msd_part1c_kernel(const MsdPart1cParams p,
                                                                                        const P1cWords w) {
    constexpr int ITEMS = p1_items(COLS), T = p1_tile(COLS), RADIX = 64;
    constexpr int ROWB = T * COLS * 8, CNTB = kMsdWaves * RADIX * 4;
    constexpr int UB = ROWB > CNTB ? ROWB : CNTB;
    __shared__ __attribute__((aligned(16))) unsigned char s_u[UB];
    __shared__ uint8_t s_pd[T];
    __shared__ int64_t s_spl[RADIX];
    __shared__ uint32_t s_bin[RADIX + 1];
    __shared__ uint32_t s_wsum[kMsdWaves];
    __shared__ int64_t s_gb[RADIX];   // output row of part b's tile-local slot 0
    __shared__ uint32_t s_ok[RADIX];
    __shared__ uint32_t s_cur[RADIX]; // rows of part b written so far by this workgroup
    int64_t *s_rows = reinterpret_cast<int64_t *>(s_u);
    uint32_t *s_wcnt = reinterpret_cast<uint32_t *>(s_u);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nb = p.nspl + 1;
    const int64_t g = blockIdx.x, t0 = g * p.chunk, t1 = min(t0 + p.chunk, p.ntiles);
    if (tid < RADIX) {
        s_spl[tid] = tid < p.nspl ? w.v[128 + tid] : INT64_MAX;
        s_cur[tid] = 0;
    }
    uint32_t *wc = s_wcnt + wave * RADIX;
    const int lrow0 = wave * ITEMS * 64 + lane;
    int64_t rows[ITEMS][COLS];
    auto load_tile = [&](int64_t t, int64_t (&r)[ITEMS][COLS]) {
        const int64_t row0 = t * T;
        const int nrows = (int)min((int64_t)T, p.n - row0);
#pragma unroll
        for (int it = 0; it < ITEMS; it++) load_row<COLS>(p.src + (row0 + min(lrow0 + it * 64, nrows - 1)) * COLS, r[it]);
    };
    if (SMJ_P1C_PF && t0 < t1) load_tile(t0, rows);
    for (int64_t t = t0; t < t1; t++) {
        zero_counters<RADIX>(wc, lane);  // (the previous tile's last barrier freed the region)
        int64_t nxt[ITEMS][COLS];
        if (!SMJ_P1C_PF) load_tile(t, rows);
        else if (t + 1 < t1) load_tile(t + 1, nxt);  // in flight while this tile is placed
        __syncthreads();                              // counters zeroed (first tile: splitters, cursors)
        const int nrows = (int)min((int64_t)T, p.n - t * T);
        uint32_t dig[ITEMS];
        uint32_t vmask = 0;
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const bool inb = lrow0 + it * 64 < nrows;
            const bool pass = !p.use_sel | (pick<COLS>(rows[it], p.sel_col) > p.sel_val);
            const bool v = inb & pass;
            const int64_t k = pick<COLS>(rows[it], p.key_col);
            uint32_t b = 0;
#pragma unroll
            for (uint32_t step = 32; step; step >>= 1) b += s_spl[b + step - 1] < k ? step : 0u;
            dig[it] = v ? b : 0u;
            vmask |= v ? (1u << it) : 0u;
        }
        wave_rank<ITEMS, 6>(dig, vmask, wc, lane);
        __syncthreads();
        (void)tile_digit_starts<RADIX>(s_wcnt, s_bin, s_wsum);
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const uint32_t d = dig[it] & 0xffffu;
            dig[it] = (d << 16) | (s_bin[d] + wc[d] + (dig[it] >> 16));  // part << 16 | staging slot
        }
        __syncthreads();  // counters read out: the region becomes the staging tile
        if (tid < nb) {
            const uint32_t c = s_bin[tid + 1] - s_bin[tid], cur = s_cur[tid];
            const uint64_t cap = (uint64_t)w.v[64 + tid];
            const bool ok = (uint64_t)cur + c <= cap;
            if (!ok) atomicOr(&p.flags[1], 1u);
            s_ok[tid] = ok ? 1u : 0u;
            s_gb[tid] = w.v[tid] + g * (int64_t)cap + (int64_t)cur - (int64_t)s_bin[tid];
            s_cur[tid] = ok ? cur + c : cur;
        }
#pragma unroll
        for (int it = 0; it < ITEMS; it++)
            if ((vmask >> it) & 1u) {
                const uint32_t slot = dig[it] & 0xffffu;
                store_row<COLS>(s_rows + (size_t)slot * COLS, rows[it]);
                s_pd[slot] = (uint8_t)(dig[it] >> 16);
            }
        __syncthreads();  // staging tile and sub-region rows published
        const uint32_t total = s_bin[nb];
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const uint32_t slot = (uint32_t)(tid + it * kMsdThreads);
            if (slot < total) {
                const uint32_t b = s_pd[slot];
                if (s_ok[b]) {
                    int64_t r[COLS];
                    load_row<COLS>(s_rows + (size_t)slot * COLS, r);
                    store_row<COLS>(p.dst + (s_gb[b] + (int64_t)slot) * COLS, r);
                }
            }
        }
        __syncthreads();  // staging tile read out
        if (SMJ_P1C_PF)
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
#pragma unroll
                for (int c = 0; c < COLS; c++) rows[it][c] = nxt[it][c];
    }
    if (tid < RADIX) p.cnt[g * RADIX + tid] = tid < nb ? s_cur[tid] : 0u;
}

// part b's tile descriptors (MsdPartAParams::desc): block b, thread g = chunk
// g's rows of part b in ceil(rows / tile) tiles, the chunks in order
__global__ __launch_bounds__(1024) void msd_p1c_desc_kernel(const uint32_t *cnt, int G, int tile, const P1cDesc d,
                                                            uint64_t *desc) {
    __shared__ uint32_t s_w[16];
    const int b = blockIdx.x, g = threadIdx.x;
    const uint32_t c = g < G ? cnt[(int64_t)g * 64 + b] : 0u;
    const uint32_t nt = (c + tile - 1) / tile;
    uint32_t tot;
    uint32_t e = block_excl_scan<16>(nt, s_w, &tot);
    uint64_t *o = desc + d.dbase[b] + e;
    const int64_t r0 = d.st[b] + (int64_t)g * d.cap[b];
    for (uint32_t i = 0; i < nt; i++)
        o[i] = ((uint64_t)(r0 + (int64_t)i * tile) << 16) | (uint64_t)min((uint32_t)tile, c - i * (uint32_t)tile);
}

// ---------------------------------------------------------------------------
// runs: per-bucket run lists over the tile-local partitions
// ---------------------------------------------------------------------------
// rows [c0, c1) of a table of ntiles rows for this wave of this segment
__device__ __forceinline__ void msd_seg_range(int64_t ntiles, int64_t &c0, int64_t &c1) {
    const int64_t L = (ntiles + kMsdSegs - 1) / kMsdSegs;
    c0 = min((int64_t)blockIdx.y * L, ntiles);
    c1 = min(c0 + L, ntiles);
    const int64_t L4 = (c1 - c0 + 3) / 4;
    const int w = threadIdx.x >> 6;
    const int64_t s0 = min(c0 + w * L4, c1);
    c1 = min(s0 + L4, c1);
    c0 = s0;
}

// grid (ceil(nb / 64), kMsdSegs) x 256: lane = bucket; rows summed and
// non-empty runs counted per segment
__device__ __forceinline__ void runs_seg_body(const uint32_t *__restrict__ offs, int64_t ntiles,
                                                           int width, int nb, uint32_t *__restrict__ segL,
                                                           uint32_t *__restrict__ segC, const int64_t *__restrict__ tmm,
                                                           int64_t *__restrict__ segmm) {
    __shared__ uint32_t partL[4][64], partC[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int a = blockIdx.x * 64 + lane;
    int64_t c0, c1;
    msd_seg_range(ntiles, c0, c1);
    if (blockIdx.x == 0) {  // min / max of the selected keys over this wave's tiles
        int64_t mn = INT64_MAX, mx = INT64_MIN;
        for (int64_t t = c0 + lane; t < c1; t += 64) {
            mn = min(mn, tmm[2 * t]);
            mx = max(mx, tmm[2 * t + 1]);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mn = min(mn, (int64_t)__shfl_xor((long long)mn, o, 64));
            mx = max(mx, (int64_t)__shfl_xor((long long)mx, o, 64));
        }
        if (lane == 0) {
            segmm[2 * (blockIdx.y * 4 + w)] = mn;
            segmm[2 * (blockIdx.y * 4 + w) + 1] = mx;
        }
    }
    uint32_t L = 0, C = 0;
    if (a < nb) {
#pragma unroll 8
        for (int64_t t = c0; t < c1; t++) {
            const uint32_t len = offs[t * width + a + 1] - offs[t * width + a];
            L += len;
            C += len ? 1u : 0u;
        }
    }
    partL[w][lane] = L;
    partC[w][lane] = C;
    __syncthreads();
    if (w == 0 && a < nb) {
        segL[blockIdx.y * kOffsA + a] = partL[0][lane] + partL[1][lane] + partL[2][lane] + partL[3][lane];
        segC[blockIdx.y * kOffsA + a] = partC[0][lane] + partC[1][lane] + partC[2][lane] + partC[3][lane];
    }
}

// The per-segment bucket partials of msd_runs_seg_kernel ([kMsdSegs][kOffsA],
// rows or runs) become exclusive prefixes over the segments, in place, and
// tot[a] = the bucket's total.  grid (kOffsA / 64, arrays) x 1024: lane =
// bucket (coalesced), wave w = segments [w S, w S + S), S = kMsdSegs / 16,
// all S loads of a lane in flight at once.
struct MsdSegScanParams {
    uint32_t *seg[4];
    uint32_t *tot[4];
};
__global__ __launch_bounds__(1024) void msd_seg_scan_kernel(const MsdSegScanParams p) {
    constexpr int NW = 16, S = kMsdSegs / NW;
    static_assert(kMsdSegs % NW == 0 && kOffsA % 64 == 0, "segment / bucket split");
    __shared__ uint32_t s_part[NW][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int a = blockIdx.x * 64 + lane;
    uint32_t *seg = p.seg[blockIdx.y];
    uint32_t v[S], sum = 0;
#pragma unroll
    for (int i = 0; i < S; i++) v[i] = seg[(w * S + i) * kOffsA + a];
#pragma unroll
    for (int i = 0; i < S; i++) sum += v[i];
    s_part[w][lane] = sum;
    __syncthreads();
    uint32_t run = 0, tot = 0;
#pragma unroll
    for (int u = 0; u < NW; u++) {
        const uint32_t q = s_part[u][lane];
        run += u < w ? q : 0u;
        tot += q;
    }
#pragma unroll
    for (int i = 0; i < S; i++) {
        seg[(w * S + i) * kOffsA + a] = run;
        run += v[i];
    }
    if (w == 0) p.tot[blockIdx.y][a] = tot;
}

// Heavy keys of bucket a = blockIdx.x: kHeavySamples rows of the bucket, both
// tables in proportion to their rows, each one row of an evenly spaced pass-A
// tile's run of the bucket, counted in an LDS hash table; a key sampled at
// least thr times -- ~kHeavyRows rows of the bucket's L --
// is heavy (the kHeavyMax most sampled when more qualify).  Runs only when the
// pass-A sample already shows skew (kHeavySkew of its keys repeated, or a
// repeated splitter) and for multi-key
// buckets over 8 kGroupCap rows; elsewhere the bucket gets none.  A missed
// heavy key only costs speed (its sub-bucket takes the oversized-group path),
// a light key taken for heavy only a single-key group of its own: the sort
// and join never depend on the sample.
constexpr int kHeavyThreads = 256;  // small: on unskewed tables every workgroup only reads the gate and exits
constexpr uint32_t kHeavySkew = 8;  // sampled keys repeated within the pass-A sample that open the gate
constexpr int kHeavySlots = 2 * kHeavySamples;  // LDS hash table of the sampled keys (load <= 1/2)
__global__ __launch_bounds__(kHeavyThreads) void msd_heavy_kernel(const MsdHeavyParams p) {
    constexpr int PER = kHeavySamples / kHeavyThreads, SPT = kHeavySlots / kHeavyThreads;
    constexpr unsigned long long kEmpty = (unsigned long long)INT64_MAX;  // (an INT64_MAX key is never counted)
    __shared__ unsigned long long s_hk[kHeavySlots];
    __shared__ uint32_t s_hc[kHeavySlots];
    __shared__ int64_t s_cand[kHeavyMax];
    __shared__ uint32_t s_skew, s_cnt;
    const int a = blockIdx.x, t = threadIdx.x;
    if (t == 0) s_skew = p.plan->skew >= kHeavySkew ? 1u : 0u;
    __syncthreads();
    for (int i = t; i + 1 < kSplA; i += kHeavyThreads)  // (every splitter pair: SMJ_BITS_A=9 has 511 splitters)
        if (p.spl[i] == p.spl[i + 1]) s_skew = 1;  // benign race: all write 1
    __syncthreads();
    const int64_t *spl = p.spl;
    const bool own = a >= 1 && a < kSplA && spl[a] == spl[a - 1] && (a == 1 || spl[a - 2] != spl[a - 1]);
    const uint32_t L0 = p.totL[0][a], L1 = p.ntab > 1 ? p.totL[1][a] : 0u, L = L0 + L1;
    if (!s_skew || own || L < 8u * kGroupCap) {
        if (t == 0) p.nheavy[a] = 0;
        return;
    }
#pragma unroll
    for (int k = 0; k < SPT; k++) {
        s_hk[t + k * kHeavyThreads] = kEmpty;
        s_hc[t + k * kHeavyThreads] = 0;
    }
    // the samples: row j of table x from an evenly spaced pass-A tile's run of the bucket
    const uint32_t n0 = p.ntab > 1 ? (uint32_t)(((uint64_t)kHeavySamples * L0 + L / 2) / L) : (uint32_t)kHeavySamples;
    int64_t key[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const uint32_t i = (uint32_t)t + (uint32_t)k * kHeavyThreads;
        const int x = i < n0 ? 0 : 1;
        const uint32_t j = x ? i - n0 : i, nx = x ? kHeavySamples - n0 : n0;
        key[k] = INT64_MAX;  // no sample
        if (j < nx && p.ntiles[x] > 0) {
            const int64_t tile = (int64_t)(((unsigned __int128)j * (uint64_t)p.ntiles[x]) / nx);
            const uint32_t *o = p.offs[x] + tile * kOffsARow;
            const uint32_t s0 = o[a], s1 = o[a + 1];  // o[kBucketsA] = the tile's rows
            if (s1 > s0) {
                const uint32_t r = s0 + (uint32_t)(((uint64_t)(j * 0x9E3779B9u) * (s1 - s0)) >> 32);
                key[k] = p.tempA[x][((int64_t)tile * p.tile[x] + r) * p.cols[x] + p.key[x]];
            }
        }
    }
    __syncthreads();
    // count them in an LDS hash table (linear probing; <= half full)
#pragma unroll
    for (int k = 0; k < PER; k++) {
        if (key[k] == INT64_MAX) continue;
        const unsigned long long u = (unsigned long long)key[k];
        uint32_t h = (uint32_t)((u * 0x9E3779B97F4A7C15ull) >> 52) & (kHeavySlots - 1);
        for (int probe = 0; probe < kHeavySlots; probe++) {
            const unsigned long long prev = atomicCAS(&s_hk[h], kEmpty, u);
            if (prev == kEmpty || prev == u) {
                atomicAdd(&s_hc[h], 1u);
                break;
            }
            h = (h + 1) & (kHeavySlots - 1);
        }
    }
    __syncthreads();
    // hits for ~kHeavyRows rows of the bucket; raised until <= kHeavyMax keys qualify
    uint32_t thr = max(3u, (uint32_t)(((uint64_t)kHeavySamples * kHeavyRows + L - 1) / L));
    for (int round = 0; round < 16; round++) {
        if (t == 0) s_cnt = 0;
        __syncthreads();
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < SPT; k++) c += s_hc[t + k * kHeavyThreads] >= thr ? 1u : 0u;
        if (c) atomicAdd(&s_cnt, c);
        __syncthreads();
        const uint32_t tot = s_cnt;
        __syncthreads();
        if (tot <= (uint32_t)kHeavyMax) break;
        thr = thr + thr / 2 + 1;
    }
    if (t == 0) s_cnt = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SPT; k++) {
        const int i = t + k * kHeavyThreads;
        if (s_hc[i] >= thr) {
            const uint32_t at = atomicAdd(&s_cnt, 1u);
            if (at < (uint32_t)kHeavyMax) s_cand[at] = (int64_t)s_hk[i];
        }
    }
    __syncthreads();
    // ascending: each candidate's rank among the (distinct) candidates
    const uint32_t m = min(s_cnt, (uint32_t)kHeavyMax);
    if ((uint32_t)t < m) {
        const int64_t v = s_cand[t];
        uint32_t r = 0;
        for (uint32_t i = 0; i < m; i++) r += s_cand[i] < v ? 1u : 0u;
        p.heavy[(int64_t)a * kHeavyMax + r] = v;
    }
    if (t == 0) p.nheavy[a] = m;
}

// one workgroup of kOffsA threads: thread = bucket.  Bucket sizes / bases of
// both tables, the global key range, and the pass-B digit of every bucket.
#ifndef SMJ_PACK_HEAVY
#define SMJ_PACK_HEAVY 0  // 1: packed pass-B rows with heavy keys too (C5 +1.7 ms, r05zzp; the single-key tier reads words)
#endif
constexpr uint32_t kWideSkew = 256;  // repeated sampled keys that keep sparse buckets narrow (msd_bases)
#ifndef SMJ_WIDE_FILL
#define SMJ_WIDE_FILL 65  // percent (0: never)
#endif
constexpr int kBasesWaves = kOffsA / 64;
constexpr uint64_t kFill = (uint64_t)kGroupCap * 15 / 16, kOne = (uint64_t)kGroupCap * 13 / 16;

// sub-buckets a final group may span, for sub-buckets of <= w keys each: a
// group's span stays within the staged kernel's counting range when one
// sub-bucket fits it, else below 2^48 (the radix tiers' sort word); the group
// kernel computes the exact span of every group.  Narrow groups (<=
// kStageRange keys) of `span` sub-buckets hold ~span Lm / D rows per table;
// well under a full group, full groups spanning more keys for the wide-span
// staged kernel cost less (round 6, r06g: C3's tables with keys over [1, 1e9]
// made groups of two sub-buckets, msd_final 3.3 ms against 1.6 at [1, 3e8]
// and 2.1 on wide groups).  SMJ_WIDE_FILL = the narrow fill (percent of
// kFill) below which a bucket goes wide.  Not when the pass-A sample repeats
// many keys (plan->skew over kWideSkew of its ~8192): few distinct keys with
// long equal-key runs fill the narrow groups whatever the interval, and the
// wide kernel hands bins over 32 rows on.  (Joining tables repeat a few: an
// S key sampled together with its R partner.)
__device__ uint32_t bases_maxspan(uint64_t w, uint64_t Lm, uint64_t D, uint32_t skew) {
    uint64_t span = w <= (uint64_t)kStageRange ? (uint64_t)kStageRange / w : ((uint64_t)1 << 48) / w;
    if (w <= (uint64_t)kStageRange && Lm > 0 && skew < kWideSkew &&
        span * Lm * 100u < (uint64_t)SMJ_WIDE_FILL * kFill * D)
        span = ((uint64_t)1 << 48) / w;
    return span >= (uint64_t)kRadB ? (uint32_t)kRadB : span ? (uint32_t)span : 1u;
}
// keys per sub-bucket of a 64-bit scale, + 1: ceil(2^64 / scale) + 1
__device__ uint64_t sub_width(uint64_t scale) {
    return (uint64_t)((((unsigned __int128)1 << 64) + scale - 1u) / scale) + 1u;
}

// The segmented pass-B digit of bucket a (MsdSeg), from its sampled keys in
// key order (msd_sample_select_kernel: positions (at(a - 1), at(a)] hold the
// bucket's ~32), one wave per bucket, a lane per sample.  The gaps between
// consecutive samples -- and from lo to the first, from the last to hi --
// are the candidates:
//  1. the largest gap G, the sum S and number c of the gaps over range / 16
//     (a cut is one of them, and cuts must sum to range / 2), and delta0 =
//     the mean of the other gaps (the spacing inside the dense parts); a
//     bucket with S < range / 2 or G under 16 delta0 has no gaps (uniform
//     keys: S ~0.4 range, G ~4 spacings);
//  2. the cuts: gaps over thr = max(32 delta0, range / 16, 4 kRadB); the
//     bucket is segmented when they sum to half its interval;
//  3. the intervals, in key order, between the cuts (the first kSegMax - 1
//     internal ones; a bucket spanning more clusters keeps the rest inside its
//     last interval).  An interval runs from its first to its last sample
//     widened by kSegMargin = 6 of its spacings on each side (rows past the
//     extreme samples: ~1 spacing's worth on average, e^-6 of one beyond 6),
//     so the gap sub-buckets stay near empty; a cut at the bottom (lo lies in
//     a gap: the previous cluster's unsampled tail sits just above lo) makes a
//     first interval [lo, lo + 6 spacings of the previous bucket's last
//     samples].  Its weight = its width in spacings (expected rows, margins
//     included: a count of ~8 samples was too noisy -- r06y, sub-buckets of
//     1000 rows); the spacing is the interval's own over 8 or more samples,
//     else the bucket's (delta, the mean of the non-cut gaps).
// Where it runs: extra workgroups of msd_runs_seg_kernel, under its other
// workgroups' time (a thread per bucket in the one-workgroup bases kernel
// cost ~6 us on the critical path, r06z11; a side-stream kernel ~15 us,
// r06z14; four extra workgroups of part_a ~18 us, r06z17).
constexpr uint64_t kSegMargin = 6;  // spacings past an interval's extreme samples
constexpr int kSegFindBlocks = 16;  // msd_runs_seg_kernel's extra workgroups (4 buckets per wave)
constexpr unsigned kRunsSegX = (kBucketsA + 63) / 64;  // their blockIdx.x
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint64_t)__shfl_xor((unsigned long long)v, o, 64));
    return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, o, 64);
    return v;
}
__device__ void seg_find(const int64_t *ss, uint32_t M, int a, int64_t lo, int64_t hi, MsdSegFind *out) {
    const int lane = threadIdx.x & 63;
    auto at = [&](int q) { return min(M - 1u, (uint32_t)(((uint64_t)(q + 1) * M) / (kSplA + 1))); };
    const uint32_t p0 = a == 0 ? 0u : at(a - 1) + 1u, p1 = a >= kSplA ? M - 1u : at(a);
    if (p1 < p0 || p1 - p0 >= 64u) return;  // (~32 per bucket; more: leave it linear)
    const uint64_t range = (uint64_t)hi - (uint64_t)lo;
    // lane j: sample p0 + j; the valid ones (in [lo, hi]) are a run of lanes
    const bool have = (uint32_t)lane <= p1 - p0;
    const int64_t k = have ? ss[p0 + lane] : hi;
    const bool in = have && k >= lo && k <= hi;
    const uint64_t vm = __ballot(in);
    const uint32_t n = (uint32_t)__popcll(vm);
    if (n < 16) return;
    const int l0 = __ffsll((long long)vm) - 1, l1 = 63 - __clzll((long long)vm);
    const int64_t up = __shfl_up((long long)k, 1, 64);
    const uint64_t g = in ? (uint64_t)k - (uint64_t)(lane == l0 ? lo : up) : 0u;  // the gap below sample lane
    const int64_t first = __shfl((long long)k, l0, 64), last = __shfl((long long)k, l1, 64);
    const uint64_t gtop0 = (uint64_t)hi - (uint64_t)last;
    // 1.
    const uint64_t r16 = range / 16u;
    const uint64_t G = max(wave_max64(g), gtop0);
    const uint64_t S = wave_sum64(g > r16 ? g : 0u) + (gtop0 > r16 ? gtop0 : 0u);
    const uint32_t c = (uint32_t)__popcll(__ballot(g > r16)) + (gtop0 > r16 ? 1u : 0u);
    if (S < range / 2u || c > n) return;
    const uint64_t delta0 = max<uint64_t>(1u, (range - S) / (n + 1u - c));
    if (G / 16u <= delta0) return;
    // 2.
    const uint64_t thr = max(max(32u * delta0, range / 16u), (uint64_t)(4 * kRadB));
    const uint64_t cm = __ballot(g > thr);  // cut below sample lane
    const bool topcut = gtop0 > thr, bottom = (cm >> l0) & 1ull;
    const uint64_t total = wave_sum64(g > thr ? g : 0u) + (topcut ? gtop0 : 0u);
    const uint32_t ncut = (uint32_t)__popcll(cm) + (topcut ? 1u : 0u);
    if (total < range / 2u || ncut == 0) return;
    const uint64_t delta = max<uint64_t>(1u, (range - total) / (n + 1u - ncut));
    const uint64_t gbot = bottom ? (uint64_t)__shfl((unsigned long long)g, l0, 64) : 0u;
    const uint64_t gtop = topcut ? gtop0 : 0u;
    // 3. (wave-uniform: the intervals are a handful; lane 0 stores them)
    uint32_t K = 0;
    auto emit = [&](int64_t st, int64_t en, uint64_t dk) {
        if (lane == 0) {
            out->st[K] = st;
            out->en[K] = en;
            out->wt[K] = (float)((double)((uint64_t)en - (uint64_t)st + 1u) / (double)dk);
        }
        K++;
    };
    if (bottom) {  // the previous bucket's tail: its last samples' spacing
        // (the middle two of its last four gaps: one of them may cross a gap)
        uint64_t dp = delta;
        if (p0 >= 5u) {
            uint64_t g4[4];
#pragma unroll
            for (int i = 0; i < 4; i++) g4[i] = (uint64_t)ss[p0 - 1 - i] - (uint64_t)ss[p0 - 2 - i];
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 3; y++)
                    if (g4[y] > g4[y + 1]) {
                        const uint64_t t2 = g4[y];
                        g4[y] = g4[y + 1], g4[y + 1] = t2;
                    }
            dp = max<uint64_t>(1u, g4[1] / 2u + g4[2] / 2u);
        }
        emit(lo, (int64_t)((uint64_t)lo + min(kSegMargin * dp, gbot / 4u)), dp);
    }
    uint64_t cuts = cm & ~(1ull << l0);  // the internal cuts (lanes whose gap below is one)
    int fl = l0;                          // the open interval's first lane
    while (true) {
        int el = l1;
        uint64_t ga = gtop;
        bool open_end = !topcut;
        const bool cut = cuts != 0 && K + 2u <= (uint32_t)kSegMax;  // (room for this interval and the last)
        if (cut) {
            const int cl = __ffsll((long long)cuts) - 1;
            cuts &= cuts - 1;
            el = cl - 1;
            ga = (uint64_t)__shfl((unsigned long long)g, cl, 64);
            open_end = false;
        }
        const int64_t f = __shfl((long long)k, fl, 64), e = __shfl((long long)k, el, 64);
        const uint32_t cnt = (uint32_t)(el - fl + 1);
        const uint64_t gb = fl == l0 ? gbot : (uint64_t)__shfl((unsigned long long)g, fl, 64);
        const uint64_t dk = cnt >= 8u ? max<uint64_t>(1u, ((uint64_t)e - (uint64_t)f) / (cnt - 1u)) : delta;
        const int64_t st = (fl == l0 && !bottom) ? lo : (int64_t)((uint64_t)f - min(kSegMargin * dk, gb / 4u));
        const int64_t en = open_end ? hi : (int64_t)((uint64_t)e + min(kSegMargin * dk, ga / 4u));
        emit(st, en, dk);
        if (!cut) break;
        fl = el + 1;
    }
    if (lane == 0) {
        out->topcut = topcut ? 1u : 0u;
        out->K = K;
    }
}

// msd_runs_seg_kernel's extra workgroups (blockIdx.x == kRunsSegX, y <
// kSegFindBlocks), a wave per bucket: seg_find over every bucket, K = 0 where
// it finds no gaps.  The end buckets' open ends (the global min / max: that
// kernel's partials) are taken as the extreme samples; msd_bases_kernel
// extends the end intervals to them.
__device__ void seg_find_all(const MsdRunsArgs &q, int blk) {
    const int lane = threadIdx.x & 63;
    const int wave = blk * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6), nw = kSegFindBlocks * (int)(blockDim.x >> 6);
    uint32_t M = lane < kSampleGatherBlocks ? (uint32_t)q.seg_samp[kSampleN + lane] : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) M += __shfl_xor(M, o, 64);
    const int64_t *ss = q.seg_samp + kSortedOff, *spl = q.seg_spl;
    const bool ok = q.seg_plan->skew < kWideSkew && M >= (uint32_t)(8 * kBucketsA) && M <= (uint32_t)kSampleN;
    for (int a = wave; a < kBucketsA; a += nw) {
        MsdSegFind *out = q.segf + a;
        if (lane == 0) out->K = 0;
        if (!ok || (a >= 1 && a < kSplA && spl[a] == spl[a - 1])) continue;  // (a heavy key's bucket / a run of repeats)
        // bucket a = (spl[a-1], spl[a]] as msd_bases_kernel has it
        const int64_t lo = a == 0 ? ss[0] : (int64_t)((uint64_t)spl[a - 1] + 1u);
        int64_t hi = a == kSplA ? ss[M - 1] : spl[a];
        if (a + 1 < kSplA && spl[a + 1] == spl[a]) hi = (int64_t)((uint64_t)spl[a] - 1u);
        if (hi > lo && (uint64_t)hi - (uint64_t)lo >= (uint64_t)kRadB) seg_find(ss, M, a, lo, hi, out);
    }
}

// msd_bases_kernel: the sub-buckets of seg_find's intervals.  The first
// interval starts at lo, the last ends at hi unless a gap was cut there (the
// end buckets: seg_find saw the extreme samples).  Sub-buckets go to the
// intervals by their weights, one gap sub-bucket after each.
__device__ void seg_finish(const MsdSegFind &f, int64_t lo, int64_t hi, uint64_t D, uint64_t Lm, uint32_t skew,
                           MsdSeg &sg) {
    const uint32_t K = f.K;
    int64_t st[kSegMax], en[kSegMax];
    float W = 0.f;
    for (uint32_t k = 0; k < K; k++) {
        st[k] = f.st[k], en[k] = f.en[k];
        W += f.wt[k];
    }
    st[0] = lo;
    if (!f.topcut) en[K - 1] = hi;
    const uint64_t dense = D - K;  // the rest: one gap sub-bucket per interval
    uint32_t db = 0;
    for (uint32_t k = 0; k < kSegMax; k++) {
        if (k >= K) {
            // unused: copies of the last interval (part_b's search may land on them)
            sg.st[k] = sg.st[K - 1], sg.s32[k] = sg.s32[K - 1], sg.pk[k] = sg.pk[K - 1], sg.ms[k] = sg.ms[K - 1];
            continue;
        }
        // (kSegMax sub-buckets held back: a float product rounded up in every
        // interval must not push the last digit past D - 1)
        const float w = f.wt[k] / W;
        uint64_t dn = max<uint64_t>(1u, (uint64_t)((float)(dense - K - kSegMax) * w));
        // and by construction: room for this interval's gap sub-bucket and two
        // digits for each interval after it
        dn = max<uint64_t>(1u, min<uint64_t>(dn, D - db - 1u - 2u * (K - 1u - k)));
        // the interval's residuals r = key - st < R (R > dn), shifted under 2^32
        const uint64_t R1 = max((uint64_t)en[k] - (uint64_t)st[k], dn);  // R - 1
        const uint32_t sh = R1 >> 32 ? 64u - (uint32_t)__clzll((long long)(R1 >> 32)) : 0u;  // bits of R1 >> 32
        const uint64_t Rs = (R1 >> sh) + 1u;  // <= 2^32
        dn = min(dn, Rs - 1u);
        const uint32_t s32 = (uint32_t)((dn << 32) / Rs);
        sg.st[k] = st[k];
        sg.s32[k] = s32;
        sg.pk[k] = db | (uint32_t)dn << 11 | sh << 22;
        // keys per sub-bucket <= (ceil(2^32 / s32) + 1) << sh
        sg.ms[k] = bases_maxspan((((1ull << 32) + s32 - 1u) / s32 + 1u) << sh, (uint64_t)((float)Lm * w), dn, skew);
        db += (uint32_t)dn + 1u;
    }
    sg.hi = hi;
    sg.nseg = K;
    for (int k = 0; k < 21; k++) sg.pad[k] = 0;
}

__global__ __launch_bounds__(kOffsA) void msd_bases_kernel(const MsdBasesParams p) {
    __shared__ uint32_t s_wsum[kBasesWaves];
    __shared__ int64_t s_mm[2 * kBasesWaves];
    const int a = threadIdx.x, lane = a & 63, wave = a >> 6;
    // global min / max of the selected keys over both tables
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    for (int x = 0; x < p.ntab; x++)  // per (segment, wave) partials of msd_runs_seg_kernel
        for (int i = a; i < kMsdSegs * 4; i += kOffsA) {
            mn = min(mn, p.segmm[x][2 * i]);
            mx = max(mx, p.segmm[x][2 * i + 1]);
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o, 64));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o, 64));
    }
    if (lane == 0) {
        s_mm[wave] = mn;
        s_mm[kBasesWaves + wave] = mx;
    }
    __syncthreads();
    for (int w = 0; w < kBasesWaves; w++) {
        mn = min(mn, s_mm[w]);
        mx = max(mx, s_mm[kBasesWaves + w]);
    }
    // packed pass-B rows: other columns in int32, every key within 2^32 of
    // any group base, and no heavy keys (msd_heavy_kernel's, or a repeated
    // splitter: they make single-key / oversized groups, whose rows the other
    // tiers read through the unpacked copy)
    const bool hv = a < kBucketsA && ((p.nheavy && p.nheavy[a] != 0u) || (a + 1 < kSplA && p.spl[a] == p.spl[a + 1]));
    const bool any_heavy = __syncthreads_or(hv) != 0;
    if (a == 0)
        p.plan->packB = p.pack_ok && p.plan->nopack == 0u && (p.pack_ok == 2 || !any_heavy || SMJ_PACK_HEAVY) && mn <= mx &&
                                (uint64_t)mx - (uint64_t)mn < (1ull << 32)
                            ? 1u : 0u;
    // rows of bucket a per table
    uint32_t Lt[2] = {0u, 0u};
    if (a < kBucketsA)
        for (int x = 0; x < p.ntab; x++) Lt[x] = p.totL[x][a];
    // pass-B digit of bucket a over the bucket's key interval [lo, hi]:
    // floor((key - lo) * D / (hi - lo + 1)) as one mulhi, or key - lo
    // when the interval holds fewer than kRadB keys.  D <= kRadB sub-buckets
    // are sized so that whole numbers of them fill a final group: at C3
    // 2 x 448 = 896 of 1024 rows instead of 2 x 381 = 762 with D = kRadB.
    int64_t lo = 0;
    uint64_t scale = 0;
    uint32_t maxspan = kRadB, s32 = 0, heavy = 0;
    bool one_key = false, seg = false;
    if (a < kBucketsA) {
        // bucket a = (spl[a-1], spl[a]] (open ends: the global min / max),
        // less a repeated splitter value, which is bucket i + 1 of its first
        // occurrence i (bucket_a); buckets inside a run of repeats are empty
        const int64_t *spl = p.spl;
        int64_t hi;
        if (a >= 1 && a < kSplA && spl[a] == spl[a - 1] && (a == 1 || spl[a - 2] != spl[a - 1])) {
            lo = hi = spl[a - 1];  // a heavy key's own bucket
        } else {
            lo = a == 0 ? mn : (int64_t)((uint64_t)spl[a - 1] + 1u);
            hi = a == kSplA ? mx : spl[a];
            if (a + 1 < kSplA && spl[a + 1] == spl[a]) hi = (int64_t)((uint64_t)spl[a] - 1u);  // repeated: not here
        }
        one_key = lo == hi;
        const uint64_t range = hi > lo ? (uint64_t)hi - (uint64_t)lo : 0u;  // interval = range + 1 keys
        if (range >= (uint64_t)kRadB) {
            // k sub-buckets of ~kFill / k rows fill a group; a bucket too big for
            // k >= 2 gets lone sub-buckets of ~kOne rows, 6 standard deviations
            // (uniform keys) below the cap: a multi-key sub-bucket over the cap
            // would leave the LDS path for the (slow) LSD fallback
            // (combined packing: groups of ~2 kFill rows of both tables)
            const uint64_t Lm = p.combined ? ((uint64_t)Lt[0] + Lt[1] + 1u) / 2u : (uint64_t)max(Lt[0], Lt[1]);
            uint64_t D = kRadB;
            if (Lm > 0 && !p.full_radix) {
                const uint64_t k = (uint64_t)kRadB * kFill / Lm;
                D = k >= 2 ? (Lm * k + kFill - 1) / kFill : (Lm + kOne - 1) / kOne;
                D = min<uint64_t>(kRadB, max<uint64_t>(kRadB / 2, D));
            }
            // the bucket's heavy keys take two sub-buckets each (their own and
            // the split of their linear sub-bucket's other keys): D - 2 m linear ones
            if (p.nheavy) {
                heavy = min(p.nheavy[a], (uint32_t)kHeavyMax);
                D = min<uint64_t>(D, (uint64_t)kRadB - 2u * heavy);
            }
            const unsigned __int128 q = ((unsigned __int128)D << 64) / ((unsigned __int128)range + 1u);
            scale = q >> 64 ? ~0ull : (uint64_t)q;
            // an interval under 2^32 keys takes a 32-bit digit, mulhi32(r, s32)
            // (one multiply in part_b instead of a 64 x 64 high product)
            if (range < 0xffffffffull) s32 = (uint32_t)(((uint64_t)D << 32) / (range + 1u));
            // keys per sub-bucket <= ceil(2^K / scale) + 1 =: w (K = 64, or 32
            // with s32; ~(range + 1) / D + 2)
            const uint64_t w = s32 ? ((1ull << 32) + s32 - 1u) / s32 + 1u : sub_width(scale);
            maxspan = bases_maxspan(w, Lm, D, p.plan->skew);
            // keys in dense intervals with wide gaps between (clustered keys)
            if (p.segf && !p.full_radix && heavy == 0u && p.plan->skew < kWideSkew && p.segf[a].K) {
                MsdSeg sg;
                seg_finish(p.segf[a], lo, hi, D, Lm, p.plan->skew, sg);
                {
                    seg = true;
                    p.seg[a] = sg;
                    scale = 1, s32 = 0, maxspan = kRadB;  // (unused: nonzero, so not single-key sub-buckets)
                    atomicAdd(&p.plan->nsegb, 1u);
                }
            }
        }
    }
    for (int x = 0; x < p.ntab; x++) {
        const uint32_t L = a < kBucketsA ? p.totL[x][a] : 0u, C = a < kBucketsA ? p.totC[x][a] : 0u;
        const uint32_t K = (L + (uint32_t)p.tile[x] - 1) / (uint32_t)p.tile[x];
        uint32_t totL, totC, totK;
        const uint32_t rs = block_excl_scan<kBasesWaves>(L, s_wsum, &totL);
        const uint32_t lb = block_excl_scan<kBasesWaves>(C, s_wsum, &totC);
        const uint32_t tb = block_excl_scan<kBasesWaves>(K, s_wsum, &totK);
        if (a < kBucketsA) {
            MsdBucket b;
            b.lo = lo;
            b.scale = scale;
            b.maxspan = maxspan;
            b.L = L;
            b.row_start = rs;
            b.list_base = lb;
            b.nruns = C;
            b.tile_base = tb;
            b.one_key = (one_key ? 1u : 0u) | (seg ? kBucketSeg : 0u) | (heavy << 8);
            b.s32 = s32;
            p.bk[x][a] = b;
        }
        if (a == 0) {
            p.plan->m[x] = totL;
            p.plan->ntilesB[x] = totK;
        }
    }
    if (a == 0) {
        p.plan->gmin = mn;
        p.plan->gmax = mx;
    }
}

// grid (kBucketsA / 4, kMsdSegs) x 256: emit the run list entries of every
// bucket for this segment, and the first run of every pass-B tile.  Wave =
// bucket, lane = tile: the segment's runs of one bucket are 64 at a time
// prefixed by two wave scans (rows, non-empty runs) and leave as consecutive
// list entries (coalesced; a lane-per-bucket loop wrote 64 scattered 8-B
// entries per store, 90 us per table at C3).  The offsA loads are strided,
// but a 128-B line of a tile's row serves 32 buckets' waves from L2.
__device__ __forceinline__ void runs_apply_body(const uint32_t *__restrict__ offs, int64_t ntiles,
                                                             int T, int TB, const uint32_t *__restrict__ segL,
                                                             const uint32_t *__restrict__ segC,
                                                             const MsdBucket *__restrict__ bk,
                                                             uint2 *__restrict__ list, uint2 *__restrict__ tinfo) {
    const int lane = threadIdx.x & 63;
    // XCD-aware block order: the eight workgroups whose bucket quads share
    // one 128-B offsA line (quads 8j .. 8j + 7 of one segment) get linear ids
    // p = 64 m + 8 r + x -- the same x, i.e. the same XCD (workgroups are
    // dealt round-robin over the 8 XCDs), one after another -- so the line
    // is fetched into one L2 once instead of into eight
    const uint32_t p = blockIdx.x + blockIdx.y * gridDim.x;
    constexpr uint32_t G8 = kBucketsA / 32;  // groups of eight quads (one offsA line) per segment
    const uint32_t x = p & 7u, r = (p >> 3) & 7u, sj = (p >> 6) * 8u + x;
    const uint32_t seg = sj / G8, quad = (sj % G8) * 8u + r;
    const int a = (int)quad * 4 + (threadIdx.x >> 6);
    const int64_t Ls = (ntiles + kMsdSegs - 1) / kMsdSegs;
    const int64_t c0 = min((int64_t)seg * Ls, ntiles), c1 = min(c0 + Ls, ntiles);
    uint32_t P = segL[seg * kOffsA + a], Q = segC[seg * kOffsA + a];  // exclusive prefixes
    const uint32_t lbase = uni32(bk[a].list_base), tbase = uni32(bk[a].tile_base);
    const uint32_t uT = (uint32_t)TB;  // pass-B tile rows (T: pass-A tile rows)
    for (int64_t t0 = c0; t0 < c1; t0 += 64) {
        const int64_t t = t0 + lane;
        uint32_t o = 0, len = 0;
        if (t < c1) {
            o = offs[t * kOffsARow + a];
            len = offs[t * kOffsARow + a + 1] - o;
        }
        const uint32_t nz = len ? 1u : 0u;
        const uint32_t il = wave_incl_scan(len, lane), iq = wave_incl_scan(nz, lane);
        if (len) {
            const uint32_t v = P + il - len, e = lbase + Q + iq - 1u;
            list[e] = make_uint2((uint32_t)(t * T) + o, v);
            for (uint32_t k = (v + uT - 1) / uT; k * uT < v + len; k++)  // pass-B tiles starting inside this run
                tinfo[tbase + k] = make_uint2((uint32_t)a, e);
        }
        P += (uint32_t)__shfl((int)il, 63, 64);
        Q += (uint32_t)__shfl((int)iq, 63, 64);
    }
}

// both tables in one launch (blockIdx.z = table): one ramp and tail instead of two
__global__ __launch_bounds__(256) void msd_runs_seg_kernel(const MsdRunsArgs a) {
    const int x = blockIdx.z;
    if (blockIdx.x == kRunsSegX) {  // the segmented digit's sample scan (dispatched early: low y)
        if (a.segf && x == 0 && blockIdx.y < (unsigned)kSegFindBlocks) seg_find_all(a, (int)blockIdx.y);
        return;
    }
    if (x >= a.ntab) return;
    runs_seg_body(x ? a.offs[1] : a.offs[0], x ? a.ntiles[1] : a.ntiles[0], kOffsARow, kBucketsA,
                  x ? a.segL[1] : a.segL[0], x ? a.segC[1] : a.segC[0], x ? a.tmm[1] : a.tmm[0],
                  x ? a.segmm[1] : a.segmm[0]);
}
__global__ __launch_bounds__(256) void msd_runs_apply_kernel(const MsdRunsArgs a) {
    const int x = blockIdx.z;
    if (x >= a.ntab) return;
    runs_apply_body(x ? a.offs[1] : a.offs[0], x ? a.ntiles[1] : a.ntiles[0], x ? a.T[1] : a.T[0],
                    x ? a.TB[1] : a.TB[0], x ? a.segL[1] : a.segL[0], x ? a.segC[1] : a.segC[0],
                    x ? a.bk[1] : a.bk[0], x ? a.list[1] : a.list[0], x ? a.tinfo[1] : a.tinfo[0]);
}

// ---------------------------------------------------------------------------
// part_b: gather a pass-B tile through the run list, stable tile-local
// partition by the 9-bit sub-bucket
// ---------------------------------------------------------------------------
// wave-uniform copies (SGPRs) of per-tile metadata loaded through vector loads
// (kernel arguments may alias the outputs, so hipcc cannot use scalar loads)
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni32((uint32_t)(v >> 32)) << 32) | uni32((uint32_t)v);
}
__device__ __forceinline__ uint2 uni_tinfo(const uint2 *t, int64_t g) {
    const uint2 v = t[g];
    return make_uint2(uni32(v.x), uni32(v.y));
}
// The same through scalar (SMEM) loads, for addresses that are wave-uniform
// (the data was written by an earlier launch: the scalar cache starts each
// launch invalidated).  SMEM loads count on lgkmcnt, so waiting for one does
// not retire the vector loads and stores in flight, as a vector load's
// vmcnt(0) did in part_b's tile loop.
#define SMJ_CONST(T) const __attribute__((address_space(4))) T
__device__ __forceinline__ uint2 sc_tinfo(const uint2 *t, int64_t g) {
    const uint64_t w = *(SMJ_CONST(uint64_t) *)uni64((uint64_t)(t + g));
    return make_uint2((uint32_t)w, (uint32_t)(w >> 32));
}
static_assert(sizeof(MsdBucket) == 48 && offsetof(MsdBucket, maxspan) == 16 && offsetof(MsdBucket, s32) == 44,
              "sc_bucket reads MsdBucket as six words");
__device__ __forceinline__ MsdBucket sc_bucket(const MsdBucket *bk, uint32_t a) {
    SMJ_CONST(uint64_t) *q = (SMJ_CONST(uint64_t) *)uni64((uint64_t)(bk + a));
    const uint64_t w2 = q[2], w3 = q[3], w4 = q[4], w5 = q[5];
    MsdBucket r;
    r.lo = (int64_t)q[0];
    r.scale = q[1];
    r.maxspan = (uint32_t)w2, r.L = (uint32_t)(w2 >> 32);
    r.row_start = (uint32_t)w3, r.list_base = (uint32_t)(w3 >> 32);
    r.nruns = (uint32_t)w4, r.tile_base = (uint32_t)(w4 >> 32);
    r.one_key = (uint32_t)w5, r.s32 = (uint32_t)(w5 >> 32);
    return r;
}
__device__ __forceinline__ MsdBucket uni_bucket(const MsdBucket *bk, uint32_t a) {
    const MsdBucket v = bk[a];
    MsdBucket r;
    r.lo = (int64_t)uni64((uint64_t)v.lo);
    r.scale = uni64(v.scale);
    r.s32 = uni32(v.s32);
    r.maxspan = uni32(v.maxspan);
    r.L = uni32(v.L);
    r.row_start = uni32(v.row_start);
    r.list_base = uni32(v.list_base);
    r.nruns = uni32(v.nruns);
    r.tile_base = uni32(v.tile_base);
    r.one_key = uni32(v.one_key);
    return r;
}

// ---------------------------------------------------------------------------
// the pass-B digit (part_b computes it, the group kernel inverts it)
// ---------------------------------------------------------------------------
// linear sub-bucket of residual r = key - lo
__device__ __forceinline__ uint32_t pb_lin(const MsdBucket &b, uint64_t r) {
    return b.s32 ? __umulhi((uint32_t)r, b.s32)  // < D: r < 2^32 in such a bucket
                 : b.scale ? min((uint32_t)__umul64hi(r, b.scale), (uint32_t)(kRadB - 1)) : (uint32_t)r;
}
// heavy keys below `key` in the bucket's sorted list hv[0, m) (m <= kHeavyMax),
// and whether key is one of them.  hv holds kHeavyMax entries, those past m
// INT64_MAX, so the search is a fixed branch-free one: every row's steps are
// plain LDS loads, and a thread's items search side by side (the guarded form,
// `pos + st <= m && ...`, compiled to a branch per step and item, and the
// items' dependent LDS loads ran one after the other: C5 part_b +12 %, r05m)
__device__ __forceinline__ uint32_t heavy_rank(const int64_t *hv, uint32_t m, int64_t key, bool &eq) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t st = kHeavyMax / 2; st >= 1; st >>= 1) pos += hv[pos + st - 1] < key ? st : 0u;
    const int64_t h = hv[pos];
    pos += h < key ? 1u : 0u;  // pos == kHeavyMax - 1: all kHeavyMax below key
    eq = h == key && pos < m;
    return pos;
}
// the digit with m heavy keys: lin + 2 c + e (order-preserving; heavy key j --
// 0-based -- alone in sub-bucket lin(h_j) + 2 j + 1)
__device__ __forceinline__ uint32_t pb_digit_heavy(uint32_t lin, const int64_t *hv, uint32_t m, int64_t key) {
    bool eq;
    const uint32_t c = heavy_rank(hv, m, key, eq);
    return lin + 2u * c + (eq ? 1u : 0u);
}

// the segmented digit (MsdSeg's first 16 words in LDS: st[0..7], s32 at 8, pk
// at 12 (u32 pairs)): the last interval starting at or below the key
// (st[0] = lo <= every key of the bucket), then its linear sub-bucket or, past
// the interval, its gap sub-bucket
__device__ __forceinline__ uint32_t pb_digit_seg(const int64_t *sg, int64_t key) {
    uint32_t k = 0;  // (the unused entries repeat the last interval: any of them gives its digit)
#pragma unroll
    for (uint32_t j = 1; j < (uint32_t)kSegMax; j++) k += key >= sg[j] ? 1u : 0u;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(sg + kSegMax);
    const uint32_t s32 = w[k], pk = w[kSegMax + k];
    const uint64_t r = ((uint64_t)key - (uint64_t)sg[k]) >> seg_sh(pk);
    const uint32_t m = (r >> 32) ? seg_dn(pk) : min(__umulhi((uint32_t)r, s32), seg_dn(pk));
    return seg_db(pk) + m;
}

// Diagnostic phase stamps of part_b (SMJ_DEBUG_MSD=1; off in production):
// [k] cycles of phase k summed over tiles (thread 0's view), [7] tiles.
// Ablation bits for smj_debug_part_b_time (timing only, output invalid):
// 2 = no row stores, 4 = synthetic rows instead of the gathers, 8 = no offsB stores,
// 16 = force the ballot ranking path, 32 = no run-list lookups (with 4),
// 64 = 40 KiB of padding LDS (one workgroup per CU)
__device__ unsigned long long g_pb_phase[8];
#define PB_STAMP(k)                                                 \
    if (SMJ_STAMPS && (p.dbg & 1) && tid == 0) {                                        \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        atomicAdd(&g_pb_phase[k], t_ - pb_t);                       \
        pb_t = t_;                                                  \
    }


constexpr int kPbFastMax = 16;  // longest sub-bucket run of a tile the atomic-rank path orders
// the same limit in msd_part_b_pipe_kernel (per quad of waves).  With the
// waves taking turns on the ballot path, runs up to 128 rows were cheaper
// ranked by the scan (C5's Zipf tiles: part_b 13.8 -> 12.9 ms at 128, 13.9
// at 256, 22.5 at 1024 -- profiles/r02bu, r02bv); with the parallel ballot
// path (SMJ_PB_SLOWPAR) 16 is best again: C5 part_b 11.3 -> 9.6 ms, 32 gives
// 9.7 (profiles/r03/r03m_ab_c5.txt); C3's tiles never take it
#ifndef SMJ_PB_FASTMAX
#define SMJ_PB_FASTMAX 16
#endif

template <int COLS>
__global__ __launch_bounds__(pb_threads(COLS), COLS == 2 ? 8 : COLS == 1 ? 2 : 4) void msd_part_b_kernel(
    const MsdPartBParams p) {
    constexpr int NT = pb_threads(COLS), NW = NT / 64, T = msd_tile_b(COLS), ITEMS = T / NT, RADIX = kRadB;
    constexpr int DPT = RADIX / NT;  // histogram digits per thread (even)
    static_assert(T % NT == 0 && RADIX % (2 * NT) == 0, "tile / histogram split");
    // One LDS region, reused per phase: (1) the run list + lookup aids (a
    // bitmap of run starts, btab[b] = entry holding tile row 64 * b: row r's
    // entry is btab[r / 64] + the run starts in (64 (r / 64), r], a popcount);
    // (2) the atomic path's tile-row permutation + the ballot path's
    // counters; (3) the staging tile.  Part_b is latency-bound: one workgroup
    // per CU instead of two costs +54 % (tools/pb_ablate.py).
    constexpr int LISTB = (T + 1) * 8, ATB = 0, BMB = T / 8, BTB = T / 64 * 2;
    constexpr int ROWB = T * COLS * 8, PERMB = T * 2, CNTB = RADIX * 4, LKB = LISTB + ATB + BMB + BTB;
    // the per-quad sub-bucket counts (below) sit past the lists, perm and
    // counters: zeroed while the list is live, dead before the tile is staged
    static_assert(NW % 4 == 0, "quads of waves");
    constexpr int QN = NW / 4, QW = (QN + 1) / 2, QB = QW * RADIX * 4;
    constexpr int QOFF0 = LKB > PERMB + CNTB ? LKB : PERMB + CNTB, QOFF = (QOFF0 + 15) / 16 * 16;
    constexpr int UB = ROWB > QOFF + QB ? ROWB : QOFF + QB;
    __shared__ __attribute__((aligned(16))) unsigned char s_u[UB];
    __shared__ uint32_t s_wsum[NW];
    __shared__ uint32_t s_slow;
    __shared__ int64_t s_hv[kHeavyMax];  // the tile's bucket's heavy keys (MsdBucket::one_key bits 8..15)
    uint16_t *s_perm = reinterpret_cast<uint16_t *>(s_u);
    uint32_t *s_cnt = reinterpret_cast<uint32_t *>(s_u + PERMB);
    int64_t *s_rows = reinterpret_cast<int64_t *>(s_u);
    uint2 *s_list = reinterpret_cast<uint2 *>(s_u);
    uint32_t *s_bm = reinterpret_cast<uint32_t *>(s_u + LISTB + ATB);
    uint16_t *s_bt = reinterpret_cast<uint16_t *>(s_u + LISTB + ATB + BMB);
    // sub-bucket counts per quad of waves (u16 halves of word (quad >> 1) *
    // RADIX + d), then each quad's first tile row of sub-bucket d
    uint32_t *s_q = reinterpret_cast<uint32_t *>(s_u + QOFF);

    // persistent over tiles g = blockIdx.x + k * gridDim.x.  The next tile's
    // metadata chain (tinfo -> bucket -> first run-list entries) is issued
    // while this tile is ranked, staged and stored, so a tile starts with
    // its run list already in registers.
    const int64_t ntl = (int64_t)p.plan->ntilesB[p.x];
    int64_t g = blockIdx.x;
    if (g >= ntl) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long pb_t = (SMJ_STAMPS && (p.dbg & 1)) ? __builtin_amdgcn_s_memtime() : 0;
    uint2 ti = uni_tinfo(p.tinfo, g);
    MsdBucket b = uni_bucket(p.bk, ti.x);
    auto runs_of = [&](const uint2 &t, const MsdBucket &bb, int64_t gg) {  // run-list entries of tile gg
        const uint32_t vv = (uint32_t)(gg - bb.tile_base) * (uint32_t)T;
        const uint32_t nr = min((uint32_t)T, bb.L - vv);
        return min(bb.list_base + bb.nruns - t.y, nr + 1u);
    };
    const uint64_t *list64 = reinterpret_cast<const uint64_t *>(p.list);
    uint64_t le = 0;  // run-list entry tid of the current tile ({x, y} as one word)
    if ((uint32_t)tid < runs_of(ti, b, g)) le = list64[ti.y + tid];
    // wait for le HERE on the prologue path: otherwise the loop-top use merges
    // this path (nothing issued after the load) with the back edge and hipcc
    // waits vmcnt(0) every tile, draining the previous tile's 64 KiB of stores
    asm volatile("" ::"v"(le));
    if (tid == 0) s_slow = 0;
    // quad of waves of this thread, its count half and word row (recomputed
    // where used: live across the tile loop they spilled)
    auto quad_of = [&]() { return (uint32_t)opaque_tid() >> 8; };
    for (; g < ntl; g += gridDim.x) {
        // per-lane values recomputed per tile (live across the loop they spill)
        const int tid = opaque_tid(), lane = tid & 63, wave = tid >> 6;
        const uint32_t v0 = (uint32_t)(g - b.tile_base) * (uint32_t)T;
        const int nrows = (int)min((uint32_t)T, b.L - v0);
        const uint32_t q0 = ti.y;
        const int J = (int)runs_of(ti, b, g);
        for (int i = tid; i < QB / 16; i += NT) reinterpret_cast<uint4 *>(s_q)[i] = make_uint4(0, 0, 0, 0);
        if (msd_heavy_count(b.one_key) && tid < kHeavyMax)  // read after two barriers; padded (heavy_rank)
            s_hv[tid] = (uint32_t)tid < msd_heavy_count(b.one_key) ? p.heavy[(int64_t)ti.x * kHeavyMax + tid] : INT64_MAX;
        if ((b.one_key & kBucketSeg) && tid < 16)  // a segmented digit instead (no heavy keys then)
            s_hv[tid] = reinterpret_cast<const int64_t *>(p.seg + ti.x)[tid];
        if (p.dbg & 32) goto lookups_done;
        if (tid < J) reinterpret_cast<uint64_t *>(s_list)[tid] = le;
        for (int j = tid + NT; j < J; j += NT)  // > NT runs: rare
            reinterpret_cast<uint64_t *>(s_list)[j] = list64[q0 + j];
        for (int i = tid; i < T / 32; i += NT) s_bm[i] = 0;
        __syncthreads();
        for (int j = tid; j < J; j += NT) {  // runs are non-empty: starts strictly increase
            const uint32_t y = s_list[j].y;
            const uint32_t s0 = y > v0 ? y - v0 : 0u;
            const uint32_t e = j + 1 < J ? s_list[j + 1].y - v0 : (uint32_t)nrows;
            if (s0 < (uint32_t)nrows) {
                atomicOr(&s_bm[s0 >> 5], 1u << (s0 & 31));
                for (uint32_t bb = (s0 + 63) >> 6; (bb << 6) < e && (bb << 6) < (uint32_t)nrows; bb++)
                    s_bt[bb] = (uint16_t)j;
            }
        }
        __syncthreads();
    lookups_done:
        PB_STAMP(0);

        const int lrow0 = wave * ITEMS * 64 + lane;
        int64_t rows[ITEMS][COLS];
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const uint32_t r = (uint32_t)min(lrow0 + it * 64, nrows - 1), bb = r >> 6;
            const uint64_t m = ((uint64_t)s_bm[2 * bb + 1] << 32 | s_bm[2 * bb]) & ((2ull << (r & 63)) - 1ull) & ~1ull;
            const uint32_t j = s_bt[bb] + (uint32_t)__popcll(m);  // run starts in (64 bb, r]
            const uint2 e = s_list[j];
            if (p.dbg & 4) {
#pragma unroll
                for (int c = 0; c < COLS; c++) rows[it][c] = b.lo + (int64_t)((v0 + r) * 7u % (b.L + 1u));
            } else {
                load_row<COLS>(p.srcA + (int64_t)(e.x + (v0 + r - e.y)) * COLS, rows[it]);
            }
        }
        const int64_t gn = g + gridDim.x;
        const uint2 tin = uni_tinfo(p.tinfo, min(gn, ntl - 1));  // prefetch 1: next tile's info
        __syncthreads();  // list dead: the region becomes the counters or the staging tile
        PB_STAMP(1);

        uint32_t dig[ITEMS];  // sub-bucket | atomic rank << 16, then the staging position
        uint32_t vmask = 0;
        const uint32_t hm = msd_heavy_count(b.one_key);  // block-uniform
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const bool v = lrow0 + it * 64 < nrows;
            const uint32_t d = pb_lin(b, (uint64_t)pick<COLS>(rows[it], p.key_col) - (uint64_t)b.lo);
            dig[it] = v ? d & (RADIX - 1) : 0u;
            vmask |= v ? (1u << it) : 0u;
        }
        if (__builtin_expect(hm != 0u, 0)) {  // heavy keys in the bucket (C5): lin + 2 c + e
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u)
                    dig[it] = pb_digit_heavy(dig[it], s_hv, hm, pick<COLS>(rows[it], p.key_col)) & (RADIX - 1);
        }
        if (__builtin_expect((b.one_key & kBucketSeg) != 0u, 0)) {  // clustered keys: the segmented digit
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) dig[it] = pb_digit_seg(s_hv, pick<COLS>(rows[it], p.key_col)) & (RADIX - 1);
        }
        // Atomic path: per quad of waves one u16 count per sub-bucket, ranks in
        // atomic order.  Stability is restored per row below among the rows
        // of its quad and sub-bucket (usually none or one other); a tile with
        // a quad's sub-bucket over kPbFastMax rows takes the ballot path
        // instead (wave_rank + per-wave counters).  (A whole-tile count and a
        // fix-up over the tile's sub-bucket run cost ~2x the fix-up rounds.)
        {
            const uint32_t quad = quad_of(), qsh = 16u * (quad & 1u), qrow = (quad >> 1) * RADIX;
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it];
                    dig[it] = d | (((atomicAdd(&s_q[qrow + d], 1u << qsh) >> qsh) & 0xffffu) << 16);
                }
        }
        const MsdBucket bn = uni_bucket(p.bk, tin.x);  // prefetch 2: its bucket
        __syncthreads();
        PB_STAMP(2);
        {  // counts -> per-quad first rows, in place; the tile's sub-bucket starts -> offsB
            uint32_t sum = 0, cmax = 0;
#pragma unroll
            for (int k = 0; k < DPT; k++)
#pragma unroll
                for (int q2 = 0; q2 < QW; q2++) {
                    const uint32_t w = s_q[q2 * RADIX + DPT * tid + k];
                    sum += (w & 0xffffu) + (w >> 16);
                    cmax = max(cmax, max(w & 0xffffu, w >> 16));
                }
            if (cmax > (uint32_t)kPbFastMax || (p.dbg & 16)) s_slow = 1;
            uint32_t tot;
            uint32_t st = block_excl_scan_nb<NW>(sum, s_wsum, &tot);  // + barrier
            uint32_t sw = 0;
#pragma unroll
            for (int k = 0; k < DPT; k++) {
                sw = (k & 1) ? sw | (st << 16) : st;
                if ((k & 1) && !(p.dbg & 8)) reinterpret_cast<uint32_t *>(p.offs + g * kOffsB)[DPT / 2 * tid + k / 2] = sw;
#pragma unroll
                for (int q2 = 0; q2 < QW; q2++) {
                    const uint32_t w = s_q[q2 * RADIX + DPT * tid + k];
                    const uint32_t b1 = st + (w & 0xffffu);
                    s_q[q2 * RADIX + DPT * tid + k] = st | (b1 << 16);
                    st = b1 + (w >> 16);
                }
            }
            static_assert(kOffsB % 2 == 0 && DPT % 2 == 0, "offsB rows 4-B aligned: starts leave two per word");
            if (tid == 0 && !(p.dbg & 8)) p.offs[g * kOffsB + RADIX] = (uint16_t)nrows;
        }
        __syncthreads();
        const bool slow = s_slow != 0;
        if (!slow) {
            const uint32_t quad = quad_of(), qsh = 16u * (quad & 1u), qrow = (quad >> 1) * RADIX;
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it] & 0xffffu;
                    s_perm[((s_q[qrow + d] >> qsh) & 0xffffu) + (dig[it] >> 16)] = (uint16_t)(lrow0 + it * 64);
                }
            __syncthreads();
            // stable rank: the rows of this quad's sub-bucket group that precede this one
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it] & 0xffffu, w = s_q[qrow + d];
                    const uint32_t st = (w >> qsh) & 0xffffu;
                    uint32_t en;  // the next quad's first row of d (quad is wave-uniform)
                    if (!(quad & 1)) en = w >> 16;
                    else if (quad + 1 < QN) en = s_q[qrow + RADIX + d] & 0xffffu;
                    else en = d + 1u < (uint32_t)RADIX ? (s_q[d + 1] & 0xffffu) : (uint32_t)nrows;
                    const uint32_t r = (uint32_t)(lrow0 + it * 64);
                    uint32_t rank = 0;
                    if (en - st > 1u)
                        for (uint32_t j = st; j < en; j++) rank += (uint32_t)s_perm[j] < r;
                    dig[it] = st + rank;
                }
        } else {
            // a sub-bucket run over kPbFastMax rows: ballot ranks (wave_rank),
            // the waves taking turns on one counter array so that the ranks
            // follow tile-row order across waves too
#pragma unroll
            for (int k = 0; k < RADIX / NT; k++) s_cnt[tid + k * NT] = 0;
#pragma unroll
            for (int it = 0; it < ITEMS; it++) dig[it] &= 0xffffu;
            __syncthreads();
            for (int w = 0; w < NW; w++) {
                if (wave == w) wave_rank<ITEMS, kBitsB>(dig, vmask, s_cnt, lane);
                __syncthreads();
            }
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it] & 0xffffu;
                    dig[it] = (s_q[d] & 0xffffu) + (dig[it] >> 16);  // quad 0's first row = the sub-bucket start
                }
        }
        __syncthreads();  // permutation / counters dead: the region becomes the staging tile
        PB_STAMP(3);
#pragma unroll
        for (int it = 0; it < ITEMS; it++)
            if ((vmask >> it) & 1u) store_row<COLS>(s_rows + (size_t)dig[it] * COLS, rows[it]);
        if (gn < ntl && (uint32_t)tid < runs_of(tin, bn, gn)) le = list64[tin.y + tid];  // prefetch 3: its runs
        __syncthreads();
        if (tid == 0) s_slow = 0;
        PB_STAMP(4);
        int64_t *dst = p.out + g * T * COLS;
        if (!(p.dbg & 2)) {
#pragma unroll
            for (int it = 0; it < ITEMS; it++) {
                const int s = min(tid + it * NT, nrows - 1);
                int64_t r[COLS];
                load_row<COLS>(s_rows + (size_t)s * COLS, r);
                store_row_nt<COLS>(dst + (size_t)s * COLS, r);
            }
        }
        PB_STAMP(5);
        if (SMJ_STAMPS && (p.dbg & 1) && tid == 0) atomicAdd(&g_pb_phase[7], 1ull);
        __syncthreads();  // staging region read out before the next tile's list lands in it
        ti = tin;
        b = bn;
    }
}

// ---- part_b, pipelined (2-column tables) ------------------------------------
// The same tile work as msd_part_b_kernel, reordered so that the NEXT tile's
// rows are gathered before THIS tile's rows are stored: its run list goes to
// a region of its own (s_nl, up to one entry per thread), built while this
// tile is ranked, and its gathers are issued between this tile's staging and
// its stores.  A vector-memory wait on gfx950 retires every older load AND
// store, so in the plain kernel the rank phase of tile k + 1 waited behind
// tile k's 64 KiB of stores; here the stores are younger than the gathers
// they used to hold up.  A next tile with more runs than threads is
// gathered after the stores, through the main region (the plain order).
#ifndef SMJ_PB_PIPE
#define SMJ_PB_PIPE 1
#endif
#ifndef SMJ_PB_NOSTORE
#define SMJ_PB_NOSTORE 0
#endif
#ifndef SMJ_PB_ONEKEY
#define SMJ_PB_ONEKEY 1  // heavy-key buckets skip the tile's counting and ranking
#endif
#ifndef SMJ_PB_SLOWPAR
#define SMJ_PB_SLOWPAR 1  // the ballot path ranks on per-wave counters in parallel (0: waves in turn)
#endif

// row -> run lookups of a tile (run list lst, start bitmap bm, 64-row block
// table bt) and the row gathers into registers
template <int COLS, int ITEMS>
__device__ __forceinline__ void pb_gather(const MsdPartBParams &p, const MsdBucket &bk, const uint2 *lst,
                                          const uint32_t *bm, const uint16_t *bt, uint32_t v0, int nrows, int lrow0,
                                          int64_t (&rows)[ITEMS][COLS]) {
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t r = (uint32_t)min(lrow0 + it * 64, nrows - 1), bb = r >> 6;
        const uint64_t m = ((uint64_t)bm[2 * bb + 1] << 32 | bm[2 * bb]) & ((2ull << (r & 63)) - 1ull) & ~1ull;
        const uint32_t j = bt[bb] + (uint32_t)__popcll(m);  // run starts in (64 bb, r]
        const uint2 e = lst[j];
        if (p.dbg & 4) {
#pragma unroll
            for (int c = 0; c < COLS; c++) rows[it][c] = bk.lo + (int64_t)((v0 + r) * 7u % (bk.L + 1u));
        } else {
            if (SMJ_PB_NTLOAD) load_row_nt<COLS>(p.srcA + (int64_t)(e.x + (v0 + r - e.y)) * COLS, rows[it]);
            else load_row<COLS>(p.srcA + (int64_t)(e.x + (v0 + r - e.y)) * COLS, rows[it]);
        }
    }
}

// the start bitmap (zeroed) and block table of a run list of J entries
template <int NT>
__device__ __forceinline__ void pb_marks(const uint2 *lst, uint32_t *bm, uint16_t *bt, int J, uint32_t v0,
                                         int nrows) {
    for (int j = opaque_tid(); j < J; j += NT) {  // runs are non-empty: starts strictly increase
        const uint32_t y = lst[j].y;
        const uint32_t s0 = y > v0 ? y - v0 : 0u;
        const uint32_t e = j + 1 < J ? lst[j + 1].y - v0 : (uint32_t)nrows;
        if (s0 < (uint32_t)nrows) {
            atomicOr(&bm[s0 >> 5], 1u << (s0 & 31));
            for (uint32_t bb = (s0 + 63) >> 6; (bb << 6) < e && (bb << 6) < (uint32_t)nrows; bb++) bt[bb] = (uint16_t)j;
        }
    }
}

// the packed pass-B word of a 2-column row (MsdPlan::packB): the key's low 32
// bits, the other column's low 32 bits above them
__device__ __forceinline__ uint64_t pb_word(const int64_t (&r)[2], int key_col) {
    return (uint64_t)(uint32_t)r[key_col] | ((uint64_t)(uint32_t)r[1 - key_col] << 32);
}

// PKM: 0 rows, 2 packed words when MsdPlan::packB (set on the device by
// msd_bases, after the host has enqueued the call: a block-uniform branch)
template <int COLS, int PKM = 0>
__global__ __launch_bounds__(pb_threads(COLS), 8) void msd_part_b_pipe_kernel(const MsdPartBParams p) {
    static_assert(PKM == 0 || COLS == 2, "packed rows: 2-column tables");
    constexpr int NT = pb_threads(COLS), NW = NT / 64, T = msd_tile_b(COLS), ITEMS = T / NT, RADIX = kRadB;
    constexpr int DPT = RADIX / NT;
    static_assert(T % NT == 0 && RADIX % (2 * NT) == 0, "tile / histogram split");
    constexpr int LISTB = (T + 1) * 8, BMB = T / 8, BTB = T / 64 * 2;
    constexpr int ROWB = T * COLS * 8, PERMB = T * 2, CNTB = RADIX * 4, LKB = LISTB + BMB + BTB;
    static_assert(NW % 4 == 0, "quads of waves");
    constexpr int QN = NW / 4, QW = (QN + 1) / 2, QB = QW * RADIX * 4;
    constexpr int QOFF0 = LKB > PERMB + CNTB ? LKB : PERMB + CNTB, QOFF = (QOFF0 + 15) / 16 * 16;
    constexpr int UB = ROWB > QOFF + QB ? ROWB : QOFF + QB;
    __shared__ __attribute__((aligned(16))) unsigned char s_u[UB];
    __shared__ uint2 s_nl[NT];          // the next tile's run list (<= NT entries)
    __shared__ uint32_t s_nbm[T / 32];  // its start bitmap
    __shared__ uint16_t s_nbt[T / 64];  // its 64-row block table
    __shared__ uint32_t s_wsum[NW];
    __shared__ uint32_t s_slow;
    __shared__ int64_t s_hv[kHeavyMax];  // the tile's bucket's heavy keys (MsdBucket::one_key bits 8..15)
    uint16_t *s_perm = reinterpret_cast<uint16_t *>(s_u);
    uint32_t *s_cnt = reinterpret_cast<uint32_t *>(s_u + PERMB);
    int64_t *s_rows = reinterpret_cast<int64_t *>(s_u);
    uint2 *s_list = reinterpret_cast<uint2 *>(s_u);
    uint32_t *s_bm = reinterpret_cast<uint32_t *>(s_u + LISTB);
    uint16_t *s_bt = reinterpret_cast<uint16_t *>(s_u + LISTB + BMB);
    uint32_t *s_q = reinterpret_cast<uint32_t *>(s_u + QOFF);

    const bool PK = PKM == 2 && uni32(p.plan->packB) != 0u;
    const int64_t ntl = (int64_t)p.plan->ntilesB[p.x];
    int64_t g = blockIdx.x;
    if (g >= ntl) return;
    const uint64_t *list64 = reinterpret_cast<const uint64_t *>(p.list);
    auto runs_of = [&](const uint2 &t, const MsdBucket &bb, int64_t gg) {  // run-list entries of tile gg
        const uint32_t vv = (uint32_t)(gg - bb.tile_base) * (uint32_t)T;
        const uint32_t nr = min((uint32_t)T, bb.L - vv);
        return min(bb.list_base + bb.nruns - t.y, nr + 1u);
    };
    auto tile_v0 = [&](const MsdBucket &bb, int64_t gg) { return (uint32_t)(gg - bb.tile_base) * (uint32_t)T; };
    auto tile_rows = [&](const MsdBucket &bb, int64_t gg) { return (int)min((uint32_t)T, bb.L - tile_v0(bb, gg)); };
    auto quad_of = [&]() { return (uint32_t)opaque_tid() >> 8; };
    // the plain order's list build in the main region (entries past the
    // first NT come straight from global memory); ends with a barrier
    auto build_main = [&](const uint2 &t, const MsdBucket &bb, int64_t gg, uint64_t le) {
        const int tid = opaque_tid();
        const int J = (int)runs_of(t, bb, gg);
        if (tid < J) reinterpret_cast<uint64_t *>(s_list)[tid] = le;
        for (int j = tid + NT; j < J; j += NT) reinterpret_cast<uint64_t *>(s_list)[j] = list64[t.y + j];
        for (int i = tid; i < T / 32; i += NT) s_bm[i] = 0;
        __syncthreads();
        pb_marks<NT>(s_list, s_bm, s_bt, J, tile_v0(bb, gg), tile_rows(bb, gg));
        __syncthreads();
    };

    uint2 ti = sc_tinfo(p.tinfo, g);
    MsdBucket b = sc_bucket(p.bk, ti.x);
    int64_t rows[ITEMS][COLS];
    {  // prologue: tile g's run list and gathers
        const int tid = opaque_tid(), lrow0 = (tid >> 6) * ITEMS * 64 + (tid & 63);
        uint64_t le = 0;
        if ((uint32_t)tid < runs_of(ti, b, g)) le = list64[ti.y + tid];
        build_main(ti, b, g, le);
        pb_gather<COLS, ITEMS>(p, b, s_list, s_bm, s_bt, tile_v0(b, g), tile_rows(b, g), lrow0, rows);
        // consumed here, so the loop top's wait counts only the back edge's
        // stores (vmcnt(stores)) instead of merging this path's vmcnt(0)
#pragma unroll
        for (int it = 0; it < ITEMS; it++)
#pragma unroll
            for (int c = 0; c < COLS; c++) asm volatile("" ::"v"(rows[it][c]));
    }
    uint2 tn = sc_tinfo(p.tinfo, min(g + (int64_t)gridDim.x, ntl - 1));  // the next tile's info
    if (opaque_tid() == 0) s_slow = 0;
    __syncthreads();  // the main list region is dead
    for (; g < ntl; g += gridDim.x) {
        const int tid = opaque_tid(), lane = tid & 63, wave = tid >> 6;
        const int64_t gn = g + gridDim.x;
        const uint32_t v0 = tile_v0(b, g);
        const int nrows = tile_rows(b, g);
        const int lrow0 = wave * ITEMS * 64 + lane;
        for (int i = tid; i < QB / 16; i += NT) reinterpret_cast<uint4 *>(s_q)[i] = make_uint4(0, 0, 0, 0);
        for (int i = tid; i < T / 32; i += NT) s_nbm[i] = 0;
        const MsdBucket bn = sc_bucket(p.bk, tn.x);  // the next tile's bucket
        // and the info of the tile after it (scalar loads: a vector load here,
        // or after the next tile's gathers as before, is waited with vmcnt(0),
        // which also retires the gathers and the previous tile's stores)
        const uint2 tn2 = sc_tinfo(p.tinfo, min(gn + (int64_t)gridDim.x, ntl - 1));
        // the tile's bucket's heavy keys (C5; block-uniform: none elsewhere).
        // Eight per wave through scalar loads: an SMEM wait is on lgkmcnt, so
        // it does not retire this tile's gathers and the previous tile's
        // stores, as the vmcnt wait of a vector load here would (every tile
        // of a heavy bucket then drained its stores: C5 part_b +1 ms, r05e)
        const uint32_t hm = msd_heavy_count(b.one_key);
        if (hm) {  // padded to kHeavyMax with INT64_MAX (heavy_rank)
            static_assert(NW * 8 > kHeavyMax, "eight heavy keys per wave, the last wave free");
            const uint32_t w8 = (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 8u;
            if (w8 < hm) {
                SMJ_CONST(int64_t) *hq =
                    (SMJ_CONST(int64_t) *)uni64((uint64_t)(p.heavy + (int64_t)ti.x * kHeavyMax + w8));
                const int64_t h0 = hq[0], h1 = hq[1], h2 = hq[2], h3 = hq[3], h4 = hq[4], h5 = hq[5], h6 = hq[6],
                              h7 = hq[7];
                const int l8 = lane & 7;
                const int64_t v = l8 == 0 ? h0 : l8 == 1 ? h1 : l8 == 2 ? h2 : l8 == 3 ? h3 : l8 == 4 ? h4
                                                                                           : l8 == 5 ? h5 : l8 == 6 ? h6 : h7;
                if (lane < 8 && w8 + (uint32_t)lane < hm) s_hv[w8 + lane] = v;
            }
            // the pads, by the last wave (it loads none: NW * 8 > kHeavyMax)
            if (wave == NW - 1 && hm + (uint32_t)lane < (uint32_t)kHeavyMax) {
                // INT64_MAX made here: left to the compiler, the constant was
                // hoisted out of the loop, spilled, and reloaded here behind a
                // vmcnt(0) that drained the tile's gathers and stores
                uint32_t lo = ~0u, hi = 0x7fffffffu;
                asm volatile("" : "+v"(lo), "+v"(hi));
                reinterpret_cast<uint2 *>(s_hv)[hm + lane] = make_uint2(lo, hi);
            }
        }
        const bool sgb = (b.one_key & kBucketSeg) != 0u;  // block-uniform: a segmented digit (clustered keys)
        if (__builtin_expect(sgb, 0)) {  // its 16 words, eight per wave of the first two (scalar loads, as above)
            const uint32_t w8 = (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 8u;
            if (w8 < 16u) {
                SMJ_CONST(int64_t) *hq = (SMJ_CONST(int64_t) *)uni64((uint64_t)(reinterpret_cast<const int64_t *>(p.seg + ti.x) + w8));
                const int64_t h0 = hq[0], h1 = hq[1], h2 = hq[2], h3 = hq[3], h4 = hq[4], h5 = hq[5], h6 = hq[6],
                              h7 = hq[7];
                const int l8 = lane & 7;
                const int64_t v = l8 == 0 ? h0 : l8 == 1 ? h1 : l8 == 2 ? h2 : l8 == 3 ? h3 : l8 == 4 ? h4
                                                                                           : l8 == 5 ? h5 : l8 == 6 ? h6 : h7;
                if (lane < 8) s_hv[w8 + lane] = v;
            }
        }
        __syncthreads();

        uint32_t dig[ITEMS];  // sub-bucket | atomic rank << 16, then the staging position
        uint32_t vmask = 0;
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const bool v = lrow0 + it * 64 < nrows;
            const uint32_t d = pb_lin(b, (uint64_t)pick<COLS>(rows[it], p.key_col) - (uint64_t)b.lo);
            dig[it] = v ? d & (RADIX - 1) : 0u;
            vmask |= v ? (1u << it) : 0u;
        }
        if (__builtin_expect(hm != 0u, 0)) {  // heavy keys in the bucket (C5): lin + 2 c + e
            // (two items at a time, no branches: four side by side spilled at 64 VGPRs)
#pragma unroll
            for (int i0 = 0; i0 < ITEMS; i0 += 2) {
#pragma unroll
                for (int it = i0; it < i0 + 2 && it < ITEMS; it++) {
                    const uint32_t hd = pb_digit_heavy(dig[it], s_hv, hm, pick<COLS>(rows[it], p.key_col)) & (RADIX - 1);
                    dig[it] = ((vmask >> it) & 1u) ? hd : dig[it];
                }
                asm volatile("" ::: "memory");
            }
        }
        if (__builtin_expect(sgb, 0)) {  // the segmented digit, one item at a time (two spilled)
#pragma unroll
            for (int it = 0; it < ITEMS; it++) {
                const uint32_t sd = pb_digit_seg(s_hv, pick<COLS>(rows[it], p.key_col)) & (RADIX - 1);
                dig[it] = ((vmask >> it) & 1u) ? sd : dig[it];
                asm volatile("" ::: "memory");
            }
        }
        // a heavy key's own bucket (one key value): every row falls in
        // sub-bucket 0 and the tile's gather order is already its stable
        // order -- no counting atomics (all on one LDS word) and no ranking
        // (cmax > SMJ_PB_FASTMAX would take the slow wave-by-wave path)
        const bool one_key = SMJ_PB_ONEKEY && (b.one_key & 1u) != 0u;  // block-uniform (SMEM)
        if (!one_key) {
            const uint32_t quad = quad_of(), qsh = 16u * (quad & 1u), qrow = (quad >> 1) * RADIX;
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it];
                    dig[it] = d | (((atomicAdd(&s_q[qrow + d], 1u << qsh) >> qsh) & 0xffffu) << 16);
                }
        } else if (tid == 0) {
            s_q[0] = (uint32_t)nrows;  // quad 0, sub-bucket 0: the whole tile (the offsB scan below)
        }
        const bool more = gn < ntl;
        const int Jn = more ? (int)runs_of(tn, bn, gn) : 0;
        uint64_t le = 0;  // the next tile's run-list entries
        if (tid < Jn) le = list64[tn.y + tid];
        __syncthreads();
        {  // counts -> per-quad first rows, in place; the tile's sub-bucket starts -> offsB
            uint32_t sum = 0, cmax = 0;
#pragma unroll
            for (int k = 0; k < DPT; k++)
#pragma unroll
                for (int q2 = 0; q2 < QW; q2++) {
                    const uint32_t w = s_q[q2 * RADIX + DPT * tid + k];
                    sum += (w & 0xffffu) + (w >> 16);
                    cmax = max(cmax, max(w & 0xffffu, w >> 16));
                }
            if (cmax > (uint32_t)SMJ_PB_FASTMAX || (p.dbg & 16)) s_slow = 1;
            uint32_t tot;
            uint32_t st = block_excl_scan_nb<NW>(sum, s_wsum, &tot);  // + barrier
            uint32_t sw = 0;
#pragma unroll
            for (int k = 0; k < DPT; k++) {
                sw = (k & 1) ? sw | (st << 16) : st;
                if (k & 1) reinterpret_cast<uint32_t *>(p.offs + g * kOffsB)[DPT / 2 * tid + k / 2] = sw;
#pragma unroll
                for (int q2 = 0; q2 < QW; q2++) {
                    const uint32_t w = s_q[q2 * RADIX + DPT * tid + k];
                    const uint32_t b1 = st + (w & 0xffffu);
                    s_q[q2 * RADIX + DPT * tid + k] = st | (b1 << 16);
                    st = b1 + (w >> 16);
                }
            }
            if (tid == 0) p.offs[g * kOffsB + RADIX] = (uint16_t)nrows;
        }
        __syncthreads();
        const bool slow = s_slow != 0;
        if (one_key) {
#pragma unroll
            for (int it = 0; it < ITEMS; it++) dig[it] = (uint32_t)(lrow0 + it * 64);  // identity (valid rows)
        } else if (!slow) {
            const uint32_t quad = quad_of(), qsh = 16u * (quad & 1u), qrow = (quad >> 1) * RADIX;
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it] & 0xffffu;
                    s_perm[((s_q[qrow + d] >> qsh) & 0xffffu) + (dig[it] >> 16)] = (uint16_t)(lrow0 + it * 64);
                }
            __syncthreads();
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it] & 0xffffu, w = s_q[qrow + d];
                    const uint32_t st = (w >> qsh) & 0xffffu;
                    uint32_t en;
                    if (!(quad & 1)) en = w >> 16;
                    else if (quad + 1 < QN) en = s_q[qrow + RADIX + d] & 0xffffu;
                    else en = d + 1u < (uint32_t)RADIX ? (s_q[d + 1] & 0xffffu) : (uint32_t)nrows;
                    const uint32_t r = (uint32_t)(lrow0 + it * 64);
                    uint32_t rank = 0;
                    if (en - st > 1u)
                        for (uint32_t j = st; j < en; j++) rank += (uint32_t)s_perm[j] < r;
                    dig[it] = st + rank;
                }
        } else if (SMJ_PB_SLOWPAR) {
            // a sub-bucket run over SMJ_PB_FASTMAX rows (Zipf tiles): every wave
            // ranks its rows on a u16 counter row of its own (NW x RADIX x 2 B =
            // the whole 64 KiB region), then one cross-wave prefix per digit.
            // The tile's sub-bucket starts (quad 0's first rows) wait in the
            // next tile's list region, idle until the staging barrier.
            static_assert(NW * RADIX * 2 <= UB && RADIX * 2 <= (int)sizeof(s_nl) && RADIX == 2 * NT,
                          "per-wave u16 counters fit the region; one packed counter pair per thread");
            uint16_t *s_st = reinterpret_cast<uint16_t *>(s_nl);
            uint16_t *cw = reinterpret_cast<uint16_t *>(s_u);
            for (int d = tid; d < RADIX; d += NT) s_st[d] = (uint16_t)(s_q[d] & 0xffffu);
#pragma unroll
            for (int it = 0; it < ITEMS; it++) dig[it] &= 0xffffu;
            __syncthreads();  // s_q read out: the region becomes the counters
            {
                uint4 *z = reinterpret_cast<uint4 *>(cw + wave * RADIX);
#pragma unroll
                for (int i = 0; i < RADIX * 2 / 16 / 64; i++) z[lane + i * 64] = make_uint4(0, 0, 0, 0);
            }
            __syncthreads();
            wave_rank16<ITEMS, kBitsB>(dig, vmask, cw + wave * RADIX, lane);
            __syncthreads();
            {  // digits 2 tid, 2 tid + 1: exclusive prefix over the waves (u16 pairs, no carry: <= T rows)
                uint32_t *c32 = reinterpret_cast<uint32_t *>(s_u);
                uint32_t run = 0;
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    const uint32_t c = c32[w * (RADIX / 2) + tid];
                    c32[w * (RADIX / 2) + tid] = run;
                    run += c;
                }
            }
            __syncthreads();
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it] & 0xffffu;
                    dig[it] = (uint32_t)s_st[d] + (uint32_t)cw[wave * RADIX + d] + (dig[it] >> 16);
                }
        } else {
#pragma unroll
            for (int k = 0; k < RADIX / NT; k++) s_cnt[tid + k * NT] = 0;
#pragma unroll
            for (int it = 0; it < ITEMS; it++) dig[it] &= 0xffffu;
            __syncthreads();
            for (int w = 0; w < NW; w++) {
                if (wave == w) wave_rank<ITEMS, kBitsB>(dig, vmask, s_cnt, lane);
                __syncthreads();
            }
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
                if ((vmask >> it) & 1u) {
                    const uint32_t d = dig[it] & 0xffffu;
                    dig[it] = (s_q[d] & 0xffffu) + (dig[it] >> 16);
                }
        }
        __syncthreads();  // permutation / counters dead: the region becomes the staging tile
        // (storing the ranked rows straight from registers instead, scattered
        // 16-B stores into the tile's region: part_b 1.58 -> 1.93 ms at C3,
        // profiles/r03/r03l_ab_c3.txt)
        int64_t *dst = p.out + g * T * COLS;
#pragma unroll
        for (int it = 0; it < ITEMS; it++)
            if ((vmask >> it) & 1u) store_row<COLS>(s_rows + (size_t)dig[it] * COLS, rows[it]);
        const bool early = more && Jn <= NT;  // block-uniform
        if (early && tid < Jn) reinterpret_cast<uint64_t *>(s_nl)[tid] = le;
        __syncthreads();  // staging tile and the next run list written
        if (tid == 0) s_slow = 0;
        if (early) {  // the next tile's gathers, ahead of this tile's stores
            pb_marks<NT>(s_nl, s_nbm, s_nbt, Jn, tile_v0(bn, gn), tile_rows(bn, gn));
            __syncthreads();
            pb_gather<COLS, ITEMS>(p, bn, s_nl, s_nbm, s_nbt, tile_v0(bn, gn), tile_rows(bn, gn), lrow0, rows);
        }
        // the stores are unconditional (a run-time ablation bit around them
        // made hipcc's wait for the next tile's rows a vmcnt(0) that also
        // retired these stores); SMJ_PB_NOSTORE=1 builds the no-store ablation
        if (!SMJ_PB_NOSTORE) {
#pragma unroll
            for (int it = 0; it < ITEMS; it++) {
                const int s = min(tid + it * NT, nrows - 1);
                int64_t r[COLS];
                load_row<COLS>(s_rows + (size_t)s * COLS, r);
                if (PK) {  // one word per row: tile g's words at [g T, g T + rows) of the u64 view
                    __builtin_nontemporal_store(pb_word(r, p.key_col), reinterpret_cast<uint64_t *>(p.out) + g * T + s);
                } else {
                    store_row_nt<COLS>(dst + (size_t)s * COLS, r);
                }
            }
        }
        __syncthreads();  // staging region read out
        if (more && !early) {  // over NT runs: the plain order, through the main region
            build_main(tn, bn, gn, le);
            pb_gather<COLS, ITEMS>(p, bn, s_list, s_bm, s_bt, tile_v0(bn, gn), tile_rows(bn, gn), lrow0, rows);
            // consumed on this path (rows younger than the stores): the loop
            // top then waits only for the early path's gathers, vmcnt(stores)
#pragma unroll
            for (int it = 0; it < ITEMS; it++)
#pragma unroll
                for (int c = 0; c < COLS; c++) asm volatile("" ::"v"(rows[it][c]));
            __syncthreads();  // the main list region is dead
        }
        ti = tn;
        tn = tn2;
        b = bn;
    }
}

// ---------------------------------------------------------------------------
// group: pack the sub-buckets of every bucket into final groups
// ---------------------------------------------------------------------------
// one workgroup of 1024 threads per bucket a; thread t owns sub-buckets
// [t*SB, t*SB + SB): per-table sub-bucket totals and prefixes, then greedy
// packing into groups, written densely in key order: bucket a's groups start
// after the groups of buckets < a, whose counts each workgroup publishes as
// soon as it has them (a look-back over at most 255 words).
// grid (kBucketsA, kGroupSlices) x 256: partial sub-bucket totals of a slice
// of the bucket's pass-B tiles (thread t owns sub-buckets [8t, 8t + 8))

__global__ __launch_bounds__(256) void msd_group_sum_kernel(const MsdGroupParams p) {
    constexpr int SB = kRadB / 256;
    const int a = blockIdx.x, sl = blockIdx.y, t = threadIdx.x;
    if (sl == 0 && t == 0) p.ngrp[a] = 0;  // msd_group_kernel's publication word (previous call: flagged)
    for (int x = 0; x < p.ntab; x++) {
        uint32_t tot[SB];
#pragma unroll
        for (int i = 0; i < SB; i++) tot[i] = 0;
        const MsdBucket bk = p.bk[x][a];
        const uint32_t K = (bk.L + (uint32_t)p.tile[x] - 1) / (uint32_t)p.tile[x];
        const uint32_t k0 = (uint32_t)(((uint64_t)K * sl) / kGroupSlices), k1 = (uint32_t)(((uint64_t)K * (sl + 1)) / kGroupSlices);
        const uint16_t *o = p.offs[x] + (int64_t)bk.tile_base * kOffsB + t * SB;
        static_assert(SB == 8 && kOffsB % 8 == 0, "one 16-B load of 8 starts per row (rows 16-B aligned)");
        if (bk.one_key & 1u) {  // a heavy key's bucket: every row is in sub-bucket 0 (C5: thousands of tiles)
            if (sl == 0 && t == 0) tot[0] = bk.L;
        } else
#pragma unroll 4
        for (uint32_t k = k0; k < k1; k++) {
            const uint16_t *r = o + (int64_t)k * kOffsB;
            const uint4 q = *reinterpret_cast<const uint4 *>(r);
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
            uint32_t prev = w[0] & 0xffffu;
#pragma unroll
            for (int i = 0; i < SB; i++) {
                const uint32_t nx = i + 1 < SB ? (w[(i + 1) >> 1] >> (16 * ((i + 1) & 1))) & 0xffffu : (uint32_t)r[SB];
                tot[i] += nx - prev;
                prev = nx;
            }
        }
        uint32_t *dst = p.part + (((int64_t)x * kBucketsA + a) * kGroupSlices + sl) * kRadB + t * SB;
#pragma unroll
        for (int i = 0; i < SB; i++) dst[i] = tot[i];
    }
}

constexpr int kGroupThreads = 1024;
constexpr uint32_t kGrpReady = 0x80000000u;  // ngrp[a]: bucket a's group count is published
constexpr int kGroupLevels = 11;  // 2^11 = kRadB: binary-lifting levels over the group starts
static_assert((1 << kGroupLevels) == kRadB, "one level per bit of a group index");
// the segmented digit's interval of sub-bucket b (the last with db <= b)
__device__ __forceinline__ uint32_t seg_of(const MsdSeg &sg, uint32_t b) {
    uint32_t k = 0;
    for (uint32_t j = 1; j < sg.nseg; j++) k = seg_db(sg.pk[j]) <= b ? j : k;
    return k;
}
// the smallest key of sub-bucket b of a segmented digit (b = one past the
// last: hi + 1): interval k's linear sub-bucket j = b - db[k] <= dn[k] starts
// at st[k] + (ceil(j 2^32 / s32[k]) << sh[k]) (j = dn[k]: the gap sub-bucket,
// the first key past en[k])
__device__ __int128 seg_lower(const MsdSeg &sg, uint32_t b) {
    const uint32_t k = seg_of(sg, b), pk = sg.pk[k], j = b - seg_db(pk);
    if (j > seg_dn(pk)) return (__int128)sg.hi + 1;
    const uint64_t q = (((uint64_t)j << 32) + sg.s32[k] - 1u) / sg.s32[k];
    return (__int128)sg.st[k] + (__int128)((unsigned __int128)q << seg_sh(pk));
}

__global__ __launch_bounds__(kGroupThreads) void msd_group_kernel(const MsdGroupParams p) {
    constexpr int NW = kGroupThreads / 64, SB = kRadB / kGroupThreads;
    __shared__ uint32_t s_P[2][kRadB + 1];          // row prefix over sub-buckets, per table (P[kRadB] = total)
    __shared__ uint16_t s_lift[kGroupLevels][kRadB + 1];  // f^(2^k): next group start after a start
    __shared__ uint16_t s_nz[kRadB + 1];            // positions of the non-empty sub-buckets, in order
    __shared__ uint16_t s_cnz[kRadB + 1];           // non-empty sub-buckets before position q
    __shared__ uint32_t s_base;
    __shared__ uint32_t s_nl[2], s_lb[2];  // this bucket's single / oversized groups: count, then list base
    __shared__ uint32_t s_wsum[NW];
    __shared__ uint16_t s_g0[kRadB], s_g1[kRadB];   // groups: sub-buckets [b0, b1)
    __shared__ int s_ng, s_a;
    __shared__ int64_t s_hk[kHeavyMax];             // the bucket's heavy keys (ascending)
    __shared__ uint16_t s_hs[kHeavyMax], s_hl[kHeavyMax];  // heavy key j's sub-bucket, and its linear sub-bucket
    __shared__ MsdSeg s_sg;                         // the bucket's segmented digit (kBucketSeg)
    // The bucket is a ticket, not blockIdx.x: dispatch order (and which XCD
    // gets a workgroup when) is undefined, so a workgroup waiting on a lower
    // blockIdx could wait on one that is not resident yet -- and with other
    // processes' kernels filling that XCD (eight ranks sharing one GPU: the
    // r03za fault) on one that never becomes resident before the spin runs
    // out.  A ticket is taken by a running workgroup, so every bucket waited
    // on belongs to a workgroup that is already executing and waits only on
    // lower tickets itself: the look-back always completes.
    if (threadIdx.x == 0) s_a = (int)atomicAdd(&p.plan->gticket, 1u);
    __syncthreads();
    const int a = s_a, t = threadIdx.x;
    uint32_t nzmask = 0;  // thread t's sub-buckets [t*SB, t*SB + SB) that hold rows
    for (int x = 0; x < 2; x++) {
        uint32_t tot[SB];
#pragma unroll
        for (int i = 0; i < SB; i++) tot[i] = 0;
        if (x < p.ntab) {
            const uint32_t *src = p.part + ((int64_t)x * kBucketsA + a) * kGroupSlices * kRadB + t * SB;
#pragma unroll
            for (int sl = 0; sl < kGroupSlices; sl++)
#pragma unroll
                for (int i = 0; i < SB; i++) tot[i] += src[(int64_t)sl * kRadB + i];
        }
        uint32_t sum = 0;
#pragma unroll
        for (int i = 0; i < SB; i++) {
            sum += tot[i];
            nzmask |= tot[i] ? 1u << i : 0u;
        }
        uint32_t all;
        uint32_t ex = block_excl_scan<NW>(sum, s_wsum, &all);
#pragma unroll
        for (int i = 0; i < SB; i++) {
            s_P[x][t * SB + i] = ex;
            ex += tot[i];
        }
        if (t == 0) s_P[x][kRadB] = all;
    }
    // compact list of the non-empty sub-buckets
    {
        uint32_t all;
        uint32_t c = block_excl_scan<NW>((uint32_t)__popc(nzmask), s_wsum, &all);
#pragma unroll
        for (int i = 0; i < SB; i++) {
            s_cnz[t * SB + i] = (uint16_t)c;
            if ((nzmask >> i) & 1u) s_nz[c++] = (uint16_t)(t * SB + i);
        }
        if (t == 0) {
            s_cnz[kRadB] = (uint16_t)all;
            s_nz[all] = (uint16_t)kRadB;  // sentinel: "no further non-empty sub-bucket"
        }
    }
    __syncthreads();
    const bool single_sub = p.bk[0][a].scale == 0;  // every sub-bucket holds one key value
    const bool sgb = (p.bk[0][a].one_key & kBucketSeg) != 0u;  // a segmented digit (MsdSeg)
    if (sgb && t < 64) reinterpret_cast<uint32_t *>(&s_sg)[t] = reinterpret_cast<const uint32_t *>(p.seg + a)[t];
    // heavy keys (msd_heavy_kernel): heavy key j alone in sub-bucket
    // s_hs[j] = lin(h_j) + 2 j + 1 -- a group of its own, flagged single-key
    // (streamed in stable order); the others' linear sub-bucket of a digit d
    // is d - 2 #{heavy sub-buckets < d}
    const uint32_t hm = msd_heavy_count(p.bk[0][a].one_key);
    if ((uint32_t)t < hm) {
        const MsdBucket &bb = p.bk[0][a];
        const int64_t h = p.heavy[(int64_t)a * kHeavyMax + t];
        const uint32_t l = pb_lin(bb, (uint64_t)h - (uint64_t)bb.lo);
        s_hk[t] = h;
        s_hl[t] = (uint16_t)l;
        s_hs[t] = (uint16_t)(l + 2u * (uint32_t)t + 1u);
    }
    __syncthreads();
    // heavy sub-buckets below d, and whether d is one
    auto heavy_below = [&](uint32_t d, bool &is) -> uint32_t {
        uint32_t pos = 0;
#pragma unroll
        for (uint32_t st = kHeavyMax; st >= 1; st >>= 1)
            if (pos + st <= hm && s_hs[pos + st - 1] < d) pos += st;
        is = pos < hm && s_hs[pos] == d;
        return pos;
    };
    // a group spans < 2^48 key values, so that (residual << idx | index) fits one
    // word in the final kernel's LDS sort
    const int maxspan = (int)p.bk[0][a].maxspan;
    // Combined packing (2-column tables, round 3): a group holds up to
    // kStRows rows of both tables together when every group of the bucket is
    // sure to fit the staged final kernel -- sub-buckets of <= kStageRange keys
    // (then maxspan keeps a group's span within the counting range) and <=
    // kStList pass-B tiles per table; elsewhere <= kGroupCap rows per table.
    bool comb = p.combined != 0;
    {
        const MsdBucket &b0 = p.bk[0][a];
        const uint64_t w = b0.scale == 0 ? 1ull
                           : b0.s32      ? ((1ull << 32) + b0.s32 - 1u) / b0.s32 + 1u
                                         : (uint64_t)((((unsigned __int128)1 << 64) + b0.scale - 1u) / b0.scale) + 1u;
        comb = comb && w * (uint64_t)b0.maxspan <= (uint64_t)kStageRange;  // (msd_bases: not a wide bucket)
        comb = comb && !sgb;  // (its gap sub-buckets span wide)
        for (int x = 0; x < p.ntab; x++)
            comb = comb && (p.bk[x][a].L + (uint32_t)p.tile[x] - 1) / (uint32_t)p.tile[x] <= (uint32_t)kStList;
    }
    // The greedy packing (a group takes consecutive non-empty sub-buckets while
    // both tables stay <= kGroupCap rows and the sub-bucket span < maxspan; a
    // sub-bucket over the cap is a group of its own), computed in parallel:
    // from a group start i the next start is f(i) = the first non-empty j > i
    // at which the R or S rows of [i, j] exceed the cap or j - i >= maxspan.
    // The starts are the orbit of the first non-empty sub-bucket under f;
    // binary lifting (f^(2^k)) gives start number s to every thread at once.
    auto next_nz = [&](int q) -> int { return q >= kRadB ? kRadB : (int)s_nz[s_cnz[q]]; };
    for (int i = t; i <= kRadB; i += kGroupThreads) {
        int f = kRadB;
        if (i < kRadB) {
            int lim = min(kRadB, i + maxspan);
            if (comb) {  // first m in [i + 2, kRadB] with the rows of both tables in [i, m) over kStRows
                const uint32_t cap = s_P[0][i] + s_P[1][i] + (uint32_t)kStRows;
                int lo = i + 2, hi = kRadB + 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (s_P[0][mid] + s_P[1][mid] > cap) hi = mid; else lo = mid + 1;
                }
                if (lo <= kRadB) lim = min(lim, lo - 1);
                else if (i + 1 <= kRadB && s_P[0][i + 1] + s_P[1][i + 1] > cap) lim = min(lim, i + 1);
            } else {
#pragma unroll
                for (int x = 0; x < 2; x++) {  // first m in [i + 2, kRadB] with P[m] - P[i] > cap: j = m - 1
                    const uint32_t cap = s_P[x][i] + (uint32_t)kGroupCap;
                    int lo = i + 2, hi = kRadB + 1;  // answer in [lo, hi); hi = none
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (s_P[x][mid] > cap) hi = mid; else lo = mid + 1;
                    }
                    if (lo <= kRadB) lim = min(lim, lo - 1);
                    else if (i + 1 <= kRadB && s_P[x][i + 1] > cap) lim = min(lim, i + 1);
                }
            }
            if (hm) {  // a heavy sub-bucket is a group of its own: stop before the next one
                bool is;
                const uint32_t c = heavy_below((uint32_t)i, is);
                if (is) lim = i + 1;
                else if (c < hm) lim = min(lim, (int)s_hs[c]);
            }
            if (sgb) {  // a group stays inside one interval's linear sub-buckets; a gap sub-bucket is its own
                const uint32_t k = seg_of(s_sg, (uint32_t)i), d0 = seg_db(s_sg.pk[k]), dn = seg_dn(s_sg.pk[k]);
                lim = (uint32_t)i >= d0 + dn ? i + 1 : min(lim, min(i + (int)s_sg.ms[k], (int)(d0 + dn)));
            }
            f = next_nz(max(lim, i + 1));
        }
        s_lift[0][i] = (uint16_t)f;
    }
    __syncthreads();
    for (int k = 1; k < kGroupLevels; k++) {
        for (int i = t; i <= kRadB; i += kGroupThreads) s_lift[k][i] = s_lift[k - 1][s_lift[k - 1][i]];
        __syncthreads();
    }
    const int s0 = next_nz(0);
    int ng_local = 0;
    for (int sidx = t; sidx < kRadB; sidx += kGroupThreads) {
        int pos = s0;
#pragma unroll
        for (int k = 0; k < kGroupLevels; k++)
            if ((sidx >> k) & 1) pos = s_lift[k][pos];
        if (pos < kRadB) {
            const int nxt = s_lift[0][pos];
            s_g0[sidx] = (uint16_t)pos;
            s_g1[sidx] = (uint16_t)(s_nz[s_cnz[nxt] - 1] + 1);  // after the last non-empty sub-bucket before nxt
            ng_local = max(ng_local, sidx + 1);
        }
    }
    {
        int m = ng_local;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
        if ((t & 63) == 0) s_wsum[t >> 6] = (uint32_t)m;
    }
    __syncthreads();
    if (t == 0) {
        int ng = 0;
        for (int w = 0; w < NW; w++) ng = max(ng, (int)s_wsum[w]);
        s_ng = ng;
        // publish this bucket's group count (msd_group_sum zeroed the word):
        // the later buckets add it to their dense base
        atomicExch(&p.ngrp[a], (uint32_t)ng | kGrpReady);
    }
    // dense base = the group counts of buckets < a, as they are published
    // (by workgroups already executing: the bucket tickets above).  Relaxed
    // atomics: nothing else this kernel writes is read back in it.
    {
        uint32_t v = 0;
        if (t < a) {
            // bounded, so the grid always drains: on exhaustion the plan's error
            // word is set, every later kernel of the call returns at entry
            // (msd_plan_failed) and msd_run returns SMJ_ERR_TIMEOUT
            uint32_t spin = 0;
            for (; spin < p.spin_limit; spin++) {
                v = __hip_atomic_load(&p.ngrp[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v & kGrpReady) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (!(v & kGrpReady)) atomicOr(&p.plan->err, 1u);
            v &= ~kGrpReady;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        __syncthreads();  // s_wsum read out above
        if ((t & 63) == 0) s_wsum[t >> 6] = v;
        __syncthreads();
        if (t == 0) {
            uint32_t base = 0;
            for (int w = 0; w < NW; w++) base += s_wsum[w];
            s_base = base;
            if (a == kBucketsA - 1) p.plan->ngroups = base + s_ng;
        }
        __syncthreads();
    }
    const uint32_t base = s_base;
    // the streamed / oversized lists: slots counted in LDS, one global
    // reservation per list and bucket (C5: ~10^4 flagged groups per call --
    // one global atomic each serialised on one L2 address, 0.13 ms per launch)
    if (t < 2) s_nl[t] = 0;
    __syncthreads();
    constexpr int GPT = kRadB / kGroupThreads;  // groups per thread (j = t + i * kGroupThreads)
    uint32_t lslot[GPT], lgi[GPT], lkind[GPT];
#pragma unroll
    for (int i = 0; i < GPT; i++) lkind[i] = 0;
    for (int j = t, i = 0; j < s_ng; j += kGroupThreads, i++) {
        const uint32_t b0 = s_g0[j], b1 = s_g1[j];
        MsdGroup gr{};
        gr.a = (uint16_t)a;
        gr.b0 = (uint16_t)b0;
        gr.b1 = (uint16_t)b1;
        gr.nR = s_P[0][b1] - s_P[0][b0];
        gr.nS = s_P[1][b1] - s_P[1][b0];
        gr.outR = p.bk[0][a].row_start + s_P[0][b0];
        gr.outS = p.ntab > 1 ? p.bk[1][a].row_start + s_P[1][b0] : 0u;
        gr.flags = 0;
        bool hv_only = false;  // the group is one heavy key's sub-bucket
        uint32_t hj = 0;
        if (hm && b1 == b0 + 1) hj = heavy_below(b0, hv_only);
        if (hv_only) {  // one key: the staged kernel's no-sort path when it fits a combined group, else streamed
            gr.flags = comb && gr.nR + gr.nS <= (uint32_t)kStRows ? (uint16_t)0 : kGroupSingle;
            gr.pad[0] = 1;  // one sub-bucket of a multi-key bucket: msd_single copies it run by run
        }
        else if (comb ? gr.nR + gr.nS > (uint32_t)kStRows : (gr.nR > (uint32_t)kGroupCap || gr.nS > (uint32_t)kGroupCap))
            gr.flags = single_sub ? kGroupSingle : kGroupBig;
#pragma unroll
        for (int x = 0; x < 2; x++) {
            gr.tb[x] = x < p.ntab ? p.bk[x][a].tile_base : 0u;
            gr.kt[x] = x < p.ntab ? (p.bk[x][a].L + (uint32_t)p.tile[x] - 1) / (uint32_t)p.tile[x] : 0u;
        }
        // key interval of sub-buckets [b0, b1): residuals r = key - lo with
        // digit(r) = floor(r * scale / 2^64) in [b0, b1) satisfy rmin(b0) <= r < rmin(b1),
        // rmin(b) = ceil(b * 2^64 / scale) (2^32 and s32 for a 32-bit digit);
        // with scale == 0 the digit is r itself
        // (with heavy keys: over the linear sub-buckets [lin(b0), lin(b1 - 1) + 1)
        // -- a superset of the group's keys -- and a heavy key's group is the key)
        const uint64_t sc = p.bk[0][a].scale;
        const uint32_t s32 = p.bk[0][a].s32;
        uint32_t l0 = b0, l1 = b1;
        if (hm) {
            bool is;
            uint32_t c = heavy_below(b0, is);
            l0 = is ? (uint32_t)s_hl[c] : b0 - 2u * c;
            c = heavy_below(b1 - 1u, is);
            l1 = (is ? (uint32_t)s_hl[c] : b1 - 1u - 2u * c) + 1u;
        }
        unsigned __int128 r0 = l0, r1 = l1;
        if (sgb) {  // the segmented digit: offsets from lo
            r0 = seg_lower(s_sg, b0) - (__int128)p.bk[0][a].lo;
            r1 = seg_lower(s_sg, b1) - (__int128)p.bk[0][a].lo;
        } else if (s32) {
            r0 = (((uint64_t)l0 << 32) + s32 - 1u) / s32;
            r1 = (((uint64_t)l1 << 32) + s32 - 1u) / s32;
        } else if (sc) {
            r0 = (((unsigned __int128)l0 << 64) + sc - 1) / sc;
            r1 = (((unsigned __int128)l1 << 64) + sc - 1) / sc;
        }
        gr.base = (int64_t)((uint64_t)p.bk[0][a].lo + (uint64_t)r0);
        const unsigned __int128 sp = r1 - r0;
        gr.span = sp > 0xffffffffu ? 0xffffffffu : (uint32_t)sp;
        if (sp > (unsigned __int128)kStageRange) {
            // a wide group (msd_final_wstage_kernel): its kStageRange bins are
            // bin(key) = mulhi64(key - base, bscale) < kStageRange over the interval
            const uint64_t bs = (uint64_t)(((unsigned __int128)kStageRange << 64) / sp);
            gr.pad[1] = (uint32_t)bs;
            gr.pad[2] = (uint32_t)(bs >> 32);
        }
        if (hv_only) {
            gr.base = s_hk[hj];
            gr.span = 1;
        }
        // dense, key-ordered index; the streamed / oversized lists
        const uint32_t gi = base + (uint32_t)j;
        if (gi >= (uint32_t)kSlots) {  // the group array's capacity (a wrong base: never stored past it)
            atomicOr(&p.plan->err, 8u);
            continue;
        }
        p.groups[gi] = gr;
        uint32_t cnt = 0;
        if (gr.flags == kGroupSingle) {
            cnt = min(gr.nR, gr.nS);
            lkind[i] = 1;
            lslot[i] = atomicAdd(&s_nl[0], 1u);
            lgi[i] = gi;
        } else if (gr.flags == kGroupBig) {
            lkind[i] = 2;
            lslot[i] = atomicAdd(&s_nl[1], 1u);
            lgi[i] = gi;
        }
        p.counts[gi] = cnt;
    }
    __syncthreads();
    if (t < 2) s_lb[t] = s_nl[t] ? atomicAdd(t ? &p.plan->nbig : &p.plan->nsingle, s_nl[t]) : 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < GPT; i++) {
        if (lkind[i] == 1) p.single_list[s_lb[0] + lslot[i]] = lgi[i];
        if (lkind[i] == 2) p.big_list[s_lb[1] + lslot[i]] = lgi[i];
    }
}

// ---------------------------------------------------------------------------
// gather of a group's rows through the pass-B tiles of its bucket
// ---------------------------------------------------------------------------
// The group's rows of table x are, in input order, the ranges
// [offsB[id][b0], offsB[id][b1]) of the bucket's pass-B tiles id.  Rows
// [V0, V1) of that sequence are visited: fn(v, src_row) for each, src_row
// indexing tempB.  s_list holds kGroupCap uint2 entries; batches of ranges.
template <class Fn>
__device__ __forceinline__ void group_gather(const MsdTab &tb, const MsdGroup &g, uint32_t V0, uint32_t V1,
                                             uint2 *s_list, uint32_t *s_wsum, Fn fn) {
    const int tid = threadIdx.x;
    const MsdBucket bk = tb.bk[g.a];
    const uint32_t K = (bk.L + (uint32_t)tb.tile - 1) / (uint32_t)tb.tile;
    if ((bk.one_key & 1u) && g.b0 == 0) {  // single-key bucket: its tiles are full and hold only sub-bucket 0
        const uint32_t base = bk.tile_base * (uint32_t)tb.tile;
        for (uint32_t v = V0 + tid; v < V1; v += kMsdThreads) fn(v, base + v);
        return;
    }
    constexpr int PER = kGroupCap / kMsdThreads;
    uint32_t carry = 0;
    for (uint32_t kb = 0; kb < K && carry < V1; kb += kGroupCap) {
        const uint32_t nb = min(K - kb, (uint32_t)kGroupCap);
        uint32_t src[PER], len[PER], sum = 0;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint32_t jj = (uint32_t)tid * PER + i;
            src[i] = len[i] = 0;
            if (jj < nb) {
                const int64_t id = (int64_t)bk.tile_base + kb + jj;
                const uint32_t lo = tb.offs[id * kOffsB + g.b0], hi = tb.offs[id * kOffsB + g.b1];
                src[i] = (uint32_t)id * (uint32_t)tb.tile + lo;
                len[i] = hi - lo;
            }
            sum += len[i];
        }
        uint32_t total;
        uint32_t ex = carry + block_excl_scan<kMsdWaves>(sum, s_wsum, &total);
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint32_t jj = (uint32_t)tid * PER + i;
            if (jj < nb) s_list[jj] = make_uint2(src[i], ex);
            ex += len[i];
        }
        __syncthreads();
        const uint32_t b0 = max(carry, V0), b1 = min(carry + total, V1);
        for (uint32_t v = b0 + tid; v < b1; v += kMsdThreads) {
            int lo = 0, hi = (int)nb - 1;  // last range starting at or before v (empty ranges skipped)
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_list[mid].y <= v) lo = mid; else hi = mid - 1;
            }
            const uint2 e = s_list[lo];
            fn(v, e.x + (v - e.y));
        }
        carry += total;
        __syncthreads();
    }
}

template <int C>
__device__ __forceinline__ void copy_row(const int64_t *__restrict__ src, int64_t *__restrict__ dst, int cols) {
    if constexpr (C > 0) {
        int64_t r[C];
        load_row<C>(src, r);
        store_row<C>(dst, r);
    } else {
        for (int c = 0; c < cols; c++) dst[c] = src[c];
    }
}

// one join row: R row r (c1 words) then S row s without column key2
template <int C1, int C2>
__device__ __forceinline__ void emit_join_row(const int64_t *__restrict__ r, const int64_t *__restrict__ s,
                                              int64_t *__restrict__ dst, int c1, int c2, int key2) {
    if constexpr (C1 == 2 && C2 == 2) {
        const i64x2 rv = *reinterpret_cast<const i64x2 *>(r);
        const i64x2 sv = *reinterpret_cast<const i64x2 *>(s);
        dst[0] = rv.x;
        dst[1] = rv.y;
        dst[2] = key2 ? sv.x : sv.y;
    } else {
        for (int c = 0; c < c1; c++) dst[c] = r[c];
        for (int c = 0, o = c1; c < c2; c++)
            if (c != key2) dst[o++] = s[c];
    }
}

// ---------------------------------------------------------------------------
// LDS radix pass over packed (residual << 16 | index) words, one table of a
// group: stable, by the 8-bit digit at `shift`.  n <= kGroupCap.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lds_radix_pass(const uint64_t *src, uint64_t *dst, int n, int shift,
                                               uint32_t *s_cnt, uint32_t *s_bin, uint32_t *s_wsum) {
    constexpr int IT = kGroupCap / kMsdThreads;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *wc = s_cnt + wave * 256;
    zero_counters<256>(wc, lane);
    uint64_t val[IT];
    uint32_t dig[IT], vmask = 0;
#pragma unroll
    for (int it = 0; it < IT; it++) {
        const int e = (wave * IT + it) * 64 + lane;
        const bool v = e < n;
        val[it] = v ? src[e] : 0ull;
        dig[it] = (uint32_t)(val[it] >> shift) & 255u;
        vmask |= v ? (1u << it) : 0u;
    }
    wave_rank<IT, 8>(dig, vmask, wc, lane);
    __syncthreads();
    tile_digit_starts<256>(s_cnt, s_bin, s_wsum);
#pragma unroll
    for (int it = 0; it < IT; it++) {
        if ((vmask >> it) & 1u) {
            const uint32_t d = dig[it] & 0xffffu;
            dst[s_bin[d] + wc[d] + (dig[it] >> 16)] = val[it];
        }
    }
    __syncthreads();
}

// first index in a[0, n) with a[i] >= k
__device__ __forceinline__ int lds_lb_u64(const uint64_t *a, int n, uint64_t k) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------
// final: per group, LDS sort of R and S, sorted rows out, zip join into slots
// ---------------------------------------------------------------------------
struct FinalSmem {
    uint64_t key[2][kGroupCap];   // raw key, then packed (residual << 16 | index), sorted
    uint32_t addr[2][kGroupCap];  // tempB row of group row v
    uint64_t tmp[kGroupCap];      // radix ping-pong / gather run list
    uint32_t cnt[kMsdWaves * 256];
    uint32_t bin[257];
    uint32_t wsum[kMsdWaves];
    int64_t mm[2 * kMsdWaves];
};

// one group; every early return is uniform over the workgroup
template <int C1, int C2>
__device__ __forceinline__ void final_group(const MsdFinalParams &p, const int64_t slot, FinalSmem &sm) {
    auto &s_key = sm.key;
    auto &s_addr = sm.addr;
    uint64_t *s_tmp = sm.tmp;
    uint32_t *s_cnt = sm.cnt, *s_bin = sm.bin, *s_wsum = sm.wsum;
    int64_t *s_mm = sm.mm;
    const MsdGroup g = p.groups[slot];
    if (g.flags) return;  // single-key / oversized groups are handled elsewhere
    const int tid = threadIdx.x;
    const int n[2] = {(int)g.nR, p.ntab > 1 ? (int)g.nS : 0};
    uint2 *s_list = reinterpret_cast<uint2 *>(s_tmp);

    // gather the keys (the rows' lines come in with them: L2-warm for later)
    int64_t mn = INT64_MAX, mx = INT64_MIN;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        if (n[x] == 0) continue;
        const MsdTab &tb = p.tab[x];
        const int cols = C1 > 0 ? (x ? C2 : C1) : tb.cols;
        group_gather(tb, g, 0u, (uint32_t)n[x], s_list, s_wsum, [&](uint32_t v, uint32_t src) {
            const int64_t k = tb.tempB[(int64_t)src * cols + tb.key];
            s_key[x][v] = (uint64_t)k;
            s_addr[x][v] = src;
            mn = min(mn, k);
            mx = max(mx, k);
        });
    }
    block_minmax<kMsdWaves>(mn, mx, s_mm);
    const uint64_t range = (uint64_t)mx - (uint64_t)mn;
    const int bits = range ? 64 - __clzll((long long)range) : 0;
    if (bits > 48) {  // residual + index do not fit one word: LSD fallback on the host side
        if (tid == 0) {
            const uint32_t idx = atomicAdd(&p.plan->nbig, 1u);
            p.big_list[idx] = (uint32_t)slot;
        }
        return;
    }
#pragma unroll
    for (int x = 0; x < 2; x++)
        for (int v = tid; v < n[x]; v += kMsdThreads)
            s_key[x][v] = (((uint64_t)s_key[x][v] - (uint64_t)mn) << 16) | (uint64_t)v;
    __syncthreads();
    const int npass = (bits + 7) >> 3;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        if (n[x] == 0) continue;
        for (int ps = 0; ps < npass; ps++) {
            const bool fwd = (ps & 1) == 0;
            lds_radix_pass(fwd ? s_key[x] : s_tmp, fwd ? s_tmp : s_key[x], n[x], 16 + 8 * ps, s_cnt, s_bin, s_wsum);
        }
        if (npass & 1) {
            for (int v = tid; v < n[x]; v += kMsdThreads) s_key[x][v] = s_tmp[v];
            __syncthreads();
        }
    }
    // sorted rows to their final places
#pragma unroll
    for (int x = 0; x < 2; x++) {
        if (n[x] == 0) continue;
        const MsdTab &tb = p.tab[x];
        const int cols = C1 > 0 ? (x ? C2 : C1) : tb.cols;
        int64_t *dst = tb.out + (int64_t)(x ? g.outS : g.outR) * cols;
        for (int v = tid; v < n[x]; v += kMsdThreads) {
            const uint32_t src = s_addr[x][s_key[x][v] & 0xffffu];
            if constexpr (C1 > 0) {
                if (x) copy_row<C2>(tb.tempB + (int64_t)src * C2, dst + (int64_t)v * C2, C2);
                else copy_row<C1>(tb.tempB + (int64_t)src * C1, dst + (int64_t)v * C1, C1);
            } else {
                copy_row<0>(tb.tempB + (int64_t)src * cols, dst + (int64_t)v * cols, cols);
            }
        }
    }
    if (!p.join) return;
    // zip join: R position i pairs with S position lbS(k) + (i - lbR(k))
    constexpr int PER = kGroupCap / kMsdThreads;
    const int nR = n[0], nS = n[1];
    uint32_t part[PER], mmask = 0;
    if (nS > 0) {
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int i = tid * PER + q;
            part[q] = 0;
            if (i < nR) {
                const uint64_t k = s_key[0][i] >> 16;
                const int lbR = lds_lb_u64(s_key[0], i + 1, k << 16);
                const int lbS = lds_lb_u64(s_key[1], nS, k << 16);
                const int j = lbS + (i - lbR);
                if (j < nS && (s_key[1][j] >> 16) == k) {
                    part[q] = (uint32_t)j;
                    mmask |= 1u << q;
                }
            }
        }
    }
    uint32_t total;
    uint32_t o = block_excl_scan<kMsdWaves>((uint32_t)__popc(mmask), s_wsum, &total);
    if (tid == 0) p.counts[slot] = total;
    if (total == 0) return;
    const int c1 = C1 > 0 ? C1 : p.tab[0].cols, c2 = C2 > 0 ? C2 : p.tab[1].cols, tc = c1 + c2 - 1;
    int64_t *dst = p.slots + (int64_t)g.outR * tc;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        if ((mmask >> q) & 1u) {
            const int i = tid * PER + q;
            const uint32_t ra = s_addr[0][s_key[0][i] & 0xffffu];
            const uint32_t sa = s_addr[1][s_key[1][part[q]] & 0xffffu];
            emit_join_row<C1, C2>(p.tab[0].tempB + (int64_t)ra * c1, p.tab[1].tempB + (int64_t)sa * c2,
                                  dst + (int64_t)o * tc, c1, c2, p.key2);
            o++;
        }
    }
}

// ---- fast path ---------------------------------------------------------------
// A group whose key range fits 21 bits (residual << 11 | row fits one 32-bit
// sort word) and whose buckets have <= kFinThreads pass-B tiles per table is
// sorted with 32-bit words, both tables ranked in the same LSD passes (four
// barriers per pass), and software-pipelined one group deep: while group i
// is written out and joined, the key gathers of group i + 1 are in flight.
// Every other group goes to the wide list (msd_final_wide_kernel).
constexpr int kFinIt = kGroupCap / kFinThreads;  // rows per table per thread
constexpr int kFinIdxBits = 10;
constexpr int kFinResBits = 32 - kFinIdxBits;     // 22-bit key residuals
static_assert(kGroupCap == (1 << kFinIdxBits), "sort word = residual << 10 | group row");

constexpr int kCountRange = 4096;  // counting-sort residual range (packed u16 bins)
constexpr int kMaxDupRun = 32;     // longest equal-key run the counting path re-orders
#ifndef SMJ_ST_MAXRUN
#define SMJ_ST_MAXRUN kMaxDupRun  // the staged kernel: longer runs take the in-LDS LSD (<= kMaxDupRun)
#endif

struct FinSmem {
    uint32_t key[2][kGroupCap];   // sort words, sorted in place (via tmp)
    uint32_t addr[2][kGroupCap];  // tempB row of group row v
    union {
        struct {
            uint32_t tmp[2][kGroupCap];  // radix ping-pong; the next group's run lists (uint2[2][kFinThreads])
            uint32_t cnt[2][kFinWaves][256];
        };
        uint32_t hist[2][kCountRange / 2];  // counting sort: two u16 bins per word
    };
    uint32_t bin[2][256];
    uint32_t wsum[2][kFinWaves];  // double-buffered block-scan wave sums
    uint32_t flag[2];
    int64_t mm[2 * kFinWaves];
};

// exclusive block scan without the trailing barrier: callers alternate wsum
// buffers so that the next scan cannot overwrite sums still being read

struct FinalPref {               // the group whose keys are in flight
    uint32_t o0[2], o1[2];       // offsB[tile][b0], offsB[tile][b1] of this thread's tile
    int64_t key[2][kFinIt];      // gathered keys (row v = tid + k * kFinThreads)
    uint32_t src[2][kFinIt];     // their tempB rows
};

__device__ __forceinline__ uint32_t fin_tiles(const MsdTab &tb, uint16_t a) {
    const uint32_t L = tb.bk[a].L;
    return (L + (uint32_t)tb.tile - 1) / (uint32_t)tb.tile;
}

__device__ __forceinline__ bool fin_fast(const MsdFinalParams &p, const MsdGroup &g) {
    return fin_tiles(p.tab[0], g.a) <= (uint32_t)kFinThreads &&
           (p.ntab < 2 || fin_tiles(p.tab[1], g.a) <= (uint32_t)kFinThreads);
}

__device__ __forceinline__ void fin_load_offs(const MsdFinalParams &p, const MsdGroup &g, uint32_t (&o0)[2],
                                              uint32_t (&o1)[2]) {
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        o0[x] = o1[x] = 0;
        if (x < p.ntab && tid < fin_tiles(p.tab[x], g.a)) {
            const int64_t id = (int64_t)p.tab[x].bk[g.a].tile_base + tid;
            o0[x] = p.tab[x].offs[id * kOffsB + g.b0];
            o1[x] = p.tab[x].offs[id * kOffsB + g.b1];
        }
    }
}

// run lists of group g from its offsB values (into sm.tmp), then the key
// gathers of its rows (fixed-step searches, interleaved over the rows)
template <int C1, int C2>
__device__ __forceinline__ void fin_issue_keys(const MsdFinalParams &p, const MsdGroup &g, FinalPref &f,
                                               FinSmem &sm, int &wsb) {
    const uint32_t tid = threadIdx.x;
    uint2 *s_list = reinterpret_cast<uint2 *>(&sm.tmp[0][0]);  // [x * kFinThreads + tile]
    const uint32_t lenR = f.o1[0] - f.o0[0], lenS = f.o1[1] - f.o0[1];
    uint32_t tot;
    const uint32_t ex = block_excl_scan_nb<kFinWaves>(lenR | (lenS << 16), sm.wsum[wsb], &tot);  // halves <= kGroupCap
    wsb ^= 1;
    uint32_t K[2];
#pragma unroll
    for (int x = 0; x < 2; x++) {
        K[x] = x < p.ntab ? fin_tiles(p.tab[x], g.a) : 0u;
        if (tid < K[x]) {
            const uint32_t id = p.tab[x].bk[g.a].tile_base + tid;
            s_list[x * kFinThreads + tid] =
                make_uint2(id * (uint32_t)p.tab[x].tile + f.o0[x], x ? (ex >> 16) : (ex & 0xffffu));
        }
    }
    __syncthreads();
    const uint32_t n[2] = {g.nR, p.ntab > 1 ? g.nS : 0u};
    uint32_t pos[2][kFinIt];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int k = 0; k < kFinIt; k++) pos[x][k] = 0;
#pragma unroll
    for (int step = kFinThreads / 2; step >= 1; step >>= 1) {  // last range starting at or before v
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int k = 0; k < kFinIt; k++) {
                const uint32_t v = tid + k * kFinThreads, q = pos[x][k] + step;
                if (q < K[x] && s_list[x * kFinThreads + q].y <= v) pos[x][k] = q;
            }
    }
#pragma unroll
    for (int x = 0; x < 2; x++) {
        const MsdTab &tb = p.tab[x];
        const int cols = C1 > 0 ? (x ? C2 : C1) : tb.cols;
#pragma unroll
        for (int k = 0; k < kFinIt; k++) {
            const uint32_t v = tid + k * kFinThreads;
            const uint2 e = s_list[x * kFinThreads + pos[x][k]];
            const uint32_t src = e.x + (v - e.y);
            f.src[x][k] = src;
            f.key[x][k] = v < n[x] ? tb.tempB[(int64_t)src * cols + tb.key] : 0;
        }
    }
}

// one stable LSD pass over both tables' sort words by the 8-bit digit at shift
__device__ __forceinline__ void fin_radix_pass(const uint32_t (*src)[kGroupCap], uint32_t (*dst)[kGroupCap],
                                               const int (&n)[2], int shift, FinSmem &sm, int &wsb) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t val[2][kFinIt], dig[2][kFinIt], vm[2];
#pragma unroll
    for (int x = 0; x < 2; x++) {
        uint32_t *wc = sm.cnt[x][wave];
        zero_counters<256>(wc, lane);
        vm[x] = 0;
#pragma unroll
        for (int it = 0; it < kFinIt; it++) {
            const int e = (wave * kFinIt + it) * 64 + lane;
            const bool v = e < n[x];
            val[x][it] = v ? src[x][e] : 0u;
            dig[x][it] = (val[x][it] >> shift) & 255u;
            vm[x] |= v ? (1u << it) : 0u;
        }
        wave_rank<kFinIt, 8>(dig[x], vm[x], wc, lane);
    }
    __syncthreads();
    uint32_t packed = 0;
    if (tid < 256) {
#pragma unroll
        for (int x = 0; x < 2; x++) {
            uint32_t c[kFinWaves];
#pragma unroll
            for (int w = 0; w < kFinWaves; w++) c[w] = sm.cnt[x][w][tid];
            uint32_t t = 0;
#pragma unroll
            for (int w = 0; w < kFinWaves; w++) {
                sm.cnt[x][w][tid] = t;
                t += c[w];
            }
            packed |= t << (16 * x);
        }
    }
    uint32_t all;
    const uint32_t ex = block_excl_scan_nb<kFinWaves>(packed, sm.wsum[wsb], &all);
    wsb ^= 1;
    if (tid < 256) {
        sm.bin[0][tid] = ex & 0xffffu;
        sm.bin[1][tid] = ex >> 16;
    }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int it = 0; it < kFinIt; it++)
            if ((vm[x] >> it) & 1u) {
                const uint32_t d = dig[x][it] & 0xffffu;
                dst[x][sm.bin[x][d] + sm.cnt[x][wave][d] + (dig[x][it] >> 16)] = val[x][it];
            }
    __syncthreads();
}

// Counting sort of both tables' sort words (residual < kCountRange): packed
// u16 histograms (LDS atomics), one block scan for both tables, scatter, and
// a re-ordering of equal-residual runs by group row (atomics place them in
// arbitrary order).  False (nothing written) when a residual repeats more
// than kMaxDupRun times: the radix path then sorts the group.
__device__ __forceinline__ bool fin_count_sort(const uint32_t (&w)[2][kFinIt], const int (&n)[2], FinSmem &sm,
                                               int &wsb) {
    const int tid = threadIdx.x;
    uint4 *h4 = reinterpret_cast<uint4 *>(&sm.hist[0][0]);
    for (int i = tid; i < kCountRange / 4; i += kFinThreads) h4[i] = make_uint4(0, 0, 0, 0);
    if (tid == 0) sm.flag[wsb] = 0;
    __syncthreads();
    uint32_t rank[2][kFinIt];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int k = 0; k < kFinIt; k++) {
            rank[x][k] = 0;
            if (w[x][k] != ~0u) {
                const uint32_t res = w[x][k] >> kFinIdxBits, sh = 16u * (res & 1u);
                rank[x][k] = (atomicAdd(&sm.hist[x][res >> 1], 1u << sh) >> sh) & 0xffffu;
            }
        }
    __syncthreads();
    // exclusive starts: thread t owns words [t*W, t*W + W) of each table's histogram
    constexpr int W = kCountRange / 2 / kFinThreads;
    uint32_t tot = 0, heavy = 0;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t h = sm.hist[x][tid * W + i];
            heavy |= ((h & 0xffffu) > (uint32_t)kMaxDupRun) | ((h >> 16) > (uint32_t)kMaxDupRun);
            t += (h & 0xffffu) + (h >> 16);
        }
        tot |= t << (16 * x);
    }
    if (heavy) sm.flag[wsb] = 1;
    uint32_t all;
    const uint32_t ex = block_excl_scan_nb<kFinWaves>(tot, sm.wsum[wsb], &all);  // its barrier publishes flag[wsb]
    const bool bail = sm.flag[wsb] != 0;
    wsb ^= 1;
    if (bail) {
        __syncthreads();  // everyone read the flag before the radix path reuses the region
        return false;
    }
#pragma unroll
    for (int x = 0; x < 2; x++) {
        uint32_t run = x ? (ex >> 16) : (ex & 0xffffu);
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t h = sm.hist[x][tid * W + i];
            sm.hist[x][tid * W + i] = run | ((run + (h & 0xffffu)) << 16);
            run += (h & 0xffffu) + (h >> 16);
        }
    }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int k = 0; k < kFinIt; k++)
            if (w[x][k] != ~0u) {
                const uint32_t res = w[x][k] >> kFinIdxBits, sh = 16u * (res & 1u);
                sm.key[x][((sm.hist[x][res >> 1] >> sh) & 0xffffu) + rank[x][k]] = w[x][k];
            }
    __syncthreads();
    // runs of one residual: insertion sort by word (= by group row), <= kMaxDupRun long
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int k = 0; k < kFinIt; k++) {
            const int q = tid * kFinIt + k;
            if (q + 1 < n[x]) {
                const uint32_t rq = sm.key[x][q] >> kFinIdxBits;
                if ((sm.key[x][q + 1] >> kFinIdxBits) == rq && (q == 0 || (sm.key[x][q - 1] >> kFinIdxBits) != rq)) {
                    int e = q + 1;
                    while (e < n[x] && (sm.key[x][e] >> kFinIdxBits) == rq) e++;
                    for (int a = q + 1; a < e; a++) {
                        const uint32_t v = sm.key[x][a];
                        int b = a - 1;
                        while (b >= q && sm.key[x][b] > v) {
                            sm.key[x][b + 1] = sm.key[x][b];
                            b--;
                        }
                        sm.key[x][b + 1] = v;
                    }
                }
            }
        }
    __syncthreads();
    return true;
}

// sort a group whose keys are in f; false when its key range is wider than
// 21 bits (the group then goes to the wide list)
__device__ __forceinline__ bool fin_sort(const MsdFinalParams &p, const MsdGroup &g, int64_t gi, const FinalPref &f,
                                         FinSmem &sm, int &wsb) {
    const int tid = threadIdx.x;
    const int n[2] = {(int)g.nR, p.ntab > 1 ? (int)g.nS : 0};
    int64_t mn = INT64_MAX, mx = INT64_MIN;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int k = 0; k < kFinIt; k++) {
            const int v = tid + k * kFinThreads;
            if (v < n[x]) {
                mn = min(mn, f.key[x][k]);
                mx = max(mx, f.key[x][k]);
                sm.addr[x][v] = f.src[x][k];
            }
        }
    block_minmax<kFinWaves>(mn, mx, sm.mm);
    const uint64_t range = (uint64_t)mx - (uint64_t)mn;
    const int bits = range ? 64 - __clzll((long long)range) : 0;
    if (bits > kFinResBits) {
        if (tid == 0) p.wide_list[atomicAdd(&p.plan->nwide, 1u)] = (uint32_t)gi;
        return false;
    }
    uint32_t w[2][kFinIt];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int k = 0; k < kFinIt; k++) {
            const int v = tid + k * kFinThreads;
            w[x][k] = v < n[x] ? ((uint32_t)((uint64_t)f.key[x][k] - (uint64_t)mn) << kFinIdxBits) | (uint32_t)v : ~0u;
        }
    if (range < (uint64_t)kCountRange && !(p.dbg & 32) && fin_count_sort(w, n, sm, wsb)) return true;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int k = 0; k < kFinIt; k++)
            if (w[x][k] != ~0u) sm.key[x][tid + k * kFinThreads] = w[x][k];
    __syncthreads();
    const int npass = (p.dbg & 2) ? 0 : (bits + 7) >> 3;
    for (int ps = 0; ps < npass; ps++) {
        const bool fwd = (ps & 1) == 0;
        fin_radix_pass(fwd ? sm.key : sm.tmp, fwd ? sm.tmp : sm.key, n, kFinIdxBits + 8 * ps, sm, wsb);
    }
    if (npass & 1) {
#pragma unroll
        for (int x = 0; x < 2; x++)
            for (int v = tid; v < n[x]; v += kFinThreads) sm.key[x][v] = sm.tmp[x][v];
        __syncthreads();
    }
    return true;
}

// # of a[0, n) below t (a sorted), n <= kGroupCap: 12 fixed steps
__device__ __forceinline__ int fin_lb(const uint32_t *a, int n, uint32_t t) {
    int pos = 0;
#pragma unroll
    for (int step = kGroupCap; step >= 1; step >>= 1)
        if (pos + step <= n && a[pos + step - 1] < t) pos += step;
    return pos;
}

// sorted rows of both tables to their final places, then the zip join
template <int C1, int C2>
__device__ __forceinline__ void fin_out_join(const MsdFinalParams &p, const MsdGroup &g, int64_t gi, FinSmem &sm,
                                             int &wsb) {
    const int tid = threadIdx.x;
    const int n[2] = {(int)g.nR, p.ntab > 1 ? (int)g.nS : 0};
    constexpr uint32_t IDX = (1u << kFinIdxBits) - 1u;
    if (p.dbg & 4) {
    } else if constexpr (C1 == 2 && C2 == 2) {
        i64x2 r[2][kFinIt];
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int k = 0; k < kFinIt; k++) {
                const int v = tid + k * kFinThreads;
                const uint32_t src = sm.addr[x][sm.key[x][v < n[x] ? v : 0] & IDX];
                r[x][k] = n[x] ? reinterpret_cast<const i64x2 *>(p.tab[x].tempB)[src] : i64x2{0, 0};
            }
#pragma unroll
        for (int x = 0; x < 2; x++) {
            i64x2 *dst = reinterpret_cast<i64x2 *>(p.tab[x].out) + (x ? g.outS : g.outR);
#pragma unroll
            for (int k = 0; k < kFinIt; k++) {
                const int v = tid + k * kFinThreads;
                if (v < n[x]) dst[v] = r[x][k];
            }
        }
    } else {
#pragma unroll
        for (int x = 0; x < 2; x++) {
            if (n[x] == 0) continue;
            const MsdTab &tb = p.tab[x];
            const int cols = C1 > 0 ? (x ? C2 : C1) : tb.cols;
            int64_t *dst = tb.out + (int64_t)(x ? g.outS : g.outR) * cols;
            for (int v = tid; v < n[x]; v += kFinThreads) {
                const uint32_t src = sm.addr[x][sm.key[x][v] & IDX];
                copy_row<0>(tb.tempB + (int64_t)src * cols, dst + (int64_t)v * cols, cols);
            }
        }
    }
    if (!p.join) return;
    // zip join: R position i pairs with S position lbS(k) + (i - lbR(k)).
    // Thread t owns R positions [t*kFinIt, t*kFinIt + kFinIt).
    const int nR = n[0], nS = n[1];
    const uint32_t *kR = sm.key[0], *kS = sm.key[1];
    uint32_t part[kFinIt], mmask = 0;
    if (nS > 0 && nR > 0 && !(p.dbg & 16)) {
        // merge-style lookups: one search for the thread's first key, then
        // short forward walks (keys ascend along the thread's positions)
        int lbR = 0, lbS = 0;
        uint32_t prev = ~0u;
#pragma unroll
        for (int q = 0; q < kFinIt; q++) {
            const int i = tid * kFinIt + q;
            part[q] = 0;
            if (i < nR) {
                const uint32_t kk = kR[i] & ~IDX;
                if (kk != prev) {
                    if (q == 0) {
                        lbR = (i > 0 && (kR[i - 1] & ~IDX) == kk) ? fin_lb(kR, i, kk) : i;
                        lbS = fin_lb(kS, nS, kk);
                    } else {
                        lbR = i;
                        int j = lbS, steps = 0;
                        while (j < nS && (kS[j] & ~IDX) < kk && steps < 16) {
                            j++;
                            steps++;
                        }
                        lbS = (j < nS && (kS[j] & ~IDX) < kk) ? fin_lb(kS, nS, kk) : j;
                    }
                    prev = kk;
                }
                const int j = lbS + (i - lbR);
                if (j < nS && (kS[j] & ~IDX) == kk) {
                    part[q] = (uint32_t)j;
                    mmask |= 1u << q;
                }
            }
        }
    }
    uint32_t total;
    uint32_t o = block_excl_scan_nb<kFinWaves>((uint32_t)__popc(mmask), sm.wsum[wsb], &total);
    wsb ^= 1;
    if (tid == 0) p.counts[gi] = total;
    if (total == 0 || (p.dbg & 8)) return;
    const int c1 = C1 > 0 ? C1 : p.tab[0].cols, c2 = C2 > 0 ? C2 : p.tab[1].cols, tc = c1 + c2 - 1;
    int64_t *dst = p.slots + (int64_t)g.outR * tc;
#pragma unroll
    for (int q = 0; q < kFinIt; q++) {
        if ((mmask >> q) & 1u) {
            const int i = tid * kFinIt + q;
            const uint32_t ra = sm.addr[0][kR[i] & IDX];
            const uint32_t sa = sm.addr[1][kS[part[q]] & IDX];
            emit_join_row<C1, C2>(p.tab[0].tempB + (int64_t)ra * c1, p.tab[1].tempB + (int64_t)sa * c2,
                                  dst + (int64_t)o * tc, c1, c2, p.key2);
            o++;
        }
    }
}

// Diagnostic phase stamps of msd_final (SMJ_DEBUG_MSD=1; off in production):
// s_memtime cycles of thread 0 per phase, summed over workgroups.
__device__ unsigned long long g_fin_phase[16];
#define FIN_STAMP(k)                                                \
    if (SMJ_STAMPS && (p.dbg & 1)) {                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ph[k] += t_ - ph_t;                                         \
        ph_t = t_;                                                  \
    }

// Packed pass-B rows (MsdPlan::packB): group g's rows of every table
// expanded from their words in tempB to 16-B rows at the same row index of
// p.shadow[x] (tempA, dead after part_b), for the tiers other than the staged
// kernel.  NT threads, a wave per pass-B tile run (every row lands at its own
// index, so the order does not matter).
template <int NT>
__device__ __forceinline__ void unpack_group(const MsdFinalParams &p, const MsdGroup &g) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int x = 0; x < p.ntab; x++) {
        const MsdTab &tb = p.tab[x];
        const uint64_t *src = reinterpret_cast<const uint64_t *>(tb.tempB);
        i64x2 *dst = reinterpret_cast<i64x2 *>(p.shadow[x]);
        const bool kc = tb.key != 0;
        auto put = [&](int64_t ix) {
            const uint64_t w = src[ix];
            const int64_t key = g.base + (int64_t)(uint32_t)((uint32_t)w - (uint32_t)g.base);
            const int64_t oth = (int64_t)(int32_t)(uint32_t)(w >> 32);
            dst[ix] = i64x2{kc ? oth : key, kc ? key : oth};
        };
        const MsdBucket bk = tb.bk[g.a];
        if ((bk.one_key & 1u) && g.b0 == 0) {  // a single-key bucket's full tiles (group_gather)
            const int64_t base = (int64_t)bk.tile_base * tb.tile, n = x ? g.nS : g.nR;
            for (int64_t v = tid; v < n; v += NT) put(base + v);
            continue;
        }
        const uint32_t K = (bk.L + (uint32_t)tb.tile - 1) / (uint32_t)tb.tile;
        for (uint32_t i = (uint32_t)wave; i < K; i += NT / 64) {
            const int64_t id = (int64_t)bk.tile_base + i;
            const uint32_t lo = tb.offs[id * kOffsB + g.b0], hi = tb.offs[id * kOffsB + g.b1];
            for (uint32_t o = lo + (uint32_t)lane; o < hi; o += 64) put(id * tb.tile + o);
        }
    }
}

// the tiers after the staged kernel read 16-B rows: with MsdPlan::packB
// (p.pk_mode == 2: the call may pack, known on the device only) those of
// p.shadow, where unpack_group expanded their groups
__device__ __forceinline__ MsdFinalParams rows_view(const MsdFinalParams &p_in) {
    MsdFinalParams p = p_in;
    if (p_in.pk_mode == 2 && uni32(p_in.plan->packB)) {
        p.tab[0].tempB = p_in.shadow[0];
        p.tab[1].tempB = p_in.shadow[1];
    }
    return p;
}

// persistent: workgroup b takes a contiguous range of dense groups (key
// order), so consecutive groups share their bucket's tiles
template <int C1, int C2>
__global__ __launch_bounds__(kFinThreads, 4) void msd_final_kernel(const MsdFinalParams p_in) {
    __shared__ FinSmem sm;
    if (msd_plan_failed(p_in.plan)) return;
    const bool unpack = C1 == 2 && p_in.pk_mode == 2 && uni32(p_in.plan->packB) != 0u;
    const MsdFinalParams p = rows_view(p_in);
    unsigned long long ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, ph_t = (SMJ_STAMPS && (p.dbg & 1)) ? __builtin_amdgcn_s_memtime() : 0;
    // contiguous mode: workgroup b walks a range of dense groups (pipelined one
    // group deep); list mode: the groups msd_final_stage_kernel handed over
    const bool lm = p.radix_list != nullptr;
    int64_t gb, ge, step;
    if (lm) {
        gb = blockIdx.x;
        ge = p.plan->nradix;
        step = gridDim.x;
    } else {
        const int64_t ng = p.plan->ngroups, per = (ng + gridDim.x - 1) / gridDim.x;
        gb = (int64_t)blockIdx.x * per;
        ge = min(ng, gb + per);
        step = 1;
    }
    if (unpack) {  // this workgroup's groups first (list mode: packing implies 2-column tables)
        for (int64_t it = gb; it < ge; it += step) {
            const MsdGroup g = p.groups[lm ? (int64_t)p.radix_list[it] : it];
            if (!g.flags) unpack_group<kFinThreads>(p_in, g);
        }
        __threadfence_block();
        __syncthreads();
    }
    FinalPref f;
    int wsb = 0;
    bool have = false;  // f holds the keys of group gi
    for (int64_t it = gb; it < ge; it += step) {
        const int64_t gi = lm ? (int64_t)p.radix_list[it] : it;
        const MsdGroup g = p.groups[gi];
        if (g.flags) {
            have = false;
            continue;
        }

        if (!fin_fast(p, g)) {
            if (threadIdx.x == 0) p.wide_list[atomicAdd(&p.plan->nwide, 1u)] = (uint32_t)gi;
            have = false;
            continue;
        }
        if (!have) {
            fin_load_offs(p, g, f.o0, f.o1);
            fin_issue_keys<C1, C2>(p, g, f, sm, wsb);
        }
        FIN_STAMP(0);
        MsdGroup gn{};
        bool nfast = false;
        if (!lm && gi + 1 < ge) {
            gn = p.groups[gi + 1];
            nfast = !gn.flags && fin_fast(p, gn);
        }
        uint32_t o0[2], o1[2];  // the next group's offsB values, in flight during the sort
        if (nfast) fin_load_offs(p, gn, o0, o1);
        FIN_STAMP(1);
        const bool ok = fin_sort(p, g, gi, f, sm, wsb);
        FIN_STAMP(2);
        if (nfast) {  // sm.tmp is free after the sort: the next run lists, its key gathers
#pragma unroll
            for (int x = 0; x < 2; x++) {
                f.o0[x] = o0[x];
                f.o1[x] = o1[x];
            }
            fin_issue_keys<C1, C2>(p, gn, f, sm, wsb);
        }
        FIN_STAMP(3);
        if (ok) fin_out_join<C1, C2>(p, g, gi, sm, wsb);
        FIN_STAMP(4);
        have = nfast;
        __syncthreads();  // LDS reused by the next group
        FIN_STAMP(5);
        if (SMJ_STAMPS && (p.dbg & 1)) ph[9]++;
    }
    if (SMJ_STAMPS && (p.dbg & 1) && threadIdx.x == 0)
        for (int k = 0; k < 10; k++) atomicAdd(&g_fin_phase[k], ph[k]);
}

// ---- 2-column staged path --------------------------------------------------------
// The common case, (key, payload) tables: every row of a group is gathered
// ONCE (16 B, lanes on consecutive rows of a pass-B tile range); its payload
// column is staged in LDS; the 32-bit sort words (key - base) << 11 | row are counting-sorted
// (base and key span come from the group record, no reduction); the zip
// join reads its run starts straight from the histogram; sorted rows and
// join rows leave through LDS as coalesced stores.  The next group's rows
// are gathered into registers while this one is sorted and written.  Groups
// outside its limits (key span > kStageRange, > kStList pass-B tiles) go to
// the radix list.
// Round 3: a group holds up to kStRows = 2048 rows of BOTH tables together
// (group rows [0, nR) are R's, [nR, nR + nS) S's; the group kernel packs
// nR + nS <= kStRows where the bucket allows it), so a skewed pair (C5: S
// has ten times R's rows) fills a group as well as a balanced one does.
constexpr int kStThreads = 512, kStWaves = kStThreads / 64;  // 3 per CU (1024-thread workgroups: slower, r01z)
#ifndef SMJ_ST_GRID
#define SMJ_ST_GRID 768
#endif
#ifndef SMJ_ST_RECS
#define SMJ_ST_RECS 16
#endif
constexpr int kStIt = kStRows / kStThreads;    // group rows per thread: tid + k * kStThreads
constexpr int kStIdx = 11;                     // sort word = residual << 11 | group row
constexpr uint32_t kStIdxMask = (1u << kStIdx) - 1u;
static_assert(kStRows == (1 << kStIdx) && kStList * 2 <= 65536, "group rows / list entries fit their fields");
constexpr int kStRange = kStageRange;
constexpr int kStRecs = SMJ_ST_RECS;           // group records per LDS chunk (two chunks in flight)

// Group-row layout of the staged kernel: R's rows are group rows [0, nR),
// S's [sp, sp + nS).  COMB (combined groups, <= kStRows rows of both tables):
// sp = nR.  Per-table groups (<= kGroupCap rows each): sp = kGroupCap, so
// items k < kStIt / 2 of a thread (group rows tid + k * kStThreads) are R's
// and the others S's -- a compile-time table per item, as the balanced
// tables (C3, C4) want it.
template <bool COMB>
struct StSplit {
    uint32_t nR, nS, sp;
    __device__ __forceinline__ StSplit(const MsdFinalParams &p, const MsdGroup &g)
        : nR(g.nR), nS(p.ntab > 1 ? g.nS : 0u), sp(COMB ? g.nR : (uint32_t)kGroupCap) {}
    __device__ __forceinline__ bool is_s(int k, uint32_t v) const { return COMB ? v >= nR : k >= kStIt / 2; }
    __device__ __forceinline__ bool valid(int k, uint32_t v) const {
        return COMB ? v < nR + nS : (k < kStIt / 2 ? v < nR : v - sp < nS);
    }
    __device__ __forceinline__ bool valid_pos(uint32_t q) const { return q < nR || q - sp < nS; }
};

// LDS: 50.4 KiB and 80 VGPRs (launch bounds: 6 waves per SIMD), so three
// workgroups share a CU (24 waves).  Only the payload column is staged: a
// row's key is the group base plus the residual in its sort word.  Same-box
// A/B against the full-row, two-per-CU kernel (profiles/r02_final_occupancy_ab.txt):
// 1.84 vs 1.91 ms and 2.00 vs 2.02 ms on two boxes; the same kernel at two
// per CU is slower (2.03 ms), and without opaque_tid (below) it spills 100 B
// per lane at 80 VGPRs and runs at 2.74 ms.
struct StSmem {
    int64_t pay[kStRows];             // payload (non-key) column, group-row order
    uint32_t key[kStRows];            // sort words, sorted: R's at [0, nR), S's at [nR, nR + nS)
    uint32_t hist[2][kStRange / 2];   // per table, packed u16 bins (zeroed for the next group during the emit)
    union {
        struct {
            uint2 list[2][kStList];          // run lists of the next group: {tempB row, table row}
            uint16_t at[kStRows];            // entry (x * kStList + j) of the non-empty range starting at group row v
            uint32_t starts[kStRows / 32];   // bitmap: a non-empty range starts at group row v
            uint16_t btab[kStRows / 64];     // entry holding group row 64 * b
        } L;
        uint32_t match[kGroupCap];           // join rows (<= min(nR, nS)): R position << 11 | S position
        uint16_t lsd[kStIt * kStWaves][128]; // in-LDS LSD: per 64-row group and digit, counts then starts
    };
    MsdGroup recs[2 * kStRecs];       // ring of this workgroup's group records
    uint32_t wsum[2][kStWaves];
    uint32_t wlen[kStWaves];          // the next group's run-length scan (st_sort)
    uint32_t wmax[2][kStWaves];       // per wave: its longest equal-key run (st_sort)
};


// Ablation bits of the staged kernel (timing only, output invalid), compiled
// in with -DSMJ_ABLATE=1 (tools/final_ablate.py through smj_debug_final_time):
// 2 = no sorted-row stores, 4 = synthetic rows instead of the gathers,
// 8 = no join rows, 16 = no equal-key fix-up rounds
#ifndef SMJ_ABLATE
#define SMJ_ABLATE 0
#endif
#define ST_ABL(bit) (SMJ_ABLATE && (p.dbg & (bit)))

template <bool COMB>
__device__ __forceinline__ bool st_ok(const MsdFinalParams &p, const MsdGroup &g) {
    const uint32_t nS = p.ntab > 1 ? g.nS : 0u;
    return !g.flags && g.span <= (uint32_t)kStRange && g.kt[0] <= (uint32_t)kStList &&
           (p.ntab < 2 || g.kt[1] <= (uint32_t)kStList) &&
           (COMB ? g.nR + nS <= (uint32_t)kStRows : g.nR <= (uint32_t)kGroupCap && nS <= (uint32_t)kGroupCap);
}

// a group the staged kernel leaves to msd_final_wstage_kernel: it would fit
// but for its key span (over kStRange values)
template <bool COMB>
__device__ __forceinline__ bool stw_ok(const MsdFinalParams &p, const MsdGroup &g) {
    const uint32_t nS = p.ntab > 1 ? g.nS : 0u;
    return !g.flags && g.span > (uint32_t)kStRange && g.kt[0] <= (uint32_t)kStList &&
           (p.ntab < 2 || g.kt[1] <= (uint32_t)kStList) &&
           (COMB ? g.nR + nS <= (uint32_t)kStRows : g.nR <= (uint32_t)kGroupCap && nS <= (uint32_t)kGroupCap);
}

__device__ __forceinline__ void st_load_offs(const MsdFinalParams &p, const MsdGroup &g, uint32_t (&o0)[2],
                                             uint32_t (&o1)[2]) {
    const uint32_t tid = opaque_tid();
#pragma unroll
    for (int x = 0; x < 2; x++) {
        o0[x] = o1[x] = 0;
        if (x < p.ntab && tid < g.kt[x]) {
            const int64_t id = (int64_t)g.tb[x] + tid;
            o0[x] = p.tab[x].offs[id * kOffsB + g.b0];
            o1[x] = p.tab[x].offs[id * kOffsB + g.b1];
        }
    }
}

__device__ unsigned long long g_st_sub[8];
#define ST_SUB(k)                                                   \
    if (SMJ_STAMPS && (p.dbg & 1) && tid == 0) {                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        atomicAdd(&g_st_sub[k], t_ - st_t);                         \
        st_t = t_;                                                  \
    }

template <bool COMB, bool PK, class SM>
__device__ __forceinline__ void st_issue_lists(const MsdFinalParams &p, const MsdGroup &g, const uint32_t (&o0)[2],
                                               const uint32_t (&o1)[2], uint32_t ex, i64x2 (&rows)[kStIt],
                                               SM &sm);

// run lists from the offsB values (union region), then the row gathers of
// group g into registers (group row v = tid + k * kStThreads).  Row v's range
// is found in O(1): the range holding the wave's first row (btab) and the last
// non-empty range starting in (64b, v] (bitmap word + at[]; the list also
// holds the group's empty ranges, so a popcount of the bitmap would not
// index it).  S's ranges start at group row nR + their table row.
template <bool COMB, bool PK, class SM>
__device__ __forceinline__ void st_issue(const MsdFinalParams &p, const MsdGroup &g, const uint32_t (&o0)[2],
                                         const uint32_t (&o1)[2], i64x2 (&rows)[kStIt], SM &sm, int &wsb) {
    const uint32_t tid = opaque_tid();
    for (uint32_t i = tid; i < kStRows / 32; i += kStThreads) sm.L.starts[i] = 0;
    const uint32_t len[2] = {o1[0] - o0[0], o1[1] - o0[1]};
    uint32_t tot;
    const uint32_t ex = block_excl_scan_nb<kStWaves>(len[0] | (len[1] << 16), sm.wsum[wsb], &tot);  // + barrier
    wsb ^= 1;
    st_issue_lists<COMB, PK, SM>(p, g, o0, o1, ex, rows, sm);
}

// st_issue after the run-length scan: ex = this thread's exclusive prefix of
// (len R | len S << 16), the start bitmap zeroed and ordered by a barrier.
// PK: tempB holds packed words (MsdPlan::packB); a row is rebuilt from its
// word and the group's base (the group spans <= kStRange keys)
template <bool COMB, bool PK, class SM>
__device__ __forceinline__ void st_issue_lists(const MsdFinalParams &p, const MsdGroup &g, const uint32_t (&o0)[2],
                                               const uint32_t (&o1)[2], uint32_t ex, i64x2 (&rows)[kStIt],
                                               SM &sm) {
    const uint32_t tid = opaque_tid(), lane = tid & 63;
    unsigned long long st_t = (SMJ_STAMPS && (p.dbg & 1)) ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t len[2] = {o1[0] - o0[0], o1[1] - o0[1]};
    const StSplit<COMB> L(p, g);
#pragma unroll
    for (int x = 0; x < 2; x++) {
        if (tid < g.kt[x] && x < p.ntab) {
            const uint32_t vs = x ? (ex >> 16) : (ex & 0xffffu);
            if (SMJ_BOUNDS) {  // a run inside its pass-B tile, and the runs adding up to the group's rows
                const uint32_t nx = x ? g.nS : g.nR;
                if (o1[x] < o0[x] || o1[x] > (uint32_t)p.tab[x].tile || (tid + 1 == g.kt[x] && vs + len[x] != nx))
                    atomicOr(&p.plan->err, 2u);
            }
            sm.L.list[x][tid] = make_uint2((g.tb[x] + tid) * (uint32_t)p.tab[x].tile + o0[x], vs);
            if (len[x]) {
                const uint32_t c = (x ? L.sp : 0u) + vs;  // group row of the range's first row
                const uint16_t e = (uint16_t)(x * kStList + tid);
                sm.L.at[c] = e;
                atomicOr(&sm.L.starts[c >> 5], 1u << (c & 31));
                for (uint32_t b = (c + 63) >> 6; b << 6 < c + len[x]; b++) sm.L.btab[b] = e;
            }
        }
    }
    __syncthreads();
    ST_SUB(4);
    const i64x2 *tB0 = reinterpret_cast<const i64x2 *>(p.tab[0].tempB);
    const i64x2 *tB1 = reinterpret_cast<const i64x2 *>(p.tab[1].tempB);
#pragma unroll
    for (int k = 0; k < kStIt; k++) {
        const uint32_t v = tid + k * kStThreads, b = v >> 6;
        i64x2 r = {0, 0};
        if (L.valid(k, v)) {
            const uint64_t m = ((uint64_t)sm.L.starts[2 * b + 1] << 32 | sm.L.starts[2 * b]) &
                               ((2ull << lane) - 1ull) & ~1ull;  // range starts in (64b, v]
            const uint32_t e = m ? sm.L.at[(b << 6) + 63 - __clzll((long long)m)] : sm.L.btab[b];
            const uint32_t x = COMB ? (e >= (uint32_t)kStList ? 1u : 0u) : (L.is_s(k, v) ? 1u : 0u);
            const uint2 le = sm.L.list[x][e - x * kStList];
            const uint32_t vt = v - (x ? L.sp : 0u);  // table row
            if (ST_ABL(4)) {
                const int64_t kk = g.base + (int64_t)((v * 3u) % max(g.span, 1u));
                if (PK) r = {(int64_t)((uint64_t)(uint32_t)kk | ((uint64_t)v << 32)), 0};
                else r = {p.tab[x].key ? (int64_t)v : kk, p.tab[x].key ? kk : (int64_t)v};
            } else {
                int64_t ix = (int64_t)le.x + (vt - le.y);
                if (SMJ_BOUNDS && (ix < 0 || ix >= p.tab[x].capB)) {
                    atomicOr(&p.plan->err, 2u);
                    ix = 0;
                }
                if constexpr (PK) {  // the raw word: decoded where st_sort consumes it (a decode here
                                     // would wait for the gather before this group's rows are written)
                    r = {(int64_t)reinterpret_cast<const uint64_t *>(x ? p.tab[1].tempB : p.tab[0].tempB)[ix], 0};
                } else {
                    r = (x ? tB1 : tB0)[ix];
                }
            }
        }
        rows[k] = r;
    }
    ST_SUB(5);
}

__device__ __forceinline__ int64_t st_key(const i64x2 &r, int key) { return key ? r.y : r.x; }

// Stable LSD sort of a group's sort words for groups whose equal-key runs are
// too long for the odd-even rounds (Zipf-skewed keys: C5).  w[k] = the word
// of group row v = tid + k * kStThreads (~0u: none; overwritten); words leave
// in sm.key sorted by (table, residual, group row).  Pass 1 sorts by the
// residual's low 6 bits, pass 2 by (table << 6 | its high 6 bits), each a
// stable counting pass: every (item, wave) group of 64 rows is ranked by wave
// ballots on the digit, and one wave prefixes the 32 groups' u16 counts per
// digit (v order = item, wave, lane; two digits per lane).
__device__ __forceinline__ void st_lsd(uint32_t (&cur)[kStIt], uint32_t nR, uint32_t sp, int n, StSmem &sm) {
    constexpr int G = kStIt * kStWaves, DB = 6, D = 128;
    static_assert(sizeof(sm.lsd) <= sizeof(sm.L), "LSD counters fit the list region");
    static_assert(kStRange <= (1 << (2 * DB)), "two 6-bit digits cover the residual");
    const int tid = opaque_tid(), lane = tid & 63, wave = tid >> 6;
    uint32_t *c32 = reinterpret_cast<uint32_t *>(&sm.lsd[0][0]);
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
        for (int i = tid; i < G * D / 2; i += kStThreads) c32[i] = 0;
        __syncthreads();
        uint32_t rk[kStIt], dg[kStIt];
#pragma unroll
        for (int k = 0; k < kStIt; k++) {
            const bool v = cur[k] != ~0u;
            const uint32_t res = cur[k] >> kStIdx;
            const uint32_t d = pass == 0 ? (res & 63u) : ((((cur[k] & kStIdxMask) >= sp) ? 64u : 0u) | (res >> DB));
            dg[k] = d;
            const uint64_t act = __ballot(v);
            uint32_t plo = (uint32_t)act, phi = (uint32_t)(act >> 32);
#pragma unroll
            for (int b = 0; b < DB + 1; b++) {
                const uint32_t sb = (uint32_t)((int32_t)(d << (31 - b)) >> 31);
                const uint64_t bb = __ballot(sb != 0u);
                plo = peer_fold(plo, (uint32_t)bb, sb);
                phi = peer_fold(phi, (uint32_t)(bb >> 32), sb);
            }
            rk[k] = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, 0u));
            const uint64_t peers = ((uint64_t)phi << 32) | plo;
            if (v && (peers >> lane) == 1ull) sm.lsd[k * kStWaves + wave][d] = (uint16_t)__popcll(peers);
        }
        __syncthreads();
        if (wave == 0) {  // lane l: digits 2l, 2l + 1 (one u32 word per group)
            uint32_t t0 = 0, t1 = 0;
#pragma unroll 8
            for (int g = 0; g < G; g++) {
                const uint32_t w2 = c32[g * (D / 2) + lane];
                t0 += w2 & 0xffffu;
                t1 += w2 >> 16;
            }
            uint32_t r0 = wave_incl_scan(t0 + t1, lane) - (t0 + t1), r1 = r0 + t0;
#pragma unroll 8
            for (int g = 0; g < G; g++) {
                const uint32_t w2 = c32[g * (D / 2) + lane];
                c32[g * (D / 2) + lane] = r0 | (r1 << 16);
                r0 += w2 & 0xffffu;
                r1 += w2 >> 16;
            }
        }
        __syncthreads();
        // (pass 2 puts S's rows right after R's: they belong at sp)
        const uint32_t shS = pass == 1 ? sp - nR : 0u;
#pragma unroll
        for (int k = 0; k < kStIt; k++)
            if (cur[k] != ~0u)
                sm.key[(uint32_t)sm.lsd[k * kStWaves + wave][dg[k]] + rk[k] + ((dg[k] & 64u) ? shS : 0u)] = cur[k];
        __syncthreads();
        if (pass == 0) {
#pragma unroll
            for (int k = 0; k < kStIt; k++) {
                const int o = tid + k * kStThreads;
                cur[k] = o < n ? sm.key[o] : ~0u;
            }
        }
    }
}

// stage + counting sort of group g whose rows are in `rows`, then the zip
// join lookups (mmask / part)
template <bool COMB, bool PK>
__device__ __forceinline__ bool st_sort(const MsdFinalParams &p, const MsdGroup &g, int64_t gi,
                                        const i64x2 (&rows)[kStIt], StSmem &sm, int &wsb, uint32_t &mmask,
                                        uint32_t (&part)[kStIt], const uint32_t (&no0)[2], const uint32_t (&no1)[2],
                                        uint32_t &nex) {
    const int tid = opaque_tid(), lane = tid & 63, wave = tid >> 6;
    unsigned long long st_t = (SMJ_STAMPS && (p.dbg & 1)) ? __builtin_amdgcn_s_memtime() : 0;
    const StSplit<COMB> L(p, g);
    const uint32_t nR = L.nR, nS = L.nS, sp = L.sp;
    const int n = (int)(nR + nS);
    uint32_t w[kStIt];  // residual << 16 | atomic rank among its table's equal residuals (~0u: no row)
    // for the next group's st_issue_lists (the list region is idle until then;
    // the barriers below order this before its atomicOr)
    for (int i = tid; i < kStRows / 32; i += kStThreads) sm.L.starts[i] = 0;
    const int kc0 = p.tab[0].key, kc1 = p.tab[1].key;
    // one key value (a heavy key's group, msd_heavy_kernel; combined layout
    // only): the gather order is already the stable sorted order -- the sort
    // words are the identity, nothing is counted, and R position i pairs with
    // S position i (below)
    const bool one = COMB && g.span == 1u;  // block-uniform
#pragma unroll
    for (int k = 0; k < kStIt; k++) {
        const int v = tid + k * kStThreads;
        w[k] = ~0u;
        if (L.valid(k, (uint32_t)v)) {
            const bool x = L.is_s(k, (uint32_t)v);
            const int kc = x ? kc1 : kc0;
            // PK: rows[k].x is the packed word -- other column in its high half,
            // the key's low 32 bits (residual from the group base: span <= kStRange)
            sm.pay[v] = PK ? (int64_t)(int32_t)(uint32_t)((uint64_t)rows[k].x >> 32) : kc ? rows[k].x : rows[k].y;
            if (one) {
                sm.key[v] = (uint32_t)v;
            } else {
                const uint32_t res = PK ? (uint32_t)rows[k].x - (uint32_t)g.base
                                        : (uint32_t)((uint64_t)st_key(rows[k], kc) - (uint64_t)g.base);
                const uint32_t sh = 16u * (res & 1u);
                w[k] = (res << 16) | ((atomicAdd(&sm.hist[x ? 1 : 0][res >> 1], 1u << sh) >> sh) & 0xffffu);
            }
        }
    }
    __syncthreads();
    ST_SUB(0);
    constexpr int W = kStRange / 2 / kStThreads;  // histogram words per thread
    uint32_t tot = 0, mrun = 0;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t h = sm.hist[x][tid * W + i], lo = h & 0xffffu, hi = h >> 16;
            mrun = max(mrun, max(lo, hi));
            t += lo + hi;
        }
        tot |= t << (16 * x);
    }
    // the longest equal-key run: a wave max, one LDS word per wave (one
    // atomicMax per thread with a run serialised ~150 of them on one word per
    // C3 group: the "bin scan" phase's 12.9k cycles, profiles/r03/r03q)
    mrun = wave_incl_max(mrun);  // lane 63: the wave's longest run
    // one barrier for two block scans: this group's bin totals and the next
    // group's run lengths (len R | len S << 16); publishes flag[wsb].
    // (Scanning the lengths in st_issue instead, after the sort: C5 final
    // 11.75 -> 12.27 ms, C3 neutral; profiles/r03/r03k_ab.txt)
    const uint32_t lens = (no1[0] - no0[0]) | ((no1[1] - no0[1]) << 16);
    const uint32_t i1 = wave_incl_scan(tot, lane), i2 = wave_incl_scan(lens, lane);
    if (lane == 63) {
        sm.wsum[wsb][wave] = i1;
        sm.wlen[wave] = i2;
        sm.wmax[wsb][wave] = mrun;
    }
    __syncthreads();
    uint32_t b1 = 0, b2 = 0;
#pragma unroll
    for (int u = 0; u < kStWaves; u++) {
        b1 += u < wave ? sm.wsum[wsb][u] : 0u;
        b2 += u < wave ? sm.wlen[u] : 0u;
    }
    uint32_t ex = b1 + i1 - tot;
    nex = b2 + i2 - lens;
    // materialise both prefixes here: left to the compiler, nex was summed
    // from the eight loaded wave totals at its use in st_issue_lists, which
    // kept 16 VGPRs live across the sort
    asm volatile("" : "+v"(ex), "+v"(nex));
    uint32_t fl = 0;
#pragma unroll
    for (int u = 0; u < kStWaves; u++) fl = max(fl, sm.wmax[wsb][u]);
    fl = fl > 1u ? fl : 0u;  // rounds of the equal-key fix-up (0: no run)
    wsb ^= 1;
    ST_SUB(1);
    bool lsd = fl > (uint32_t)SMJ_ST_MAXRUN;  // block-uniform
    if (lsd && tid == 0) atomicAdd(&p.plan->nlsd, 1u);
    // One key value per table (keys of ~1000 rows per table, a group each: a
    // run that long is the whole table part): the gather order is the stable
    // order, no LSD -- each row's rank becomes its table row, so the scatter
    // below places it there, and no rounds follow.  Checked only on the LSD
    // branch (C3 never takes it).
    if (lsd) {  // a bin holding all of a table's rows (an empty table: any bin)
        uint32_t f = 0;
#pragma unroll
        for (int x = 0; x < 2; x++) {
            const uint32_t nx = x ? nS : nR;
#pragma unroll
            for (int i = 0; i < W; i++) {
                const uint32_t h = sm.hist[x][tid * W + i];
                f |= ((h & 0xffffu) == nx || (h >> 16) == nx) ? (1u << x) : 0u;
            }
        }
        const int fr = __syncthreads_or((int)(f & 1u)), fs = __syncthreads_or((int)(f & 2u));
        if (fr && fs) {
#pragma unroll
            for (int k = 0; k < kStIt; k++)
                if (w[k] != ~0u) {
                    const uint32_t v = (uint32_t)(tid + k * kStThreads);
                    w[k] = (w[k] & 0xffff0000u) | (L.is_s(k, v) ? v - sp : v);
                }
            lsd = false;
            fl = 0;
        }
    }
#pragma unroll
    for (int x = 0; x < 2; x++) {  // per-table starts (table rows)
        uint32_t run = x ? (ex >> 16) : (ex & 0xffffu);
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t h = sm.hist[x][tid * W + i];
            sm.hist[x][tid * W + i] = run | ((run + (h & 0xffffu)) << 16);
            run += (h & 0xffffu) + (h >> 16);
        }
    }
    __syncthreads();
    if (lsd) {  // an equal-key run over kMaxDupRun: stable LSD instead of scatter + rounds
#pragma unroll
        for (int k = 0; k < kStIt; k++)
            if (w[k] != ~0u) w[k] = ((w[k] >> 16) << kStIdx) | (uint32_t)(tid + k * kStThreads);
        st_lsd(w, nR, sp, n, sm);
    } else {
#pragma unroll
        for (int k = 0; k < kStIt; k++)
            if (w[k] != ~0u) {
                const uint32_t v = (uint32_t)(tid + k * kStThreads), x = L.is_s(k, v) ? 1u : 0u;
                const uint32_t res = w[k] >> 16, sh = 16u * (res & 1u);
                sm.key[(x ? sp : 0u) + ((sm.hist[x][res >> 1] >> sh) & 0xffffu) + (w[k] & 0xffffu)] =
                    (res << kStIdx) | v;
            }
        __syncthreads();
    }
    ST_SUB(2);
    // equal residuals were placed in atomic order: odd-even transposition
    // rounds (as many as the longest run) order every run by group row.  A
    // pair across the R / S boundary never swaps (R's group rows are the
    // smaller).  (Measured slower: ranking each run member by a scan of its
    // run, r01k; the run's first thread insertion-sorting the run, r01ah:
    // 2.81 vs 2.32 ms.)
    static_assert(kStRows / 2 == 2 * kStThreads, "two compare-exchanges per thread and round");
    // (Measured and dropped in round 5: runs of <= 8 rows ordered in one pass
    // by the thread holding a run's first position, +0.08 ms -- one lane
    // holds its wave; profiles/r05/r05d.)
    for (uint32_t rd = 0; rd < ((ST_ABL(16) || lsd) ? 0u : fl); rd++) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t q = 2u * (uint32_t)(tid + h * kStThreads) + (rd & 1u);
            if (L.valid_pos(q) && L.valid_pos(q + 1)) {
                const uint32_t a = sm.key[q], b = sm.key[q + 1];
                if ((a >> kStIdx) == (b >> kStIdx) && a > b) {
                    sm.key[q] = b;
                    sm.key[q + 1] = a;
                }
            }
        }
        __syncthreads();
    }
    ST_SUB(3);
    // zip join from the histogram starts: R position i with residual r pairs
    // with S position startS(r) + (i - startR(r)) while i - startR(r) < countS(r)
    mmask = 0;
    // R positions tid * JI + q (consecutive per thread: the block scan of the
    // match counts keeps R order); per-table groups have <= kGroupCap R rows
    constexpr int JI = COMB ? kStIt : kStIt / 2;
#pragma unroll
    for (int q = 0; q < kStIt; q++) part[q] = 0;
    if (one) {
        if (p.join) {
#pragma unroll
            for (int q = 0; q < JI; q++) {
                const uint32_t i = (uint32_t)tid * JI + q;
                if (i < nR && i < nS) {
                    part[q] = i;
                    mmask |= 1u << q;
                }
            }
        }
    } else if (p.join && nR > 0 && nS > 0) {
#pragma unroll
        for (int q = 0; q < JI; q++) {
            const uint32_t i = (uint32_t)tid * JI + q;
            if (i < nR) {
                const uint32_t res = sm.key[i] >> kStIdx, sh = 16u * (res & 1u);
                const uint32_t sR = (sm.hist[0][res >> 1] >> sh) & 0xffffu;
                const uint32_t hS = sm.hist[1][res >> 1];
                const uint32_t sS = (hS >> sh) & 0xffffu;
                const uint32_t eS = (res & 1u) ? ((res + 1u < (uint32_t)kStRange) ? (sm.hist[1][(res + 1) >> 1] & 0xffffu)
                                                                                 : nS)
                                               : (hS >> 16);
                const uint32_t occ = i - sR;
                if (occ < eS - sS) {
                    part[q] = sS + occ;
                    mmask |= 1u << q;
                }
            }
        }
    }
    return true;
}

// sorted rows out (coalesced), join rows out (word-coalesced); the histogram
// is zeroed for the next group here (no one reads it after the lookups)
// WIDE (msd_final_wstage_kernel): keys come from k64 (group-row order), not
// from the group base and the sort word's residual
template <bool COMB, bool WIDE = false>
__device__ __forceinline__ void st_emit(const MsdFinalParams &p, const MsdGroup &g, int64_t gi, StSmem &sm,
                                        int &wsb, uint32_t mmask, const uint32_t (&part)[kStIt],
                                        const int64_t *k64 = nullptr) {
    const int tid = opaque_tid();
    const StSplit<COMB> L(p, g);
    {
        uint4 *h4 = reinterpret_cast<uint4 *>(&sm.hist[0][0]);
        for (int i = tid; i < kStRange / 4; i += kStThreads) h4[i] = make_uint4(0, 0, 0, 0);
    }
    i64x2 *dR = reinterpret_cast<i64x2 *>(p.tab[0].out) + g.outR;
    i64x2 *dS = reinterpret_cast<i64x2 *>(p.tab[1].out) + g.outS - L.sp;  // S row q - sp
    const int kc0 = p.tab[0].key, kc1 = p.tab[1].key;
#pragma unroll
    for (int k = 0; k < kStIt; k++) {
        const uint32_t q = tid + k * kStThreads;
        if (L.valid(k, q) && !ST_ABL(2)) {
            const bool x = L.is_s(k, q);
            const uint32_t w = sm.key[q];
            const int64_t key = WIDE ? k64[w & kStIdxMask] : g.base + (int64_t)(w >> kStIdx);
            const int64_t pay = sm.pay[w & kStIdxMask];
            const int kc = x ? kc1 : kc0;
            i64x2 r;
            r.x = kc ? pay : key;
            r.y = kc ? key : pay;
            __builtin_nontemporal_store(r, (x ? dS : dR) + q);  // final rows: streamed
        }
    }
    if (!p.join || ST_ABL(8)) return;
    const uint32_t *kS = sm.key + L.sp;
    uint32_t total;
    uint32_t o = block_excl_scan_nb<kStWaves>((uint32_t)__popc(mmask), sm.wsum[wsb], &total);
    wsb ^= 1;
    if (tid == 0) p.counts[gi] = total;
    if (total == 0) return;
    constexpr int JI = COMB ? kStIt : kStIt / 2;  // as in st_sort
#pragma unroll
    for (int q = 0; q < JI; q++)
        if ((mmask >> q) & 1u) sm.match[o++] = (((uint32_t)tid * JI + q) << kStIdx) | part[q];
    __syncthreads();
    // output word wd = row * 3 + column: R key, R payload, S payload
    int64_t *dst = p.slots + (int64_t)g.outR * 3;
    // fixed trip count (total <= kGroupCap), see st_load_recs
    constexpr int EMIT_IT = (3 * kGroupCap + kStThreads - 1) / kStThreads;
#pragma unroll
    for (int it = 0; it < EMIT_IT; it++) {
        const uint32_t wd = tid + it * kStThreads;
        if (wd < total * 3u) {
            const uint32_t row = wd / 3u, c = wd - row * 3u;
            const uint32_t m = sm.match[row];
            int64_t val;
            if (c < 2) {  // R's columns: the key from the sort word, the payload staged
                const uint32_t w = sm.key[m >> kStIdx];
                val = (int)c == kc0 ? (WIDE ? k64[w & kStIdxMask] : g.base + (int64_t)(w >> kStIdx))
                                    : sm.pay[w & kStIdxMask];
            } else {      // S's column other than key2: its payload
                val = sm.pay[kS[m & kStIdxMask] & kStIdxMask];
            }
            __builtin_nontemporal_store(val, dst + wd);  // join slots: read back by msd_compact only
        }
    }
}

// copy the records of this workgroup's local groups [t0, t0 + kStRecs) into
// ring half h (local group t is dense group g0 + t * gs): one word per thread,
// no loop -- a dynamic-count load loop here would make hipcc's waitcnt pass
// give up counting, and every group's prefetched rows would then be consumed
// behind a vmcnt(0) that also drains the previous group's stores
template <class SM>
__device__ __forceinline__ void st_load_recs(const MsdFinalParams &p, int64_t g0, int64_t gs, int64_t t0,
                                             int64_t cnt, SM &sm, int h) {
    constexpr int WORDS = sizeof(MsdGroup) / 8;
    static_assert(kStRecs * WORDS <= kStThreads, "at most one record word per thread");
    int64_t *dst = reinterpret_cast<int64_t *>(&sm.recs[h * kStRecs]);
    const int i = opaque_tid();
    const int64_t t = t0 + i / WORDS;
    if (i < kStRecs * WORDS && t < cnt) dst[i] = reinterpret_cast<const int64_t *>(p.groups + g0 + t * gs)[i % WORDS];
}

// persistent staged kernel.  XCD-aware schedule: the dense (key-ordered)
// groups are cut into kXcdSlots contiguous ranges, one per set of blocks
// sharing an XCD (blocks b, b + 8, ... -- MI355X_MICROARCH.md, workgroup
// dispatch), and the set's blocks interleave over their range (block j of the
// set takes groups j, j + gs, ...).  Groups in flight on one XCD are then
// neighbours in key order: the pass-B tile lines and offsB lines two
// neighbouring groups share are fetched into that XCD's L2 once.
constexpr int kXcdSlots = 8;
#ifndef SMJ_ST_MINW
#define SMJ_ST_MINW 6
#endif
template <bool COMB, bool PK>
__device__ __forceinline__ void st_body(const MsdFinalParams &p, StSmem &sm) {
    const int64_t ng = p.plan->ngroups;
    const int64_t gs = gridDim.x / kXcdSlots;  // blocks per XCD set
    const int64_t xr = (ng + kXcdSlots - 1) / kXcdSlots;
    const int64_t x0 = (int64_t)(blockIdx.x % kXcdSlots) * xr, x1 = min(ng, x0 + xr);
    const int64_t g0 = x0 + blockIdx.x / kXcdSlots;  // local group t = dense group g0 + t * gs
    const int64_t cnt = x1 > g0 ? (x1 - g0 + gs - 1) / gs : 0;
    unsigned long long ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, ph_t = (SMJ_STAMPS && (p.dbg & 1)) ? __builtin_amdgcn_s_memtime() : 0;
    {
        uint4 *h4 = reinterpret_cast<uint4 *>(&sm.hist[0][0]);
        for (int i = opaque_tid(); i < kStRange / 4; i += kStThreads) h4[i] = make_uint4(0, 0, 0, 0);
    }
    if (0 < cnt) st_load_recs(p, g0, gs, 0, cnt, sm, 0);
    if (kStRecs < cnt) st_load_recs(p, g0, gs, kStRecs, cnt, sm, 1);
    __syncthreads();
    i64x2 cur[kStIt];
    int wsb = 0;
    uint32_t nwst = 0;  // wide groups left to msd_final_wstage_kernel (block-uniform)
    bool have = false;  // cur holds the rows of group gi
    for (int64_t li = 0; li < cnt; li++) {
        const int64_t gi = g0 + li * gs;
        if (li >= kStRecs && li % kStRecs == 0) {  // entering chunk c: fetch chunk c + 1 into the other half
            const int64_t c = li / kStRecs;
            __syncthreads();
            if (li + kStRecs < cnt) st_load_recs(p, g0, gs, li + kStRecs, cnt, sm, (int)((c + 1) & 1));
            __syncthreads();
        }
        const MsdGroup &g = sm.recs[li % (2 * kStRecs)];  // fields read from LDS where used (register pressure)
        if (g.flags) {
            have = false;
            continue;
        }
        if (!st_ok<COMB>(p, g)) {
            if (stw_ok<COMB>(p, g)) {  // a wide group: the wide-span kernels' (msd_back launches them)
                nwst++;
                have = false;
                continue;
            }
            // (the group kernel packs over kGroupCap rows of a table only where
            // every group fits this kernel: the radix tier takes <= kGroupCap)
            if (opaque_tid() == 0) {
                // the radix tier stages <= kGroupCap rows per table in LDS: a
                // group over that is only flagged (the call fails), never listed
                if (g.nR > (uint32_t)kGroupCap || (p.ntab > 1 && g.nS > (uint32_t)kGroupCap))
                    atomicOr(&p.plan->err, 4u);
                else
                    p.radix_list[atomicAdd(&p.plan->nradix, 1u)] = (uint32_t)gi;
            }
            have = false;
            continue;
        }
        if (!have) {
            uint32_t o0[2], o1[2];
            st_load_offs(p, g, o0, o1);
            st_issue<COMB, PK>(p, g, o0, o1, cur, sm, wsb);
            __syncthreads();  // the list region is reused by the join
        }
        FIN_STAMP(0);
        bool nfit = false;
        const MsdGroup &gn = sm.recs[(li + 1) % (2 * kStRecs)];
        uint32_t o0[2] = {0, 0}, o1[2] = {0, 0};
        if (li + 1 < cnt) {
            nfit = st_ok<COMB>(p, gn);
            if (nfit) st_load_offs(p, gn, o0, o1);
        }
        FIN_STAMP(1);
        uint32_t mmask = 0, part[kStIt];
        uint32_t nex;  // the next group's run-length prefix, scanned with this group's bins
        const bool ok = st_sort<COMB, PK>(p, g, gi, cur, sm, wsb, mmask, part, o0, o1, nex);  // cur is staged in LDS here
        FIN_STAMP(2);
        // st_issue_lists writes only the list region (unused by the sort; its
        // start bitmap was zeroed, and its run lengths scanned, inside
        // st_sort), and its barrier orders the sort's last histogram reads
        // before st_emit zeroes the histogram; st_emit writes `match`
        // (aliasing the list) only after its own scan barrier, which every
        // wave reaches after its st_issue_lists reads.  Without a next group
        // one barrier does both.
        if (nfit)  // the next group's rows: in flight while this one is written out
            st_issue_lists<COMB, PK>(p, gn, o0, o1, nex, cur, sm);
        else
            __syncthreads();
        FIN_STAMP(3);
        if (ok) {
            st_emit<COMB>(p, g, gi, sm, wsb, mmask, part);
        } else {  // hand-over: the histogram still needs zeroing
            uint4 *h4 = reinterpret_cast<uint4 *>(&sm.hist[0][0]);
            for (int i = opaque_tid(); i < kStRange / 4; i += kStThreads) h4[i] = make_uint4(0, 0, 0, 0);
        }
        FIN_STAMP(4);
        have = nfit;
        __syncthreads();
        FIN_STAMP(5);
        if (SMJ_STAMPS && (p.dbg & 1)) ph[9]++;
    }
    if (nwst && opaque_tid() == 0) atomicAdd(&p.plan->nwst, nwst);
    if (SMJ_STAMPS && (p.dbg & 1) && opaque_tid() == 0)
        for (int k = 0; k < 10; k++) atomicAdd(&g_fin_phase[k], ph[k]);
}

template <bool COMB, int PKM = 0>
__global__ __launch_bounds__(kStThreads, SMJ_ST_MINW) void msd_final_stage_kernel(const MsdFinalParams p) {
    __shared__ StSmem sm;
    if (msd_plan_failed(p.plan)) return;
    constexpr bool PK = PKM == 1;
    if (PKM == 2) {  // the layout is known on the device only: both bodies, one block-uniform branch
        if (uni32(p.plan->packB)) st_body<COMB, true>(p, sm);
        else st_body<COMB, false>(p, sm);
        return;
    }
    st_body<COMB, PK>(p, sm);
}

// ---- wide-span staged path (round 6) ----------------------------------------
// Groups whose keys span more than kStRange values -- every group of a table
// with full-range int64 keys (SURVEY 8(d)'s C3-wide: a pass-B sub-bucket then
// spans ~2^45 keys) -- went to the radix tier, which handed them to the 64-bit
// LSD kernel (msd_final_wide_kernel: C3-wide msd_final 9.7 ms).  Here they
// take the staged kernel's shape: rows gathered once into registers (the next
// group's during this one's emit), staged in LDS with their FULL keys (k64),
// a counting sort over kStRange monotone bins bin(key) = mulhi64(key - base,
// bscale) (MsdGroup::pad[1..2], msd_group_kernel), then odd-even rounds that
// order each bin by (key, group row) -- the narrow kernel's equal-residual
// rounds with a key compare -- and the zip join by key within each bin
// (cpu_app.c:204-266: occurrence i of a key in R pairs with occurrence i in
// S).  Staging the keys costs LDS: layouts below.  A bin over SMJ_ST_MAXRUN
// rows (keys clustered inside the group's interval) hands the group to the
// radix tier before anything is written.
// LDS layouts of the wide-span kernels: PayT = the staged other column,
// KT = the staged key (int64; uint32 = key - group base with packed pass-B
// rows, whose keys lie within 2^32 of every group base), HB = bins per table.
// <int32, uint32, 4096> (packed rows) and <int32, int64, 2048> (rows whose
// other column fits int32, MsdPlan::nopack == 0) take 50.7 KiB: three
// workgroups per CU, as the narrow kernel; <int64, int64, 4096> (any rows)
// 66.6 KiB: two.
template <class PayT, class KT, int HB>
struct StwSmemT {
    PayT pay[kStRows];              // other column, group-row order
    KT kk[kStRows];                 // keys, group-row order
    uint32_t key[kStRows];          // sort words bin << kStIdx | group row, sorted
    uint32_t hist[2][HB / 2];       // per table, packed u16 bins
    union {
        struct {
            uint2 list[2][kStList];
            uint16_t at[kStRows];
            uint32_t starts[kStRows / 32];
            uint16_t btab[kStRows / 64];
        } L;
        uint32_t match[kGroupCap];
    };
    MsdGroup recs[2 * kStRecs];
    uint32_t wsum[2][kStWaves];
    uint32_t wlen[kStWaves];
    uint32_t wmax[2][kStWaves];
    static constexpr int kBins = HB;
    using PayType = PayT;
};
using StwSmemP = StwSmemT<int32_t, uint32_t, kStRange>;      // packed pass-B rows
using StwSmemR = StwSmemT<int32_t, int64_t, kStRange / 2>;   // 16-B rows, other column in int32
using StwSmem64 = StwSmemT<int64_t, int64_t, kStRange>;      // 16-B rows

template <class SM>
__device__ __forceinline__ int64_t stw_key(const SM &sm, const MsdGroup &g, uint32_t v) {
    if constexpr (sizeof(sm.kk[0]) == 4) return g.base + (int64_t)sm.kk[v];
    else return (int64_t)sm.kk[v];
}

// stage + bin sort + in-bin rounds of wide group g, then the zip join lookups
template <bool COMB, bool PK, class SM>
__device__ __forceinline__ bool stw_sort(const MsdFinalParams &p, const MsdGroup &g, const i64x2 (&rows)[kStIt],
                                         SM &sm, int &wsb, uint32_t &mmask, uint32_t (&part)[kStIt],
                                         const uint32_t (&no0)[2], const uint32_t (&no1)[2], uint32_t &nex) {
    constexpr int HB = SM::kBins;
    constexpr int BSH = HB == kStRange ? 0 : HB == kStRange / 2 ? 1 : 2;  // bins from the record's kStRange-bin scale
    static_assert(HB == (kStRange >> BSH), "bins per table");
    const int tid = opaque_tid(), lane = tid & 63, wave = tid >> 6;
    const StSplit<COMB> L(p, g);
    const uint32_t nR = L.nR, nS = L.nS, sp = L.sp;
    const uint64_t bscale = (uint64_t)g.pad[1] | ((uint64_t)g.pad[2] << 32);
    uint32_t w[kStIt];  // bin << 16 | atomic rank among its table's rows of that bin (~0u: no row)
    for (int i = tid; i < kStRows / 32; i += kStThreads) sm.L.starts[i] = 0;  // for the next st_issue_lists
    const int kc0 = p.tab[0].key, kc1 = p.tab[1].key;
#pragma unroll
    for (int k = 0; k < kStIt; k++) {
        const int v = tid + k * kStThreads;
        w[k] = ~0u;
        if (L.valid(k, (uint32_t)v)) {
            const bool x = L.is_s(k, (uint32_t)v);
            const int kc = x ? kc1 : kc0;
            // PK: the packed word's key half is exact from the base (packB: every key
            // within 2^32 of every group base)
            const uint64_t r = PK ? (uint64_t)((uint32_t)rows[k].x - (uint32_t)g.base)
                                  : (uint64_t)st_key(rows[k], kc) - (uint64_t)g.base;
            const int64_t pay = PK ? (int64_t)(int32_t)(uint32_t)((uint64_t)rows[k].x >> 32) : kc ? rows[k].x : rows[k].y;
            sm.pay[v] = (typename SM::PayType)pay;
            if constexpr (sizeof(sm.kk[0]) == 4) sm.kk[v] = (uint32_t)r;
            else sm.kk[v] = (int64_t)((uint64_t)g.base + r);
            const uint32_t bin = min((uint32_t)(__umul64hi(r, bscale) >> BSH), (uint32_t)HB - 1u);
            const uint32_t sh = 16u * (bin & 1u);
            w[k] = (bin << 16) | ((atomicAdd(&sm.hist[x ? 1 : 0][bin >> 1], 1u << sh) >> sh) & 0xffffu);
        }
    }
    __syncthreads();
    constexpr int W = HB / 2 / kStThreads;
    uint32_t tot = 0, mrun = 0;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t h = sm.hist[x][tid * W + i], lo = h & 0xffffu, hi = h >> 16;
            mrun = max(mrun, max(lo, hi));
            t += lo + hi;
        }
        tot |= t << (16 * x);
    }
    mrun = wave_incl_max(mrun);
    const uint32_t lens = (no1[0] - no0[0]) | ((no1[1] - no0[1]) << 16);
    const uint32_t i1 = wave_incl_scan(tot, lane), i2 = wave_incl_scan(lens, lane);
    if (lane == 63) {
        sm.wsum[wsb][wave] = i1;
        sm.wlen[wave] = i2;
        sm.wmax[wsb][wave] = mrun;
    }
    __syncthreads();
    uint32_t b1 = 0, b2 = 0;
#pragma unroll
    for (int u = 0; u < kStWaves; u++) {
        b1 += u < wave ? sm.wsum[wsb][u] : 0u;
        b2 += u < wave ? sm.wlen[u] : 0u;
    }
    uint32_t ex = b1 + i1 - tot;
    nex = b2 + i2 - lens;
    asm volatile("" : "+v"(ex), "+v"(nex));
    uint32_t fl = 0;
#pragma unroll
    for (int u = 0; u < kStWaves; u++) fl = max(fl, sm.wmax[wsb][u]);
    wsb ^= 1;
    // block-uniform: the radix tier sorts it (p.dbg bits 16..23: a test's lower limit + 1)
    const uint32_t maxrun = (p.dbg >> 16) & 0xff ? (uint32_t)((p.dbg >> 16) & 0xff) - 1u : (uint32_t)SMJ_ST_MAXRUN;
    if (fl > maxrun) return false;
    fl = fl > 1u ? fl : 0u;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        uint32_t run = x ? (ex >> 16) : (ex & 0xffffu);
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t h = sm.hist[x][tid * W + i];
            sm.hist[x][tid * W + i] = run | ((run + (h & 0xffffu)) << 16);
            run += (h & 0xffffu) + (h >> 16);
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kStIt; k++)
        if (w[k] != ~0u) {
            const uint32_t v = (uint32_t)(tid + k * kStThreads), x = L.is_s(k, v) ? 1u : 0u;
            const uint32_t bin = w[k] >> 16, sh = 16u * (bin & 1u);
            sm.key[(x ? sp : 0u) + ((sm.hist[x][bin >> 1] >> sh) & 0xffffu) + (w[k] & 0xffffu)] = (bin << kStIdx) | v;
        }
    __syncthreads();
    // rows of one bin were placed in atomic order: odd-even rounds (as many as
    // the longest bin) order each bin by (key, group row) -- group rows ascend
    // in input order within a table, so this is the stable order.  A pair
    // across the R / S boundary never swaps.  (kk: the key, or its offset from
    // the group base -- the same order.)
    for (uint32_t rd = 0; rd < fl; rd++) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t q = 2u * (uint32_t)(tid + h * kStThreads) + (rd & 1u);
            if (L.valid_pos(q) && L.valid_pos(q + 1) && (q < sp) == (q + 1 < sp)) {
                const uint32_t a = sm.key[q], b = sm.key[q + 1];
                if ((a >> kStIdx) == (b >> kStIdx)) {
                    const auto ka = sm.kk[a & kStIdxMask], kb = sm.kk[b & kStIdxMask];
                    if (ka > kb || (ka == kb && a > b)) {
                        sm.key[q] = b;
                        sm.key[q + 1] = a;
                    }
                }
            }
        }
        __syncthreads();
    }
    // zip join: R position i holding key k is occurrence occ = i - (first R
    // position of k) of its key; it pairs with S position (first S position
    // of k) + occ while that still holds k.  Keys are sorted within a bin and a
    // key never leaves its bin, so both searches stay inside the bin (<=
    // SMJ_ST_MAXRUN positions).
    mmask = 0;
    constexpr int JI = COMB ? kStIt : kStIt / 2;
#pragma unroll
    for (int q = 0; q < kStIt; q++) part[q] = 0;
    if (p.join && nR > 0 && nS > 0) {
        const uint32_t *kS = sm.key + sp;
#pragma unroll
        for (int q = 0; q < JI; q++) {
            const uint32_t i = (uint32_t)tid * JI + q;
            if (i < nR) {
                const uint32_t wi = sm.key[i], bin = wi >> kStIdx, sh = 16u * (bin & 1u);
                const uint32_t hS = sm.hist[1][bin >> 1];
                const uint32_t sS = (hS >> sh) & 0xffffu;
                const uint32_t eS = (bin & 1u) ? ((bin + 1u < (uint32_t)HB) ? (sm.hist[1][(bin + 1) >> 1] & 0xffffu) : nS)
                                               : (hS >> 16);
                if (sS == eS) continue;  // no S row in the bin
                const auto kk = sm.kk[wi & kStIdxMask];
                const uint32_t sR = (sm.hist[0][bin >> 1] >> sh) & 0xffffu;
                uint32_t f = i;
                while (f > sR && sm.kk[sm.key[f - 1] & kStIdxMask] == kk) f--;
                const uint32_t occ = i - f;
                uint32_t j = sS;
                while (j < eS && sm.kk[kS[j] & kStIdxMask] < kk) j++;
                if (j + occ < eS && sm.kk[kS[j + occ] & kStIdxMask] == kk) {
                    part[q] = j + occ;
                    mmask |= 1u << q;
                }
            }
        }
    }
    return true;
}

// sorted rows out (coalesced), join rows out (word-coalesced); the histogram
// is zeroed for the next group here (st_emit's shape, keys from kk)
template <bool COMB, class SM>
__device__ __forceinline__ void stw_emit(const MsdFinalParams &p, const MsdGroup &g, int64_t gi, SM &sm, int &wsb,
                                         uint32_t mmask, const uint32_t (&part)[kStIt]) {
    const int tid = opaque_tid();
    const StSplit<COMB> L(p, g);
    {
        uint4 *h4 = reinterpret_cast<uint4 *>(&sm.hist[0][0]);
        for (int i = tid; i < SM::kBins / 4; i += kStThreads) h4[i] = make_uint4(0, 0, 0, 0);
    }
    i64x2 *dR = reinterpret_cast<i64x2 *>(p.tab[0].out) + g.outR;
    i64x2 *dS = reinterpret_cast<i64x2 *>(p.tab[1].out) + g.outS - L.sp;  // S row q - sp
    const int kc0 = p.tab[0].key, kc1 = p.tab[1].key;
#pragma unroll
    for (int k = 0; k < kStIt; k++) {
        const uint32_t q = tid + k * kStThreads;
        if (L.valid(k, q)) {
            const bool x = L.is_s(k, q);
            const uint32_t v = sm.key[q] & kStIdxMask;
            const int64_t key = stw_key(sm, g, v), pay = (int64_t)sm.pay[v];
            const int kc = x ? kc1 : kc0;
            i64x2 r;
            r.x = kc ? pay : key;
            r.y = kc ? key : pay;
            __builtin_nontemporal_store(r, (x ? dS : dR) + q);
        }
    }
    if (!p.join) return;
    const uint32_t *kS = sm.key + L.sp;
    uint32_t total;
    uint32_t o = block_excl_scan_nb<kStWaves>((uint32_t)__popc(mmask), sm.wsum[wsb], &total);
    wsb ^= 1;
    if (tid == 0) p.counts[gi] = total;
    if (total == 0) return;
    constexpr int JI = COMB ? kStIt : kStIt / 2;
#pragma unroll
    for (int q = 0; q < JI; q++)
        if ((mmask >> q) & 1u) sm.match[o++] = (((uint32_t)tid * JI + q) << kStIdx) | part[q];
    __syncthreads();
    int64_t *dst = p.slots + (int64_t)g.outR * 3;
    constexpr int EMIT_IT = (3 * kGroupCap + kStThreads - 1) / kStThreads;
#pragma unroll
    for (int it = 0; it < EMIT_IT; it++) {
        const uint32_t wd = tid + it * kStThreads;
        if (wd < total * 3u) {
            const uint32_t row = wd / 3u, c = wd - row * 3u;
            const uint32_t m = sm.match[row];
            int64_t val;
            if (c < 2) {
                const uint32_t v = sm.key[m >> kStIdx] & kStIdxMask;
                val = (int)c == kc0 ? stw_key(sm, g, v) : (int64_t)sm.pay[v];
            } else {
                val = (int64_t)sm.pay[kS[m & kStIdxMask] & kStIdxMask];
            }
            __builtin_nontemporal_store(val, dst + wd);
        }
    }
}

// persistent over the dense groups with the staged kernel's XCD-aware
// schedule, taking only the wide groups (stw_ok) the staged kernel skipped
int g_wide_maxrun = -1;
template <bool COMB, bool PK, class SM>
__device__ __forceinline__ void stw_body(const MsdFinalParams &p, SM &sm) {
    const int64_t ng = p.plan->ngroups;
    const int64_t gs = gridDim.x / kXcdSlots;
    const int64_t xr = (ng + kXcdSlots - 1) / kXcdSlots;
    const int64_t x0 = (int64_t)(blockIdx.x % kXcdSlots) * xr, x1 = min(ng, x0 + xr);
    const int64_t g0 = x0 + blockIdx.x / kXcdSlots;
    const int64_t cnt = x1 > g0 ? (x1 - g0 + gs - 1) / gs : 0;
    {
        uint4 *h4 = reinterpret_cast<uint4 *>(&sm.hist[0][0]);
        for (int i = opaque_tid(); i < SM::kBins / 4; i += kStThreads) h4[i] = make_uint4(0, 0, 0, 0);
    }
    if (0 < cnt) st_load_recs(p, g0, gs, 0, cnt, sm, 0);
    if (kStRecs < cnt) st_load_recs(p, g0, gs, kStRecs, cnt, sm, 1);
    __syncthreads();
    i64x2 cur[kStIt];
    int wsb = 0;
    bool have = false;  // cur holds the rows of group gi
    for (int64_t li = 0; li < cnt; li++) {
        const int64_t gi = g0 + li * gs;
        if (li >= kStRecs && li % kStRecs == 0) {
            const int64_t c = li / kStRecs;
            __syncthreads();
            if (li + kStRecs < cnt) st_load_recs(p, g0, gs, li + kStRecs, cnt, sm, (int)((c + 1) & 1));
            __syncthreads();
        }
        const MsdGroup &g = sm.recs[li % (2 * kStRecs)];
        if (!stw_ok<COMB>(p, g)) {  // the staged kernel's, or listed by it
            have = false;
            continue;
        }
        if (!have) {
            uint32_t o0[2], o1[2];
            st_load_offs(p, g, o0, o1);
            st_issue<COMB, PK>(p, g, o0, o1, cur, sm, wsb);
            __syncthreads();
        }
        bool nfit = false;
        const MsdGroup &gn = sm.recs[(li + 1) % (2 * kStRecs)];
        uint32_t o0[2] = {0, 0}, o1[2] = {0, 0};
        if (li + 1 < cnt) {
            nfit = stw_ok<COMB>(p, gn);
            if (nfit) st_load_offs(p, gn, o0, o1);
        }
        uint32_t mmask = 0, part[kStIt], nex;
        const bool ok = stw_sort<COMB, PK>(p, g, cur, sm, wsb, mmask, part, o0, o1, nex);
        // the join lookups read the histogram, which does not alias the list
        // region st_issue_lists writes; its barrier orders them before the
        // emit zeroes the histogram
        if (nfit)
            st_issue_lists<COMB, PK>(p, gn, o0, o1, nex, cur, sm);
        else
            __syncthreads();
        if (ok) {
            stw_emit<COMB>(p, g, gi, sm, wsb, mmask, part);
        } else {  // a bin over SMJ_ST_MAXRUN rows: the radix tier's (nothing was written)
            if (opaque_tid() == 0) {
                if (g.nR > (uint32_t)kGroupCap || (p.ntab > 1 && g.nS > (uint32_t)kGroupCap))
                    atomicOr(&p.plan->err, 4u);  // over the radix tier's LDS (combined groups are never wide)
                else
                    p.radix_list[atomicAdd(&p.plan->nradix, 1u)] = (uint32_t)gi;
            }
            uint4 *h4 = reinterpret_cast<uint4 *>(&sm.hist[0][0]);
            for (int i = opaque_tid(); i < SM::kBins / 4; i += kStThreads) h4[i] = make_uint4(0, 0, 0, 0);
        }
        have = nfit;
        __syncthreads();
    }
}

// the layout a call's wide groups take (block-uniform, from the plan): 0 =
// packed rows, 1 = 16-B rows whose other column fits int32 (part_a checked it:
// a call that may pack, p.shadow[0]), 2 = any 16-B rows
__device__ __forceinline__ int stw_layout(const MsdFinalParams &p) {
    if (uni32(p.plan->packB)) return 0;
    return p.shadow[0] && uni32(p.plan->nopack) == 0u ? 1 : 2;
}

// layouts 0 and 1: three workgroups per CU
constexpr int kStwGrid = SMJ_ST_GRID;
template <bool COMB>
__global__ __launch_bounds__(kStThreads, SMJ_ST_MINW) void msd_final_wstage_kernel(const MsdFinalParams p) {
    __shared__ union {
        StwSmemP pk;
        StwSmemR rw;
    } sm;
    if (msd_plan_failed(p.plan) || uni32(p.plan->nwst) == 0u) return;
    const int lay = stw_layout(p);
    if (lay == 0) stw_body<COMB, true>(p, sm.pk);
    else if (lay == 1) stw_body<COMB, false>(p, sm.rw);
}

// layout 2: two workgroups per CU
constexpr int kStw64Grid = 512;
template <bool COMB>
__global__ __launch_bounds__(kStThreads, 4) void msd_final_wstage64_kernel(const MsdFinalParams p) {
    __shared__ StwSmem64 sm;
    if (msd_plan_failed(p.plan) || uni32(p.plan->nwst) == 0u || stw_layout(p) != 2) return;
    stw_body<COMB, false>(p, sm);
}

// Packed pass-B rows: the single-key and oversized groups (msd_group's
// lists) unpacked for the host-launched tiers (smj_api.hip msd_fallback,
// which launches this only when the call packed and has such groups); the
// radix tier unpacks its own groups.
constexpr int kUnpackGrid = 1024;
__global__ __launch_bounds__(256) void msd_unpack_groups_kernel(const MsdFinalParams p) {
    if (msd_plan_failed(p.plan) || p.plan->packB == 0u) return;
    // (the single-key tier reads the packed words itself: MsdFinalParams::pk_mode 3)
    const uint32_t nb = p.plan->nbig;
    for (uint32_t e = blockIdx.x; e < nb; e += gridDim.x) unpack_group<256>(p, p.groups[p.big_list[e]]);
}

hipError_t launch_msd_unpack_groups(const MsdFinalParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_unpack_groups_kernel, dim3(kUnpackGrid), dim3(256), 0, s, p);
    return hipGetLastError();
}

// groups of the wide list (key range over 22 bits, or a bucket with more than
// kFinThreads pass-B tiles): the generic 64-bit path, persistent over the list
template <int C1, int C2>
__global__ __launch_bounds__(kMsdThreads, 2) void msd_final_wide_kernel(const MsdFinalParams p_in) {
    __shared__ FinalSmem sm;
    if (msd_plan_failed(p_in.plan)) return;
    const MsdFinalParams p = rows_view(p_in);  // (its groups come from the radix list: unpacked there)
    const uint32_t nw = p.plan->nwide;
    for (uint32_t i = blockIdx.x; i < nw; i += gridDim.x) {
        final_group<C1, C2>(p, p.wide_list[i], sm);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// oversized multi-key groups of a small key span (2-column tables)
// ---------------------------------------------------------------------------
// A sub-bucket over kGroupCap rows that holds more than one key value (a
// Zipf-skewed table, BASELINE C5: a key with thousands of rows next to light
// ones) used to leave the device pipeline for the host-driven fallback
// (gather, 64-bit LSD sort, zip join of every such group).  When its keys
// span at most kStRange values (and it has at most kBgMaxRows rows per
// table) it is sorted here instead, one workgroup per group, by a two-pass
// counting sort over the residual r = key - base: pass 1 counts every r of
// both tables through LDS atomics; the counts become exclusive output starts
// (and the zip join's per-r pair counts min(cR, cS) an exclusive prefix of
// join rows); pass 2 streams the rows again in chunks of kGroupCap, and the
// waves of the workgroup take turns in input order: a wave ranks its rows
// among equal residuals with wave ballots (wave_rank) on top of the running
// start of each r and advances it -- so equal keys keep their input order --
// and every row is stored straight to its place.  The join rows are then
// built from the two sorted output ranges (occurrence i of r in R with
// occurrence i in S, cpu_app.c:204-266) into the group's slot range, and
// counts[g] = their number, as the staged kernel does.
constexpr int kBgIt = kGroupCap / kMsdThreads;  // chunk rows per thread
#ifndef SMJ_BG_AGG
#define SMJ_BG_AGG 1  // bg_count: the wave's rows of its first residual counted by one atomic
#endif
#ifndef SMJ_BG_ABL
#define SMJ_BG_ABL 0  // timing ablation (output invalid): 1 = no counting pass, 2 = no row pass, 4 = no join rows
#endif
constexpr uint32_t kBgLarge = 8 * kGroupCap;  // groups over this many rows (either table) are dealt first
static_assert(kBgSeg % kGroupCap == 0 && kStRange % (4 * kMsdThreads) == 0, "giant jobs: whole chunks, uint4 counts");
constexpr int kBgIds = 256;     // compact residual ids of the parallel ranking (more distinct keys: the
                                // wave-serial ranking)
constexpr int kBgBlk = 2048;    // 64-row blocks of a row range a block table covers (131072 rows)
struct BgSmem {                 // 69 KiB: two workgroups per CU
    uint32_t end[2][kStRange];   // per residual: row count, then the running start of its output rows
    union {
        uint2 list[2][kGroupCap];    // per table: {tempB row, group row} of each pass-B tile's run
        uint32_t jst[kStRange + 1];  // once the rows are placed: the exclusive prefix over residuals of
                                     // min(countR, countS) (join rows)
    };
    uint8_t id[kStRange];        // residual -> compact id (the group's distinct residuals in order)
    uint16_t rid[kBgIds];        // compact id -> residual
    uint32_t wcnt[kMsdWaves][kBgIds];  // per wave and id: rows of the chunk, then their first output row
    uint16_t blk[2][kBgBlk];     // per table: the run holding row bv0 + 64 b (bg_blocks)
    uint32_t bv0[2], nblk[2];    // the rows the block table covers start at bv0 (nblk == 0: no table)
    uint32_t nid;                // distinct residuals (> kBgIds: wave-serial ranking)
    uint32_t nl[2];              // runs per table
    uint32_t wsum[kMsdWaves];
    uint32_t ticket;
};

__device__ __forceinline__ bool bg_dev(const MsdGroup &g) {  // sorted on the device (either kernel)
    return g.flags == kGroupBig && msd_big_on_device(g.span, g.kt[0], g.kt[1]);
}
__device__ __forceinline__ bool bg_giant(const MsdGroup &g, uint32_t bg_max) {  // by jobs (msd_giant_*)
    return bg_dev(g) && max(g.nR, g.nS) > bg_max;
}
__device__ __forceinline__ bool bg_ok(const MsdGroup &g, uint32_t bg_max) {  // by one workgroup (msd_big_stage_kernel)
    return bg_dev(g) && max(g.nR, g.nS) <= bg_max;
}

// wave_rank with 32-bit positions: pos[it] = wc[digit] + the row's rank among
// the wave's earlier rows of its digit (items in order, lanes in order);
// the wave's last row of each digit advances wc[digit]
template <int ITEMS, int DBITS>
__device__ __forceinline__ void bg_rank(const uint32_t (&dig)[ITEMS], uint32_t vmask, uint32_t *wc, int lane,
                                        uint32_t (&pos)[ITEMS]) {
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
            pos[it] = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, base));
            const uint64_t peers = ((uint64_t)phi << 32) | plo;
            if ((peers >> lane) == 1ull) wc[dd] = base + (uint32_t)__popcll(peers);
        }
    }
}

// row v of table x's group sequence: its tempB row (the last run starting at or before v)
__device__ __forceinline__ uint32_t bg_src(const uint2 *lst, uint32_t nl, uint32_t v) {
    uint32_t lo = 0, hi = nl - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (lst[mid].y <= v) lo = mid; else hi = mid - 1;
    }
    const uint2 e = lst[lo];
    return e.x + (v - e.y);
}

// O(1)-ish row -> run lookup for rows [v0, v1) of table X (after bg_lists):
// blk[b] = the run holding row v0 + 64 b; a lookup walks on from there over
// the runs starting inside the block (groups of Zipf tables: ~10-row runs)
__device__ __forceinline__ void bg_blocks(BgSmem &sm, int X, uint32_t n, uint32_t v0, uint32_t v1) {
    const int tid = threadIdx.x;
    const uint32_t nb = (v1 - v0 + 63) >> 6, nl = sm.nl[X];
    if (tid == 0) {
        sm.bv0[X] = v0;
        sm.nblk[X] = nb <= (uint32_t)kBgBlk ? nb : 0u;
    }
    if (nb <= (uint32_t)kBgBlk && v1 > v0) {
#pragma unroll
        for (int i = 0; i < kBgIt; i++) {
            const uint32_t j = (uint32_t)tid * kBgIt + i;
            if (j >= nl) continue;
            const uint32_t y0 = max(sm.list[X][j].y, v0), y1 = min(j + 1 < nl ? sm.list[X][j + 1].y : n, v1);
            if (y0 >= y1) continue;
            for (uint32_t b = (y0 - v0 + 63) >> 6; b <= (y1 - 1 - v0) >> 6; b++) sm.blk[X][b] = (uint16_t)j;
        }
    }
    __syncthreads();
}
__device__ __forceinline__ uint32_t bg_src_blk(const BgSmem &sm, int X, uint32_t v) {
    const uint2 *lst = sm.list[X];
    const uint32_t nl = sm.nl[X];
    if (sm.nblk[X]) {
        uint32_t j = sm.blk[X][(v - sm.bv0[X]) >> 6];
        for (int k = 0; k < 8 && j + 1 < nl && lst[j + 1].y <= v; k++) j++;
        if (!(j + 1 < nl && lst[j + 1].y <= v)) return lst[j].x + (v - lst[j].y);
    }
    return bg_src(lst, nl, v);
}

// the group's run list per table (one block scan each), then a barrier
__device__ __forceinline__ void bg_lists(const MsdFinalParams &p, const MsdGroup &g, BgSmem &sm) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        if (x >= p.ntab) break;
        const MsdTab &tb = p.tab[x];
        uint32_t src[kBgIt], len[kBgIt], sum = 0;
#pragma unroll
        for (int i = 0; i < kBgIt; i++) {
            const uint32_t j = (uint32_t)tid * kBgIt + i;
            src[i] = len[i] = 0;
            if (j < g.kt[x]) {
                const int64_t id = (int64_t)g.tb[x] + j;
                const uint32_t lo = tb.offs[id * kOffsB + g.b0], hi = tb.offs[id * kOffsB + g.b1];
                src[i] = (uint32_t)id * (uint32_t)tb.tile + lo;
                len[i] = hi - lo;
                if (SMJ_BOUNDS && (hi < lo || hi > (uint32_t)tb.tile)) {
                    atomicOr(&p.plan->err, 2u);
                    len[i] = 0;
                }
            }
            sum += len[i];
        }
        uint32_t total;
        uint32_t ex = block_excl_scan<kMsdWaves>(sum, sm.wsum, &total);
#pragma unroll
        for (int i = 0; i < kBgIt; i++) {
            const uint32_t j = (uint32_t)tid * kBgIt + i;
            if (j < g.kt[x]) sm.list[x][j] = make_uint2(src[i], ex);
            ex += len[i];
        }
        if (tid == 0) sm.nl[x] = g.kt[x];
    }
    __syncthreads();
}

// residual counts of rows [v0, v1) of table X into cnt (LDS atomics)
template <int X>
__device__ __forceinline__ void bg_count(const MsdFinalParams &p, const MsdGroup &g, uint32_t v0, uint32_t v1,
                                         BgSmem &sm, uint32_t *cnt) {
    constexpr int U = 4 * kBgIt;  // rows per thread in flight (four chunks): the pass is latency-bound
    const MsdTab &tb = p.tab[X];
    const i64x2 *tB = reinterpret_cast<const i64x2 *>(tb.tempB);
    const int tid = threadIdx.x;
    for (uint32_t c0 = v0; c0 < v1; c0 += U * kMsdThreads) {
        int64_t k[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            const uint32_t v = c0 + tid + i * kMsdThreads;
            k[i] = 0;
            if (v < v1) {
                const i64x2 r = tB[bg_src_blk(sm, X, v)];
                k[i] = tb.key ? r.y : r.x;
            }
        }
        // the rows of the wave's first active residual (Zipf groups: usually
        // the heavy key's) are counted by one atomic instead of colliding on
        // one LDS word, lane by lane
#pragma unroll
        for (int i = 0; i < U; i++) {
            const bool v = c0 + tid + i * kMsdThreads < v1;
            const uint32_t r = (uint32_t)((uint64_t)k[i] - (uint64_t)g.base);
            const uint64_t act = __ballot(v);
            if (act == 0) continue;
            const int lead = __ffsll((unsigned long long)act) - 1;
            const uint32_t r0 = (uint32_t)__shfl((int)r, lead, 64);
            const uint64_t same = __ballot(v && r == r0);
            if (SMJ_BG_AGG && v && r == r0) {
                if ((threadIdx.x & 63) == lead) atomicAdd(&cnt[r0], (uint32_t)__popcll(same));
            } else if (v) {
                atomicAdd(&cnt[r], 1u);
            }
        }
    }
}

// rows [v0, v1) of table X to their places: chunks in input order, the
// waves taking turns (wave-major, item, lane = input order within a chunk);
// end[r] = the next output row of residual r, advanced
template <int X>
__device__ __forceinline__ void bg_scatter(const MsdFinalParams &p, const MsdGroup &g, uint32_t v0, uint32_t v1,
                                           BgSmem &sm) {
    const MsdTab &tb = p.tab[X];
    const i64x2 *tB = reinterpret_cast<const i64x2 *>(tb.tempB);
    i64x2 *dst = reinterpret_cast<i64x2 *>(tb.out) + (X ? g.outS : g.outR);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the chunk's rows of this thread (input order: wave, item, lane)
    auto load = [&](uint32_t c0, i64x2 (&rows)[kBgIt], uint32_t &vm) {
        vm = 0;
#pragma unroll
        for (int i = 0; i < kBgIt; i++) {
            const uint32_t v = c0 + (uint32_t)(wave * kBgIt + i) * 64u + (uint32_t)lane;
            rows[i] = i64x2{0, 0};
            if (v < v1) {
                rows[i] = tB[bg_src_blk(sm, X, v)];
                vm |= 1u << i;
            }
        }
    };
    i64x2 cur[kBgIt];
    uint32_t vmask;
    load(v0, cur, vmask);
    for (uint32_t c0 = v0; c0 < v1; c0 += kGroupCap) {
        // the next chunk's rows are in flight while this one is ranked and stored
        i64x2 nxt[kBgIt];
        uint32_t vnext = 0;
        if (c0 + kGroupCap < v1) load(c0 + kGroupCap, nxt, vnext);
        uint32_t dig[kBgIt];
#pragma unroll
        for (int i = 0; i < kBgIt; i++)
            dig[i] = ((vmask >> i) & 1u) ? (uint32_t)((uint64_t)(tb.key ? cur[i].y : cur[i].x) - (uint64_t)g.base) : 0u;
        uint32_t pos[kBgIt];
        for (int w = 0; w < kMsdWaves; w++) {
            if (wave == w) bg_rank<kBgIt, 12>(dig, vmask, sm.end[X], lane, pos);
            __syncthreads();
        }
#pragma unroll
        for (int i = 0; i < kBgIt; i++)  // plain stores: a join read-back goes through L1
            if ((vmask >> i) & 1u) dst[pos[i]] = cur[i];
#pragma unroll
        for (int i = 0; i < kBgIt; i++) cur[i] = nxt[i];
        vmask = vnext;
    }
}

// compact ids of the group's distinct residuals (sm.end = the residual
// counts of both tables): id[r] = #{distinct residuals < r}, rid[id] = r,
// nid = their number.  Ends with a barrier.
__device__ __forceinline__ void bg_build_ids(BgSmem &sm) {
    constexpr int RP = kStRange / kMsdThreads;
    const int tid = threadIdx.x;
    uint32_t f = 0, sum = 0;
#pragma unroll
    for (int j = 0; j < RP; j++) {
        const int r = tid * RP + j;
        const bool nz = (sm.end[0][r] | sm.end[1][r]) != 0u;
        f |= nz ? (1u << j) : 0u;
        sum += nz ? 1u : 0u;
    }
    uint32_t all;
    uint32_t ex = block_excl_scan<kMsdWaves>(sum, sm.wsum, &all);
    if (all <= (uint32_t)kBgIds) {
#pragma unroll
        for (int j = 0; j < RP; j++)
            if ((f >> j) & 1u) {
                const int r = tid * RP + j;
                sm.id[r] = (uint8_t)ex;
                sm.rid[ex] = (uint16_t)r;
                ex++;
            }
    }
    if (tid == 0) sm.nid = all;
    __syncthreads();
}

// bg_scatter with the waves ranking in parallel (the group has <= kBgIds
// distinct residuals): per chunk of kGroupCap rows (input order = wave,
// item, lane) each wave ranks its rows by ballots on the 8-bit compact id and
// counts them per id; one thread per id then turns the per-wave counts into
// the waves' first output rows (running start end[r] + the earlier waves'
// rows) and advances end[r].  Two barriers per chunk instead of eight waves
// in turn.
// one chunk of kGroupCap rows of table X (rows in input order = wave, item,
// lane; vmask: valid items) to their places by the parallel ranking
template <int X>
__device__ __forceinline__ void bg_place_ids(const MsdFinalParams &p, const MsdGroup &g, const i64x2 (&cur)[kBgIt],
                                             uint32_t vmask, BgSmem &sm) {
    const MsdTab &tb = p.tab[X];
    i64x2 *dst = reinterpret_cast<i64x2 *>(tb.out) + (X ? g.outS : g.outR);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nid = sm.nid;
    uint32_t *wc = sm.wcnt[wave];
    for (int i = lane; i < kBgIds; i += 64) wc[i] = 0;  // this wave's counters (read by this wave only below)
    uint32_t dig[kBgIt], pos[kBgIt];
#pragma unroll
    for (int i = 0; i < kBgIt; i++)
        dig[i] = ((vmask >> i) & 1u)
                     ? (uint32_t)sm.id[(uint32_t)((uint64_t)(tb.key ? cur[i].y : cur[i].x) - (uint64_t)g.base)]
                     : 0u;
    bg_rank<kBgIt, 8>(dig, vmask, wc, lane, pos);  // pos = rank among the wave's rows of the id
    __syncthreads();
    if (tid < (int)nid) {  // id tid: the waves' first rows, then the running start advanced
        const uint32_t r = sm.rid[tid];
        uint32_t run = sm.end[X][r];
#pragma unroll
        for (int w = 0; w < kMsdWaves; w++) {
            const uint32_t c = sm.wcnt[w][tid];
            sm.wcnt[w][tid] = run;
            run += c;
        }
        sm.end[X][r] = run;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kBgIt; i++)
        if ((vmask >> i) & 1u) dst[wc[dig[i]] + pos[i]] = cur[i];
    // no barrier: a wave zeroes and reads only its own counter row, and the id
    // threads of the next chunk write after its first barrier
}

// row v of table X's group sequence, input-order mapping of chunk c0
template <int X>
__device__ __forceinline__ void bg_load_chunk(const MsdFinalParams &p, const BgSmem &sm, uint32_t c0, uint32_t v1,
                                              i64x2 (&rows)[kBgIt], uint32_t &vm) {
    const i64x2 *tB = reinterpret_cast<const i64x2 *>(p.tab[X].tempB);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    vm = 0;
#pragma unroll
    for (int i = 0; i < kBgIt; i++) {
        const uint32_t v = c0 + (uint32_t)(wave * kBgIt + i) * 64u + (uint32_t)lane;
        rows[i] = i64x2{0, 0};
        if (v < v1) {
            rows[i] = tB[bg_src_blk(sm, X, v)];
            vm |= 1u << i;
        }
    }
}

// bg_scatter with the waves ranking in parallel (the group has <= kBgIds
// distinct residuals): per chunk of kGroupCap rows (input order = wave,
// item, lane) each wave ranks its rows by ballots on the 8-bit compact id and
// counts them per id; one thread per id then turns the per-wave counts into
// the waves' first output rows (running start end[r] + the earlier waves'
// rows) and advances end[r].  Two barriers per chunk instead of eight waves
// in turn.
template <int X>
__device__ __forceinline__ void bg_scatter_ids(const MsdFinalParams &p, const MsdGroup &g, uint32_t v0, uint32_t v1,
                                               BgSmem &sm) {
    i64x2 cur[kBgIt];
    uint32_t vmask;
    bg_load_chunk<X>(p, sm, v0, v1, cur, vmask);
    for (uint32_t c0 = v0; c0 < v1; c0 += kGroupCap) {
        i64x2 nxt[kBgIt];  // the next chunk's rows are in flight while this one is ranked and stored
        uint32_t vnext = 0;
        if (c0 + kGroupCap < v1) bg_load_chunk<X>(p, sm, c0 + kGroupCap, v1, nxt, vnext);
        bg_place_ids<X>(p, g, cur, vmask, sm);
#pragma unroll
        for (int i = 0; i < kBgIt; i++) cur[i] = nxt[i];
        vmask = vnext;
    }
}

// join rows [j0, j1) of group g: row j of residual r (jst[r] <= j < jst[r + 1])
// pairs occurrence i = j - jst[r] of r in R and in S, whose sorted output
// rows start at startR(r), startS(r) (ends: those of r - 1)
__device__ __forceinline__ void bg_join(const MsdFinalParams &p, const MsdGroup &g, uint32_t j0, uint32_t j1,
                                        const BgSmem &sm, bool ends) {
    const i64x2 *oR = reinterpret_cast<const i64x2 *>(p.tab[0].out) + g.outR;
    const i64x2 *oS = reinterpret_cast<const i64x2 *>(p.tab[1].out) + g.outS;
    const int ks = p.tab[1].key;
    int64_t *slot = p.slots + (int64_t)g.outR * 3;
    for (uint32_t j = j0 + threadIdx.x; j < j1; j += kMsdThreads) {
        int lo = 0, hi = kStRange - 1;  // the residual of join row j: last r with jst[r] <= j
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (sm.jst[mid] <= j) lo = mid; else hi = mid - 1;
        }
        const uint32_t i = j - sm.jst[lo];
        const uint32_t sR = ends ? (lo ? sm.end[0][lo - 1] : 0u) : sm.end[0][lo];
        const uint32_t sS = ends ? (lo ? sm.end[1][lo - 1] : 0u) : sm.end[1][lo];
        const i64x2 rr = oR[sR + i], rs = oS[sS + i];
        slot[3 * (int64_t)j] = rr.x;
        slot[3 * (int64_t)j + 1] = rr.y;
        slot[3 * (int64_t)j + 2] = ks ? rs.x : rs.y;
    }
}

// per-residual counts c[x][r] in sm.end -> exclusive output starts, and
// min(cR, cS) -> the join-row prefix jst (jst[kStRange] = the join rows);
// returns the join rows.  Ends with a barrier.
__device__ __forceinline__ uint32_t bg_starts(BgSmem &sm, bool join, bool with_jst) {
    constexpr int RP = kStRange / kMsdThreads;
    const int tid = threadIdx.x;
    uint32_t c[3][RP], sum[3] = {0, 0, 0};
#pragma unroll
    for (int j = 0; j < RP; j++) {
        const int r = tid * RP + j;
        c[0][j] = sm.end[0][r];
        c[1][j] = sm.end[1][r];
        c[2][j] = join ? min(c[0][j], c[1][j]) : 0u;
#pragma unroll
        for (int q = 0; q < 3; q++) sum[q] += c[q][j];
    }
    uint32_t ex[3], tot[3];
#pragma unroll
    for (int q = 0; q < 3; q++) ex[q] = block_excl_scan<kMsdWaves>(sum[q], sm.wsum, &tot[q]);
#pragma unroll
    for (int j = 0; j < RP; j++) {
        const int r = tid * RP + j;
        sm.end[0][r] = ex[0];
        sm.end[1][r] = ex[1];
        if (with_jst) sm.jst[r] = ex[2];
#pragma unroll
        for (int q = 0; q < 3; q++) ex[q] += c[q][j];
    }
    if (tid == 0 && with_jst) sm.jst[kStRange] = tot[2];
    __syncthreads();
    return tot[2];
}

// after the rows are placed (sm.end = the end of each residual's rows): the
// join-row prefix jst, into the run lists' (now idle) region.  Ends with a barrier.
__device__ __forceinline__ void bg_jst_from_ends(BgSmem &sm) {
    constexpr int RP = kStRange / kMsdThreads;
    const int tid = threadIdx.x;
    uint32_t c[RP], sum = 0;
    uint32_t pR = tid ? sm.end[0][tid * RP - 1] : 0u, pS = tid ? sm.end[1][tid * RP - 1] : 0u;
#pragma unroll
    for (int j = 0; j < RP; j++) {
        const int r = tid * RP + j;
        const uint32_t eR = sm.end[0][r], eS = sm.end[1][r];
        c[j] = min(eR - pR, eS - pS);
        pR = eR;
        pS = eS;
        sum += c[j];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan<kMsdWaves>(sum, sm.wsum, &tot);  // (its barriers: the run lists are dead)
#pragma unroll
    for (int j = 0; j < RP; j++) {
        sm.jst[tid * RP + j] = ex;
        ex += c[j];
    }
    if (tid == 0) sm.jst[kStRange] = tot;
    __syncthreads();
}

// SMJ_STAMPS builds, p.dbg bit 5: cycles per oversized group by size class
// (log2 of its larger table's rows: [0..31]), groups per class, and cycles per
// phase (lists, count, starts, scatter, join) -> smj_debug_big_times
__device__ unsigned long long g_bg_cls[2][32], g_bg_ph[8];
#define BG_STAMP(k)                                                              \
    if (SMJ_STAMPS && (p.dbg & 32) && tid == 0) {                                \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
        atomicAdd(&g_bg_ph[k], t_ - bg_t);                                       \
        bg_t = t_;                                                               \
    }

__global__ __launch_bounds__(kMsdThreads, 2) void msd_big_stage_kernel(const MsdFinalParams p) {
    __shared__ BgSmem sm;
    if (msd_plan_failed(p.plan)) return;
    const uint32_t nbig = p.plan->nbig;
    const int tid = threadIdx.x;
    const bool join = p.join && p.ntab > 1;
    unsigned long long bg_t = 0, bg_g = 0;
    // dynamic tickets over the (unordered) list, twice: the groups over
    // kBgLarge rows first, so that the longest ones do not start last
    for (int round = 0; round < 2; round++)
    for (;;) {
        __syncthreads();  // LDS of the previous group / ticket read out
        if (tid == 0) sm.ticket = atomicAdd(&p.plan->bgticket[round], 1u);
        __syncthreads();
        const uint32_t bi = sm.ticket;
        if (bi >= nbig) break;
        const uint32_t gi = p.big_list[bi];
        const MsdGroup g = p.groups[gi];
        if (round == 0 && bg_giant(g, p.bg_max)) {  // over kBgMaxRows rows: split into jobs (msd_giant_*)
            const uint32_t nseg = (max(g.nR, p.ntab > 1 ? g.nS : 0u) + p.bg_seg - 1) / p.bg_seg;
            if (tid == 0) {
                const uint32_t base = atomicAdd(&p.plan->njobs, nseg), idx = atomicAdd(&p.plan->ngiant, 1u);
                p.giant[idx] = make_uint4(gi, base, nseg, 0u);
                sm.ticket = base;
                sm.nl[0] = idx;
            }
            __syncthreads();
            for (uint32_t k = tid; k < nseg; k += kMsdThreads) p.gmap[sm.ticket + k] = sm.nl[0];
            continue;
        }
        if (!bg_ok(g, p.bg_max)) continue;  // block-uniform: a giant, or left to the host fallback
        if ((max(g.nR, g.nS) > kBgLarge) != (round == 0)) continue;
        if (SMJ_STAMPS && (p.dbg & 32) && tid == 0) bg_g = bg_t = __builtin_amdgcn_s_memtime();
        for (int i = tid; i < 2 * kStRange; i += kMsdThreads) (&sm.end[0][0])[i] = 0;
        bg_lists(p, g, sm);
        bg_blocks(sm, 0, g.nR, 0, g.nR);
        if (p.ntab > 1) bg_blocks(sm, 1, g.nS, 0, g.nS);
        BG_STAMP(0);
        if (!(SMJ_BG_ABL & 1)) {  // pass 1: residual counts of both tables
            bg_count<0>(p, g, 0, g.nR, sm, sm.end[0]);
            if (p.ntab > 1) bg_count<1>(p, g, 0, g.nS, sm, sm.end[1]);
        }
        __syncthreads();
        BG_STAMP(1);
        bg_build_ids(sm);
        const uint32_t J = bg_starts(sm, join, false);
        if (tid == 0) {
            p.counts[gi] = J;
            atomicAdd(&p.plan->nbigdev, 1u);
        }
        BG_STAMP(2);
        if (!(SMJ_BG_ABL & 2)) {  // pass 2
            if (sm.nid <= (uint32_t)kBgIds) {
                bg_scatter_ids<0>(p, g, 0, g.nR, sm);
                if (p.ntab > 1) bg_scatter_ids<1>(p, g, 0, g.nS, sm);
            } else {
                bg_scatter<0>(p, g, 0, g.nR, sm);
                if (p.ntab > 1) bg_scatter<1>(p, g, 0, g.nS, sm);
            }
        }
        BG_STAMP(3);
        if (join && !(SMJ_BG_ABL & 4)) {  // join rows from the sorted output ranges (written above by this workgroup)
            // workgroup scope is enough: only this workgroup's own rows are read
            // back, from the CU that wrote them.  (__threadfence()'s agent scope
            // writes back the XCD's whole L2 on gfx950 -- 20 of C5's ms.)
            __threadfence_block();
            __syncthreads();
            bg_jst_from_ends(sm);
            bg_join(p, g, 0, J, sm, true);
        }
        BG_STAMP(4);
        if (SMJ_STAMPS && (p.dbg & 32) && tid == 0) {
            const int c = 31 - __clz(max(max(g.nR, g.nS), 1u));
            atomicAdd(&g_bg_cls[0][c], bg_t - bg_g);
            atomicAdd(&g_bg_cls[1][c], 1ull);
        }
    }
}

hipError_t read_big_times(unsigned long long *out72) {
    hipError_t e = hipMemcpyFromSymbol(out72, HIP_SYMBOL(g_bg_cls), sizeof(g_bg_cls));
    if (e != hipSuccess) return e;
    e = hipMemcpyFromSymbol(out72 + 64, HIP_SYMBOL(g_bg_ph), sizeof(g_bg_ph));
    if (e != hipSuccess) return e;
    static const unsigned long long z[64] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_bg_cls), z, sizeof(g_bg_cls));
    return hipMemcpyToSymbol(HIP_SYMBOL(g_bg_ph), z, sizeof(g_bg_ph));
}

// Groups over kBgMaxRows rows (the largest Zipf groups: up to ~1e6 rows, one
// workgroup would take ~17 ms): the same counting sort split into jobs of
// kBgSeg rows per table, in three launches -- per-job residual counts to
// global memory (gh[job][table][r]); each job's output starts (the group's
// totals scanned + the counts of its earlier jobs) and its rows scattered;
// the join rows, kBgSeg per job.  Jobs of one group are numbered
// giant[i].y + s; gmap[job] = i.
struct GiantJob {
    uint32_t gi, s, nseg, job0;
};
__device__ __forceinline__ GiantJob giant_job(const MsdFinalParams &p, uint32_t t) {
    const uint4 e = p.giant[p.gmap[t]];
    return GiantJob{e.x, t - e.y, e.z, e.y};
}

__global__ __launch_bounds__(kMsdThreads, 2) void msd_giant_count_kernel(const MsdFinalParams p) {
    __shared__ BgSmem sm;
    if (msd_plan_failed(p.plan)) return;
    const uint32_t nj = p.plan->njobs;
    for (uint32_t t = blockIdx.x; t < nj; t += gridDim.x) {
        const GiantJob jb = giant_job(p, t);
        const MsdGroup g = p.groups[jb.gi];
        for (int i = threadIdx.x; i < 2 * kStRange; i += kMsdThreads) (&sm.end[0][0])[i] = 0;
        bg_lists(p, g, sm);
        const uint32_t v0 = jb.s * p.bg_seg;
        bg_blocks(sm, 0, g.nR, min(v0, g.nR), min(v0 + p.bg_seg, g.nR));
        if (p.ntab > 1) bg_blocks(sm, 1, g.nS, min(v0, g.nS), min(v0 + p.bg_seg, g.nS));
        bg_count<0>(p, g, min(v0, g.nR), min(v0 + p.bg_seg, g.nR), sm, sm.end[0]);
        if (p.ntab > 1) bg_count<1>(p, g, min(v0, g.nS), min(v0 + p.bg_seg, g.nS), sm, sm.end[1]);
        __syncthreads();
        uint32_t *h = p.gh + (int64_t)t * 2 * kStRange;
        for (int i = threadIdx.x; i < 2 * kStRange; i += kMsdThreads) h[i] = (&sm.end[0][0])[i];
        __syncthreads();
    }
}

// the group's residual totals (all its jobs) into sm.end, and into pre[x][r]
// (per thread: residuals tid * RP + j) the counts of the jobs before s
__device__ __forceinline__ void giant_totals(const MsdFinalParams &p, const GiantJob &jb, BgSmem &sm,
                                             uint32_t (&pre)[2][kStRange / kMsdThreads]) {
    constexpr int RP = kStRange / kMsdThreads;
    const int tid = threadIdx.x;
#pragma unroll
    for (int x = 0; x < 2; x++) {
        uint32_t tot[RP];
#pragma unroll
        for (int j = 0; j < RP; j++) tot[j] = pre[x][j] = 0;
        for (uint32_t q = 0; q < jb.nseg; q++) {
            const uint4 *h = reinterpret_cast<const uint4 *>(p.gh + ((int64_t)(jb.job0 + q) * 2 + x) * kStRange) + tid * (RP / 4);
#pragma unroll
            for (int u = 0; u < RP / 4; u++) {
                const uint4 v = h[u];
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    tot[4 * u + k] += w[k];
                    if (q < jb.s) pre[x][4 * u + k] += w[k];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < RP; j++) sm.end[x][tid * RP + j] = tot[j];
    }
    __syncthreads();
}

__global__ __launch_bounds__(kMsdThreads, 2) void msd_giant_scatter_kernel(const MsdFinalParams p) {
    __shared__ BgSmem sm;
    constexpr int RP = kStRange / kMsdThreads;
    if (msd_plan_failed(p.plan)) return;
    const uint32_t nj = p.plan->njobs;
    const bool join = p.join && p.ntab > 1;
    for (uint32_t t = blockIdx.x; t < nj; t += gridDim.x) {
        const GiantJob jb = giant_job(p, t);
        const MsdGroup g = p.groups[jb.gi];
        uint32_t pre[2][RP];
        giant_totals(p, jb, sm, pre);
        bg_build_ids(sm);
        bg_starts(sm, join, false);
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int j = 0; j < RP; j++) sm.end[x][threadIdx.x * RP + j] += pre[x][j];
        bg_lists(p, g, sm);  // (its barrier also orders the starts above)
        const uint32_t v0 = jb.s * p.bg_seg;
        bg_blocks(sm, 0, g.nR, min(v0, g.nR), min(v0 + p.bg_seg, g.nR));
        if (p.ntab > 1) bg_blocks(sm, 1, g.nS, min(v0, g.nS), min(v0 + p.bg_seg, g.nS));
        if (sm.nid <= (uint32_t)kBgIds) {
            bg_scatter_ids<0>(p, g, min(v0, g.nR), min(v0 + p.bg_seg, g.nR), sm);
            if (p.ntab > 1) bg_scatter_ids<1>(p, g, min(v0, g.nS), min(v0 + p.bg_seg, g.nS), sm);
        } else {
            bg_scatter<0>(p, g, min(v0, g.nR), min(v0 + p.bg_seg, g.nR), sm);
            if (p.ntab > 1) bg_scatter<1>(p, g, min(v0, g.nS), min(v0 + p.bg_seg, g.nS), sm);
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kMsdThreads, 2) void msd_giant_join_kernel(const MsdFinalParams p) {
    __shared__ BgSmem sm;
    constexpr int RP = kStRange / kMsdThreads;
    if (msd_plan_failed(p.plan)) return;
    const uint32_t nj = p.plan->njobs;
    const bool join = p.join && p.ntab > 1;
    for (uint32_t t = blockIdx.x; t < nj; t += gridDim.x) {
        const GiantJob jb = giant_job(p, t);
        const MsdGroup g = p.groups[jb.gi];
        uint32_t pre[2][RP];
        giant_totals(p, jb, sm, pre);
        const uint32_t J = bg_starts(sm, join, true);  // sm.end = the starts
        if (jb.s == 0 && threadIdx.x == 0) {
            p.counts[jb.gi] = J;
            atomicAdd(&p.plan->nbigdev, 1u);
        }
        const uint32_t j0 = jb.s * p.bg_seg;
        if (join && j0 < J) bg_join(p, g, j0, min(J, j0 + p.bg_seg), sm, false);
        __syncthreads();
    }
}

static const unsigned long long zero8_pb[8] = {0};
hipError_t read_msd_phases(unsigned long long *out16) {
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_fin_phase), sizeof(unsigned long long) * 10);
    if (e != hipSuccess) return e;
    e = hipMemcpyFromSymbol(out16 + 10, HIP_SYMBOL(g_st_sub), sizeof(unsigned long long) * 6);
    if (e != hipSuccess) return e;
    e = hipMemcpyFromSymbol(out16 + 16, HIP_SYMBOL(g_pb_phase), sizeof(unsigned long long) * 8);
    if (e != hipSuccess) return e;
    hipMemcpyToSymbol(HIP_SYMBOL(g_pb_phase), zero8_pb, sizeof(zero8_pb));
    static const unsigned long long zero8[8] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_st_sub), zero8, sizeof(zero8));
    static const unsigned long long zero[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_fin_phase), zero, sizeof(zero));
}

// ---------------------------------------------------------------------------
// single-key oversized groups: already in stable order; copy and zip
// ---------------------------------------------------------------------------
// row ix of table tb's pass-B rows: a packed word (MsdPlan::packB, pk) rebuilt
// from group g's base, or the 16-B row
__device__ __forceinline__ i64x2 pb_row(const MsdTab &tb, const MsdGroup &g, int64_t ix, bool pk) {
    if (!pk) return reinterpret_cast<const i64x2 *>(tb.tempB)[ix];
    const uint64_t w = reinterpret_cast<const uint64_t *>(tb.tempB)[ix];
    const int64_t key = g.base + (int64_t)(uint32_t)((uint32_t)w - (uint32_t)g.base);
    const int64_t oth = (int64_t)(int32_t)(uint32_t)(w >> 32);
    return tb.key ? i64x2{oth, key} : i64x2{key, oth};
}

// grid = work items (dense group, chunk of kGroupCap group rows).  With
// p.pk_mode == 3 the pass-B rows are packed words (2-column tables), read
// and rebuilt here (no unpacked copy for this tier)
template <int C1, int C2>
__global__ __launch_bounds__(kMsdThreads) void msd_single_kernel(const MsdFinalParams p, const uint2 *work) {
    __shared__ uint64_t s_tmp[kGroupCap];
    __shared__ uint32_t s_addr[2][kGroupCap];
    __shared__ uint32_t s_wsum[kMsdWaves];
    if (msd_plan_failed(p.plan)) return;
    const uint2 w = work[blockIdx.x];
    const MsdGroup g = p.groups[w.x];
    const int tid = threadIdx.x;
    if (w.y & kSingleRuns) {
        // a heavy key's sub-bucket b0 of a multi-key bucket (msd_heavy_kernel):
        // rows [V0, V1) of each table, kSingleRunRows a work item.  The group's
        // rows are one run per pass-B tile of the bucket; the runs' places are
        // the prefix of the earlier runs (a scan of their offsB lengths), and
        // the runs meeting [V0, V1) are copied run by run (a wave per run,
        // coalesced) -- no per-row search.  The zip join is read back from
        // the sorted rows just written (workgroup fence).
        uint2 *s_run = reinterpret_cast<uint2 *>(s_tmp);  // {tempB row, output row} per tile of a batch
        uint32_t *s_len = s_addr[0];
        const int lane = tid & 63, wave = tid >> 6;
        const uint32_t V0 = (w.y & ~kSingleRuns) * kSingleRunRows;
#pragma unroll
        for (int x = 0; x < 2; x++) {
            const uint32_t nx = x ? (p.ntab > 1 ? g.nS : 0u) : g.nR;
            if (V0 >= nx) continue;
            const uint32_t V1 = min(V0 + kSingleRunRows, nx);
            const MsdTab &tb = p.tab[x];
            const int cols = C1 > 0 ? (x ? C2 : C1) : tb.cols;
            const MsdBucket bk = tb.bk[g.a];
            const uint32_t K = (bk.L + (uint32_t)tb.tile - 1) / (uint32_t)tb.tile;
            int64_t *dst = tb.out + (int64_t)(x ? g.outS : g.outR) * cols;
            uint32_t carry = 0;
            for (uint32_t kb = 0; kb < K && carry < V1; kb += kMsdThreads) {
                const uint32_t nb = min(K - kb, (uint32_t)kMsdThreads);
                uint32_t len = 0, src = 0;
                if ((uint32_t)tid < nb) {
                    const int64_t id = (int64_t)bk.tile_base + kb + tid;
                    const uint32_t lo = tb.offs[id * kOffsB + g.b0], hi = tb.offs[id * kOffsB + g.b1];
                    src = (uint32_t)id * (uint32_t)tb.tile + lo;
                    len = hi - lo;
                }
                uint32_t total;
                const uint32_t ex = carry + block_excl_scan<kMsdWaves>(len, s_wsum, &total);
                if ((uint32_t)tid < nb) {
                    s_run[tid] = make_uint2(src, ex);
                    s_len[tid] = len;
                }
                __syncthreads();
                for (uint32_t j = (uint32_t)wave; j < nb; j += kMsdWaves) {
                    const uint2 e = s_run[j];
                    const uint32_t r0 = e.y < V0 ? V0 - e.y : 0u, r1 = min(s_len[j], V1 > e.y ? V1 - e.y : 0u);
                    for (uint32_t r = r0 + (uint32_t)lane; r < r1; r += 64) {
                        if constexpr (C1 == 2 && C2 == 2) {
                            reinterpret_cast<i64x2 *>(dst)[e.y + r] = pb_row(tb, g, (int64_t)(e.x + r), p.pk_mode == 3);
                        } else if constexpr (C1 > 0) {
                            if (x) copy_row<C2>(tb.tempB + (int64_t)(e.x + r) * C2, dst + (int64_t)(e.y + r) * C2, C2);
                            else copy_row<C1>(tb.tempB + (int64_t)(e.x + r) * C1, dst + (int64_t)(e.y + r) * C1, C1);
                        } else {
                            copy_row<0>(tb.tempB + (int64_t)(e.x + r) * cols, dst + (int64_t)(e.y + r) * cols, cols);
                        }
                    }
                }
                carry += total;
                __syncthreads();
            }
        }
        if (!p.join) return;
        const uint32_t m = min(g.nR, p.ntab > 1 ? g.nS : 0u);
        if (V0 >= m) return;
        __threadfence_block();  // the sorted rows written above, visible to the whole workgroup
        __syncthreads();
        const uint32_t V1 = min(V0 + kSingleRunRows, m);
        const int c1 = C1 > 0 ? C1 : p.tab[0].cols, c2 = C2 > 0 ? C2 : p.tab[1].cols, tc = c1 + c2 - 1;
        const int64_t *oR = p.tab[0].out + (int64_t)g.outR * c1, *oS = p.tab[1].out + (int64_t)g.outS * c2;
        int64_t *dj = p.slots + (int64_t)g.outR * tc;
        for (uint32_t v = V0 + tid; v < V1; v += kMsdThreads)
            emit_join_row<C1, C2>(oR + (int64_t)v * c1, oS + (int64_t)v * c2, dj + (int64_t)v * tc, c1, c2, p.key2);
        return;
    }
    const uint32_t V0 = w.y * (uint32_t)kGroupCap;
    const uint32_t n[2] = {g.nR, p.ntab > 1 ? g.nS : 0u};
    uint2 *s_list = reinterpret_cast<uint2 *>(s_tmp);
#pragma unroll
    for (int x = 0; x < 2; x++) {
        if (V0 >= n[x]) continue;
        const uint32_t V1 = min(V0 + (uint32_t)kGroupCap, n[x]);
        group_gather(p.tab[x], g, V0, V1, s_list, s_wsum, [&](uint32_t v, uint32_t src) { s_addr[x][v - V0] = src; });
    }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; x++) {
        if (V0 >= n[x]) continue;
        const MsdTab &tb = p.tab[x];
        const int cols = C1 > 0 ? (x ? C2 : C1) : tb.cols;
        const uint32_t V1 = min(V0 + (uint32_t)kGroupCap, n[x]);
        int64_t *dst = tb.out + (int64_t)(x ? g.outS : g.outR) * cols;
        for (uint32_t v = V0 + tid; v < V1; v += kMsdThreads) {
            const uint32_t src = s_addr[x][v - V0];
            if constexpr (C1 == 2 && C2 == 2) {
                reinterpret_cast<i64x2 *>(dst)[v] = pb_row(tb, g, (int64_t)src, p.pk_mode == 3);
            } else if constexpr (C1 > 0) {
                if (x) copy_row<C2>(tb.tempB + (int64_t)src * C2, dst + (int64_t)v * C2, C2);
                else copy_row<C1>(tb.tempB + (int64_t)src * C1, dst + (int64_t)v * C1, C1);
            } else {
                copy_row<0>(tb.tempB + (int64_t)src * cols, dst + (int64_t)v * cols, cols);
            }
        }
    }
    if (!p.join) return;
    const uint32_t m = min(n[0], n[1]);
    if (V0 >= m) return;
    const uint32_t V1 = min(V0 + (uint32_t)kGroupCap, m);
    const int c1 = C1 > 0 ? C1 : p.tab[0].cols, c2 = C2 > 0 ? C2 : p.tab[1].cols, tc = c1 + c2 - 1;
    int64_t *dst = p.slots + (int64_t)g.outR * tc;
    for (uint32_t v = V0 + tid; v < V1; v += kMsdThreads) {
        if constexpr (C1 == 2 && C2 == 2) {
            if (p.pk_mode == 3) {  // packed rows: rebuilt (emit_join_row's 2-column layout)
                const i64x2 rv = pb_row(p.tab[0], g, (int64_t)s_addr[0][v - V0], true);
                const i64x2 sv = pb_row(p.tab[1], g, (int64_t)s_addr[1][v - V0], true);
                int64_t *d = dst + (int64_t)v * tc;
                d[0] = rv.x;
                d[1] = rv.y;
                d[2] = p.key2 ? sv.x : sv.y;
                continue;
            }
        }
        emit_join_row<C1, C2>(p.tab[0].tempB + (int64_t)s_addr[0][v - V0] * c1,
                              p.tab[1].tempB + (int64_t)s_addr[1][v - V0] * c2, dst + (int64_t)v * tc, c1, c2,
                              p.key2);
    }
}

// Batched fallback for oversized multi-key groups (smj_api.hip msd_fallback):
// the groups are disjoint key ranges in key order, so gathering all of them
// (in group order) into one buffer, one stable sort of that buffer and one
// zip join of the two sorted buffers give every group's sort and join at once.
// work item = {dense group, first group row V0 of the chunk, buffer row of V0, -}
__global__ __launch_bounds__(kMsdThreads) void msd_gather_list_kernel(const MsdTab tb, const MsdGroup *groups,
                                                                      const uint4 *work, int64_t *dst) {
    __shared__ uint64_t s_tmp[kGroupCap];
    __shared__ uint32_t s_wsum[kMsdWaves];
    const uint4 w = work[blockIdx.x];
    const MsdGroup g = groups[w.x];
    const uint32_t nx = tb.x ? g.nS : g.nR;
    const uint32_t V0 = w.y, V1 = min(V0 + (uint32_t)kGroupCap, nx);
    const int64_t d0 = w.z;
    group_gather(tb, g, V0, V1, reinterpret_cast<uint2 *>(s_tmp), s_wsum, [&](uint32_t v, uint32_t src) {
        copy_row<0>(tb.tempB + (int64_t)src * tb.cols, dst + (d0 + (v - V0)) * tb.cols, tb.cols);
    });
}

// the host fallback's view of the oversized groups: out[i] = groups[list[i]]
// for the nsingle single-key then nbig oversized list entries (copied to the
// host instead of every dense group record)
__global__ __launch_bounds__(256) void msd_pick_groups_kernel(const MsdGroup *__restrict__ groups,
                                                              const uint32_t *__restrict__ single_list,
                                                              const uint32_t *__restrict__ big_list, uint32_t nsingle,
                                                              uint32_t nbig, MsdGroup *__restrict__ out) {
    constexpr int W = sizeof(MsdGroup) / 8;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one 8-B word of one record
    const int64_t r = i / W;
    if (r >= (int64_t)nsingle + nbig) return;
    const uint32_t slot = r < nsingle ? single_list[r] : big_list[r - nsingle];
    reinterpret_cast<int64_t *>(out)[i] = reinterpret_cast<const int64_t *>(groups + slot)[i % W];
}
hipError_t launch_msd_pick_groups(const MsdGroup *groups, const uint32_t *single_list, const uint32_t *big_list,
                                  uint32_t nsingle, uint32_t nbig, MsdGroup *out, hipStream_t s) {
    const int64_t words = ((int64_t)nsingle + nbig) * (int64_t)(sizeof(MsdGroup) / 8);
    if (words == 0) return hipSuccess;
    hipLaunchKernelGGL(msd_pick_groups_kernel, dim3(blocks_for(words, 256)), dim3(256), 0, s, groups, single_list,
                       big_list, nsingle, nbig, out);
    return hipGetLastError();
}

// work item = {source row, destination row, rows, -}: contiguous row runs
__global__ __launch_bounds__(256) void msd_seg_copy_kernel(const int64_t *__restrict__ src, int64_t *__restrict__ dst,
                                                           const uint4 *work, int cols) {
    const uint4 w = work[blockIdx.x];
    const int64_t *a = src + (int64_t)w.x * cols;
    int64_t *b = dst + (int64_t)w.y * cols;
    const int64_t words = (int64_t)w.z * cols;
    for (int64_t i = threadIdx.x; i < words; i += 256) b[i] = a[i];
}

// first index in [0, n) whose key is >= k (upper: > k)
__device__ __forceinline__ int64_t key_bound(const int64_t *J, int64_t n, int tc, int kc, int64_t k, bool upper) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int64_t v = J[mid * tc + kc];
        if (upper ? v <= k : v < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// one workgroup per oversized group: its join rows are the rows of the
// batched join J whose key lies in [first, last] of the group's sorted R rows;
// copied to the group's slot rows, their number to counts.
// work item = {dense group, first row of the group in the sorted R buffer, nR, nS}
__global__ __launch_bounds__(256) void msd_big_split_kernel(const int64_t *__restrict__ J, const int64_t *nJp, int tc,
                                                            const int64_t *__restrict__ Rs, int c1, int key1,
                                                            const uint4 *work, const MsdGroup *groups,
                                                            int64_t *__restrict__ slots, uint32_t *counts) {
    const uint4 w = work[blockIdx.x];
    if (w.z == 0 || w.w == 0) {
        if (threadIdx.x == 0) counts[w.x] = 0;
        return;
    }
    const int64_t nJ = *nJp;
    const int64_t kmin = Rs[(int64_t)w.y * c1 + key1], kmax = Rs[((int64_t)w.y + w.z - 1) * c1 + key1];
    const int64_t lo = key_bound(J, nJ, tc, key1, kmin, false), hi = key_bound(J, nJ, tc, key1, kmax, true);
    if (threadIdx.x == 0) counts[w.x] = (uint32_t)(hi - lo);
    const int64_t *a = J + lo * tc;
    int64_t *b = slots + (int64_t)groups[w.x].outR * tc;
    const int64_t words = (hi - lo) * tc;
    for (int64_t i = threadIdx.x; i < words; i += 256) b[i] = a[i];
}

// pack the join slots: dense group g has counts[g] rows at slot row outR.
// One wave per group (persistent over the groups), 8 words per lane in
// flight per round; the next group's count / slot / offset are loaded while
// this one is copied.  Groups over kGroupCap join rows (only oversized ones
// have them) are left to msd_compact_big_kernel; the speculative launch
// before the fallback (after_fallback == 0) does nothing when the plan has
// oversized groups, as the launch after it packs everything.
__global__ __launch_bounds__(256) void msd_compact_kernel(const int64_t *__restrict__ slots,
                                                          const MsdGroup *__restrict__ groups,
                                                          const uint32_t *__restrict__ counts,
                                                          const uint32_t *__restrict__ offs,
                                                          const MsdPlan *__restrict__ plan, int tc,
                                                          int64_t *__restrict__ out, int after_fallback) {
    constexpr int U = 8;
    const int lane = threadIdx.x & 63;
    if (msd_plan_failed(plan)) return;
    // (speculative call: a no-op while some groups' counts are still to come --
    // the host-driven tiers' groups, and the final tiers launched by msd_back)
    if (!after_fallback && plan->nsingle + plan->nbig + plan->nradix + plan->nwst > 0) return;
    const int64_t ng = plan->ngroups, step = (int64_t)gridDim.x * 4;
    int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= ng) return;
    auto cnt = [&](int64_t i) {
        const uint32_t c = counts[i];
        return c > (uint32_t)kGroupCap ? 0u : c;
    };
    uint32_t c = cnt(g), o = offs[g], r = groups[g].outR;
    for (; g < ng; g += step) {
        const int64_t gn = g + step;
        uint32_t cn = 0, on = 0, rn = 0;
        if (gn < ng) {
            cn = cnt(gn);
            on = offs[gn];
            rn = groups[gn].outR;
        }
        const int64_t nw = (int64_t)c * tc;
        const int64_t *src = slots + (int64_t)r * tc;
        int64_t *dst = out + (int64_t)o * tc;
        for (int64_t i0 = 0; i0 < nw; i0 += 64 * U) {
            int64_t v[U];
#pragma unroll
            for (int k = 0; k < U; k++) {
                const int64_t i = i0 + k * 64 + lane;
                if (i < nw) v[k] = src[i];
            }
#pragma unroll
            for (int k = 0; k < U; k++) {
                const int64_t i = i0 + k * 64 + lane;
                if (i < nw) dst[i] = v[k];
            }
        }
        c = cn;
        o = on;
        r = rn;
    }
}

// the groups with more than kGroupCap join rows, in chunks: work item =
// {dense group, chunk}; chunks past the group's count (the host sizes the
// list by min(nR, nS)) and groups at or under kGroupCap do nothing
__global__ __launch_bounds__(256) void msd_compact_big_kernel(const int64_t *__restrict__ slots,
                                                              const MsdGroup *__restrict__ groups,
                                                              const uint32_t *__restrict__ counts,
                                                              const uint32_t *__restrict__ offs, const uint2 *work,
                                                              int tc, int64_t *__restrict__ out) {
    const uint2 w = work[blockIdx.x];
    const uint32_t c = counts[w.x], v0 = w.y * kCompactChunk;
    if (c <= (uint32_t)kGroupCap || v0 >= c) return;
    const uint32_t v1 = min(c, v0 + kCompactChunk);
    const int64_t *src = slots + ((int64_t)groups[w.x].outR + v0) * tc;
    int64_t *dst = out + ((int64_t)offs[w.x] + v0) * tc;
    const int64_t nw = (int64_t)(v1 - v0) * tc;
    for (int64_t i = threadIdx.x; i < nw; i += 256) dst[i] = src[i];
}

// exclusive scan of the dense group counts in two launches over chunks of
// kCountChunk groups (256 threads x 16): msd_count_part_kernel sums each
// chunk, msd_count_scan_kernel adds the sums of the chunks before its own
// (one wave) and scans its chunk; the chunk holding the last group writes
// plan->joined = total.  grid kCountChunks x 256 (chunks past ngroups exit).
constexpr int kCountPer = 16, kCountChunk = 256 * kCountPer;
constexpr int kCountChunks = (kSlots + kCountChunk - 1) / kCountChunk;
static_assert(kCountChunks <= 256, "one wave (<= 4 sums per lane) adds the earlier chunks");
__device__ __forceinline__ void count_load(const uint32_t *counts, int64_t ng, int64_t i0, uint32_t (&v)[kCountPer]) {
    if (i0 + kCountPer <= ng) {
        const uint4 *c4 = reinterpret_cast<const uint4 *>(counts + i0);
#pragma unroll
        for (int q = 0; q < kCountPer / 4; q++) {
            const uint4 u = c4[q];
            v[4 * q] = u.x;
            v[4 * q + 1] = u.y;
            v[4 * q + 2] = u.z;
            v[4 * q + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kCountPer; k++) v[k] = i0 + k < ng ? counts[i0 + k] : 0u;
    }
}

__global__ __launch_bounds__(256) void msd_count_part_kernel(const uint32_t *__restrict__ counts,
                                                             uint32_t *__restrict__ part, const MsdPlan *plan) {
    __shared__ uint32_t s_w[4];
    if (msd_plan_failed(plan)) return;
    const int64_t ng = plan->ngroups, c0 = (int64_t)blockIdx.x * kCountChunk;
    if (c0 >= ng) return;
    const int tid = threadIdx.x, lane = tid & 63;
    uint32_t v[kCountPer], sum = 0;
    count_load(counts, ng, c0 + (int64_t)tid * kCountPer, v);
#pragma unroll
    for (int k = 0; k < kCountPer; k++) sum += v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) s_w[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0) part[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ __launch_bounds__(256) void msd_count_scan_kernel(const uint32_t *__restrict__ counts,
                                                             const uint32_t *__restrict__ part,
                                                             uint32_t *__restrict__ offs, MsdPlan *plan) {
    __shared__ uint32_t s_w[4], s_base;
    if (msd_plan_failed(plan)) return;
    const int64_t ng = plan->ngroups, c0 = (int64_t)blockIdx.x * kCountChunk;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (ng == 0) {
        if (blockIdx.x == 0 && tid == 0) plan->joined = 0;
        return;
    }
    if (c0 >= ng) return;
    const int64_t i0 = c0 + (int64_t)tid * kCountPer;
    uint32_t v[kCountPer], sum = 0;
    count_load(counts, ng, i0, v);
    if (wave == 0) {
        const int b = (int)blockIdx.x;
        uint32_t e = 0;
#pragma unroll
        for (int q = 0; q < (kCountChunks + 63) / 64; q++) e += lane + 64 * q < b ? part[lane + 64 * q] : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
        if (lane == 0) s_base = e;
    }
#pragma unroll
    for (int k = 0; k < kCountPer; k++) sum += v[k];
    const uint32_t incl = wave_incl_scan(sum, lane);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t run = s_base + incl - sum;
    for (int w = 0; w < wave; w++) run += s_w[w];
    uint32_t o[kCountPer];
#pragma unroll
    for (int k = 0; k < kCountPer; k++) {
        o[k] = run;
        run += v[k];
    }
    if (i0 + kCountPer <= ng) {
        uint4 *o4 = reinterpret_cast<uint4 *>(offs + i0);
#pragma unroll
        for (int q = 0; q < kCountPer / 4; q++) o4[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < kCountPer; k++)
            if (i0 + k < ng) offs[i0 + k] = o[k];
    }
    if (c0 + kCountChunk >= ng && tid == 255) plan->joined = (int64_t)run;  // thread 255 ends the chunk
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_msd_sample(const MsdSampleParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_sample_gather_kernel, dim3(kSampleGatherBlocks), dim3(256), 0, s, p);
    hipLaunchKernelGGL(msd_sample_select_kernel, dim3(kSampleN / kSelSamples), dim3(1024), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_sample_gather(const MsdSampleParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_sample_gather_kernel, dim3(kSampleGatherBlocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

// the one-pass partition's per-call words for smj_dev_partition_regions: the
// region starts / capacities arrive as kernel arguments (stream-ordered, no
// host staging buffer that a second call could overwrite), the ticket /
// overflow / timeout flags are zeroed
__global__ void p1_set_words_kernel(const P1Words w, int64_t *oc, uint32_t *flags) {
    const int t = threadIdx.x;
    if (t < 192) oc[t] = w.v[t];
    if (t < 4) flags[t] = 0u;
}

// after the partition: out = overflow (bit 0) | look-back timeout (bit 1) |
// a packed row did not fit (bit 2)
__global__ void p1_finish_kernel(const uint32_t *flags, int64_t *out) {
    if (threadIdx.x == 0) *out = (flags[1] ? 1 : 0) | (flags[2] ? 2 : 0) | (flags[3] ? 4 : 0);
}

hipError_t launch_p1_words(const P1Words &w, int64_t *oc, uint32_t *flags, hipStream_t s) {
    hipLaunchKernelGGL(p1_set_words_kernel, dim3(1), dim3(192), 0, s, w, oc, flags);
    return hipGetLastError();
}

hipError_t launch_p1_finish(const uint32_t *flags, int64_t *out, hipStream_t s) {
    hipLaunchKernelGGL(p1_finish_kernel, dim3(1), dim3(64), 0, s, flags, out);
    return hipGetLastError();
}

hipError_t launch_msd_part1(const MsdPart1Params &p, int cols, hipStream_t s) {
    if (p.ntiles <= 0) return hipSuccess;
    // one tile per workgroup: a persistent form that took its next ticket
    // ahead (its rows in flight during the look-back) ran 17.7 vs 14.4 ms at
    // C4 -- the taken-ahead tiles publish late and every successor's look-back
    // waits on them (profiles/r03/r03o_ab_c4.txt)
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((msd_part1_kernel<C>), dim3((unsigned)p.ntiles), dim3(kMsdThreads), 0, s, p));
    return hipGetLastError();
}

template <class K>
static int64_t resident_blocks(K kernel, int threads, size_t dyn_lds);

int msd_part1c_grid(int cols) {
    static int g[9] = {0};
    if (cols < 1 || cols > 8) return 0;  // (SMJ_COLS_SWITCH)
    if (!g[cols]) SMJ_COLS_SWITCH(cols, g[cols] = (int)std::min<int64_t>(1024, resident_blocks(msd_part1c_kernel<C>, kMsdThreads, 0)));
    const char *e = getenv("SMJ_P1C_GRID");  // tests: fewer chunks of more tiles at small sizes
    return e && atoi(e) > 0 ? std::min(g[cols], atoi(e)) : g[cols];
}

hipError_t launch_msd_part1c(const MsdPart1cParams &p, const P1cWords &w, int cols, int grid, hipStream_t s) {
    if (p.ntiles <= 0) return hipSuccess;
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((msd_part1c_kernel<C>), dim3((unsigned)grid), dim3(kMsdThreads), 0, s, p, w));
    return hipGetLastError();
}

hipError_t launch_p1c_desc(const uint32_t *cnt, int G, int nb, int tile, const P1cDesc &d, uint64_t *desc, hipStream_t s) {
    if (G > 1024 || nb > 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(msd_p1c_desc_kernel, dim3((unsigned)nb), dim3(1024), 0, s, cnt, G, tile, d, desc);
    return hipGetLastError();
}

static int64_t pa_tiles(const MsdPartAParams &p, int cols) {
    return p.n <= 0 ? 0 : p.desc ? p.ntiles : (int64_t)blocks_for(p.n, msd_tile_a(cols));
}

hipError_t launch_msd_part_a(const MsdPartAParams &p, int cols, hipStream_t s) {
    if (p.n <= 0) return hipSuccess;
    return launch_msd_part_a_tiles(p, cols, 0, pa_tiles(p, cols), s);
}


hipError_t launch_msd_part_a_tiles(const MsdPartAParams &p_in, int cols, int64_t t0, int64_t t1, hipStream_t s) {
    if (p_in.n <= 0 || t1 <= t0) return hipSuccess;
    MsdPartA2 q{};
    q.t[0] = p_in;
    q.t[0].tile0 = (int)t0;
    q.tiles0 = (unsigned)(t1 - t0);
    const unsigned nb = q.tiles0;
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((msd_part_a_kernel<C>), dim3(nb), dim3(pa_threads(C)), 0, s, q));
    return hipGetLastError();
}

hipError_t launch_msd_part_a2(const MsdPartAParams &a, const MsdPartAParams &b, int cols, hipStream_t s) {
    MsdPartA2 q{};
    q.t[0] = a;
    q.t[1] = b;
    q.t[0].tile0 = q.t[1].tile0 = 0;
    q.tiles0 = (unsigned)pa_tiles(a, cols);
    const unsigned tiles1 = (unsigned)pa_tiles(b, cols);
    if (q.tiles0 + tiles1 == 0) return hipSuccess;
    const unsigned nb = q.tiles0 + tiles1;
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((msd_part_a_kernel<C>), dim3(nb), dim3(pa_threads(C)), 0, s, q));
    return hipGetLastError();
}

hipError_t launch_msd_sample_select(const MsdSampleParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_sample_select_kernel, dim3(kSampleN / kSelSamples), dim3(1024), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_runs_seg(const MsdRunsArgs &a, hipStream_t s) {
    static_assert(kSegFindBlocks <= kMsdSegs, "the scan's workgroups are a column of the grid");
    const dim3 grid(kRunsSegX + (a.segf ? 1u : 0u), kMsdSegs, a.ntab);
    hipLaunchKernelGGL(msd_runs_seg_kernel, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_msd_seg_scan(uint32_t *const *seg, uint32_t *const *tot, int narr, hipStream_t s) {
    MsdSegScanParams p{};
    for (int i = 0; i < narr; i++) {
        p.seg[i] = seg[i];
        p.tot[i] = tot[i];
    }
    hipLaunchKernelGGL(msd_seg_scan_kernel, dim3(kOffsA / 64, narr), dim3(1024), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_bases(const MsdBasesParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_bases_kernel, dim3(1), dim3(kOffsA), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_heavy(const MsdHeavyParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_heavy_kernel, dim3(kBucketsA), dim3(kHeavyThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_runs_apply(const MsdRunsArgs &a, hipStream_t s) {
    static_assert(kBucketsA % 4 == 0, "four buckets (waves) per workgroup");
    static_assert(kBucketsA % 32 == 0 && kMsdSegs % 8 == 0, "runs_apply_body's XCD-aware block order");
    const dim3 grid(kBucketsA / 4, kMsdSegs, a.ntab);
    hipLaunchKernelGGL(msd_runs_apply_kernel, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

// resident workgroups of a `threads`-thread kernel on the current device
// (occupancy x CUs), cached per kernel and LDS pad
// resident workgroups of `kernel` on the whole device, cached per kernel and
// LDS pad (kernels of one signature share K: the cache is keyed by address)
template <class K>
static int64_t resident_blocks(K kernel, int threads, size_t dyn_lds) {
    static std::mutex mu;
    static std::map<std::pair<const void *, size_t>, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    int &c = cache[{reinterpret_cast<const void *>(kernel), dyn_lds}];
    if (!c) {
        int dev = 0, per = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, dyn_lds) != hipSuccess || per < 1)
            return kMsdPartBGrid;
        c = per * cus;
    }
    return c;
}

// packed pass-B rows are written by the pipelined part_b only (2-column
// tables); SMJ_PACKB=0 turns them off (A/B), =2 packs skewed tables too
// (tests: the unpacked copy for the single-key / oversized tiers)
int msd_packb_mode() {
    const char *e = getenv("SMJ_PACKB");
    const int m = e ? atoi(e) : 1;
    return SMJ_PB_PIPE && m >= 0 && m <= 2 ? m : 0;
}

hipError_t launch_msd_part_b(const MsdPartBParams &p_in, int cols, int64_t max_tiles, hipStream_t s, bool pb_pack) {
    if (max_tiles <= 0) return hipSuccess;
    static const int dbg = getenv("SMJ_DEBUG_MSD") ? atoi(getenv("SMJ_DEBUG_MSD")) : 0;
    MsdPartBParams p = p_in;
    p.dbg = p_in.dbg ? p_in.dbg : dbg;  // explicit ablation bits (smj_debug_part_b_time) or SMJ_DEBUG_MSD
    const size_t pad = (p.dbg & 64) ? 40960 : 0;  // ablation: dynamic LDS pad -> 1 workgroup per CU
    // persistent: exactly the resident workgroups (tiles are dealt statically)
    SMJ_COLS_SWITCH(cols, {
        const unsigned grid =
            (unsigned)std::min<int64_t>(max_tiles, resident_blocks(msd_part_b_kernel<C>, pb_threads(C), pad));
        if (C == 2 && SMJ_PB_PIPE) {
            const unsigned gp = (unsigned)std::min<int64_t>(
                max_tiles, resident_blocks(msd_part_b_pipe_kernel<2>, pb_threads(2), pad));
            // rows, or packed words when MsdPlan::packB (known on the device only)
            if (pb_pack) hipLaunchKernelGGL((msd_part_b_pipe_kernel<2, 2>), dim3(gp), dim3(pb_threads(2)), pad, s, p);
            else hipLaunchKernelGGL((msd_part_b_pipe_kernel<2, 0>), dim3(gp), dim3(pb_threads(2)), pad, s, p);
        } else {
            hipLaunchKernelGGL((msd_part_b_kernel<C>), dim3(grid), dim3(pb_threads(C)), pad, s, p);
        }
    });
    return hipGetLastError();
}

hipError_t launch_msd_group(const MsdGroupParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_group_sum_kernel, dim3(kBucketsA, kGroupSlices), dim3(256), 0, s, p);
    hipLaunchKernelGGL(msd_group_kernel, dim3(kBucketsA), dim3(kGroupThreads), 0, s, p);
    return hipGetLastError();
}

// oversized multi-key groups of a small key span (2-column tables; the
// rest: host fallback), launched by the host once the plan shows some
hipError_t launch_msd_big(const MsdFinalParams &p_in, hipStream_t s) {
    static const unsigned bg_grid = (unsigned)resident_blocks(msd_big_stage_kernel, kMsdThreads, 0);
    static const int dbg = getenv("SMJ_DEBUG_BIG") ? 32 : 0;
    MsdFinalParams p = p_in;
    p.dbg |= dbg;
    hipLaunchKernelGGL(msd_big_stage_kernel, dim3(bg_grid), dim3(kMsdThreads), 0, s, p);
    // the groups over the one-workgroup limit it registered, as jobs (no-ops without)
    hipLaunchKernelGGL(msd_giant_count_kernel, dim3(bg_grid), dim3(kMsdThreads), 0, s, p);
    hipLaunchKernelGGL(msd_giant_scatter_kernel, dim3(bg_grid), dim3(kMsdThreads), 0, s, p);
    hipLaunchKernelGGL(msd_giant_join_kernel, dim3(bg_grid), dim3(kMsdThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_final(const MsdFinalParams &p_in, hipStream_t s) {
    static const int dbg = getenv("SMJ_DEBUG_MSD") ? atoi(getenv("SMJ_DEBUG_MSD")) : 0;
    MsdFinalParams p = p_in;
    p.dbg = p_in.dbg ? p_in.dbg : dbg;  // explicit bits (smj_debug_final_time) or SMJ_DEBUG_MSD
    const size_t pad = (p.dbg & 64) ? 40960 : 0;  // ablation: dynamic LDS pad -> 1 workgroup per CU
    const bool two = p.tab[0].cols == 2 && (p.ntab == 1 || p.tab[1].cols == 2);
    if (two) {
        constexpr int kStGrid = SMJ_ST_GRID;
        static_assert(kStGrid % kXcdSlots == 0, "whole XCD sets");
        const unsigned sg = pad ? kStGrid / 2 : kStGrid;
        // rows or packed words in tempB (MsdPlan::packB, set on the device):
        // both layouts' launches go in, the other returns at entry
        if (p.combined) {
            if (p.shadow[0]) hipLaunchKernelGGL((msd_final_stage_kernel<true, 2>), dim3(sg), dim3(kStThreads), pad, s, p);
            else hipLaunchKernelGGL((msd_final_stage_kernel<true, 0>), dim3(sg), dim3(kStThreads), pad, s, p);
        } else {
            if (p.shadow[0]) hipLaunchKernelGGL((msd_final_stage_kernel<false, 2>), dim3(sg), dim3(kStThreads), pad, s, p);
            else hipLaunchKernelGGL((msd_final_stage_kernel<false, 0>), dim3(sg), dim3(kStThreads), pad, s, p);
        }
        // (the wide-span kernels and the radix / 64-bit tiers: launch_msd_final_tiers,
        // from msd_back once the plan shows groups for them)
    } else {
        MsdFinalParams q = p;
        q.radix_list = nullptr;  // contiguous mode
        hipLaunchKernelGGL((msd_final_kernel<0, 0>), dim3(kMsdFinalGrid), dim3(kFinThreads), 0, s, q);
        hipLaunchKernelGGL((msd_final_wide_kernel<0, 0>), dim3(kMsdFinalGrid), dim3(kMsdThreads), 0, s, q);
    }
    return hipGetLastError();
}

// 2-column tables: the groups the staged kernel did not sort -- the wide
// groups (msd_final_wstage_kernel, or msd_final_wstage64_kernel with 64-bit
// payloads: the other returns at entry), then the radix tier over the
// handed-over groups and the 64-bit tier over what it passes on.  The host
// launches these only when the plan shows such groups (msd_back): in C3 /
// C4 / C5 the staged kernel sorts every group, and launches that return at
// entry still take CU slots behind a concurrent part's kernels (C4's trace,
// profiles/r06/r06o).  (Sorting the wide groups inside the staged kernel's
// own walk, in views of its LDS, made its narrow path slower: C4 msd_final
// 14.64-14.71 -> 15.39-15.50 ms, profiles/r06/r06p.)
hipError_t launch_msd_final_tiers(const MsdFinalParams &p_in, hipStream_t s) {
    MsdFinalParams p = p_in;
    if (g_wide_maxrun >= 0) p.dbg |= (min(g_wide_maxrun, 254) + 1) << 16;
    if (p.combined) {
        if (p.shadow[0]) hipLaunchKernelGGL((msd_final_wstage_kernel<true>), dim3(kStwGrid), dim3(kStThreads), 0, s, p);
        hipLaunchKernelGGL((msd_final_wstage64_kernel<true>), dim3(kStw64Grid), dim3(kStThreads), 0, s, p);
    } else {
        if (p.shadow[0]) hipLaunchKernelGGL((msd_final_wstage_kernel<false>), dim3(kStwGrid), dim3(kStThreads), 0, s, p);
        hipLaunchKernelGGL((msd_final_wstage64_kernel<false>), dim3(kStw64Grid), dim3(kStThreads), 0, s, p);
    }
    MsdFinalParams q = p;
    q.pk_mode = p.shadow[0] ? 2 : -1;  // packed rows possible: the tiers unpack / read the shadow on the device
    hipLaunchKernelGGL((msd_final_kernel<2, 2>), dim3(kMsdFinalGrid), dim3(kFinThreads), 0, s, q);
    q.radix_list = nullptr;
    hipLaunchKernelGGL((msd_final_wide_kernel<2, 2>), dim3(kMsdFinalGrid), dim3(kMsdThreads), 0, s, q);
    return hipGetLastError();
}

hipError_t launch_msd_single(const MsdFinalParams &p, const uint2 *work, int64_t nwork, hipStream_t s) {
    if (nwork <= 0) return hipSuccess;
    if (p.tab[0].cols == 2 && (p.ntab == 1 || p.tab[1].cols == 2))
        hipLaunchKernelGGL((msd_single_kernel<2, 2>), dim3((unsigned)nwork), dim3(kMsdThreads), 0, s, p, work);
    else
        hipLaunchKernelGGL((msd_single_kernel<0, 0>), dim3((unsigned)nwork), dim3(kMsdThreads), 0, s, p, work);
    return hipGetLastError();
}

hipError_t launch_msd_gather_list(const MsdTab &tb, const MsdGroup *groups, const uint4 *work, int64_t nwork,
                                  int64_t *dst, hipStream_t s) {
    if (nwork <= 0) return hipSuccess;
    hipLaunchKernelGGL(msd_gather_list_kernel, dim3((unsigned)nwork), dim3(kMsdThreads), 0, s, tb, groups, work, dst);
    return hipGetLastError();
}

hipError_t launch_msd_seg_copy(const int64_t *src, int64_t *dst, const uint4 *work, int64_t nwork, int cols,
                               hipStream_t s) {
    if (nwork <= 0) return hipSuccess;
    hipLaunchKernelGGL(msd_seg_copy_kernel, dim3((unsigned)nwork), dim3(256), 0, s, src, dst, work, cols);
    return hipGetLastError();
}

hipError_t launch_msd_big_split(const int64_t *J, const int64_t *nJ, int tc, const int64_t *Rs, int c1, int key1,
                                const uint4 *work, int64_t nwork, const MsdGroup *groups, int64_t *slots,
                                uint32_t *counts, hipStream_t s) {
    if (nwork <= 0) return hipSuccess;
    hipLaunchKernelGGL(msd_big_split_kernel, dim3((unsigned)nwork), dim3(256), 0, s, J, nJ, tc, Rs, c1, key1, work,
                       groups, slots, counts);
    return hipGetLastError();
}

hipError_t launch_msd_compact(const int64_t *slots, const MsdGroup *groups, const uint32_t *counts,
                              const uint32_t *offs, const MsdPlan *plan, int tc, int64_t *out, int after_fallback,
                              hipStream_t s) {
    hipLaunchKernelGGL(msd_compact_kernel, dim3(2048), dim3(256), 0, s, slots, groups, counts, offs, plan, tc, out,
                       after_fallback);
    return hipGetLastError();
}

hipError_t launch_msd_compact_big(const int64_t *slots, const MsdGroup *groups, const uint32_t *counts,
                                  const uint32_t *offs, const uint2 *work, int64_t nwork, int tc, int64_t *out,
                                  hipStream_t s) {
    if (nwork <= 0) return hipSuccess;
    hipLaunchKernelGGL(msd_compact_big_kernel, dim3((unsigned)nwork), dim3(256), 0, s, slots, groups, counts, offs,
                       work, tc, out);
    return hipGetLastError();
}

hipError_t launch_msd_count_scan(const uint32_t *counts, uint32_t *part, uint32_t *offs, MsdPlan *plan,
                                 hipStream_t s) {
    hipLaunchKernelGGL(msd_count_part_kernel, dim3(kCountChunks), dim3(256), 0, s, counts, part, plan);
    hipLaunchKernelGGL(msd_count_scan_kernel, dim3(kCountChunks), dim3(256), 0, s, counts, part, offs, plan);
    return hipGetLastError();
}

}  // namespace smj
