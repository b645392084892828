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
//             LDS) and keeps 127 splitters; pass-A bucket of a key =
//             2 * #{splitters < key} + (key == that splitter): 255 buckets,
//             the odd ones hold exactly one key value (heavy keys).
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

#include <stdlib.h>

#include <algorithm>

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
#pragma unroll
    for (int w = 0; w < NW; w++) {
        mn = min(mn, s_mm[w]);
        mx = max(mx, s_mm[NW + w]);
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

// Per-digit cross-wave exclusive prefixes (in place in s_wcnt[wave][digit])
// and tile-local exclusive digit starts s_bin[0..RADIX] (s_bin[RADIX] = the
// tile's row count).  Thread t owns digits [t * DPT, t * DPT + DPT).  Ends
// with a barrier.
template <int RADIX>
__device__ __forceinline__ uint32_t tile_digit_starts(uint32_t *s_wcnt, uint32_t *s_bin, uint32_t *s_wsum) {
    constexpr int DPT = RADIX > kMsdThreads ? RADIX / kMsdThreads : 1;
    const int tid = threadIdx.x;
    uint32_t tot[DPT], sum = 0;
#pragma unroll
    for (int j = 0; j < DPT; j++) {
        const int d = tid * DPT + j;
        uint32_t t = 0;
        if (d < RADIX) {
#pragma unroll
            for (int w = 0; w < kMsdWaves; w++) {
                const uint32_t c = s_wcnt[w * RADIX + d];
                s_wcnt[w * RADIX + d] = t;
                t += c;
            }
        }
        tot[j] = t;
        sum += t;
    }
    uint32_t all;
    uint32_t ex = block_excl_scan<kMsdWaves>(sum, s_wsum, &all);
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

// pass-A bucket of a key: 2 * #{splitters < key} + (key == that splitter)
__device__ __forceinline__ uint32_t bucket_a(const int64_t *s_spl, int64_t k) {
    int pos = 0;
#pragma unroll
    for (int step = 64; step >= 1; step >>= 1)
        pos += (s_spl[pos + step - 1] < k) ? step : 0;  // index <= 126: 127 = 2^7 - 1 splitters
    const bool eq = pos < kSplA && s_spl[pos < kSplA ? pos : kSplA - 1] == k;
    return 2u * (uint32_t)pos + (eq ? 1u : 0u);
}

// ---------------------------------------------------------------------------
// sample -> splitters
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void msd_sample_kernel(const MsdSampleParams p) {
    constexpr int N = 2 * kSampleMax;  // 16 Ki keys = 128 KiB of LDS
    __shared__ int64_t s_key[N];
    __shared__ uint32_t s_wsum[16];
    const int tid = threadIdx.x;
    uint32_t valid = 0;
    for (int j = tid; j < N; j += 1024) {
        int64_t k = INT64_MAX;
        const int x = j >= kSampleMax ? 1 : 0;
        const int jj = j - x * kSampleMax;
        const MsdTable &t = p.tab[x];
        if (x < p.ntab && t.n > 0) {
            const int64_t ns = min(t.n, (int64_t)kSampleMax);
            if (jj < ns) {
                const int64_t r = ((2 * (int64_t)jj + 1) * t.n) / (2 * ns);
                const int64_t *row = t.src + r * t.cols;
                if (!t.use_sel || row[t.sel_col] > t.sel_val) {
                    k = row[t.key_col];
                    valid++;
                }
            }
        }
        s_key[j] = k;
    }
    // valid sample count
    {
        uint32_t v = valid;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((tid & 63) == 0) s_wsum[tid >> 6] = v;
    }
    __syncthreads();
    uint32_t M = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) M += s_wsum[w];
    // bitonic sort ascending (invalid samples are INT64_MAX: they sort behind every valid key)
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int q = tid; q < N / 2; q += 1024) {
                const int i = (q / j) * 2 * j + (q % j);
                const int l = i + j;
                const int64_t a = s_key[i], b = s_key[l];
                const bool up = (i & k) == 0;
                if ((a > b) == up) {
                    s_key[i] = b;
                    s_key[l] = a;
                }
            }
            __syncthreads();
        }
    }
    if (tid < kSplA) {
        int64_t s = INT64_MAX;
        if (M > 0) {
            const uint32_t at = min(M - 1, (uint32_t)(((uint64_t)(tid + 1) * M) / (kSplA + 1)));
            s = s_key[at];
        }
        p.spl[tid] = s;
    }
}

// ---------------------------------------------------------------------------
// part_a: select + stable tile-local partition by pass-A bucket
// ---------------------------------------------------------------------------
template <int COLS>
__global__ __launch_bounds__(kMsdThreads, 2) void msd_part_a_kernel(const MsdPartAParams p) {
    constexpr int ITEMS = msd_items(COLS), T = msd_tile(COLS), RADIX = kOffsA;
    constexpr int ROWB = T * COLS * 8, CNTB = kMsdWaves * RADIX * 4;
    constexpr int UB = ROWB > CNTB ? ROWB : CNTB;
    __shared__ __attribute__((aligned(16))) unsigned char s_u[UB];
    __shared__ int64_t s_spl[kSplA + 1];
    __shared__ uint32_t s_bin[RADIX + 1];
    __shared__ uint32_t s_wsum[kMsdWaves];
    __shared__ int64_t s_mm[2 * kMsdWaves];
    int64_t *s_rows = reinterpret_cast<int64_t *>(s_u);
    uint32_t *s_wcnt = reinterpret_cast<uint32_t *>(s_u);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t t = blockIdx.x, row0 = t * T;
    const int nrows = (int)min((int64_t)T, p.n - row0);
    uint32_t *wc = s_wcnt + wave * RADIX;
    if (tid < kSplA) s_spl[tid] = p.spl[tid];
    zero_counters<RADIX>(wc, lane);
    const int lrow0 = wave * ITEMS * 64 + lane;
    int64_t rows[ITEMS][COLS];
#pragma unroll
    for (int it = 0; it < ITEMS; it++)
        load_row<COLS>(p.src + (row0 + min(lrow0 + it * 64, nrows - 1)) * COLS, rows[it]);
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
    wave_rank<ITEMS, 8>(dig, vmask, wc, lane);
    __syncthreads();
    const uint32_t total = tile_digit_starts<RADIX>(s_wcnt, s_bin, s_wsum);
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t d = dig[it] & 0xffffu;
        dig[it] = s_bin[d] + wc[d] + (dig[it] >> 16);
    }
    block_minmax<kMsdWaves>(mn, mx, s_mm);  // its barriers also retire the counters
#pragma unroll
    for (int it = 0; it < ITEMS; it++)
        if ((vmask >> it) & 1u) store_row<COLS>(s_rows + (size_t)dig[it] * COLS, rows[it]);
    if (tid < RADIX) p.offs[t * kOffsA + tid] = s_bin[tid];  // s_bin[255] = total (bucket 255 is never used)
    if (tid == 0) {
        p.tmm[2 * t] = mn;
        p.tmm[2 * t + 1] = mx;
    }
    __syncthreads();
    if (total > 0) {
        int64_t *dst = p.out + row0 * COLS;
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const uint32_t s = min((uint32_t)(tid + it * kMsdThreads), total - 1u);
            int64_t r[COLS];
            load_row<COLS>(s_rows + (size_t)s * COLS, r);
            store_row<COLS>(dst + (size_t)s * COLS, r);
        }
    }
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
__global__ __launch_bounds__(256) void msd_runs_seg_kernel(const uint32_t *__restrict__ offs, int64_t ntiles,
                                                           int width, int nb, uint32_t *__restrict__ segL,
                                                           uint32_t *__restrict__ segC) {
    __shared__ uint32_t partL[4][64], partC[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int a = blockIdx.x * 64 + lane;
    int64_t c0, c1;
    msd_seg_range(ntiles, c0, c1);
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

// one workgroup of 256: thread = bucket.  Bucket sizes / bases of both
// tables, the global key range, and the pass-B digit of every bucket.
__global__ __launch_bounds__(256) void msd_bases_kernel(const MsdBasesParams p) {
    __shared__ uint32_t s_wsum[4];
    __shared__ int64_t s_mm[8];
    const int a = threadIdx.x, lane = a & 63, wave = a >> 6;
    // global min / max of the selected keys over both tables
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    for (int x = 0; x < p.ntab; x++)
        for (int64_t t = a; t < p.ntiles[x]; t += 256) {
            mn = min(mn, p.tmm[x][2 * t]);
            mx = max(mx, p.tmm[x][2 * t + 1]);
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o, 64));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o, 64));
    }
    if (lane == 0) {
        s_mm[wave] = mn;
        s_mm[4 + wave] = mx;
    }
    __syncthreads();
    for (int w = 0; w < 4; w++) {
        mn = min(mn, s_mm[w]);
        mx = max(mx, s_mm[4 + w]);
    }
    // pass-B digit of bucket a over the bucket's key interval [lo, hi]:
    // floor((key - lo) * kRadB / (hi - lo + 1)) as one mulhi, or key - lo
    // when the interval holds fewer than kRadB keys
    int64_t lo = 0;
    uint64_t scale = 0;
    uint32_t maxspan = kRadB;
    if (a < kBucketsA) {
        const int i = a >> 1;
        int64_t hi;
        if (a & 1) {
            lo = hi = p.spl[i];
        } else {
            lo = i == 0 ? mn : (int64_t)((uint64_t)p.spl[i - 1] + 1u);
            hi = i == kSplA ? mx : (int64_t)((uint64_t)p.spl[i] - 1u);
        }
        const uint64_t range = hi > lo ? (uint64_t)hi - (uint64_t)lo : 0u;  // interval = range + 1 keys
        if (range >= (uint64_t)kRadB) {
            const unsigned __int128 one73 = (unsigned __int128)1 << (64 + kBitsB);
            const unsigned __int128 q = one73 / ((unsigned __int128)range + 1u);
            scale = q >> 64 ? ~0ull : (uint64_t)q;
            // keys per sub-bucket <= ceil((range + 1) / kRadB) + 1: spans keep group ranges < 2^48
            const uint64_t w = (range >> kBitsB) + 2u;
            const uint64_t span = ((uint64_t)1 << 48) / w;
            maxspan = span >= (uint64_t)kRadB ? (uint32_t)kRadB : span ? (uint32_t)span : 1u;
        }
    }
    for (int x = 0; x < p.ntab; x++) {
        uint32_t L = 0, C = 0;
        if (a < kBucketsA)
            for (int s = 0; s < kMsdSegs; s++) {
                L += p.segL[x][s * kOffsA + a];
                C += p.segC[x][s * kOffsA + a];
            }
        const uint32_t K = (L + (uint32_t)p.tile[x] - 1) / (uint32_t)p.tile[x];
        uint32_t totL, totC, totK;
        const uint32_t rs = block_excl_scan<4>(L, s_wsum, &totL);
        const uint32_t lb = block_excl_scan<4>(C, s_wsum, &totC);
        const uint32_t tb = block_excl_scan<4>(K, s_wsum, &totK);
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

// grid (ceil(nb / 64), kMsdSegs) x 256: emit the run list entries of every
// bucket (lane) for this segment, and the first run of every pass-B tile
__global__ __launch_bounds__(256) void msd_runs_apply_kernel(const uint32_t *__restrict__ offs, int64_t ntiles,
                                                             int T, const uint32_t *__restrict__ segL,
                                                             const uint32_t *__restrict__ segC,
                                                             const MsdBucket *__restrict__ bk,
                                                             uint2 *__restrict__ list, uint2 *__restrict__ tinfo) {
    __shared__ uint32_t partL[4][64], partC[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int a = blockIdx.x * 64 + lane;
    const bool ok = a < kBucketsA;
    int64_t c0, c1;
    msd_seg_range(ntiles, c0, c1);
    uint32_t L = 0, C = 0;
    if (ok)
#pragma unroll 8
        for (int64_t t = c0; t < c1; t++) {
            const uint32_t len = offs[t * kOffsA + a + 1] - offs[t * kOffsA + a];
            L += len;
            C += len ? 1u : 0u;
        }
    partL[w][lane] = L;
    partC[w][lane] = C;
    __syncthreads();
    if (!ok) return;
    uint32_t P = 0, Q = 0;
    for (int s = 0; s < (int)blockIdx.y; s++) {
        P += segL[s * kOffsA + a];
        Q += segC[s * kOffsA + a];
    }
    for (int v = 0; v < w; v++) {
        P += partL[v][lane];
        Q += partC[v][lane];
    }
    const MsdBucket b = bk[a];
    const uint32_t uT = (uint32_t)T;
    for (int64_t t = c0; t < c1; t++) {
        const uint32_t o = offs[t * kOffsA + a];
        const uint32_t len = offs[t * kOffsA + a + 1] - o;
        if (len) {
            list[b.list_base + Q] = make_uint2((uint32_t)(t * T) + o, P);
            const uint32_t k = (P + uT - 1) / uT;  // the pass-B tile starting inside this run, if any
            if (k * uT < P + len) tinfo[b.tile_base + k] = make_uint2((uint32_t)a, b.list_base + Q);
            Q++;
            P += len;
        }
    }
}

// ---------------------------------------------------------------------------
// part_b: gather a pass-B tile through the run list, stable tile-local
// partition by the 9-bit sub-bucket
// ---------------------------------------------------------------------------
template <int COLS>
__global__ __launch_bounds__(kMsdThreads, 2) void msd_part_b_kernel(const MsdPartBParams p) {
    constexpr int ITEMS = msd_items(COLS), T = msd_tile(COLS), RADIX = kRadB;
    constexpr int ROWB = T * COLS * 8, CNTB = kMsdWaves * RADIX * 4, LISTB = (T + 1) * 8;
    constexpr int UB0 = ROWB > CNTB ? ROWB : CNTB;
    constexpr int UB = UB0 > LISTB ? UB0 : LISTB;
    __shared__ __attribute__((aligned(16))) unsigned char s_u[UB];
    __shared__ uint32_t s_bin[RADIX + 1];
    __shared__ uint32_t s_wsum[kMsdWaves];
    int64_t *s_rows = reinterpret_cast<int64_t *>(s_u);
    uint32_t *s_wcnt = reinterpret_cast<uint32_t *>(s_u);
    uint2 *s_list = reinterpret_cast<uint2 *>(s_u);

    const int64_t g = blockIdx.x;
    if (g >= (int64_t)p.plan->ntilesB[p.x]) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint2 ti = p.tinfo[g];
    const MsdBucket b = p.bk[ti.x];
    const uint32_t v0 = (uint32_t)(g - b.tile_base) * (uint32_t)T;
    const int nrows = (int)min((uint32_t)T, b.L - v0);
    const uint32_t q0 = ti.y;
    const int J = (int)min(b.list_base + b.nruns - q0, (uint32_t)nrows + 1u);
    for (int j = tid; j < J; j += kMsdThreads) s_list[j] = p.list[q0 + j];
    __syncthreads();

    const int lrow0 = wave * ITEMS * 64 + lane;
    int64_t rows[ITEMS][COLS];
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t v = v0 + (uint32_t)min(lrow0 + it * 64, nrows - 1);
        int lo = 0, hi = J - 1;  // last run starting at or before v
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_list[mid].y <= v) lo = mid; else hi = mid - 1;
        }
        const uint2 e = s_list[lo];
        load_row<COLS>(p.srcA + (int64_t)(e.x + (v - e.y)) * COLS, rows[it]);
    }
    __syncthreads();  // list dead: the region becomes the counters
    uint32_t *wc = s_wcnt + wave * RADIX;
    zero_counters<RADIX>(wc, lane);

    uint32_t dig[ITEMS];
    uint32_t vmask = 0;
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const bool v = lrow0 + it * 64 < nrows;
        const uint64_t r = (uint64_t)pick<COLS>(rows[it], p.key_col) - (uint64_t)b.lo;
        const uint32_t d = b.scale ? min((uint32_t)__umul64hi(r, b.scale), (uint32_t)(RADIX - 1)) : (uint32_t)r;
        dig[it] = v ? d & (RADIX - 1) : 0u;
        vmask |= v ? (1u << it) : 0u;
    }
    wave_rank<ITEMS, kBitsB>(dig, vmask, wc, lane);
    __syncthreads();
    tile_digit_starts<RADIX>(s_wcnt, s_bin, s_wsum);
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t d = dig[it] & 0xffffu;
        dig[it] = s_bin[d] + wc[d] + (dig[it] >> 16);
    }
    __syncthreads();  // counters dead: the region becomes the staging tile
#pragma unroll
    for (int it = 0; it < ITEMS; it++)
        if ((vmask >> it) & 1u) store_row<COLS>(s_rows + (size_t)dig[it] * COLS, rows[it]);
    for (int d = tid; d <= RADIX; d += kMsdThreads) p.offs[g * kOffsB + d] = s_bin[d];  // s_bin[RADIX] = nrows
    __syncthreads();
    int64_t *dst = p.out + g * T * COLS;
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const int s = min(tid + it * kMsdThreads, nrows - 1);
        int64_t r[COLS];
        load_row<COLS>(s_rows + (size_t)s * COLS, r);
        store_row<COLS>(dst + (size_t)s * COLS, r);
    }
}

// ---------------------------------------------------------------------------
// group: pack the sub-buckets of every bucket into final groups
// ---------------------------------------------------------------------------
// one workgroup of kRadB threads per bucket a (thread = sub-bucket): per-table
// sub-bucket totals, their prefixes, greedy packing into groups written to
// slots a * kRadB + j.  msd_group_pack_kernel then lays them out densely.
__global__ __launch_bounds__(kRadB) void msd_group_kernel(const MsdGroupParams p) {
    constexpr int NW = kRadB / 64;
    __shared__ uint32_t s_tot[2][kRadB];
    __shared__ uint32_t s_pre[2][kRadB];
    __shared__ uint32_t s_wsum[NW];
    __shared__ uint16_t s_g0[kRadB], s_g1[kRadB];  // groups: sub-buckets [b0, b1)
    __shared__ int s_ng;
    const int a = blockIdx.x, b = threadIdx.x;
    for (int x = 0; x < 2; x++) {
        uint32_t tot = 0;
        if (x < p.ntab) {
            const MsdBucket bk = p.bk[x][a];
            const uint32_t K = (bk.L + (uint32_t)p.tile[x] - 1) / (uint32_t)p.tile[x];
            const uint32_t *o = p.offs[x] + (int64_t)bk.tile_base * kOffsB + b;
#pragma unroll 4
            for (uint32_t k = 0; k < K; k++) tot += o[(int64_t)k * kOffsB + 1] - o[(int64_t)k * kOffsB];
        }
        uint32_t all;
        const uint32_t ex = block_excl_scan<NW>(tot, s_wsum, &all);
        s_tot[x][b] = tot;
        s_pre[x][b] = ex;
    }
    __syncthreads();
    const bool single_sub = (a & 1) || p.bk[0][a].scale == 0;  // every sub-bucket holds one key value
    // a group spans < 2^48 key values, so that (residual << 16 | index) fits one
    // word in the final kernel's LDS sort
    const int maxspan = (int)p.bk[0][a].maxspan;
    if (b == 0) {  // greedy packing; a group that is over the cap holds exactly one sub-bucket
        int ng = 0, b0 = -1, last = -1;
        uint32_t cr = 0, cs = 0;
        for (int j = 0; j < kRadB; j++) {
            const uint32_t r = s_tot[0][j], s = s_tot[1][j];
            if (r + s == 0) continue;
            if (b0 >= 0 && (cr + r > (uint32_t)kGroupCap || cs + s > (uint32_t)kGroupCap || j - b0 >= maxspan)) {
                s_g0[ng] = (uint16_t)b0;
                s_g1[ng] = (uint16_t)(last + 1);
                ng++;
                b0 = -1;
                cr = cs = 0;
            }
            if (b0 < 0) b0 = j;
            cr += r;
            cs += s;
            last = j;
        }
        if (b0 >= 0) {
            s_g0[ng] = (uint16_t)b0;
            s_g1[ng] = (uint16_t)(last + 1);
            ng++;
        }
        s_ng = ng;
        p.ngrp[a] = (uint32_t)ng;
    }
    __syncthreads();
    const int j = b;
    if (j >= s_ng) return;
    const uint32_t b0 = s_g0[j], b1 = s_g1[j];
    MsdGroup gr{};
    gr.a = (uint16_t)a;
    gr.b0 = (uint16_t)b0;
    gr.b1 = (uint16_t)b1;
    gr.nR = s_pre[0][b1 - 1] + s_tot[0][b1 - 1] - s_pre[0][b0];
    gr.nS = s_pre[1][b1 - 1] + s_tot[1][b1 - 1] - s_pre[1][b0];
    gr.outR = p.bk[0][a].row_start + s_pre[0][b0];
    gr.outS = p.ntab > 1 ? p.bk[1][a].row_start + s_pre[1][b0] : 0u;
    gr.flags = 0;
    if (gr.nR > (uint32_t)kGroupCap || gr.nS > (uint32_t)kGroupCap) gr.flags = single_sub ? kGroupSingle : kGroupBig;
    p.slot_groups[(int64_t)a * kRadB + j] = gr;
}

// grid kBucketsA x 256: bucket a's groups -> dense (key-ordered) indices
// base_a + j; join counts of single-key groups; fallback lists
__global__ __launch_bounds__(256) void msd_group_pack_kernel(const MsdGroupParams p) {
    __shared__ uint32_t s_base;
    const int a = blockIdx.x, tid = threadIdx.x;
    if (tid < 64) {
        uint32_t v = 0;
        for (int i = tid; i < a; i += 64) v += p.ngrp[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (tid == 0) s_base = v;
    }
    __syncthreads();
    const uint32_t base = s_base, ng = p.ngrp[a];
    if (a == kBucketsA - 1 && tid == 0) p.plan->ngroups = base + ng;
    for (uint32_t j = tid; j < ng; j += 256) {
        const MsdGroup g = p.slot_groups[(int64_t)a * kRadB + j];
        const uint32_t gi = base + j;
        p.groups[gi] = g;
        uint32_t cnt = 0;
        if (g.flags == kGroupSingle) {
            cnt = min(g.nR, g.nS);
            p.single_list[atomicAdd(&p.plan->nsingle, 1u)] = gi;
        } else if (g.flags == kGroupBig) {
            p.big_list[atomicAdd(&p.plan->nbig, 1u)] = gi;
        }
        p.counts[gi] = cnt;
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
    if ((g.a & 1) && g.b0 == 0) {  // single-key bucket: its tiles are full and hold only sub-bucket 0
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

// persistent: workgroup b takes dense groups b, b + grid, ... (key order)
template <int C1, int C2>
__global__ __launch_bounds__(kMsdThreads, 2) void msd_final_kernel(const MsdFinalParams p) {
    __shared__ FinalSmem sm;
    const int64_t ng = p.plan->ngroups;
    for (int64_t gi = blockIdx.x; gi < ng; gi += gridDim.x) {
        final_group<C1, C2>(p, gi, sm);
        __syncthreads();  // LDS reused by the next group
    }
}

// ---------------------------------------------------------------------------
// single-key oversized groups: already in stable order; copy and zip
// ---------------------------------------------------------------------------
// grid = work items (dense group, chunk of kGroupCap group rows)
template <int C1, int C2>
__global__ __launch_bounds__(kMsdThreads) void msd_single_kernel(const MsdFinalParams p, const uint2 *work) {
    __shared__ uint64_t s_tmp[kGroupCap];
    __shared__ uint32_t s_addr[2][kGroupCap];
    __shared__ uint32_t s_wsum[kMsdWaves];
    const uint2 w = work[blockIdx.x];
    const MsdGroup g = p.groups[w.x];
    const int tid = threadIdx.x;
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
            if constexpr (C1 > 0) {
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
    for (uint32_t v = V0 + tid; v < V1; v += kMsdThreads)
        emit_join_row<C1, C2>(p.tab[0].tempB + (int64_t)s_addr[0][v - V0] * c1,
                              p.tab[1].tempB + (int64_t)s_addr[1][v - V0] * c2, dst + (int64_t)v * tc, c1, c2,
                              p.key2);
}

// gather a group's rows of table x into a contiguous buffer (LSD fallback)
__global__ __launch_bounds__(kMsdThreads) void msd_gather_kernel(const MsdTab tb, const MsdGroup *groups,
                                                                 uint32_t slot, int64_t *dst) {
    __shared__ uint64_t s_tmp[kGroupCap];
    __shared__ uint32_t s_wsum[kMsdWaves];
    const MsdGroup g = groups[slot];
    const uint32_t nx = tb.x ? g.nS : g.nR;
    const uint32_t V0 = blockIdx.x * (uint32_t)kGroupCap;
    if (V0 >= nx) return;
    const uint32_t V1 = min(V0 + (uint32_t)kGroupCap, nx);
    group_gather(tb, g, V0, V1, reinterpret_cast<uint2 *>(s_tmp), s_wsum, [&](uint32_t v, uint32_t src) {
        copy_row<0>(tb.tempB + (int64_t)src * tb.cols, dst + (int64_t)v * tb.cols, tb.cols);
    });
}

// pack the join slots: dense group g has counts[g] rows at slot row outR
// (persistent over the groups)
__global__ __launch_bounds__(256) void msd_compact_kernel(const int64_t *__restrict__ slots,
                                                          const MsdGroup *__restrict__ groups,
                                                          const uint32_t *__restrict__ counts,
                                                          const uint32_t *__restrict__ offs,
                                                          const MsdPlan *__restrict__ plan, int tc,
                                                          int64_t *__restrict__ out) {
    const int64_t ng = plan->ngroups;
    for (int64_t g = blockIdx.x; g < ng; g += gridDim.x) {
        const uint32_t c = counts[g];
        if (c == 0) continue;
        const int64_t nw = (int64_t)c * tc;
        const int64_t *src = slots + (int64_t)groups[g].outR * tc;
        int64_t *dst = out + (int64_t)offs[g] * tc;
        for (int64_t i = threadIdx.x; i < nw; i += 256) dst[i] = src[i];
    }
}

// exclusive scan of the dense group counts (one workgroup of 1024, rounds of
// 16 Ki staged through LDS); plan->joined = total
__global__ __launch_bounds__(1024) void msd_count_scan_kernel(const uint32_t *__restrict__ counts,
                                                              uint32_t *__restrict__ offs, MsdPlan *plan) {
    constexpr int PER = 16, ROUND = 1024 * PER;
    __shared__ uint32_t s_c[ROUND];
    __shared__ uint32_t s_w[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t ng = plan->ngroups;
    uint32_t carry = 0;
    for (int64_t base = 0; base < ng; base += ROUND) {
        const int64_t n = min((int64_t)ROUND, ng - base);
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
    if (tid == 0) plan->joined = (int64_t)carry;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_msd_sample(const MsdSampleParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_sample_kernel, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_part_a(const MsdPartAParams &p, int cols, hipStream_t s) {
    if (p.n <= 0) return hipSuccess;
    const unsigned grid = blocks_for(p.n, msd_tile(cols));
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((msd_part_a_kernel<C>), dim3(grid), dim3(kMsdThreads), 0, s, p));
    return hipGetLastError();
}

hipError_t launch_msd_runs_seg(const uint32_t *offs, int64_t ntiles, uint32_t *segL, uint32_t *segC,
                               hipStream_t s) {
    const dim3 grid((kBucketsA + 63) / 64, kMsdSegs);
    hipLaunchKernelGGL(msd_runs_seg_kernel, grid, dim3(256), 0, s, offs, ntiles, kOffsA, kBucketsA, segL, segC);
    return hipGetLastError();
}

hipError_t launch_msd_bases(const MsdBasesParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_bases_kernel, dim3(1), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_runs_apply(const uint32_t *offs, int64_t ntiles, int T, const uint32_t *segL,
                                 const uint32_t *segC, const MsdBucket *bk, uint2 *list, uint2 *tinfo,
                                 hipStream_t s) {
    const dim3 grid((kBucketsA + 63) / 64, kMsdSegs);
    hipLaunchKernelGGL(msd_runs_apply_kernel, grid, dim3(256), 0, s, offs, ntiles, T, segL, segC, bk, list, tinfo);
    return hipGetLastError();
}

hipError_t launch_msd_part_b(const MsdPartBParams &p, int cols, int64_t max_tiles, hipStream_t s) {
    if (max_tiles <= 0) return hipSuccess;
    SMJ_COLS_SWITCH(cols, hipLaunchKernelGGL((msd_part_b_kernel<C>), dim3((unsigned)max_tiles), dim3(kMsdThreads),
                                             0, s, p));
    return hipGetLastError();
}

hipError_t launch_msd_group(const MsdGroupParams &p, hipStream_t s) {
    hipLaunchKernelGGL(msd_group_kernel, dim3(kBucketsA), dim3(kRadB), 0, s, p);
    hipLaunchKernelGGL(msd_group_pack_kernel, dim3(kBucketsA), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_msd_final(const MsdFinalParams &p, hipStream_t s) {
    if (p.tab[0].cols == 2 && (p.ntab == 1 || p.tab[1].cols == 2))
        hipLaunchKernelGGL((msd_final_kernel<2, 2>), dim3(kMsdFinalGrid), dim3(kMsdThreads), 0, s, p);
    else
        hipLaunchKernelGGL((msd_final_kernel<0, 0>), dim3(kMsdFinalGrid), dim3(kMsdThreads), 0, s, p);
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

hipError_t launch_msd_gather(const MsdTab &tb, const MsdGroup *groups, uint32_t slot, int64_t rows, int64_t *dst,
                             hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(msd_gather_kernel, dim3(blocks_for(rows, kGroupCap)), dim3(kMsdThreads), 0, s, tb, groups,
                       slot, dst);
    return hipGetLastError();
}

hipError_t launch_msd_compact(const int64_t *slots, const MsdGroup *groups, const uint32_t *counts,
                              const uint32_t *offs, const MsdPlan *plan, int tc, int64_t *out, hipStream_t s) {
    hipLaunchKernelGGL(msd_compact_kernel, dim3(2048), dim3(256), 0, s, slots, groups, counts, offs, plan, tc, out);
    return hipGetLastError();
}

hipError_t launch_msd_count_scan(const uint32_t *counts, uint32_t *offs, MsdPlan *plan, hipStream_t s) {
    hipLaunchKernelGGL(msd_count_scan_kernel, dim3(1), dim3(1024), 0, s, counts, offs, plan);
    return hipGetLastError();
}

}  // namespace smj
