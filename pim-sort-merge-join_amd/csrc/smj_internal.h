// smj_internal.h -- shared between the HIP kernels (smj_kernels.hip) and the
// C-ABI layer (smj_api.hip).  Not installed; the public contract is smj.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace smj {

// ---------------------------------------------------------------------------
// Sort geometry.  One onesweep pass = one launch of onesweep_kernel: every
// 512-lane workgroup ranks one tile of rows in LDS (wave64 ballot matching on
// the digit bits), publishes its per-digit counts, resolves its global digit
// offsets by decoupled look-back over its predecessors' status words, and
// scatters the tile through LDS so that each digit's run leaves as coalesced
// 16-B-per-lane stores.
// ---------------------------------------------------------------------------
#ifndef SMJ_SORT_THREADS
#define SMJ_SORT_THREADS 1024
#endif
#ifndef SMJ_RADIX_BITS
#define SMJ_RADIX_BITS 10
#endif
constexpr int kSortThreads = SMJ_SORT_THREADS;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kRadixBits = SMJ_RADIX_BITS;       // digit width of the radix passes
constexpr int kRadix = 1 << kRadixBits;          // 1024 bins
constexpr int kNumPos = (64 + kRadixBits - 1) / kRadixBits;  // 7 digit positions
constexpr int kBucketBits = 6;                   // multi-GPU partition: <= 64 buckets
constexpr int kMaxSplitters = (1 << kBucketBits) - 1;

// rows per thread per tile: a tile is 64 KiB of rows whatever the row width
__host__ __device__ constexpr int sort_items(int cols) { return cols == 1 ? 8 : cols >= 8 ? 2 : (16 / cols); }
__host__ __device__ constexpr int sort_tile_rows(int cols) { return sort_items(cols) * kSortThreads; }

// A pass is processed in chunks of kChunkTiles consecutive tiles (one
// workgroup per chunk in the scatter kernel); the [chunk][digit] count table
// is scanned in kScanSegs segments.
constexpr int kChunkTiles = 8;
__host__ __device__ constexpr int64_t chunk_rows(int cols) { return (int64_t)kChunkTiles * sort_tile_rows(cols); }
constexpr int kScanSegs = 16;

// Join / merge geometry: one workgroup per merge-path tile of kJoinTile
// merged elements (R-piece + S-piece).
constexpr int kJoinThreads = 512;
constexpr int kJoinPer = 8;
constexpr int kJoinTile = kJoinThreads * kJoinPer;  // 4096 (merge); the join adapts:
// merged elements per join tile: both pieces must fit in 64 KiB of LDS as rows
__host__ __device__ constexpr int join_tile_size(int c1, int c2) {
    return (c1 > c2 ? c1 : c2) <= 2 ? 4096 : (c1 > c2 ? c1 : c2) <= 4 ? 2048 : 1024;
}

// Look-back status word: [31:30] flag, [29:0] count.
constexpr uint32_t kFlagAgg = 1u << 30;
constexpr uint32_t kFlagInc = 2u << 30;
constexpr uint32_t kValueMask = (1u << 30) - 1;

struct SortPlan {
    uint32_t m;          // rows that passed the select
    int32_t npasses;     // radix passes to run (>= 1 when m > 0)
    int32_t pos[8];      // digit position (0..kNumPos-1) of pass k
    uint32_t pad[2];
};

// Device scratch counters.  {tile, count} are zeroed before every launch
// (8-byte memset).
struct Counters {
    uint32_t tile;       // dynamic tile id
    uint32_t count;      // rows emitted (select-only passes)
    uint32_t pad[2];
};

// ---- launchers (smj_kernels.hip) ------------------------------------------
// All return hipSuccess or the launch error.  `prof` tags are recorded by
// the caller.

// all-digit histograms (ghist[kNumPos][kRadix]) + digit-0 counts per chunk of
// the first pass (table0[chunks][kRadix])
hipError_t launch_hist_radix(const int64_t *src, int64_t n, int cols, int use_select, int sel_col,
                             int64_t sel_val, int key_col, uint64_t key_base, uint32_t *ghist, uint32_t *table0,
                             hipStream_t s);
hipError_t launch_plan(uint32_t *ghist, SortPlan *plan, hipStream_t s);
enum DigitKind { DIGIT_RADIX = 0, DIGIT_ZERO = 1, DIGIT_BUCKET = 2 };
// One scatter pass: rows of src (with the WHERE predicate when use_select)
// are moved stably into dst in the order of their digit.
struct PassSpec {
    const int64_t *src;
    int64_t nsrc;
    int64_t *dst;
    int cols, use_select, sel_col, key_col;
    int64_t sel_val;
    DigitKind kind;
    uint64_t key_base;    // DIGIT_RADIX: digit = ((key ^ 2^63) - key_base) >> shift
    int shift;
    const int64_t *spl;   // DIGIT_BUCKET: host array of nspl sorted splitters
    int nspl;
    int64_t *trash;       // device scratch, kSortThreads * 16 int64 (ITEMS * COLS <= 16)
};
int pass_radix(const PassSpec &ps);
int64_t pass_chunks(const PassSpec &ps);
// table: pass_chunks * pass_radix u32; segsum: kScanSegs * pass_radix u32;
// base: pass_radix global exclusive digit starts (nullptr = 0).
hipError_t launch_chunk_hist(const PassSpec &ps, uint32_t *table, hipStream_t s);
hipError_t launch_chunk_scan(const PassSpec &ps, uint32_t *table, uint32_t *segsum, const uint32_t *base,
                             hipStream_t s);
hipError_t launch_chunk_scatter(const PassSpec &ps, uint32_t *table, Counters *ctr, hipStream_t s);
// chunk_scan with the digit bases computed on the device (exclusive prefix of
// the digit totals, written to base[radix]); the totals go to counts[radix]
hipError_t launch_chunk_scan_dev(const PassSpec &ps, uint32_t *table, uint32_t *segsum, uint32_t *base,
                                 unsigned long long *counts, hipStream_t s);
hipError_t launch_hist_bucket(const int64_t *src, int64_t n, int cols, int use_select, int sel_col,
                              int64_t sel_val, int key_col, const int64_t *spl, int nspl,
                              unsigned long long *gcount, long long *gminmax, hipStream_t s);
// run_start may be nullptr (merge); for the join it gets, per tile, the first
// A row carrying the key of A[apart[t]]
hipError_t launch_merge_partition(const int64_t *a, int64_t na, int ca, int ka, const int64_t *b,
                                  int64_t nb, int cb, int kb, int64_t *apart, int64_t *run_start, int64_t ntiles,
                                  int tile, hipStream_t s);
// join phases: 0 = tiles (slots + counts), 1 = scan counts (offs, *out_rows),
// 2 = compact slots into out
hipError_t launch_join(const int64_t *R, int64_t nr, int c1, int key1, const int64_t *S, int64_t ns, int c2,
                       int key2, const int64_t *apart, const int64_t *run_start, int64_t ntiles, int64_t *slots,
                       uint32_t *counts, uint32_t *offs, int64_t *out, int64_t *out_rows, int phase,
                       hipStream_t s);
hipError_t launch_merge_tiles(const int64_t *a, int64_t na, const int64_t *b, int64_t nb, int cols,
                              int key_col, const int64_t *apart, int64_t ntiles, int64_t *out,
                              hipStream_t s);
hipError_t read_phase_cycles(unsigned long long *out16);
// T = UINT64 (ktype 1) / DOUBLE (2): order-preserving map of the colmask
// columns onto int64 (inverse = 0) or back (inverse = 1); src may equal dst
hipError_t launch_key_map(const int64_t *src, int64_t *dst, int64_t rows, int cols, uint32_t colmask, int ktype,
                          int inverse, hipStream_t s);
// index-sort path for wide rows (smj_kernels.hip): (key, row id) pairs, row
// gathers by id, joined rows from (key, R id, S id) triples
hipError_t launch_row_pairs(const int64_t *src, int64_t n, int cols, int key, int use_sel, int sel_col,
                            int64_t sel_val, int ktype, int64_t row0, int64_t *out, hipStream_t s);
hipError_t launch_gather_rows(const int64_t *src0, int64_t n0, const int64_t *src1, int cols, const int64_t *ids,
                              int id_stride, int id_col, int64_t m, int64_t *dst, hipStream_t s);
hipError_t launch_join_gather(const int64_t *R, int c1, const int64_t *S, int c2, int key2, const int64_t *jp,
                              int64_t J, int64_t *out, hipStream_t s);
hipError_t launch_gen_uniform(int64_t *out, int64_t row0, int64_t rows, uint64_t seed,
                              uint64_t key_range, hipStream_t s);
hipError_t launch_gen_wide(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t plant_seed,
                           int64_t plant_rows, hipStream_t s);
hipError_t launch_gen_zipf(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, int64_t domain,
                           double theta, double zeta_n, hipStream_t s);
// distributed splitters (smj_dev_dist_sample / smj_dev_dist_splitters)
constexpr int kDistHdr = 5;         // [valid samples, samples of R, of S, rows of R, of S]
constexpr int kDistMaxParts = 64;   // splitters + 1 (the partition kernels' <= 64 buckets)
struct DistSampleArgs {
    const int64_t *t[2];
    int64_t n[2];
    int cols[2], key[2];
    int samples;
    int64_t *buf;                   // kDistHdr + 2 samples words
};
struct DistSelectArgs {
    const int64_t *all;             // world rows of `stride` words (gathered sample buffers)
    int64_t stride;
    int world, parts, use_q;
    int32_t q20[kDistMaxParts];     // stage fractions << 20 (use_q)
    int64_t *out;                   // parts words: parts - 1 splitters, then L
};
hipError_t launch_dist_sample(const DistSampleArgs &a, hipStream_t s);
hipError_t launch_dist_select(const DistSelectArgs &a, hipStream_t s);
// *out = sum over rows i of hash(pos0 + i, row i) mod 2^64 (smj_dev_digest)
hipError_t launch_digest(const int64_t *rows, int64_t n, int cols, int64_t pos0, uint64_t *out, hipStream_t s);

// ---------------------------------------------------------------------------
// MSD sample-sort pipeline (smj_msd.hip): sample -> part_a -> runs -> part_b
// -> group -> final (+ single / LSD fallback) -> compact.  DESIGN.md §3.
// ---------------------------------------------------------------------------
constexpr int kMsdThreads = 512;
constexpr int kMsdWaves = kMsdThreads / 64;
// rows per thread of a tile: a tile is <= 64 KiB of rows whatever the width
__host__ __device__ constexpr int msd_items(int cols) {
    return cols == 1 ? 16 : cols == 2 ? 8 : cols == 3 ? 5 : cols == 4 ? 4 : cols == 5 ? 3 : 2;
}
__host__ __device__ constexpr int msd_tile(int cols) { return kMsdThreads * msd_items(cols); }
// pass-A tiles: 2-column tables take 8192-row tiles (1024 threads, 128 KiB of
// staged rows, one workgroup per CU) with SMJ_PA_BIG=1, so that the bucket
// runs part_b gathers are ~32 rows long instead of ~16
#ifndef SMJ_PA_BIG
#define SMJ_PA_BIG 0
#endif
__host__ __device__ constexpr int pa_threads(int cols) { return (SMJ_PA_BIG && cols == 2) ? 1024 : kMsdThreads; }
// SMJ_PA_ITEMS: rows per thread of a 2-column pass-A tile (8: 4096 rows, two
// workgroups per CU; 6: 3072 rows, three)
#ifndef SMJ_PA_ITEMS
#define SMJ_PA_ITEMS 8
#endif
__host__ __device__ constexpr int pa_items(int cols) { return cols == 2 ? SMJ_PA_ITEMS : msd_items(cols); }
__host__ __device__ constexpr int msd_tile_a(int cols) { return pa_threads(cols) * pa_items(cols); }
__host__ __device__ constexpr int pa_waves_per_eu(int cols) {
    return pa_threads(cols) != kMsdThreads ? 4 : pa_items(cols) >= 8 ? 4 : 6;
}
// pass-B tiles (rows); part_b runs 1024 threads x 4 rows for 2-column tables
// (64 VGPRs, 2 x 16 waves per CU: part_b is latency-bound)
__host__ __device__ constexpr int msd_tile_b(int cols) { return msd_tile(cols); }
__host__ __device__ constexpr int pb_threads(int cols) { return cols == 2 ? 1024 : kMsdThreads; }
// Pass A: 255 sampled splitters, 256 buckets (an 8-bit digit).  Bucket a
// holds the keys in (spl[a-1], spl[a]]; a key value the sample saw more than
// once (spl[i] == spl[i+1]: a heavy key) gets bucket i + 1 to itself, and the
// buckets between its repeated splitters stay empty (bucket_a, msd_bases).
// At C3 a bucket holds ~3.9e5 rows per table, i.e. ~96 pass-B tiles whose
// runs a final group gathers (127 splitters and an odd single-key bucket per
// splitter -- the round-1 layout -- gave ~191 tiles of half the run length,
// and buckets over the final stage's 256-tile list from ~1.3e8 rows on).
#ifndef SMJ_BITS_A
#define SMJ_BITS_A 8
#endif
constexpr int kBitsA = SMJ_BITS_A;           // pass-A digit bits
constexpr int kBucketsA = 1 << kBitsA;       // 256 pass-A buckets
constexpr int kSplA = kBucketsA - 1;         // 255 pass-A splitters
constexpr int kOffsA = kBucketsA;            // per-bucket arrays (segment partials, bucket records)
constexpr int kOffsARow = kBucketsA + 8;     // offsA row (u32): 256 bucket starts + the tile's row count, 16-B padded
constexpr int kBitsB = 11;
constexpr int kRadB = 1 << kBitsB;         // 2048 pass-B sub-buckets per bucket
constexpr int kOffsB = kRadB + 8;          // offsB row (u16): 2048 starts + the tile's row count, padded to 16 B
constexpr int kGroupCap = 1024;            // rows per table in one final group (LDS)
constexpr int kStRows = 2 * kGroupCap;     // rows of both tables in one group of the staged final kernel
#ifndef SMJ_ST_LIST
#define SMJ_ST_LIST 256
#endif
constexpr int kStList = SMJ_ST_LIST;       // pass-B tiles per bucket and table a staged group may span
constexpr int kStageRange = 4096;          // key range of the staged final path's counting sort
#ifndef SMJ_BG_MAX_ROWS
#define SMJ_BG_MAX_ROWS 65536  // C5: 65536 beats 131072 and 32768 (profiles/r03/r03za/ab_c5_bg_max.txt)
#endif
constexpr uint32_t kBgMaxRows = SMJ_BG_MAX_ROWS;  // rows per table of an oversized group one workgroup sorts
constexpr uint32_t kBgSeg = 32768;               // rows per table of a job of a larger group (msd_giant_*)
// an oversized multi-key group sorted on the device (msd_big_stage_kernel /
// msd_giant_*, 2-column tables): keys spanning <= kStageRange values and a
// run list that fits LDS; the others take the host-driven fallback
// (smj_api.hip msd_fallback)
__host__ __device__ inline bool msd_big_on_device(uint32_t span, uint32_t ktR, uint32_t ktS) {
    return span <= (uint32_t)kStageRange && ktR <= (uint32_t)kGroupCap && ktS <= (uint32_t)kGroupCap;
}
// the thresholds in force: kBgMaxRows / kBgSeg, or SMJ_BG_MAX_ROWS / SMJ_BG_SEG
// from the environment (tests: giant groups at small sizes; the segment a
// multiple of kGroupCap)
// smj_debug_wide_maxrun: msd_final_wstage_kernel's bin limit override (-1: none)
extern int g_wide_maxrun;
struct MsdBgLimits {
    uint32_t max_rows, seg;
};
MsdBgLimits msd_bg_limits();
constexpr int kSlots = kBucketsA * kRadB;  // group slots (bucket-major = key order); groups <= kSlots
constexpr int kFinThreads = 256;           // final kernel workgroup (4 per CU)
constexpr int kFinWaves = kFinThreads / 64;
constexpr int kMsdFinalGrid = 1024;        // persistent final kernel: 4 workgroups per CU
constexpr int kMsdPartBGrid = 512;         // persistent part_b: 2 workgroups per CU
constexpr int kSampleMax = 4096;           // sampled keys per table
#ifndef SMJ_MSD_SEGS
#define SMJ_MSD_SEGS 256
#endif
constexpr int kMsdSegs = SMJ_MSD_SEGS;     // segments of the run scans (x 4 waves: ~24 tiles per lane at 1e8 rows)
constexpr int kGroupSlices = 8;            // tile slices per bucket in msd_group_sum_kernel
constexpr uint16_t kGroupEmpty = 1, kGroupSingle = 2, kGroupBig = 4;
// msd_single_kernel work item {group, kSingleRuns | c}: rows [c R, (c + 1) R)
// of a heavy key's sub-bucket (MsdGroup::pad[0] = 1), R = kSingleRunRows,
// copied run by run; else {group, chunk c of kGroupCap rows}
constexpr uint32_t kSingleRuns = 0x80000000u;
constexpr uint32_t kSingleRunRows = 8 * 1024;

struct MsdTable {        // an input table as the sampler and part_a see it
    const int64_t *src;
    int64_t n;
    int cols, key_col, use_sel, sel_col;
    int64_t sel_val;
    const uint64_t *desc = nullptr;  // a chunked part's tile descriptors (MsdPartAParams::desc), ntiles of tile rows
    int64_t ntiles = 0;
    int tile = 0;
    // packed input (2-column tables, no select; smj_dev_sort_merge_join_begin_pk):
    // row i is the one word src[i] = (int32 key - pkk) | (int32 other - pkp) << 32
    int pk = 0;
    int64_t pkk = 0, pkp = 0;
};
struct MsdSampleParams {
    MsdTable tab[2];
    int ntab;
    int64_t *spl;        // out: kSplA splitters
    int64_t *samp;       // scratch: 2 kSampleMax samples + per-block valid counts; then (select kernel, out)
                         // the valid samples in key order at samp + kSortedOff
    struct MsdPlan *plan;  // out (select kernel): plan->skew, sampled keys with an equal partner (nullptr: not counted)
};
struct MsdPartAParams {
    const int64_t *src;
    int64_t n;
    int use_sel, sel_col, key_col, tile0;  // tile0: first tile of this launch (staged H2D: one launch per chunk)
    int64_t sel_val;
    const int64_t *spl;
    int64_t *out;        // tempA: tile t's rows at [t*T, t*T + m_t)
    uint32_t *offs;      // [tiles][kOffsARow]
    int64_t *tmm;        // [tiles][2] min / max selected key
    // a part of the chunked partition (msd_part1c_kernel): tile t's rows are
    // desc[t] >> 16 (a row of src) and the desc[t] & 0xffff rows after it, in
    // order; ntiles tiles.  nullptr: tile t = rows [t T, t T + T) of src
    const uint64_t *desc = nullptr;
    int64_t ntiles = 0;
    int pk = 0;                  // packed input (MsdTable::pk)
    int64_t pkk = 0, pkp = 0;
    uint32_t *nopack = nullptr;  // 2-column tables: MsdPlan::nopack, set when a row's other column does not fit int32
};
struct MsdPartA2 {       // one part_a launch over up to two tables
    MsdPartAParams t[2];
    unsigned tiles0;     // blocks [0, tiles0) take table 0's tiles, the rest table 1's
};
// samp + kSortedOff: the select kernel's samples in key order (msd_bases_kernel's segmented digit)
constexpr int kSortedOff = 2 * kSampleMax + 64;
constexpr int kSampScratch = kSortedOff + 2 * kSampleMax + 64;  // int64 words of MsdScratch::samp (+ the
                                                                 // over-read of seg_plan's fixed-count loads)
// A segmented pass-B digit (MsdBucket::one_key bit 1, kBucketSeg): a bucket
// whose sampled keys sit in up to kSegMax dense intervals separated by wide
// empty gaps (clustered keys: an interval straddling two clusters 2^40 apart
// put both clusters' rows into one or two linear sub-buckets).  Interval k,
// [st[k], en[k]], gets dn[k] linear sub-buckets from db[k] on and the one
// after them holds the keys past en[k] up to st[k + 1] (the gap; keys in the
// gap are rare but legal):
//   k = the last interval with st[k] <= key (k = 0 below st[1]),
//   r = (key - st[k]) >> sh[k],
//   digit = db[k] + (r >= 2^32 ? dn[k] : min(dn[k], mulhi32(r, s32[k]))),
//   s32[k] = 2^32 dn[k] / (((en[k] - st[k]) >> sh[k]) + 1)   (keys <= en[k]: < dn[k]),
// sh[k] the shift that brings the interval under 2^32 (a 32-bit multiply in
// part_b).  st[0] = the bucket's lo, so every key of the bucket has an interval.
constexpr int kSegMax = 8;
constexpr uint32_t kBucketSeg = 2u;  // MsdBucket::one_key bit: the bucket's digit is MsdSeg's
struct MsdSeg {
    int64_t st[kSegMax];   // interval starts, ascending (st[0] = lo; unused entries repeat the last)
    uint32_t s32[kSegMax]; // interval scales
    uint32_t pk[kSegMax];  // db | dn << 11 | sh << 22
    int64_t hi;            // the bucket's last key
    uint32_t ms[kSegMax];  // sub-buckets a final group of the interval may span (MsdBucket::maxspan)
    uint32_t nseg, pad[21];
};
// seg_find's intervals of a bucket (extra workgroups of msd_runs_seg_kernel)
// for msd_bases_kernel, which sizes their sub-buckets
struct MsdSegFind {
    int64_t st[kSegMax], en[kSegMax];
    float wt[kSegMax];   // expected rows (width in sample spacings)
    uint32_t K, topcut;  // K = 0: not segmented; topcut: the last interval ends before hi
    uint32_t pad[6];
};
__host__ __device__ inline uint32_t seg_db(uint32_t pk) { return pk & 0x7ffu; }
__host__ __device__ inline uint32_t seg_dn(uint32_t pk) { return (pk >> 11) & 0x7ffu; }
__host__ __device__ inline uint32_t seg_sh(uint32_t pk) { return pk >> 22; }
static_assert(sizeof(MsdSeg) == 256 && offsetof(MsdSeg, hi) == 128, "part_b loads st, s32, pk: 16 words");
struct MsdBucket {       // per pass-A bucket and table
    int64_t lo;          // pass-B digit (common to R and S): with r = key - lo,
    uint64_t scale;      //   scale == 0: r (interval < kRadB keys: one key per sub-bucket)
                         //   else min(kRadB - 1, mulhi(r, scale)), scale = 2^64 * kRadB / (hi - lo + 1)
    uint32_t maxspan;    // sub-buckets a final group may span (its key range stays < 2^48)
    uint32_t L;          // rows of this table in the bucket
    uint32_t row_start;  // first sorted-output row of the bucket
    uint32_t list_base;  // first run-list entry
    uint32_t nruns;      // run-list entries
    uint32_t tile_base;  // first pass-B tile
    uint32_t one_key;    // bit 0: the bucket's interval is a single key value (a heavy key's bucket);
                         // bit 1 (kBucketSeg): the pass-B digit is the segmented one (MsdSeg; scale,
                         // s32 and maxspan unused);
                         // bits 8..15: m, the bucket's heavy keys (msd_heavy_kernel): the pass-B digit
                         // is then d = lin(r) + 2 c + e over D - 2 m linear sub-buckets, c = heavy keys
                         // below the key, e = the key is one -- every heavy key a sub-bucket of its own
    uint32_t s32;        // != 0 (interval < 2^32 keys): the digit is mulhi32(r, s32) instead
};
// Heavy keys of a multi-key pass-A bucket (C5's Zipf tables: keys with
// thousands of rows next to light ones, which made oversized sub-buckets for
// msd_big_stage / msd_giant_*): found from a sample of the bucket's rows,
// <= kHeavyMax per bucket, each given a sub-bucket of its own by the pass-B
// digit -- a single-key group, streamed in stable order by msd_single_kernel
constexpr int kHeavyMax = 64;
#ifndef SMJ_HEAVY_SAMPLES
#define SMJ_HEAVY_SAMPLES 1024  // (2048: msd_heavy 0.44 -> 0.28 ms per C5 step at 1024, C5 -0.2 ms; r05zc)
#endif
constexpr int kHeavySamples = SMJ_HEAVY_SAMPLES;  // sampled rows per bucket (both tables)
constexpr uint32_t kHeavyRows = 768;  // a key is heavy from ~this many rows (sample hits scaled)
__host__ __device__ inline uint32_t msd_heavy_count(uint32_t one_key_word) { return (one_key_word >> 8) & 0xffu; }
struct MsdHeavyParams {
    const int64_t *tempA[2];   // pass-A tiles (msd_part_a)
    const uint32_t *offs[2];   // [tiles][kOffsARow] bucket starts
    int64_t ntiles[2];
    int tile[2], cols[2], key[2];  // pass-A tile rows, columns, key column
    const uint32_t *totL[2];   // rows per bucket (msd_seg_scan_kernel)
    const int64_t *spl;        // pass-A splitters
    int ntab;
    int64_t *heavy;            // out: [kBucketsA][kHeavyMax] ascending heavy keys
    uint32_t *nheavy;          // out: [kBucketsA] their count
    const struct MsdPlan *plan;  // plan->skew (msd_sample_select)
};
struct MsdPlan {         // device-side pipeline state (zeroed per call)
    uint32_t m[2];       // selected rows per table
    uint32_t ntilesB[2]; // pass-B tiles per table
    uint32_t nsingle, nbig;
    int64_t gmin, gmax;
    int64_t joined;      // written by the count scan
    uint32_t ngroups;    // dense groups (key order)
    uint32_t nwide;      // groups for the 64-bit final path
    uint32_t nradix;     // groups for the radix-sort final path
    uint32_t nlsd;       // staged groups sorted by the in-LDS LSD (equal-key runs over kMaxDupRun)
    uint32_t nbigdev;    // oversized multi-key groups sorted on the device (msd_big_stage_kernel)
    uint32_t bgticket[2];// msd_big_stage_kernel's group tickets (large groups first, then the rest)
    uint32_t ngiant;     // groups over kBgMaxRows rows registered as jobs
    uint32_t njobs;      // their jobs
    uint32_t err;        // bit 0: a cross-workgroup wait gave up (msd_group_kernel) -> SMJ_ERR_TIMEOUT;
                         // bit 1: inconsistent run metadata (SMJ_BOUNDS builds) -> SMJ_ERR_HIP;
                         // bit 2: a combined group missed the staged kernel (a bug) -> SMJ_ERR_HIP;
                         // bit 3: a dense group index past kSlots (a bug) -> SMJ_ERR_HIP.
                         // Every kernel after msd_group_kernel returns at entry once err != 0
                         // (msd_plan_failed), so a failed plan never drives a gather or a store.
    uint32_t gticket;    // msd_group_kernel: bucket tickets, taken in the order workgroups start
    uint32_t skew;       // msd_sample_select: sampled keys that another sample repeats (skew: msd_heavy_kernel runs)
    // Packed pass-B rows (2-column tables): part_b writes each row as ONE word
    // (uint32) key | (uint32) other << 32 -- the key's low 32 bits and the
    // other column, which must fit int32 -- so it writes, and the staged final
    // kernel gathers, 8 B per row instead of 16.  A key is rebuilt from its
    // group's base: base + (uint32)(lo32 - (uint32)base), exact while
    // key - base < 2^32 (the staged kernel's groups span <= 4096 keys; every
    // group lies in [gmin, gmax], so packB requires gmax - gmin < 2^32).  The
    // other final tiers read 16-B rows that msd_unpack_groups_kernel expands
    // into tempA (dead after part_b) for exactly the groups the staged kernel
    // does not take.
    uint32_t nopack;     // part_a: a selected row's other column does not fit int32
    uint32_t packB;      // msd_bases: pass-B rows are packed in this call
    uint32_t nwst;       // groups of a key span over kStageRange left by the staged kernel to
                         // msd_final_wstage_kernel (full-range keys: SURVEY 8(d)'s C3-wide)
    uint32_t nsegb;      // msd_bases: buckets given a segmented pass-B digit (MsdSeg)
};
// A kernel launched after msd_group_kernel reads the plan's error word first:
// a set bit means the dense group array may hold slots this call never wrote.
__device__ __forceinline__ bool msd_plan_failed(const MsdPlan *pl) {
    return __builtin_expect(*(const volatile uint32_t *)&pl->err != 0u, 0);
}
constexpr uint32_t kMsdSpinLimit = 1u << 26;  // polls before a cross-workgroup wait gives up
struct MsdBasesParams {
    const uint32_t *totL[2];   // rows / runs of each bucket over all pass-A tiles (msd_seg_scan_kernel)
    const uint32_t *totC[2];
    const int64_t *segmm[2];   // [kMsdSegs * 4][2] min / max partials
    int64_t ntiles[2];
    int tile[2];
    int ntab;
    int full_radix;            // ablation (SMJ_PASSB_FULL=1): D = kRadB pass-B sub-buckets in every bucket
    int combined;              // 2-column tables: final groups of <= 2 kGroupCap rows of both tables together
    const int64_t *spl;
    MsdBucket *bk[2];
    MsdPlan *plan;
    int pack_ok;               // msd_packb_mode() with 2-column tables: MsdPlan::packB may be set (2: despite skew)
    const uint32_t *nheavy;    // [kBucketsA] heavy keys per bucket (msd_heavy_kernel), nullptr = none
    const MsdSegFind *segf;    // [kBucketsA] intervals (msd_runs_seg_kernel); nullptr = none (SMJ_SEG=0)
    MsdSeg *seg;               // out: [kBucketsA] segmented digits
};
struct MsdPartBParams {
    const int64_t *srcA;
    int64_t *out;        // tempB: pass-B tile g at rows [g*T, g*T + rows)
    const uint2 *list;
    const uint2 *tinfo;  // per pass-B tile: {bucket, first run-list entry}
    const MsdBucket *bk;
    const MsdPlan *plan;
    uint16_t *offs;      // [tilesB][kOffsB] tile-local sub-bucket starts
    int key_col, x;
    int dbg;             // SMJ_DEBUG_MSD: phase stamps (tools/msd_phases.py)
    const int64_t *heavy;  // [kBucketsA][kHeavyMax] heavy keys (MsdBucket::one_key bits 8..15: how many)
    const MsdSeg *seg;     // [kBucketsA] segmented digits (MsdBucket::one_key & kBucketSeg)
};
struct MsdGroup {        // one final group: sub-buckets [b0, b1) of bucket a
    uint16_t a, flags, b0, b1;
    uint32_t nR, nS, outR, outS;
    uint32_t tb[2];      // first pass-B tile of the bucket, per table
    uint32_t kt[2];      // pass-B tiles of the bucket, per table
    int64_t base;        // smallest key the group's sub-buckets can hold
    uint32_t span;       // keys the group's sub-buckets can hold (saturated): key - base < span
    uint32_t pad[3];     // [0]: 1 = one heavy key's sub-bucket (msd_single); [1], [2]: a group spanning
                         // over kStageRange keys, the low / high half of its bin scale (msd_final_wstage_kernel)
};
struct MsdGroupParams {
    const uint16_t *offs[2];
    const MsdBucket *bk[2];
    int tile[2];
    int ntab;
    uint32_t *part;         // [2][kBucketsA][kGroupSlices][kRadB] partial sub-bucket totals
    uint32_t *ngrp;         // [kBucketsA] groups per bucket | kGrpReady (published for the later buckets)
    MsdGroup *groups;       // dense, key order
    uint32_t *counts;       // dense: join rows per group (single-key groups: known here)
    MsdPlan *plan;
    uint32_t *single_list, *big_list;  // dense group indices
    int combined;           // as MsdBasesParams::combined
    uint32_t spin_limit;    // polls of the look-back before it gives up (kMsdSpinLimit; 0 in the forced-timeout test)
    const int64_t *heavy;   // as MsdPartBParams::heavy
    const MsdSeg *seg;      // as MsdPartBParams::seg
};
struct MsdTab {          // a table as the final kernels see it
    const int64_t *tempB;
    const uint16_t *offs;
    const MsdBucket *bk;
    int64_t *out;        // sorted rows
    int tile, cols, key, x;
    int64_t capB;        // rows tempB holds (SMJ_BOUNDS builds check gathers against it)
};
struct MsdFinalParams {
    MsdTab tab[2];
    const MsdGroup *groups;
    int64_t *slots;      // join rows of group s at slot row groups[s].outR
    uint32_t *counts;
    MsdPlan *plan;
    uint32_t *big_list;
    uint32_t *single_list = nullptr;  // msd_group's single-key groups (msd_unpack_groups_kernel)
    uint32_t *wide_list; // dense indices of groups for msd_final_wide_kernel
    uint32_t *radix_list;// groups for the radix tier (msd_final_kernel in list mode; nullptr = contiguous mode)
    uint4 *giant;        // groups over kBgMaxRows rows: {dense group, first job, jobs}
    uint32_t *gmap;      // job -> its giant entry
    uint32_t *gh;        // [job][2][kStageRange] residual counts of each job's rows
    uint32_t bg_max, bg_seg;  // msd_bg_limits()
    int ntab, join, key2, dbg;
    int combined;        // the group kernel packed combined groups (staged kernel: R rows then S rows in one sort)
    int64_t *shadow[2] = {nullptr, nullptr};  // packB: 16-B rows of the groups the staged kernel does not take
                                              // (tempA, >= capB rows); nullptr: packing off for the call
    int pk_mode = -1;    // 2: the call may pack its pass-B rows (MsdPlan::packB, known on the device only) --
                         // the radix / wide tiers then read p.shadow; -1: rows
};

// ---- C-ABI internals shared by smj_api.hip and smj_host.hip -------------------
// frees every library-owned device / pinned buffer (smj_finalize)
void api_free_all();
// Device memory the library owns goes through these: hipMalloc / hipFree plus
// the held-byte account behind smj_scratch_bytes / smj_set_scratch_limit.
hipError_t dev_alloc_raw(void **p, size_t n);
hipError_t dev_free(void *p);
template <class X>
inline hipError_t dev_alloc(X **p, size_t n) { return dev_alloc_raw(reinterpret_cast<void **>(p), n); }
int64_t dev_held_bytes();
// after a top-level call: release every scratch buffer when the library holds
// more than the caller's limit (smj_set_scratch_limit); the call's work is done
void trim_if_over_limit();
int open_jobs();  // smj_dev_sort_merge_join_begin jobs not yet ended (all threads)
// worker threads of the multi-device host API give each device of the set its
// own scratch (several may map to one physical device); -1 = per device
void set_scratch_slot(int slot);
// the fused pipeline on host tables copied in chunks that overlap part_a
// (smj_api.hip); SMJ_ERR_UNSUPPORTED where the plain path must run instead
int msd_staged_sort_merge_join(const int64_t *hR, int64_t nr, int c1, int sc1, int64_t sv1, int key1,
                               const int64_t *hS, int64_t ns, int c2, int sc2, int64_t sv2, int key2, int64_t *dR,
                               int64_t *dS, int64_t *dRs, int64_t *dSs, int64_t *dJ, int64_t *h_rows, hipStream_t s,
                               hipStream_t copy, hipEvent_t landed);

// the partitioned mode's one-pass range partition (msd_part1_kernel): its
// tile (SMJ_P1_ITEMS rows per thread for 2-column tables; fewer rows = less
// LDS = more workgroups per CU to hide the look-back) and occupancy
#ifndef SMJ_P1_ITEMS
#define SMJ_P1_ITEMS 8
#endif
__host__ __device__ constexpr int p1_items(int cols) { return cols == 2 ? SMJ_P1_ITEMS : msd_items(cols); }
__host__ __device__ constexpr int p1_tile(int cols) { return kMsdThreads * p1_items(cols); }
__host__ __device__ constexpr int p1_waves_per_eu(int cols) { return p1_items(cols) >= 8 ? 4 : p1_items(cols) >= 6 ? 6 : 8; }
struct MsdPart1Params {
    const int64_t *src;
    int64_t n;
    int use_sel, sel_col, key_col, nspl;
    int64_t sel_val;
    const int64_t *spl;          // device: nspl part splitters (part of a key = #{splitters < key})
    const int64_t *oc;           // device [128]: region start of part b (rows), then its capacity
    int64_t *dst;                // staging buffer of the regions
    unsigned long long *status;  // [ntiles][nspl + 1] look-back words, zeroed
    long long *tot;              // [nspl + 1]: rows per part (written by the last tile)
    uint32_t *flags;             // [0] tile ticket, [1] a region overflowed, [2] look-back timeout,
                                 // [3] a packed row did not fit (pk); zeroed
    int64_t ntiles;
    // packed output (2-column tables; smj_dev_partition_regions_pk): row = one
    // word (int32 key - pkk) | (int32 other - pkp) << 32, differences taken
    // mod 2^64 -- a row whose differences do not fit int32 sets flags[3]
    int pk = 0;
    int64_t pkk = 0, pkp = 0;
};
hipError_t launch_unpack_rows(const int64_t *packed, int64_t n, int key_col, int64_t pkk, int64_t pkp, int64_t *out,
                              hipStream_t s);
hipError_t launch_msd_part1(const MsdPart1Params &p, int cols, hipStream_t s);
// The chunked one-pass partition (msd_part1c_kernel): no look-back.  A
// persistent grid of G workgroups; workgroup g takes the consecutive tiles
// [g K, g K + K) in order and appends part b's rows to its own sub-region
// [st[b] + g cap[b], + cap[b]) of the staging buffer, so part b = the G
// sub-regions' filled prefixes in g order (input order).  cnt[g * 64 + b] =
// the rows it wrote there; flags[1] = a sub-region overflowed.  The part's
// tile descriptors for part_a then come from msd_p1c_desc_kernel.
struct P1cWords {  // sub-region starts of part b [0, 64) and per-chunk capacities [64, 128), rows; splitters [128, 192)
    int64_t v[192];
};
struct MsdPart1cParams {
    const int64_t *src;
    int64_t n;
    int use_sel, sel_col, key_col, nspl;
    int64_t sel_val;
    int64_t *dst;
    uint32_t *cnt;               // [G][64] rows per (chunk, part)
    uint32_t *flags;             // [1]: a sub-region overflowed (zeroed by the caller)
    int64_t ntiles, chunk;       // p1_tile rows per tile; tiles per workgroup
};
hipError_t launch_msd_part1c(const MsdPart1cParams &p, const P1cWords &w, int cols, int grid, hipStream_t s);
int msd_part1c_grid(int cols);   // resident workgroups of the chunked partition (G)
// part b's part_a tile descriptors at desc + dbase[b]: chunk g's rows in tiles
// of tile rows (the last one partial), chunks in order
struct P1cDesc {
    int64_t st[64], cap[64], dbase[64];
};
hipError_t launch_p1c_desc(const uint32_t *cnt, int G, int nb, int tile, const P1cDesc &d, uint64_t *desc, hipStream_t s);
struct P1Words {  // region starts [0, 64) and capacities [64, 128), rows; splitters [128, 192)
    int64_t v[192];
};
hipError_t launch_p1_words(const P1Words &w, int64_t *oc, uint32_t *flags, hipStream_t s);
hipError_t launch_p1_finish(const uint32_t *flags, int64_t *out, hipStream_t s);
hipError_t launch_msd_sample(const MsdSampleParams &p, hipStream_t s);
// the sample gather alone: samp[x * kSampleMax + j] = sampled key j of table x
// (INT64_MAX for a row the select drops or a missing row), samp[2 kSampleMax
// + b] = valid samples of gather block b (blocks [0, 16) sample table 0)
hipError_t launch_msd_sample_gather(const MsdSampleParams &p, hipStream_t s);
constexpr int kSampleGatherBlocksH = 2 * kSampleMax / 256;
hipError_t launch_msd_part_a(const MsdPartAParams &p, int cols, hipStream_t s);
// both tables (the same column count) in one launch: no tail between them
hipError_t launch_msd_part_a2(const MsdPartAParams &a, const MsdPartAParams &b, int cols, hipStream_t s);
// tiles [t0, t1) only (their rows must be resident: the staged host path)
hipError_t launch_msd_part_a_tiles(const MsdPartAParams &p, int cols, int64_t t0, int64_t t1, hipStream_t s);
// the splitter selection alone, over samples already in p.samp (host-side gather)
hipError_t launch_msd_sample_select(const MsdSampleParams &p, hipStream_t s);
// per-bucket run sums and counts per segment; also the selected-key min / max
// per (segment, wave): segmm[kMsdSegs * 4][2] (256 entries, INT64_MAX / MIN when empty)
struct MsdRunsArgs {     // msd_runs_seg / msd_runs_apply over both tables (blockIdx.z = table)
    const uint32_t *offs[2];
    int64_t ntiles[2];
    uint32_t *segL[2], *segC[2];
    const int64_t *tmm[2];
    int64_t *segmm[2];
    // the segmented digit's sample scan (seg_find_all, extra workgroups of msd_runs_seg_kernel; segf =
    // nullptr: none): samples in key order (MsdSampleParams::samp), splitters, plan->skew.  (Before T:
    // a host source's macro T = int64_t turns `int T[2]` into a member named int64_t.)
    const int64_t *seg_samp = nullptr;
    const int64_t *seg_spl = nullptr;
    const MsdPlan *seg_plan = nullptr;
    MsdSegFind *segf = nullptr;
    int T[2], TB[2];
    const MsdBucket *bk[2];
    uint2 *list[2], *tinfo[2];
    int ntab;
};
hipError_t launch_msd_runs_seg(const MsdRunsArgs &a, hipStream_t s);

hipError_t launch_msd_seg_scan(uint32_t *const *seg, uint32_t *const *tot, int narr, hipStream_t s);
hipError_t launch_msd_bases(const MsdBasesParams &p, hipStream_t s);
hipError_t launch_msd_heavy(const MsdHeavyParams &p, hipStream_t s);
hipError_t launch_msd_runs_apply(const MsdRunsArgs &a, hipStream_t s);
// pb_pack: the call may pack its pass-B rows (MsdPlan::packB decides on the device)
hipError_t launch_msd_part_b(const MsdPartBParams &p, int cols, int64_t max_tiles, hipStream_t s, bool pb_pack = false);
hipError_t launch_msd_group(const MsdGroupParams &p, hipStream_t s);
hipError_t launch_msd_final(const MsdFinalParams &p, hipStream_t s);
hipError_t launch_msd_final_tiers(const MsdFinalParams &p, hipStream_t s);  // 2-column: wide-span kernels, radix, 64-bit tiers
int msd_packb_mode();
// the single-key / oversized groups' rows unpacked into MsdFinalParams::shadow (packed calls)
hipError_t launch_msd_unpack_groups(const MsdFinalParams &p, hipStream_t s);  // packed pass-B rows (MsdPlan::packB): 0 off, 1 on unskewed tables, 2 forced (SMJ_PACKB)
hipError_t launch_msd_big(const MsdFinalParams &p, hipStream_t s);
hipError_t launch_msd_single(const MsdFinalParams &p, const uint2 *work, int64_t nwork, hipStream_t s);
// out[i] = groups[list[i]] over the single-key then oversized list entries
hipError_t launch_msd_pick_groups(const MsdGroup *groups, const uint32_t *single_list, const uint32_t *big_list,
                                  uint32_t nsingle, uint32_t nbig, MsdGroup *out, hipStream_t s);
// batched fallback (oversized multi-key groups): see smj_msd.hip
hipError_t launch_msd_gather_list(const MsdTab &tb, const MsdGroup *groups, const uint4 *work, int64_t nwork,
                                  int64_t *dst, hipStream_t s);
hipError_t launch_msd_seg_copy(const int64_t *src, int64_t *dst, const uint4 *work, int64_t nwork, int cols,
                               hipStream_t s);
hipError_t launch_msd_big_split(const int64_t *J, const int64_t *nJ, int tc, const int64_t *Rs, int c1, int key1,
                                const uint4 *work, int64_t nwork, const MsdGroup *groups, int64_t *slots,
                                uint32_t *counts, hipStream_t s);
// groups with at most kGroupCap join rows; after_fallback == 0: nothing when the plan has oversized groups
hipError_t launch_msd_compact(const int64_t *slots, const MsdGroup *groups, const uint32_t *counts,
                              const uint32_t *offs, const MsdPlan *plan, int tc, int64_t *out, int after_fallback,
                              hipStream_t s);
// groups over kGroupCap join rows: work = {dense group, chunk of kCompactChunk rows}
constexpr uint32_t kCompactChunk = 4096;
hipError_t launch_msd_compact_big(const int64_t *slots, const MsdGroup *groups, const uint32_t *counts,
                                  const uint32_t *offs, const uint2 *work, int64_t nwork, int tc, int64_t *out,
                                  hipStream_t s);
hipError_t read_msd_phases(unsigned long long *out16);  // diagnostic (SMJ_DEBUG_MSD=1)
// diagnostic (SMJ_STAMPS build, SMJ_DEBUG_BIG=1): [0..31] cycles and [32..63]
// groups of msd_big_stage_kernel per log2 size class, [64..71] cycles per phase
hipError_t read_big_times(unsigned long long *out72);
// exclusive scan of the plan->ngroups dense group counts -> offs, total -> plan->joined
hipError_t launch_msd_count_scan(const uint32_t *counts, uint32_t *part, uint32_t *offs, MsdPlan *plan,
                                 hipStream_t s);
// exclusive scan of n u32 counts -> offs, total -> *total (one workgroup)
hipError_t launch_count_scan(const uint32_t *counts, int64_t n, uint32_t *offs, int64_t *total, hipStream_t s);

}  // namespace smj
