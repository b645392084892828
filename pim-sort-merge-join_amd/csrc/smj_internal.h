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
constexpr int kBucketBits = 4;                   // multi-GPU partition: <= 16 buckets
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
    uint32_t err;        // set by kernels when a look-back wait timed out
    uint32_t pad;
};

// Device scratch counters.  {tile, count} are zeroed before every launch
// (8-byte memset); err is sticky for the whole API call.
struct Counters {
    uint32_t tile;       // dynamic tile id
    uint32_t count;      // rows emitted (select-only passes)
    uint32_t err;        // look-back wait timed out
    uint32_t pad;
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
hipError_t launch_gen_uniform(int64_t *out, int64_t row0, int64_t rows, uint64_t seed,
                              uint64_t key_range, hipStream_t s);
hipError_t launch_gen_zipf(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, int64_t domain,
                           double theta, double zeta_n, hipStream_t s);

}  // namespace smj
