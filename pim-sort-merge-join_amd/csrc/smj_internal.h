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
constexpr int kSortThreads = 512;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kRadixBits = 10;                   // digit width of the radix passes
constexpr int kRadix = 1 << kRadixBits;          // 1024 bins
constexpr int kNumPos = (64 + kRadixBits - 1) / kRadixBits;  // 7 digit positions
constexpr int kBucketBits = 4;                   // multi-GPU partition: <= 16 buckets
constexpr int kMaxSplitters = (1 << kBucketBits) - 1;

// rows per thread per tile: a tile is 64 KiB of rows whatever the row width
__host__ __device__ constexpr int sort_items(int cols) { return cols >= 8 ? 2 : (16 / cols); }
__host__ __device__ constexpr int sort_tile_rows(int cols) { return sort_items(cols) * kSortThreads; }

// Join / merge geometry: one workgroup per merge-path tile of kJoinTile
// merged elements (R-piece + S-piece).
constexpr int kJoinThreads = 512;
constexpr int kJoinPer = 8;
constexpr int kJoinTile = kJoinThreads * kJoinPer;  // 4096

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

hipError_t launch_hist_radix(const int64_t *src, int64_t n, int cols, int use_select, int sel_col,
                             int64_t sel_val, int key_col, uint64_t key_base, uint32_t *ghist,
                             hipStream_t s);
hipError_t launch_plan(uint32_t *ghist, SortPlan *plan, hipStream_t s);
hipError_t launch_radix_pass(const int64_t *src, int64_t nsrc, int64_t *dst, int cols,
                             int use_select, int sel_col, int64_t sel_val, int key_col,
                             uint64_t key_base, int shift, const uint32_t *bin_base,
                             uint32_t *status, Counters *ctr, hipStream_t s);
hipError_t launch_compact_pass(const int64_t *src, int64_t nsrc, int64_t *dst, int cols,
                               int sel_col, int64_t sel_val, uint32_t *status, Counters *ctr,
                               hipStream_t s);
hipError_t launch_hist_bucket(const int64_t *src, int64_t n, int cols, int use_select, int sel_col,
                              int64_t sel_val, int key_col, const int64_t *spl, int nspl,
                              unsigned long long *gcount, long long *gminmax, hipStream_t s);
hipError_t launch_bucket_pass(const int64_t *src, int64_t nsrc, int64_t *dst, int cols,
                              int use_select, int sel_col, int64_t sel_val, int key_col,
                              const int64_t *spl, int nspl, const uint32_t *bin_base,
                              uint32_t *status, Counters *ctr, hipStream_t s);
hipError_t launch_merge_partition(const int64_t *a, int64_t na, int ca, int ka, const int64_t *b,
                                  int64_t nb, int cb, int kb, int64_t *apart, int64_t ntiles,
                                  hipStream_t s);
hipError_t launch_join_tiles(const int64_t *R, int64_t nr, int c1, int key1, const int64_t *S,
                             int64_t ns, int c2, int key2, const int64_t *apart, int64_t ntiles,
                             int64_t *out, int64_t *out_rows, uint32_t *status, Counters *ctr,
                             hipStream_t s);
hipError_t launch_merge_tiles(const int64_t *a, int64_t na, const int64_t *b, int64_t nb, int cols,
                              int key_col, const int64_t *apart, int64_t ntiles, int64_t *out,
                              hipStream_t s);
hipError_t launch_gen_uniform(int64_t *out, int64_t row0, int64_t rows, uint64_t seed,
                              uint64_t key_range, hipStream_t s);
hipError_t launch_gen_zipf(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, int64_t domain,
                           double theta, double zeta_n, hipStream_t s);

}  // namespace smj
