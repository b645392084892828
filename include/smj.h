/*
 * smj.h -- C-ABI of libsmj_hip.so, the MI355X sort-merge-join library.
 *
 * This is the drop-in boundary for the reference's DPU path.  The reference
 * host (sort-merge-join/app.c) drives four UPMEM kernels through the UPMEM
 * host API (include/dpu/dpu.h): dpu_alloc / dpu_load / dpu_prepare_xfer /
 * dpu_push_xfer / dpu_launch / dpu_free.  Each entry point below replaces one
 * reference kernel together with the transfers around it; the comment on
 * each cites the reference interface it replaces.
 *
 * Conventions (mirroring dpu_error_t, include/dpu/dpu_error.h:19):
 *   - every int-returning call returns SMJ_OK (0) or a negative SMJ_ERR_*;
 *   - SMJ_ASSERT() mirrors DPU_ASSERT (include/dpu/dpu.h:130-144): print and
 *     exit(EXIT_FAILURE) on error;
 *   - host-pointer calls are blocking (like dpu_launch(set, DPU_SYNCHRONOUS),
 *     app.c:247) and not re-entrant; one host thread drives the library;
 *   - tables are row-major T[row_num * col_num] (common.h).  The library's
 *     cells are 64-bit; the entry points below take int64 tables (the
 *     reference default, INT64).  Builds with T = uint64_t / double (common.h
 *     UINT64 / DOUBLE) reach the fused pipeline through the *_typed entry
 *     points; smj_sort_merge_join / smj_dev_sort_merge_join map to them;
 *   - row counts must be < 2^31 per table (dpu_block_t.row_num is an int,
 *     common.h:17) and col_num in [1, 1024].  Tables over 1.6e8 rows are
 *     range-partitioned on the key inside the library (in one pass into
 *     part regions of ~1.3-1.6x the table of library scratch when the device
 *     has room, else counted and scattered in place; the regions stay
 *     allocated for the next call until smj_trim / smj_finalize (or a
 *     budget, smj_set_scratch_limit), and are released when they cannot all
 *     be had; two parts are in flight at once, on two library streams with
 *     two sets of per-part scratch, both kept the same way -- ~5 GB each at
 *     1e9 x 1e9), tables over 8 columns
 *     are sorted as (key, row id) pairs and gathered; the
 *     LSD and partition entry points take 1..8 columns (else
 *     SMJ_ERR_UNSUPPORTED).
 *
 * Two layers:
 *   smj_*      host pointers, exactly the reference's data flow (app.c);
 *   smj_dev_*  device pointers + a HIP stream, for device-resident pipelines
 *              (bench.py, the multi-GPU driver).  No torch types anywhere.
 */
#ifndef SMJ_H
#define SMJ_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string.h>

#include "common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (dpu_error_t analogue) ------------------------------- */
#define SMJ_OK 0
#define SMJ_ERR_INVALID (-1)      /* bad argument / descriptor             */
#define SMJ_ERR_HIP (-2)          /* a HIP runtime call failed             */
#define SMJ_ERR_NOMEM (-3)        /* device or host allocation failed      */
#define SMJ_ERR_NODEVICE (-4)     /* no gfx950 device / smj_init missing   */
#define SMJ_ERR_TOO_LARGE (-5)    /* row count >= 2^31 or over 1024 columns */
#define SMJ_ERR_TIMEOUT (-6)      /* an in-kernel look-back wait timed out */
#define SMJ_ERR_UNSUPPORTED (-7)

#define SMJ_MAX_COLS 1024  /* tables over 8 columns take the index-sort path */
#define SMJ_MAX_ROWS ((int64_t)1 << 31)

const char *smj_strerror(int code);

/* DPU_ASSERT analogue (include/dpu/dpu.h:130-144). */
#define SMJ_ASSERT(stmt)                                                              \
    do {                                                                              \
        int smj_assert_rc_ = (stmt);                                                  \
        if (smj_assert_rc_ != SMJ_OK) {                                               \
            fprintf(stderr, "%s:%d(%s): SMJ error in %s: %s\n", __FILE__, __LINE__,   \
                    __func__, #stmt, smj_strerror(smj_assert_rc_));                   \
            exit(EXIT_FAILURE);                                                       \
        }                                                                             \
    } while (0)

/* Phase timing in the reference's three buckets (app.c:136-138, :763-772):
 * host->device copies, device kernels, device->host copies (milliseconds). */
typedef struct {
    double cpu_gpu_ms;
    double gpu_ms;
    double gpu_cpu_ms;
} smj_timing_t;

/* ---- lifetime ----------------------------------------------------------- */
/* Replaces dpu_alloc(NR_DPUS, profile, &set) (include/dpu/dpu.h:164; called
 * at app.c:175,315,422,638): the device set of the host-pointer API is GPUs
 * 0 .. n_gpus - 1 (n_gpus <= 0 or over the visible count: all visible).
 * Returns the number of GPUs in the set (>= 1) or a negative error.  With
 * more than one, smj_sort_merge_join and smj_sort shard their tables over
 * every GPU of the set (range partition + one exchange over xGMI, one host
 * worker thread per GPU); smj_select / smj_merge / smj_join run on the
 * first. */
int smj_init(int n_gpus);
/* The device set as an explicit list of HIP device ids; an id may repeat
 * (several shards on one GPU: tests the sharded path on one device).
 * Returns n or a negative error. */
int smj_init_devices(const int *device_ids, int n);
/* Size of the current device set (0 before smj_init). */
int smj_device_count(void);
/* Replaces dpu_free(set) (include/dpu/dpu.h:189; app.c:307,402,503,761):
 * releases the device set and every library-owned buffer. */
void smj_finalize(void);
/* Returns every device buffer the library holds -- per-call scratch, the
 * partitioned mode's part regions and second scratch set, the device set's
 * staging buffers -- once the work on them has drained (it synchronises the
 * devices).  The device set and its streams stay; the next call allocates
 * again.  The per-phase dpu_free of the reference (app.c:307,402,503,761)
 * without ending the set.  SMJ_ERR_INVALID while a
 * smj_dev_sort_merge_join_begin job is open. */
int smj_trim(void);
/* Device bytes the library holds now (scratch of every kind). */
int64_t smj_scratch_bytes(void);
/* A byte budget: a pipeline call that ends with the library holding more
 * than `bytes` trims (smj_trim) before it returns.  -1 (the default, or the
 * environment's SMJ_SCRATCH_LIMIT): keep scratch for the next call. */
void smj_set_scratch_limit(int64_t bytes);
/* Version string of the library build. */
const char *smj_version(void);

/* ---- host-pointer API: one call per reference kernel ------------------- */

/* select.c (main :63-194; host side app.c:172-307):
 *   out <- rows of `in` with row[select_col] > select_val (signed 64-bit),
 *   input order kept.  bl->col_num / bl->row_num describe `in`; `out` must
 *   hold bl->row_num rows; *out_rows gets the kept count. */
int smj_select(const dpu_block_t *bl, const int64_t *in, int64_t *out, int select_col, int64_t select_val,
               int *out_rows);

/* sort_dpu.c (main :189-328; host side app.c:309-406) + the merge tree:
 *   stable ascending sort of bl->row_num rows on row[key_col] (signed),
 *   in place from the caller's view.  Stability matches cpu_app.c
 *   insertion_sort_in_cpu (:172-202), the parity target. */
int smj_sort(const dpu_block_t *bl, int64_t *rows, int key_col);

/* merge_dpu.c (main :55-223; host tournament app.c:412-547):
 *   out <- stable merge of two sorted runs a (bl1) and b (bl2) on key_col;
 *   equal keys take run a first.  bl1->col_num must equal bl2->col_num;
 *   out holds bl1->row_num + bl2->row_num rows. */
int smj_merge(const dpu_block_t *bl1, const int64_t *a, const dpu_block_t *bl2, const int64_t *b,
              int key_col, int64_t *out);

/* join.c (main :58-266; host splitters app.c:585-692):
 *   1:1 zip merge join of two tables sorted on key1 / key2 (cpu_app.c
 *   join_in_cpu :204-266).  Output row = all R columns then the S columns
 *   except key2 (c1 + c2 - 1 columns), rows in key order.  *out is
 *   malloc'd by the library and free()'d by the caller (app.c:679,759);
 *   *out_rows gets the joined row count. */
int smj_join(const dpu_block_t *r, const int64_t *R, const dpu_block_t *s, const int64_t *S, int key1,
             int key2, int64_t **out, int64_t *out_rows);

/* The whole app.c pipeline (select -> sort -> merge -> join, :172-692) in one
 * call.  On one GPU the tables cross PCIe in chunks on a copy stream while the
 * first partition pass runs on the chunks already landed (a table that fits
 * one chunk takes one copy), and the result comes back through pinned slots
 * by several host threads.  With a device set of n > 1 GPUs (smj_init(n) /
 * smj_init_devices) the tables are range-partitioned on the key over the
 * GPUs, exchanged over xGMI, and each GPU sorts and joins its key range; the
 * result is the GPUs' outputs in key order.  *out is malloc'd (caller frees).
 * timing may be NULL. */
int smj_sort_merge_join(const dpu_block_t *r, const int64_t *R, const dpu_block_t *s, const int64_t *S,
                        int select_col1, int64_t select_val1, int select_col2, int64_t select_val2,
                        int key1, int key2, int64_t **out, int64_t *out_rows, smj_timing_t *timing);

/* ---- device-pointer API ------------------------------------------------ */
/* All smj_dev_* calls enqueue on `stream` (a hipStream_t, NULL = the legacy
 * default stream) on the CURRENT HIP device and use library-owned scratch
 * memory for that device (grow-only; calls on one device must be serialised
 * on one stream).  Buffers must be distinct unless stated. */

/* Stable select + sort (fused): out <- sort_stable(select(in)).  When
 * use_select == 0 every row is kept.  Runs the MSD sample-sort pipeline
 * (sample splitters -> two tile-local partition passes -> LDS sort of final
 * groups); key_base is accepted for ABI stability and only used by the LSD
 * variant below.  Blocks until the row count is known; *out_rows gets it. */
int smj_dev_select_sort(const int64_t *in, int64_t n_rows, int col_num, int use_select, int select_col,
                        int64_t select_val, int key_col, uint64_t key_base, int64_t *out, int64_t *out_rows,
                        void *stream);

/* The same select + sort on the LSD radix path (hist -> 10-bit chunk passes);
 * kept as the fallback of the MSD pipeline for groups it cannot sort in LDS
 * and for comparison.  Same contract as smj_dev_select_sort. */
int smj_dev_select_sort_lsd(const int64_t *in, int64_t n_rows, int col_num, int use_select, int select_col,
                            int64_t select_val, int key_col, uint64_t key_base, int64_t *out, int64_t *out_rows,
                            void *stream);

/* The whole hot path on device-resident tables in one pipeline (app.c
 * :172-692 / cpu_app.c main :303-364): select (row[sel_col] > sel_val when
 * use_sel), stable sort on the key, and the 1:1 zip join.  R_sorted / S_sorted
 * get the sorted selected rows (nr x c1 / ns x c2 capacity), out the joined
 * rows (min(nr, ns) x (c1 + c2 - 1) capacity).  Synchronises once at the end
 * (twice when oversized single-key or multi-key groups need the fallback);
 * h_rows[0..2] = selected rows of R, of S, joined rows. */
int smj_dev_sort_merge_join(const int64_t *R, int64_t nr, int c1, int use_sel1, int sel_col1, int64_t sel_val1, int key1,
                            const int64_t *S, int64_t ns, int c2, int use_sel2, int sel_col2, int64_t sel_val2, int key2,
                            int64_t *R_sorted, int64_t *S_sorted, int64_t *out, int64_t *h_rows, void *stream);

/* smj_dev_sort_merge_join in two halves.  _begin validates the arguments,
 * enqueues the pipeline up to its sort/join kernel on `stream` and returns at
 * once with *job; _end enqueues the compaction of the joined rows into `out`,
 * waits, and fills h_rows exactly as smj_dev_sort_merge_join does (the job is
 * released whatever it returns).  Between the two the calling thread may do
 * anything but start another smj_dev_* pipeline call (the job holds the
 * thread's scratch; a second _begin returns SMJ_ERR_INVALID): the multi-GPU
 * driver posts its next stage's transfers there, and `out`'s place may be
 * chosen only then.  Inputs and R_sorted / S_sorted must stay valid until _end
 * returns.  Tables over 1.6e8 rows, over 8 columns or empty run whole inside
 * _end.  (Replaces nothing in the reference: app.c's DPU launches are
 * synchronous, app.c:247; this is the asynchronous form a device-resident
 * caller needs.) */
int smj_dev_sort_merge_join_begin(const int64_t *R, int64_t nr, int c1, int use_sel1, int sel_col1, int64_t sel_val1,
                                  int key1, const int64_t *S, int64_t ns, int c2, int use_sel2, int sel_col2,
                                  int64_t sel_val2, int key2, int64_t *R_sorted, int64_t *S_sorted, void *stream,
                                  void **job);
int smj_dev_sort_merge_join_end(void *job, int64_t *out, int64_t *h_rows);

/* Stable select alone (a stable compaction). *out_rows is written after a
 * stream synchronisation. */
int smj_dev_select(const int64_t *in, int64_t n_rows, int col_num, int select_col, int64_t select_val, int64_t *out,
                   int64_t *out_rows, void *stream);

/* Stable merge of sorted runs a (na rows) and b (nb rows) -> out. Async. */
int smj_dev_merge(const int64_t *a, int64_t na, const int64_t *b, int64_t nb, int col_num, int key_col,
                  int64_t *out, void *stream);

/* 1:1 zip join of sorted R (nr x c1) and S (ns x c2) into out, which must
 * hold min(nr, ns) rows of (c1 + c2 - 1) columns.  The joined row count is
 * written to *d_out_rows (DEVICE int64) asynchronously; if h_out_rows is not
 * NULL the call synchronises and also stores it there. */
int smj_dev_join(const int64_t *R, int64_t nr, int c1, const int64_t *S, int64_t ns, int c2, int key1,
                 int key2, int64_t *out, int64_t *d_out_rows, int64_t *h_out_rows, void *stream);

/* Multi-GPU range partition, step 1: counts of selected rows
 * per destination bucket, bucket(k) = #{splitters < k} over n_split sorted
 * splitters (n_split + 1 <= 64 buckets), plus the min / max selected key.
 * Synchronises; h_counts gets n_split + 1 entries, h_minmax 2 (INT64_MAX /
 * INT64_MIN when nothing is selected). */
int smj_dev_partition_count(const int64_t *in, int64_t n_rows, int col_num, int use_select,
                            int select_col, int64_t select_val, int key_col, const int64_t *d_splitters,
                            int n_split, int64_t *h_counts, int64_t *h_minmax, void *stream);

/* Step 2: stable scatter of the selected rows into bucket-contiguous `out`
 * (bucket b starts at the exclusive prefix of h_counts).  Async. */
int smj_dev_partition_scatter(const int64_t *in, int64_t n_rows, int col_num, int use_select,
                              int select_col, int64_t select_val, int key_col, const int64_t *d_splitters,
                              int n_split, const int64_t *h_counts, int64_t *out, void *stream);

/* Steps 1 + 2 in one call (what smj/dist.py runs): stable scatter of the
 * selected rows into bucket-contiguous `out` (room for n_rows rows), bucket
 * starts computed on the device; h_counts gets the n_split + 1 bucket
 * counts.  Reads the table twice (count + scatter) instead of three times.
 * Synchronises. */
int smj_dev_partition(const int64_t *in, int64_t n_rows, int col_num, int use_select, int select_col,
                      int64_t select_val, int key_col, const int64_t *d_splitters, int n_split, int64_t *out,
                      int64_t *h_counts, void *stream);

/* The same partition split for a distributed driver that must not stall
 * the stream (smj/dist.py): splitters are HOST values, nothing synchronises.
 * smj_dev_partition_plan counts the selected rows per (chunk, bucket) into
 * d_plan (smj_partition_plan_bytes(n_rows, col_num, n_split) bytes of device
 * memory, caller-owned) and turns them into absolute stable output starts;
 * the n_split + 1 bucket counts land in d_counts (DEVICE int64).
 * smj_dev_partition_apply then writes the bucket-contiguous copy from that
 * plan (same table, splitters and select).  A plan outlives other calls, so
 * a caller can count every table first, exchange the counts, and scatter
 * later without reading a table a third time. */
size_t smj_partition_plan_bytes(int64_t n_rows, int col_num, int n_split);
int smj_dev_partition_plan(const int64_t *in, int64_t n_rows, int col_num, int use_select, int select_col,
                           int64_t select_val, int key_col, const int64_t *h_splitters, int n_split, void *d_plan,
                           int64_t *d_counts, void *stream);
int smj_dev_partition_apply(const int64_t *in, int64_t n_rows, int col_num, int use_select, int select_col,
                            int64_t select_val, int key_col, const int64_t *h_splitters, int n_split,
                            const void *d_plan, int64_t *out, void *stream);

/* The partition in ONE read of the table, for a driver that can size the
 * buckets' destinations from a key sample (smj/dist.py): bucket b's selected
 * rows go, stably, to out rows [h_region[b], h_region[b] + count_b), where
 * h_region[0..n_split] are ascending, disjoint region starts and
 * h_region[n_split + 1 + b] region b's capacity (rows; out must hold the last
 * region).  d_counts (DEVICE int64, n_split + 2 entries) gets the n_split + 1
 * exact bucket counts and d_counts[n_split + 1] = 0, or bit 0 set when a
 * bucket outgrew its region (that region's contents are then unspecified --
 * nothing is written past it -- and the caller re-partitions with plan /
 * apply; the counts stay exact) / bit 1 when the decoupled
 * look-back timed out (a bug).  Decoupled look-back over 4096-row tiles
 * (msd_part1_kernel); nothing synchronises; <= 64 buckets, 1..8 columns. */
int smj_dev_partition_regions(const int64_t *in, int64_t n_rows, int col_num, int use_select, int select_col,
                              int64_t select_val, int key_col, const int64_t *h_splitters, int n_split,
                              const int64_t *h_region, int64_t *out, int64_t *d_counts, void *stream);

/* Synthetic 2-column table (key, payload) for rows [row0, row0 + rows):
 * key = 1 + floor(splitmix64(g + seed * 0xD1B54A32D192ED03) * key_range / 2^64),
 * payload = g (the global row index).  Identical to the oracle's
 * smj_ref_gen_uniform.  Async. */
int smj_dev_gen_uniform(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t key_range,
                        void *stream);

/* Zipf(theta) keys over [1, domain]: rank r is drawn with
 * Gray et al.'s closed-form approximation (SIGMOD'94 "Quickly generating
 * billion-record synthetic databases", as used by YCSB) from uniform
 * u = splitmix64(g + seed * 0xD1B54A32D192ED03) / 2^64, and the key is the
 * rank scattered over [1, domain] by a bijective affine hash so hot keys are
 * spread over the key space.  zeta_n = smj_zipf_zeta(domain, theta).
 * payload = g.  Async. */
int smj_dev_gen_zipf(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, int64_t domain,
                     double theta, double zeta_n, void *stream);
/* sum_{i=1..n} i^-theta (host). */
double smj_zipf_zeta(int64_t n, double theta);

/* C3-wide (SURVEY 8(d) stress input): full-range signed int64 keys.  Row g's
 * own key is (int64) h with h = splitmix64(g + seed * 0xD1B54A32D192ED03);
 * when plant_rows > 0, a third of the rows (d = splitmix64(h ^
 * 0x2545F4914F6CDD1D), mulhi(d, 3) == 0) instead take the key row
 * r = mulhi(splitmix64(d), plant_rows) has in the table generated with
 * plant_seed (R), so they join.  payload = g.  Identical to the oracle's
 * smj_ref_gen_wide.  Async. */
int smj_dev_gen_wide(int64_t *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t plant_seed,
                     int64_t plant_rows, void *stream);

/* Order-sensitive digest of a row-major table slice whose first row sits at
 * global position pos0:
 *   *d_digest (DEVICE uint64) = sum_i h(pos0 + i, row i) mod 2^64, with
 *   h(p, r) = f(... f(f(mix(p ^ 0x5851F42D4C957F2D) + r[0]) + r[1]) ... + r[c-1])
 * and mix = splitmix64's finaliser (x += 0x9E3779B97F4A7C15 then the two
 * xor-shift-multiply rounds).  Digests of consecutive slices at their global
 * positions sum to the digest of the whole, so a distributed result (one slice
 * per rank, rank order) is checked against a single call by adding numbers.
 * Async.  (The reference has no result checker at all -- SURVEY 4: no tests;
 * this is the verification the multi-GPU bench line carries.) */
int smj_dev_digest(const int64_t *rows, int64_t n_rows, int col_num, int64_t pos0, uint64_t *d_digest,
                   void *stream);

/* Splitters of the range-partitioned multi-GPU path (the
 * reference deals rows to DPUs by count, app.c:155-218, and has no key
 * ranges).  Two device steps around the caller's all_gather:
 *   smj_dev_dist_sample: d_buf (DEVICE, 5 + 2 samples words) = the header
 *     [c0 + c1, c0, c1, nR, nS], then the keys of rows j (n - 1) / (c - 1),
 *     j < c = min(samples, n), of R then S, then INT64_MAX pads.
 *   smj_dev_dist_splitters: d_all = world such buffers back to back (stride
 *     words each); d_out (DEVICE, parts words) = the keys at sorted positions
 *     max(0, (q + 1) L / parts - 1), or max(0, q20[q] L / 2^20 - 1) when q20
 *     (HOST, parts - 1 fractions << 20) is given, q < parts - 1, then L (the
 *     valid samples of all ranks; L = 0: every splitter 0).  parts <= 64.
 * Async. */
int smj_dev_dist_sample(const int64_t *R, int64_t nR, int colsR, int keyR, const int64_t *S, int64_t nS, int colsS,
                        int keyS, int samples, int64_t *d_buf, void *stream);
int smj_dev_dist_splitters(const int64_t *d_all, int world, int64_t stride, int parts, const int32_t *q20,
                           int64_t *d_out, void *stream);

/* Packed exchange rows (frame-of-reference packing of the
 * range-partitioned rows before they cross xGMI): a 2-column row
 * (key in column key_col, the other column o) travels as ONE int64 word
 *   w = (uint32)(key - key_base) | (uint64)(uint32)(o - other_base) << 32,
 * differences taken mod 2^64; it round-trips iff both differences fit int32.
 *   smj_dev_partition_regions_pk: smj_dev_partition_regions of a 2-column
 *     table writing packed words (out: one int64 per row of every region);
 *     d_counts[n_split + 1] gets bit 2 (4) when some row did not fit -- the
 *     caller then re-partitions unpacked (the output is not usable).
 *   smj_dev_unpack_rows: n packed words -> n x 2 rows.
 *   smj_dev_sort_merge_join_begin_pk: smj_dev_sort_merge_join_begin on two
 *     2-column tables without a select, either of them packed (pkX = 1; rows
 *     of <= 1.6e8 per table, else SMJ_ERR_UNSUPPORTED: unpack first); ended by
 *     smj_dev_sort_merge_join_end.
 * Async. */
int smj_dev_partition_regions_pk(const int64_t *in, int64_t n, int use_select, int select_col, int64_t select_val,
                                 int key_col, const int64_t *h_splitters, int n_split, const int64_t *h_region,
                                 int64_t *out, int64_t *d_counts, int64_t key_base, int64_t other_base, void *stream);
int smj_dev_unpack_rows(const int64_t *d_packed, int64_t n, int key_col, int64_t key_base, int64_t other_base,
                        int64_t *d_out, void *stream);
int smj_dev_sort_merge_join_begin_pk(const int64_t *R, int64_t nR, int key1, int pk1, int64_t key_base1,
                                     int64_t other_base1, const int64_t *S, int64_t nS, int key2, int pk2,
                                     int64_t key_base2, int64_t other_base2, int64_t *R_sorted, int64_t *S_sorted,
                                     void *stream, void **job);

/* ---- T = UINT64 / DOUBLE (common.h:3-9) ------------- */
/* The fused pipeline with keys and select values compared as key_type
 * (uint64 or IEEE double, as cpu_app.c compiled with that T): tables are
 * 8-byte cells; select values are passed as their bit patterns.  The key and
 * select columns are mapped order-preservingly onto int64 for the pipeline
 * and back for the outputs.  DOUBLE: -0.0 equals +0.0 (and comes back as
 * +0.0 in those columns); NaN keys are not supported. */
#define SMJ_KEY_INT64 0
#define SMJ_KEY_UINT64 1
#define SMJ_KEY_DOUBLE 2
int smj_sort_merge_join_typed(int key_type, const dpu_block_t *r, const void *R, const dpu_block_t *s,
                              const void *S, int select_col1, uint64_t sel_bits1, int select_col2,
                              uint64_t sel_bits2, int key1, int key2, void **out, int64_t *out_rows,
                              smj_timing_t *timing);
int smj_dev_sort_merge_join_typed(int key_type, const void *R, int64_t nr, int c1, int use_sel1, int sel_col1,
                                  uint64_t sel_bits1, int key1, const void *S, int64_t ns, int c2, int use_sel2,
                                  int sel_col2, uint64_t sel_bits2, int key2, void *R_sorted, void *S_sorted,
                                  void *out, int64_t *h_rows, void *stream);

#if defined(UINT64) || defined(DOUBLE)
#ifdef UINT64
#define SMJ_KEY_TYPE SMJ_KEY_UINT64
#else
#define SMJ_KEY_TYPE SMJ_KEY_DOUBLE
#endif
static inline uint64_t smj_T_bits(T v)
{
    uint64_t u;
    memcpy(&u, &v, sizeof u);
    return u;
}
static inline int smj_T_sort_merge_join(const dpu_block_t *r, const T *R, const dpu_block_t *s, const T *S,
                                        int select_col1, T select_val1, int select_col2, T select_val2, int key1,
                                        int key2, T **out, int64_t *out_rows, smj_timing_t *timing)
{
    return smj_sort_merge_join_typed(SMJ_KEY_TYPE, r, R, s, S, select_col1, smj_T_bits(select_val1), select_col2,
                                     smj_T_bits(select_val2), key1, key2, (void **)out, out_rows, timing);
}
static inline int smj_T_dev_sort_merge_join(const T *R, int64_t nr, int c1, int use_sel1, int sel_col1, T sel_val1,
                                            int key1, const T *S, int64_t ns, int c2, int use_sel2, int sel_col2,
                                            T sel_val2, int key2, T *R_sorted, T *S_sorted, T *out, int64_t *h_rows,
                                            void *stream)
{
    return smj_dev_sort_merge_join_typed(SMJ_KEY_TYPE, R, nr, c1, use_sel1, sel_col1, smj_T_bits(sel_val1), key1, S,
                                         ns, c2, use_sel2, sel_col2, smj_T_bits(sel_val2), key2, R_sorted, S_sorted,
                                         out, h_rows, stream);
}
/* the app.c drop-in calls stay as written */
#define smj_sort_merge_join smj_T_sort_merge_join
#define smj_dev_sort_merge_join smj_T_dev_sort_merge_join
#else
#define SMJ_KEY_TYPE SMJ_KEY_INT64
#endif

/* ---- diagnostics ------------------------------------------------------- */
/* Counters of the last MSD pipeline call: out4[0] = single-key groups
 * streamed without a sort, out4[1] = groups sorted / joined by the LSD
 * fallback, out4[2] / out4[3] = selected rows of R / S. */
void smj_debug_msd_stats(int64_t *out4);
/* Final-stage group counts of the last MSD pipeline call: out3[0] = LDS
 * (dense) groups, out3[1] = radix-tier groups, out3[2] = 64-bit-tier groups. */
void smj_debug_msd_groups(int64_t *out3);
/* The same plus out4[3] = staged groups whose equal-key runs (over 32 rows)
 * were ordered by the in-LDS stable LSD instead of the transposition rounds. */
void smj_debug_msd_tiers(int64_t *out4);
/* Run every pipeline call in the partitioned mode with `parts` key-range
 * parts (tests); 0 = automatic (tables over 1.6e8 rows). */
void smj_debug_force_parts(int parts);
/* Polls the pipeline's cross-workgroup look-back makes before it gives up
 * and the call returns SMJ_ERR_TIMEOUT (tests: 0 forces the timeout path);
 * a negative value restores the default (2^26). */
void smj_debug_spin_limit(int64_t polls);
/* Rows (R + S, after the WHERE clause) each device of the set received in
 * the last sharded call (load balance); returns the device count, writes at
 * most `max` entries. */
int smj_debug_shard_rows(int64_t *out, int max);

/* ---- profiling ---------------------------------------------------------- */
/* When enabled, every kernel launch is bracketed by hipEvents recorded on
 * the stream it is launched on, tagged with the kernel's name and its
 * algorithmic byte count.  smj_prof_report() synchronises, writes
 * a JSON object {name: {"launches", "ms", "bytes"}} into buf and resets. */
void smj_prof_enable(int on);
int smj_prof_report(char *buf, size_t buflen);

#ifdef __cplusplus
}
#endif
#endif /* SMJ_H */
