/*
 * cpu_ref.h -- CPU ORACLE for the sort-merge-join path.  TEST INFRASTRUCTURE.
 *
 * A from-scratch C restatement of the reference's CPU pipeline
 * (sort-merge-join/cpu_app.c).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / the CPU
 * baseline -- never as the product path.
 *
 * Parity pinning: the restatement is checked against golden outputs produced
 * by the reference cpu_app.c functions themselves (compiled from
 * /root/reference by oracle/Makefile into oracle/_ref/, see
 * tests/golden/make_goldens.py): bundled data1 x data2 (sha256 f4088e9f...),
 * the 10k pair (sha256 0a881f37...) and the SURVEY 8(c) known-answer test.
 */
#ifndef SMJ_CPU_REF_H
#define SMJ_CPU_REF_H

#include <stdint.h>
#include "common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* cpu_app.c:15-44.  Column count = strtok(",") tokens of the first fgets
 * line; row count = fgets lines - 1 (1024-byte line buffer).  Returns 0 or -1
 * when the file cannot be opened. */
int smj_ref_csv_size(const char *path, int *col_num, int *row_num);

/* cpu_app.c:46-79.  Allocates *out (calloc: cells the reference leaves
 * uninitialised read 0 here) and fills it with atoi() of every token;
 * atoi wraps to 32 bits and is sign-extended into T. */
int smj_ref_load_csv(const char *path, int col_num, int row_num, T **out);

/* cpu_app.c:81-112.  Stable compaction of rows with row[select_col] >
 * select_val (signed 64-bit compare).  Replaces *arr (freed) and *row_num. */
int smj_ref_select(int col_num, int64_t *row_num, T **arr, int select_col, T select_val);

/* Same select, out-of-place, no allocation (out must hold row_num rows). */
int64_t smj_ref_select_into(int col_num, int64_t row_num, const T *in, int select_col, T select_val, T *out);

/* cpu_app.c:172-202.  The reference algorithm: O(n^2) stable insertion sort
 * ascending on row[key] ('>' compare at :186). Used for the CPU baseline. */
void smj_ref_insertion_sort(int col_num, int64_t row_num, int key, T *arr);

/* Same output order as smj_ref_insertion_sort (stable, ascending on row[key]),
 * O(n log n) bottom-up merge sort, so parity checks finish in seconds. */
int smj_ref_stable_sort(int col_num, int64_t row_num, int key, T *arr);

/* cpu_app.c:204-266.  1:1 "zip" merge join of two sorted tables: on equal keys
 * both cursors advance, so key k yields min(cnt_R(k), cnt_S(k)) rows pairing
 * the i-th R occurrence with the i-th S occurrence.  Output row = all R
 * columns followed by the S columns except key2 (total c1 + c2 - 1).
 * *out is malloc'd (caller frees); returns the joined row count or -1. */
int64_t smj_ref_join(int c1, int64_t r1, const T *a, int c2, int64_t r2, const T *b,
                     int key1, int key2, T **out);

/* Count-only pass of smj_ref_join (cpu_app.c:211-227). */
int64_t smj_ref_join_count(int c1, int64_t r1, const T *a, int c2, int64_t r2, const T *b,
                           int key1, int key2);

/* cpu_app.c:268-301.  Header col1..colN, rows of "%ld" joined by ',' with
 * '\n' line ends.  Returns 0 or -1. */
int smj_ref_save_csv(const char *path, int col_num, int64_t row_num, const T *arr);

/* The whole cpu_app.c main() pipeline (:324-350): load, select, sort, join,
 * save.  use_insertion selects the reference O(n^2) sort.  Returns joined
 * rows or -1; *elapsed_ms gets the load->join wall time (cpu_app.c:329,347). */
int64_t smj_ref_pipeline_csv(const char *path1, const char *path2, const char *out_path,
                             int sel_col1, T sel_val1, int sel_col2, T sel_val2,
                             int key1, int key2, int use_insertion, double *elapsed_ms);

/* ---- synthetic tables (build-owned) ----------------------- */
/* C3-wide synthetic keys (the device's smj_dev_gen_wide). */
void smj_ref_gen_wide(T *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t plant_seed, int64_t plant_rows);
/* splitmix64 finaliser. */
uint64_t smj_ref_splitmix64(uint64_t x);
/* Fill rows [row0, row0 + rows) of a 2-column table (key, payload): the key of
 * global row g is 1 + floor(h(g) * key_range / 2^64) with
 * h(g) = splitmix64(g + seed * 0xD1B54A32D192ED03), payload = g.  Keys are
 * therefore iid uniform in [1, key_range]; the table is identical however it
 * is sharded. */
void smj_ref_gen_uniform(T *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t key_range);
/* Zipf(theta) keys over [1, n] of global rows [row0, row0 + rows) (the
 * device generator's restatement; zetan = sum_{i<=n} i^-theta). */
void smj_ref_gen_zipf(T *out, int64_t row0, int64_t rows, uint64_t seed, int64_t n, double theta, double zetan);

/* The checker's side of smj_dev_digest (include/smj.h): sum over rows i of
 * h(pos0 + i, row i) mod 2^64, h(p, r) = f(..f(f(m(p ^ 0x5851F42D4C957F2D) +
 * r[0]) + r[1]).. + r[c-1]), f = m = splitmix64 (cells as their 64-bit
 * patterns).  Not part of cpu_app.c: the reference has no result checker. */
uint64_t smj_ref_digest(const void *rows, int64_t row_num, int col_num, int64_t pos0);

#ifdef __cplusplus
}
#endif
#endif
