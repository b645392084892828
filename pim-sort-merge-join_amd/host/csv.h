/*
 * csv.h -- CSV ingest / egress of the sort-merge-join host (product code).
 *
 * Contract, identical to the reference host
 * (sort-merge-join/app.c:28-92 ingest, app.c:720-755 egress; the same code
 * is in cpu_app.c:15-79 / :268-301):
 *   - columns = number of ','-separated tokens (empty fields collapsed) of the
 *     header line; rows = physical lines - 1, where a "line" is what one
 *     fgets() into a 1024-byte buffer returns (longer lines count twice);
 *   - every token is converted with atoi() semantics: leading white space,
 *     optional sign, decimal digits, strtol saturation at the 64-bit limits,
 *     then truncation to a 32-bit int, sign-extended into T;
 *   - token k of data line r lands in cell r*cols + k (no per-row bound, as
 *     in the reference; cells past the table end are dropped, cells the
 *     reference leaves uninitialised read 0);
 *   - output: header "col1,...,colN\n", rows "%ld" joined by ',' + '\n'.
 */
#ifndef SMJ_HOST_CSV_H
#define SMJ_HOST_CSV_H

#include <stdint.h>

#include "common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Parses the whole file; *out is malloc'd (rows*cols cells).  Returns 0 or -1
 * (errno set) when the file cannot be read. */
int smj_csv_load(const char *path, int *col_num, int *row_num, T **out);

/* Writes the result table.  Returns 0 or -1. */
int smj_csv_save(const char *path, int col_num, int64_t row_num, const T *arr);

/* Threads for smj_csv_load / smj_csv_save: n >= 1 fixes
 * the count (1 = the serial code), 0 = SMJ_CSV_THREADS, else OMP_NUM_THREADS,
 * else min(online CPUs, 16).  Small files use fewer threads.  The result is
 * byte-identical whatever the count. */
void smj_csv_set_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
