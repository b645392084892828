/*
 * common.h -- row layout contract (reference: sort-merge-join/common.h:1-34).
 *
 * A table is a row-major array T[row_num * col_num]; T is the element type
 * selected by one of INT64 (default) / UINT64 / DOUBLE exactly as in the
 * reference (common.h:1-9).  The library's cells are 8 bytes whatever T is:
 * a C host compiled with -DUINT64 or -DDOUBLE reaches the same pipeline
 * through smj.h's *_typed entry points (smj_sort_merge_join maps to them),
 * which compare keys and select values as T.
 *
 * dpu_block_t is the 12-byte block descriptor the reference host pushes to
 * every DPU kernel (common.h:13-18, e.g. app.c:226, :447).  The C-ABI in
 * smj.h takes the same descriptor so a caller can hand over exactly what it
 * used to push to the DPUs.
 */
#ifndef SMJ_COMMON_H
#define SMJ_COMMON_H

#include <stdint.h>

#if !defined(INT64) && !defined(UINT64) && !defined(DOUBLE)
#define INT64
#endif

#ifdef UINT64
#define T uint64_t
#elif defined(INT64)
#define T int64_t
#elif defined(DOUBLE)
#define T double
#endif

/* Reference DPU MRAM read granule (common.h:11).  Not used by the GPU path. */
#define CACHE_SIZE 256

typedef struct
{
    int table_num; /* 0 = first table (R), 1 = second table (S)          */
    int col_num;   /* columns per row                                     */
    int row_num;   /* rows in this block                                  */
} dpu_block_t;

typedef struct
{
    int table_num;
    int dpu_id;    /* reference: DPU index; here: GPU / partition index   */
    int col_num;
    int row_num;
    T *arr;
} dpu_result_t;

typedef struct
{
    int tasklet_id;
    int row_num;
    T *arr;
} tasklet_result_t;

#endif /* SMJ_COMMON_H */
