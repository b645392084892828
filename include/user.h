/*
 * user.h -- compile-time configuration contract of the sort-merge-join path.
 *
 * Same macro names and default values as the reference's
 * sort-merge-join/user.h:1-13 so that a host program written against the
 * reference configuration builds unchanged against this library.
 *
 *   NR_DPUS       reference: number of UPMEM DPUs (user.h:3).  Here it is kept
 *                 only for source compatibility; the GPU count is NR_GPUS.
 *   NR_TASKLETS   reference: hardware threads per DPU (user.h:4).  Unused on
 *                 MI355X (a workgroup is 512 lanes); kept for compatibility.
 *   SELECT_COL{1,2} / SELECT_VAL{1,2}
 *                 WHERE row[SELECT_COL] > SELECT_VAL on table 1 / table 2
 *                 (user.h:6-10, applied at cpu_app.c:336-337).
 *   JOIN_KEY{1,2} join-key column of table 1 / table 2 (user.h:12-13).
 */
#ifndef SMJ_USER_H
#define SMJ_USER_H

/* #define DEBUG */

#ifndef NR_DPUS
#define NR_DPUS 64
#endif
#ifndef NR_TASKLETS
#define NR_TASKLETS 16
#endif

/* MI355X: GPUs of one node the join is range-partitioned over. */
#ifndef NR_GPUS
#define NR_GPUS 1
#endif

#ifndef SELECT_COL1
#define SELECT_COL1 0
#endif
#ifndef SELECT_VAL1
#define SELECT_VAL1 5000
#endif

#ifndef SELECT_COL2
#define SELECT_COL2 0
#endif
#ifndef SELECT_VAL2
#define SELECT_VAL2 5000
#endif

#ifndef JOIN_KEY1
#define JOIN_KEY1 0
#endif
#ifndef JOIN_KEY2
#define JOIN_KEY2 0
#endif

#endif /* SMJ_USER_H */
