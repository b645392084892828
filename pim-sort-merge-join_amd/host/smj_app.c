/*
 * smj_app.c -- the MI355X replacement of the reference host program
 * (sort-merge-join/app.c).  Same command line (app.c:130-131):
 *
 *   smj_app data1.csv data2.csv [-o result.csv] [--select c1 v1 c2 v2] [--keys k1 k2]
 *           [--gpus N | --devices i,j,...]
 *
 * --gpus N (default NR_GPUS, user.h) is the device set smj_init gets, the
 * way NR_DPUS sizes dpu_alloc; --devices lists HIP device ids explicitly and
 * may repeat one (the sharded path on a single GPU).
 *
 * Loads both CSVs with the reference's ingest semantics (app.c:153-159),
 * runs select -> sort -> merge -> join on the GPU through the C-ABI in
 * include/smj.h (where app.c used dpu_alloc/dpu_load/dpu_push_xfer/
 * dpu_launch/dpu_free), writes ./data/result.csv (app.c:720) and prints the
 * reference's timing banner (app.c:763-772) with GPU in place of DPU.
 * Configuration defaults come from include/user.h exactly as in the
 * reference.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "common.h"
#include "csv.h"
#include "smj.h"
#include "user.h"

static double now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

int main(int argc, char **argv)
{
    const char *in1 = NULL, *in2 = NULL, *out_path = "./data/result.csv";
    int sc1 = SELECT_COL1, sc2 = SELECT_COL2, k1 = JOIN_KEY1, k2 = JOIN_KEY2;
    long long sv1 = SELECT_VAL1, sv2 = SELECT_VAL2;
    int ngpus = NR_GPUS, ndev = 0, devs[64];
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-o") && i + 1 < argc) {
            out_path = argv[++i];
        } else if (!strcmp(argv[i], "--select") && i + 4 < argc) {
            sc1 = atoi(argv[++i]);
            sv1 = strtoll(argv[++i], NULL, 10);
            sc2 = atoi(argv[++i]);
            sv2 = strtoll(argv[++i], NULL, 10);
        } else if (!strcmp(argv[i], "--keys") && i + 2 < argc) {
            k1 = atoi(argv[++i]);
            k2 = atoi(argv[++i]);
        } else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) {
            ngpus = atoi(argv[++i]);
        } else if (!strcmp(argv[i], "--devices") && i + 1 < argc) {
            for (char *t = strtok(argv[++i], ","); t && ndev < 64; t = strtok(NULL, ",")) devs[ndev++] = atoi(t);
        } else if (!in1) {
            in1 = argv[i];
        } else if (!in2) {
            in2 = argv[i];
        } else {
            fprintf(stderr, "unexpected argument %s\n", argv[i]);
            return 2;
        }
    }
    if (!in1 || !in2) {
        fprintf(stderr, "usage: %s data1.csv data2.csv [-o result.csv] [--select c1 v1 c2 v2] "
                        "[--keys k1 k2] [--gpus N | --devices i,j,...]\n", argv[0]);
        return 2;
    }

    /* ingest (app.c:153-159) */
    double t0 = now_ms();
    int c1 = 0, r1 = 0, c2 = 0, r2 = 0;
    T *a = NULL, *b = NULL;
    if (smj_csv_load(in1, &c1, &r1, &a) || smj_csv_load(in2, &c2, &r2, &b)) {
        perror("Failed to open file");
        return EXIT_FAILURE;
    }
    double t_load = now_ms() - t0;
    if (sc1 >= c1 || sc2 >= c2 || k1 >= c1 || k2 >= c2) {
        fprintf(stderr, "select/join column out of range (tables have %d and %d columns)\n", c1, c2);
        return EXIT_FAILURE;
    }

    /* dpu_alloc -> smj_init */
    const int got = ndev ? smj_init_devices(devs, ndev) : smj_init(ngpus);
    if (got < 1) {
        fprintf(stderr, "smj_init: %s\n", smj_strerror(got < 0 ? got : SMJ_ERR_NODEVICE));
        return EXIT_FAILURE;
    }
    dpu_block_t bl1 = {0, c1, r1}, bl2 = {1, c2, r2};
    T *res = NULL;
    int64_t j = 0;
    smj_timing_t tm = {0, 0, 0};
    SMJ_ASSERT(smj_sort_merge_join(&bl1, a, &bl2, b, sc1, (T)sv1, sc2, (T)sv2, k1, k2, &res, &j, &tm));

    /* egress (app.c:720-755) */
    double t1 = now_ms();
    if (smj_csv_save(out_path, c1 + c2 - 1, j, res)) {
        perror("Failed to open file");
        return EXIT_FAILURE;
    }
    double t_save = now_ms() - t1;

    printf("\n");
    printf("######### GPU #########\n");
    printf("### SORT-MERGE-JOIN ###\n");
    printf("         EXEC TIME     \n");
    printf("CPU-GPU  %f\n", tm.cpu_gpu_ms);
    printf("GPU      %f\n", tm.gpu_ms);
    printf("GPU-CPU  %f\n", tm.gpu_cpu_ms);
    printf("-----------------------\n");
    printf("TOTAL %f\n", tm.cpu_gpu_ms + tm.gpu_ms + tm.gpu_cpu_ms);
    printf("#######################\n");
    printf("rows %lld on %d GPU(s) (csv load %.3f ms, save %.3f ms)\n\n", (long long)j, got, t_load, t_save);

    free(res);
    free(a);
    free(b);
    smj_finalize();
    return 0;
}
