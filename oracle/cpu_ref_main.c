/*
 * cpu_ref_main.c -- command-line front end of the CPU oracle (test
 * infrastructure).  Same CLI as the reference cpu_app (cpu_app.c:303-307):
 *
 *   cpu_ref data1.csv data2.csv [out.csv] [--insertion]
 *           [--select c1 v1 c2 v2] [--keys k1 k2]
 *
 * Defaults come from include/user.h.  Prints the reference's timing banner
 * (cpu_app.c:352-358) and, when out.csv is given, writes the join result
 * (cpu_app.c:350, enabled here).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cpu_ref.h"
#include "user.h"

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s data1.csv data2.csv [out.csv] [--insertion] "
                        "[--select c1 v1 c2 v2] [--keys k1 k2]\n", argv[0]);
        return 2;
    }
    const char *out = NULL;
    int insertion = 0;
    int sc1 = SELECT_COL1, sc2 = SELECT_COL2, k1 = JOIN_KEY1, k2 = JOIN_KEY2;
    long long sv1 = SELECT_VAL1, sv2 = SELECT_VAL2;
    for (int i = 3; i < argc; i++) {
        if (!strcmp(argv[i], "--insertion")) {
            insertion = 1;
        } else if (!strcmp(argv[i], "--select") && i + 4 < argc) {
            sc1 = atoi(argv[++i]);
            sv1 = strtoll(argv[++i], NULL, 10);
            sc2 = atoi(argv[++i]);
            sv2 = strtoll(argv[++i], NULL, 10);
        } else if (!strcmp(argv[i], "--keys") && i + 2 < argc) {
            k1 = atoi(argv[++i]);
            k2 = atoi(argv[++i]);
        } else {
            out = argv[i];
        }
    }
    double ms = 0;
    int64_t j = smj_ref_pipeline_csv(argv[1], argv[2], out, sc1, (T)sv1, sc2, (T)sv2, k1, k2,
                                     insertion, &ms);
    if (j < 0) {
        perror("cpu_ref");
        return 1;
    }
    printf("\n######### CPU #########\n### SORT-MERGE-JOIN ###\n       EXEC TIME       \n");
    printf("Time (ms): %f\t\n", ms);
    printf("Joined rows: %lld\n#######################\n", (long long)j);
    return 0;
}
