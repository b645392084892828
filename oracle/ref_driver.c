/*
 * ref_driver.c -- drives the REAL reference functions (test infrastructure).
 *
 * oracle/Makefile compiles /root/reference/sort-merge-join/cpu_app.c, where
 * it lies, into oracle/_ref/libcpu_app_ref.so with its main() renamed; this
 * driver (our own code) calls the reference's own set_csv_size / load_csv /
 * select_in_cpu / insertion_sort_in_cpu / join_in_cpu / save_to_csv in the
 * order of cpu_app.c:main (:324-350), with save_to_csv enabled and the
 * user.h SELECT/JOIN values overridable, so the goldens under tests/golden/
 * are produced by the reference implementation itself.
 *
 *   ref_driver data1.csv data2.csv out.csv [c1 v1 c2 v2 k1 k2]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

/* Signatures of cpu_app.c (T = int64_t, common.h:1-6). */
void set_csv_size(const char *filename, int *col_num, int *row_num);
void load_csv(const char *filename, int col_num, int row_num, int64_t **test_array);
void select_in_cpu(int col_num, int *row_num, int64_t **test_array, int64_t select_col, int64_t select_val);
void insertion_sort_in_cpu(int col_num, int row_num, int key, int64_t **test_array);
void join_in_cpu(int col_num_1, int row_num_1, int64_t *test_array_1, int col_num_2, int row_num_2,
                 int64_t *test_array_2, int key1, int key2);
void save_to_csv(const char *filename, int col_num, int row_num, int64_t *test_array);
extern int64_t *result;
extern int result_row_num;
extern int result_col_num;

int main(int argc, char **argv)
{
    if (argc != 4 && argc != 10) {
        fprintf(stderr, "usage: %s d1.csv d2.csv out.csv [c1 v1 c2 v2 k1 k2]\n", argv[0]);
        return 2;
    }
    long long c1 = 0, v1 = 5000, c2 = 0, v2 = 5000, k1 = 0, k2 = 0; /* user.h:6-13 */
    if (argc == 10) {
        c1 = atoll(argv[4]);
        v1 = strtoll(argv[5], NULL, 10);
        c2 = atoll(argv[6]);
        v2 = strtoll(argv[7], NULL, 10);
        k1 = atoll(argv[8]);
        k2 = atoll(argv[9]);
    }
    int cn1 = 0, rn1 = 0, cn2 = 0, rn2 = 0;
    int64_t *a = NULL, *b = NULL;
    set_csv_size(argv[1], &cn1, &rn1);
    set_csv_size(argv[2], &cn2, &rn2);
    load_csv(argv[1], cn1, rn1, &a);
    load_csv(argv[2], cn2, rn2, &b);
    select_in_cpu(cn1, &rn1, &a, c1, v1);
    select_in_cpu(cn2, &rn2, &b, c2, v2);
    insertion_sort_in_cpu(cn1, rn1, (int)k1, &a);
    insertion_sort_in_cpu(cn2, rn2, (int)k2, &b);
    join_in_cpu(cn1, rn1, a, cn2, rn2, b, (int)k1, (int)k2);
    save_to_csv(argv[3], result_col_num, result_row_num, result);
    printf("%d\n", result_row_num);
    return 0;
}
