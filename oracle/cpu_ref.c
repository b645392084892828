/*
 * cpu_ref.c -- CPU ORACLE (test infrastructure only; see cpu_ref.h).
 *
 * Restates sort-merge-join/cpu_app.c function by function; each function
 * cites the reference lines it follows.  Parity pinned by tests/golden/
 * (outputs of the reference cpu_app.c functions themselves).
 */
#define _POSIX_C_SOURCE 200809L
#include "cpu_ref.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* cpu_app.c:15-44 */
int smj_ref_csv_size(const char *path, int *col_num, int *row_num)
{
    FILE *f = fopen(path, "r");
    if (!f)
        return -1;
    char line[1024];
    int first = 1;
    *col_num = 0;
    *row_num = 0;
    while (fgets(line, sizeof(line), f)) {
        if (first) {
            first = 0;
            for (char *tok = strtok(line, ","); tok; tok = strtok(NULL, ","))
                (*col_num)++;
        }
        (*row_num)++;
    }
    (*row_num)--;
    fclose(f);
    return 0;
}

/* cpu_app.c:46-79.  Token k of data line r lands in cell r*col_num + k, with
 * no per-row bound (extra tokens spill into the following row, as in the
 * reference); writes past the end of the table are dropped instead of being
 * undefined behaviour. */
int smj_ref_load_csv(const char *path, int col_num, int row_num, T **out)
{
    int64_t cells = (int64_t)col_num * (row_num > 0 ? row_num : 0);
    T *arr = (T *)calloc(cells > 0 ? (size_t)cells : 1, sizeof(T));
    if (!arr)
        return -1;
    FILE *f = fopen(path, "r");
    if (!f) {
        free(arr);
        return -1;
    }
    char line[1024];
    int64_t row = 0;
    if (!fgets(line, sizeof(line), f)) { /* header */
        fclose(f);
        *out = arr;
        return 0;
    }
    while (fgets(line, sizeof(line), f)) {
        int64_t col = 0;
        for (char *tok = strtok(line, ","); tok; tok = strtok(NULL, ",")) {
            int64_t idx = row * col_num + col;
            if (idx < cells)
                arr[idx] = (T)atoi(tok); /* int -> T sign extension, as :71 */
            col++;
        }
        row++;
    }
    fclose(f);
    *out = arr;
    return 0;
}

/* cpu_app.c:81-112 (count pass :86-92, copy pass :96-106) */
int64_t smj_ref_select_into(int col_num, int64_t row_num, const T *in, int select_col, T select_val, T *out)
{
    int64_t j = 0;
    for (int64_t i = 0; i < row_num; i++) {
        if (in[i * col_num + select_col] > select_val) {
            memcpy(out + j * col_num, in + i * col_num, sizeof(T) * col_num);
            j++;
        }
    }
    return j;
}

int smj_ref_select(int col_num, int64_t *row_num, T **arr, int select_col, T select_val)
{
    const T *in = *arr;
    int64_t cnt = 0;
    for (int64_t i = 0; i < *row_num; i++)
        if (in[i * col_num + select_col] > select_val)
            cnt++;
    T *res = (T *)malloc((size_t)(cnt > 0 ? cnt : 1) * col_num * sizeof(T));
    if (!res)
        return -1;
    smj_ref_select_into(col_num, *row_num, in, select_col, select_val, res);
    free(*arr);
    *arr = res;
    *row_num = cnt;
    return 0;
}

/* cpu_app.c:172-202: take row i, shift rows with key > its key one slot up. */
void smj_ref_insertion_sort(int col_num, int64_t row_num, int key, T *arr)
{
    T tmp[64];
    T *t = col_num <= 64 ? tmp : (T *)malloc(sizeof(T) * col_num);
    for (int64_t i = 1; i < row_num; i++) {
        memcpy(t, arr + i * col_num, sizeof(T) * col_num);
        int64_t j = i - 1;
        while (j >= 0 && arr[j * col_num + key] > t[key]) {
            memcpy(arr + (j + 1) * col_num, arr + j * col_num, sizeof(T) * col_num);
            j--;
        }
        memcpy(arr + (j + 1) * col_num, t, sizeof(T) * col_num);
    }
    if (t != tmp)
        free(t);
}

/* Stable bottom-up merge sort; ties keep the left (earlier) row first, which
 * is exactly the order insertion sort produces. */
int smj_ref_stable_sort(int col_num, int64_t row_num, int key, T *arr)
{
    if (row_num < 2)
        return 0;
    const size_t w = sizeof(T) * col_num;
    T *buf = (T *)malloc(w * row_num);
    if (!buf)
        return -1;
    /* runs of 16 by insertion sort first */
    const int64_t RUN = 16;
    for (int64_t s = 0; s < row_num; s += RUN) {
        int64_t e = s + RUN < row_num ? s + RUN : row_num;
        smj_ref_insertion_sort(col_num, e - s, key, arr + s * col_num);
    }
    T *src = arr, *dst = buf;
    for (int64_t width = RUN; width < row_num; width *= 2) {
        for (int64_t lo = 0; lo < row_num; lo += 2 * width) {
            int64_t mid = lo + width < row_num ? lo + width : row_num;
            int64_t hi = lo + 2 * width < row_num ? lo + 2 * width : row_num;
            int64_t i = lo, j = mid, k = lo;
            while (i < mid && j < hi) {
                if (src[j * col_num + key] < src[i * col_num + key]) {
                    memcpy(dst + k * col_num, src + j * col_num, w);
                    j++;
                } else {
                    memcpy(dst + k * col_num, src + i * col_num, w);
                    i++;
                }
                k++;
            }
            if (i < mid)
                memcpy(dst + k * col_num, src + i * col_num, w * (mid - i)), k += mid - i;
            if (j < hi)
                memcpy(dst + k * col_num, src + j * col_num, w * (hi - j));
        }
        T *t = src;
        src = dst;
        dst = t;
    }
    if (src != arr)
        memcpy(arr, src, w * row_num);
    free(buf);
    return 0;
}

/* cpu_app.c:211-227 */
int64_t smj_ref_join_count(int c1, int64_t r1, const T *a, int c2, int64_t r2, const T *b,
                           int key1, int key2)
{
    int64_t cnt = 0, i = 0, j = 0;
    while (i < r1 && j < r2) {
        T ka = a[i * c1 + key1], kb = b[j * c2 + key2];
        if (ka == kb) {
            cnt++;
            i++;
            j++;
        } else if (ka < kb) {
            i++;
        } else {
            j++;
        }
    }
    return cnt;
}

/* cpu_app.c:204-266 */
int64_t smj_ref_join(int c1, int64_t r1, const T *a, int c2, int64_t r2, const T *b,
                     int key1, int key2, T **out)
{
    const int tc = c1 + c2 - 1;
    int64_t cnt = smj_ref_join_count(c1, r1, a, c2, r2, b, key1, key2);
    T *res = (T *)malloc(sizeof(T) * (size_t)(cnt > 0 ? cnt : 1) * tc);
    if (!res)
        return -1;
    int64_t i = 0, j = 0, o = 0;
    while (i < r1 && j < r2) {
        T ka = a[i * c1 + key1], kb = b[j * c2 + key2];
        if (ka == kb) {
            T *row = res + o * tc;
            memcpy(row, a + i * c1, sizeof(T) * c1);
            for (int c = 0, k = 0; c < c2; c++)
                if (c != key2)
                    row[c1 + k++] = b[j * c2 + c];
            o++;
            i++;
            j++;
        } else if (ka < kb) {
            i++;
        } else {
            j++;
        }
    }
    *out = res;
    return cnt;
}

/* cpu_app.c:268-301 */
int smj_ref_save_csv(const char *path, int col_num, int64_t row_num, const T *arr)
{
    FILE *f = fopen(path, "w");
    if (!f)
        return -1;
    for (int i = 1; i <= col_num; i++)
        fprintf(f, i < col_num ? "col%d," : "col%d", i);
    fputc('\n', f);
    for (int64_t r = 0; r < row_num; r++) {
        for (int c = 0; c < col_num; c++)
            fprintf(f, c < col_num - 1 ? "%ld," : "%ld", (long)arr[r * col_num + c]);
        fputc('\n', f);
    }
    fclose(f);
    return 0;
}

static double now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* cpu_app.c:303-361 (with save_to_csv enabled when out_path != NULL). */
int64_t smj_ref_pipeline_csv(const char *path1, const char *path2, const char *out_path,
                             int sel_col1, T sel_val1, int sel_col2, T sel_val2,
                             int key1, int key2, int use_insertion, double *elapsed_ms)
{
    int c1, r1, c2, r2;
    if (smj_ref_csv_size(path1, &c1, &r1) || smj_ref_csv_size(path2, &c2, &r2))
        return -1;
    double t0 = now_ms();
    T *a = NULL, *b = NULL;
    if (smj_ref_load_csv(path1, c1, r1, &a) || smj_ref_load_csv(path2, c2, r2, &b))
        return -1;
    int64_t n1 = r1, n2 = r2;
    smj_ref_select(c1, &n1, &a, sel_col1, sel_val1);
    smj_ref_select(c2, &n2, &b, sel_col2, sel_val2);
    if (use_insertion) {
        smj_ref_insertion_sort(c1, n1, key1, a);
        smj_ref_insertion_sort(c2, n2, key2, b);
    } else {
        smj_ref_stable_sort(c1, n1, key1, a);
        smj_ref_stable_sort(c2, n2, key2, b);
    }
    T *res = NULL;
    int64_t j = smj_ref_join(c1, n1, a, c2, n2, b, key1, key2, &res);
    double t1 = now_ms();
    if (elapsed_ms)
        *elapsed_ms = t1 - t0;
    if (out_path && j >= 0)
        smj_ref_save_csv(out_path, c1 + c2 - 1, j, res);
    free(a);
    free(b);
    free(res);
    return j;
}

uint64_t smj_ref_splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

uint64_t smj_ref_digest(const void *rows, int64_t row_num, int col_num, int64_t pos0)
{
    const uint64_t *r = (const uint64_t *)rows;
    uint64_t acc = 0;
    for (int64_t i = 0; i < row_num; i++) {
        uint64_t h = smj_ref_splitmix64((uint64_t)(pos0 + i) ^ 0x5851F42D4C957F2DULL);
        for (int c = 0; c < col_num; c++) h = smj_ref_splitmix64(h + r[i * col_num + c]);
        acc += h;
    }
    return acc;
}

void smj_ref_gen_uniform(T *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t key_range)
{
    const uint64_t salt = seed * 0xD1B54A32D192ED03ULL;
    for (int64_t i = 0; i < rows; i++) {
        uint64_t g = (uint64_t)(row0 + i);
        uint64_t h = smj_ref_splitmix64(g + salt);
        uint64_t k = (uint64_t)(((unsigned __int128)h * key_range) >> 64);
        out[2 * i] = (T)(1 + k);
        out[2 * i + 1] = (T)g;
    }
}

/* Zipf(theta) keys over [1, domain], the restatement of the
 * device generator gen_zipf_kernel (pim-sort-merge-join_amd/csrc/smj_kernels.hip):
 * global row g draws u = splitmix64(g + seed * 0xD1B54A32D192ED03) / 2^64
 * (53 bits), the rank by Gray et al.'s inverse CDF approximation (ranks 1
 * and 2 exact), scattered over the domain by rank * 2654435761 + 12345 mod
 * domain; payload = g.  A function of g only: the table is the same however
 * it is sharded. */
void smj_ref_gen_zipf(T *out, int64_t row0, int64_t rows, uint64_t seed, int64_t n, double theta, double zetan)
{
    const uint64_t salt = seed * 0xD1B54A32D192ED03ULL;
    const double alpha = 1.0 / (1.0 - theta);
    const double zeta2 = 1.0 + pow(0.5, theta);
    const double eta = (1.0 - pow(2.0 / (double)n, 1.0 - theta)) / (1.0 - zeta2 / zetan);
    for (int64_t i = 0; i < rows; i++) {
        const uint64_t g = (uint64_t)(row0 + i);
        const double u = (double)(smj_ref_splitmix64(g + salt) >> 11) * 0x1.0p-53;
        const double uz = u * zetan;
        int64_t rank;
        if (uz < 1.0) rank = 1;
        else if (uz < zeta2) rank = 2;
        else rank = 1 + (int64_t)((double)n * pow(eta * u - eta + 1.0, alpha));
        rank = rank < 1 ? 1 : (rank > n ? n : rank);
        const uint64_t key = (uint64_t)(((unsigned __int128)(uint64_t)(rank - 1) * 2654435761ULL + 12345u) %
                                        (unsigned __int128)(uint64_t)n);
        out[2 * i] = (T)(key + 1);
        out[2 * i + 1] = (T)g;
    }
}

/* C3-wide (SURVEY 8(d) stress input), the restatement of the device generator
 * gen_wide_kernel (pim-sort-merge-join_amd/csrc/smj_kernels.hip, smj.h
 * smj_dev_gen_wide): row g's own key is the full 64-bit splitmix64(g + seed *
 * 0xD1B54A32D192ED03) read as a signed int64; with plant_rows > 0 a third of
 * the rows (d = splitmix64(key ^ 0x2545F4914F6CDD1D), floor(3 d / 2^64) == 0)
 * take the key of row floor(splitmix64(d) * plant_rows / 2^64) of the
 * plant_seed table instead.  payload = g. */
void smj_ref_gen_wide(T *out, int64_t row0, int64_t rows, uint64_t seed, uint64_t plant_seed, int64_t plant_rows)
{
    const uint64_t salt = seed * 0xD1B54A32D192ED03ULL, psalt = plant_seed * 0xD1B54A32D192ED03ULL;
    for (int64_t i = 0; i < rows; i++) {
        const uint64_t g = (uint64_t)(row0 + i);
        uint64_t key = smj_ref_splitmix64(g + salt);
        if (plant_rows > 0) {
            const uint64_t d = smj_ref_splitmix64(key ^ 0x2545F4914F6CDD1DULL);
            if ((uint64_t)(((unsigned __int128)d * 3u) >> 64) == 0) {
                const uint64_t r = (uint64_t)(((unsigned __int128)smj_ref_splitmix64(d) * (uint64_t)plant_rows) >> 64);
                key = smj_ref_splitmix64(r + psalt);
            }
        }
        out[2 * i] = (T)(int64_t)key;
        out[2 * i + 1] = (T)g;
    }
}
