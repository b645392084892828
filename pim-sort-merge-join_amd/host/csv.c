/*
 * csv.c -- CSV ingest / egress with the reference's exact semantics (csv.h).
 *
 * The file is read in one go and cut into the same "lines" the reference's
 * fgets(line, 1024, f) loop sees (app.c:40, :78): up to and including '\n',
 * at most 1023 bytes.  Tokens are maximal runs without ',' (strtok(",")
 * collapses empty fields, app.c:80-86) and end at a NUL byte like a C string.
 */
#define _GNU_SOURCE
#include "csv.h"

#include <errno.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define SMJ_FGETS_MAX 1023 /* char line[1024] */

static int read_all(const char *path, char **buf, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return -1;
    size_t cap = 1 << 20, n = 0;
    char *b = (char *)malloc(cap + 1);
    if (!b) {
        fclose(f);
        return -1;
    }
    for (;;) {
        if (n == cap) {
            cap *= 2;
            char *nb = (char *)realloc(b, cap + 1);
            if (!nb) {
                free(b);
                fclose(f);
                return -1;
            }
            b = nb;
        }
        size_t r = fread(b + n, 1, cap - n, f);
        n += r;
        if (r == 0)
            break;
    }
    fclose(f);
    b[n] = '\0';
    *buf = b;
    *len = n;
    return 0;
}

/* One fgets() line starting at p: returns its length (>= 1) or 0 at EOF. */
static size_t next_line(const char *p, const char *end)
{
    if (p >= end)
        return 0;
    size_t lim = (size_t)(end - p) < SMJ_FGETS_MAX ? (size_t)(end - p) : SMJ_FGETS_MAX;
    const char *nl = (const char *)memchr(p, '\n', lim);
    return nl ? (size_t)(nl - p) + 1 : lim;
}

/* glibc atoi(): (int) strtol(s, NULL, 10) -- saturate at long, wrap to int. */
static int atoi_like(const char *s, const char *end)
{
    while (s < end && (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\v' || *s == '\f' || *s == '\r'))
        s++;
    int neg = 0;
    if (s < end && (*s == '+' || *s == '-')) {
        neg = *s == '-';
        s++;
    }
    unsigned long acc = 0;
    int over = 0;
    const unsigned long lim = neg ? (unsigned long)LONG_MAX + 1ul : (unsigned long)LONG_MAX;
    for (; s < end && *s >= '0' && *s <= '9'; s++) {
        unsigned d = (unsigned)(*s - '0');
        if (over || acc > (lim - d) / 10) {
            over = 1;
            continue;
        }
        acc = acc * 10 + d;
    }
    long v;
    if (over)
        v = neg ? LONG_MIN : LONG_MAX;
    else
        v = neg ? (long)(0ul - acc) : (long)acc;
    return (int)(unsigned int)(unsigned long)v; /* low 32 bits, as the (int) cast */
}

/* Visit the strtok(",") tokens of one line; returns the token count. */
typedef void (*tok_fn)(void *ctx, const char *b, const char *e);
static int tokens(const char *p, size_t len, tok_fn fn, void *ctx)
{
    const char *end = p + len;
    const char *z = (const char *)memchr(p, '\0', len); /* C-string end */
    if (z)
        end = z;
    int k = 0;
    while (p < end) {
        while (p < end && *p == ',')
            p++;
        if (p >= end)
            break;
        const char *b = p;
        while (p < end && *p != ',')
            p++;
        if (fn)
            fn(ctx, b, p);
        k++;
    }
    return k;
}

struct fill_ctx {
    T *arr;
    int64_t idx, cells;
};

static void fill_tok(void *vctx, const char *b, const char *e)
{
    struct fill_ctx *c = (struct fill_ctx *)vctx;
    if (c->idx >= 0 && c->idx < c->cells)
        c->arr[c->idx] = (T)atoi_like(b, e);
    c->idx++;
}

int smj_csv_load(const char *path, int *col_num, int *row_num, T **out)
{
    char *buf;
    size_t len;
    if (read_all(path, &buf, &len))
        return -1;
    const char *p = buf, *end = buf + len;
    /* pass 1: header columns + line count (set_csv_size, app.c:28-57) */
    int cols = 0;
    int64_t lines = 0;
    for (size_t l; (l = next_line(p, end)) > 0; p += l) {
        if (lines == 0)
            cols = tokens(p, l, NULL, NULL);
        lines++;
    }
    int64_t rows = lines > 0 ? lines - 1 : 0;
    if (rows > INT_MAX) {
        free(buf);
        errno = EFBIG;
        return -1;
    }
    int64_t cells = (int64_t)cols * rows;
    T *arr = (T *)calloc(cells > 0 ? (size_t)cells : 1, sizeof(T));
    if (!arr) {
        free(buf);
        return -1;
    }
    /* pass 2: load_csv (app.c:59-92) */
    p = buf;
    size_t l = next_line(p, end); /* header */
    p += l;
    int64_t row = 0;
    struct fill_ctx ctx = {arr, 0, cells};
    for (; (l = next_line(p, end)) > 0; p += l, row++) {
        ctx.idx = row * cols;
        tokens(p, l, fill_tok, &ctx);
    }
    free(buf);
    *col_num = cols;
    *row_num = (int)rows;
    *out = arr;
    return 0;
}

static char *put_i64(char *o, int64_t v)
{
    char tmp[24];
    int n = 0;
    uint64_t u = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
    do {
        tmp[n++] = (char)('0' + u % 10);
        u /= 10;
    } while (u);
    if (v < 0)
        *o++ = '-';
    while (n)
        *o++ = tmp[--n];
    return o;
}

int smj_csv_save(const char *path, int col_num, int64_t row_num, const T *arr)
{
    FILE *f = fopen(path, "w");
    if (!f)
        return -1;
    for (int i = 1; i <= col_num; i++)
        fprintf(f, i < col_num ? "col%d," : "col%d", i);
    fputc('\n', f);
    const size_t CH = 1 << 20;
    char *buf = (char *)malloc(CH + 64 * (size_t)(col_num + 1));
    if (!buf) {
        fclose(f);
        return -1;
    }
    char *o = buf;
    for (int64_t r = 0; r < row_num; r++) {
        const T *row = arr + r * col_num;
        for (int c = 0; c < col_num; c++) {
            o = put_i64(o, (int64_t)row[c]);
            *o++ = c < col_num - 1 ? ',' : '\n';
        }
        if ((size_t)(o - buf) >= CH) {
            fwrite(buf, 1, (size_t)(o - buf), f);
            o = buf;
        }
    }
    fwrite(buf, 1, (size_t)(o - buf), f);
    free(buf);
    return fclose(f) == 0 ? 0 : -1;
}
