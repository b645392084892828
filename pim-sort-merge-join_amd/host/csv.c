/*
 * csv.c -- CSV ingest / egress with the reference's exact semantics (csv.h).
 *
 * The file is read in one go and cut into the same "lines" the reference's
 * fgets(line, 1024, f) loop sees (app.c:40, :78): up to and including '\n',
 * at most 1023 bytes.  Tokens are maximal runs without ',' (strtok(",")
 * collapses empty fields, app.c:80-86) and end at a NUL byte like a C string.
 *
 * Both directions run on a pool of threads.  Ingest:
 * an fgets() line always restarts after a '\n', so the file is cut into
 * chunks at newlines and every chunk is counted, then parsed, on its own;
 * the only cross-row effect of the reference loop -- a row with more tokens
 * than the header spills into the next rows' cells -- is replayed in row
 * order afterwards.  Egress: rows are formatted in parallel slices and
 * written in order.  One thread runs the serial code (the semantics'
 * reference, kept below).
 */
#define _GNU_SOURCE
#include "csv.h"

#include <errno.h>
#include <limits.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

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

static int csv_load_serial(const char *path, int *col_num, int *row_num, T **out)
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

static int csv_save_serial(const char *path, int col_num, int64_t row_num, const T *arr)
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

/* ------------------------------------------------------------------------ */
/* parallel ingest / egress                                                 */
/* ------------------------------------------------------------------------ */
static int g_csv_threads = 0; /* 0: SMJ_CSV_THREADS, OMP_NUM_THREADS, min(ncpu, 16) */

void smj_csv_set_threads(int n) { g_csv_threads = n; }

static int csv_threads(size_t work, size_t per)
{
    int n = g_csv_threads;
    const char *e;
    if (n > 0) /* explicit: no size cap (the tests force threads on small files) */
        return n > 64 ? 64 : n;
    if ((e = getenv("SMJ_CSV_THREADS")) != NULL)
        n = atoi(e);
    if (n <= 0 && (e = getenv("OMP_NUM_THREADS")) != NULL)
        n = atoi(e);
    if (n <= 0) {
        long c = sysconf(_SC_NPROCESSORS_ONLN);
        n = c > 16 ? 16 : c > 0 ? (int)c : 1;
    }
    if (n > 64)
        n = 64;
    size_t most = work / per + 1; /* at least `per` units of work per thread */
    if ((size_t)n > most)
        n = (int)most;
    return n < 1 ? 1 : n;
}

struct spill {
    int64_t row;
    size_t off, len; /* the line's bytes */
};

struct load_job {
    const char *b, *e;  /* chunk [b, e): whole lines */
    int64_t row0, rows; /* first row, line count */
    int cols;
    int64_t cells;
    T *arr;
    uint16_t *ntok;     /* tokens per row (a line holds <= 512) */
    const char *base;
    struct spill *sp;   /* rows with more tokens than cols */
    size_t nsp, csp;
    int err;
};

static void *load_count(void *vj)
{
    struct load_job *j = (struct load_job *)vj;
    int64_t n = 0;
    for (const char *p = j->b; p < j->e;) {
        size_t l = next_line(p, j->e);
        p += l;
        n++;
    }
    j->rows = n;
    return NULL;
}

struct own_ctx {
    T *arr;
    int64_t base, cells;
    int cols, k;
};

static void own_tok(void *vctx, const char *b, const char *e)
{
    struct own_ctx *c = (struct own_ctx *)vctx;
    if (c->k < c->cols && c->base + c->k < c->cells)
        c->arr[c->base + c->k] = (T)atoi_like(b, e);
    c->k++;
}

static void *load_parse(void *vj)
{
    struct load_job *j = (struct load_job *)vj;
    int64_t r = j->row0;
    for (const char *p = j->b; p < j->e; r++) {
        size_t l = next_line(p, j->e);
        struct own_ctx c = {j->arr, r * j->cols, j->cells, j->cols, 0};
        const int k = tokens(p, l, own_tok, &c);
        j->ntok[r] = (uint16_t)k;
        if (k > j->cols) {
            if (j->nsp == j->csp) {
                size_t nc = j->csp ? 2 * j->csp : 64;
                struct spill *ns = (struct spill *)realloc(j->sp, nc * sizeof *ns);
                if (!ns) {
                    j->err = 1;
                    return NULL;
                }
                j->sp = ns;
                j->csp = nc;
            }
            j->sp[j->nsp].row = r;
            j->sp[j->nsp].off = (size_t)(p - j->base);
            j->sp[j->nsp].len = l;
            j->nsp++;
        }
        p += l;
    }
    return NULL;
}

struct spill_ctx {
    T *arr;
    const uint16_t *ntok;
    int64_t base, cells;
    int cols, k;
};

/* token k of a spilling row: cell base + k lands in row r' = idx / cols;
 * the last writer in the reference's row order wins -- row r' itself when
 * it has a token for that column, else the latest spilling row */
static void spill_tok(void *vctx, const char *b, const char *e)
{
    struct spill_ctx *c = (struct spill_ctx *)vctx;
    if (c->k >= c->cols) {
        const int64_t idx = c->base + c->k;
        if (idx < c->cells && (int64_t)c->ntok[idx / c->cols] <= idx % c->cols)
            c->arr[idx] = (T)atoi_like(b, e);
    }
    c->k++;
}

int smj_csv_load(const char *path, int *col_num, int *row_num, T **out)
{
    char *buf;
    size_t len;
    if (read_all(path, &buf, &len))
        return -1;
    const char *end = buf + len;
    int nt = csv_threads(len, (size_t)4 << 20);
    if (nt == 1) {
        free(buf);
        return csv_load_serial(path, col_num, row_num, out);
    }
    size_t hl = next_line(buf, end);
    const int cols = hl ? tokens(buf, hl, NULL, NULL) : 0;
    const char *p0 = buf + hl;
    struct load_job *jobs = (struct load_job *)calloc((size_t)nt, sizeof *jobs);
    pthread_t *th = (pthread_t *)calloc((size_t)nt, sizeof *th);
    if (!jobs || !th) {
        free(jobs);
        free(th);
        free(buf);
        return -1;
    }
    const char *cut = p0;
    for (int t = 0; t < nt; t++) { /* chunks end right after a '\n' (or at EOF) */
        const char *e = t + 1 == nt ? end : p0 + (size_t)(end - p0) * (size_t)(t + 1) / (size_t)nt;
        if (e < cut)
            e = cut;
        if (e < end && e > cut) {
            const char *nl = (const char *)memchr(e - 1, '\n', (size_t)(end - (e - 1)));
            e = nl ? nl + 1 : end;
        }
        jobs[t].b = cut;
        jobs[t].e = e;
        jobs[t].base = buf;
        cut = e;
    }
    for (int t = 0; t < nt; t++)
        pthread_create(&th[t], NULL, load_count, &jobs[t]);
    int64_t rows = 0;
    for (int t = 0; t < nt; t++) {
        pthread_join(th[t], NULL);
        jobs[t].row0 = rows;
        rows += jobs[t].rows;
    }
    int rc = -1;
    T *arr = NULL;
    uint16_t *ntok = NULL;
    if (rows > INT_MAX) {
        errno = EFBIG;
        goto done;
    }
    const int64_t cells = (int64_t)cols * rows;
    arr = (T *)calloc(cells > 0 ? (size_t)cells : 1, sizeof(T));
    ntok = (uint16_t *)malloc((size_t)(rows > 0 ? rows : 1) * sizeof *ntok);
    if (!arr || !ntok)
        goto done;
    for (int t = 0; t < nt; t++) {
        jobs[t].cols = cols;
        jobs[t].cells = cells;
        jobs[t].arr = arr;
        jobs[t].ntok = ntok;
        pthread_create(&th[t], NULL, load_parse, &jobs[t]);
    }
    int err = 0;
    for (int t = 0; t < nt; t++) {
        pthread_join(th[t], NULL);
        err |= jobs[t].err;
    }
    if (err)
        goto done;
    for (int t = 0; t < nt; t++) /* spills, in row order */
        for (size_t i = 0; i < jobs[t].nsp; i++) {
            const struct spill *sp = &jobs[t].sp[i];
            struct spill_ctx c = {arr, ntok, sp->row * cols, cells, cols, 0};
            tokens(buf + sp->off, sp->len, spill_tok, &c);
        }
    *col_num = cols;
    *row_num = (int)rows;
    *out = arr;
    arr = NULL;
    rc = 0;
done:
    for (int t = 0; t < nt; t++)
        free(jobs[t].sp);
    free(jobs);
    free(th);
    free(arr);
    free(ntok);
    free(buf);
    return rc;
}

struct save_job {
    const T *arr;
    int cols;
    int64_t r0, r1;
    char *buf;
    size_t cap, len;
};

static void *save_fmt(void *vj)
{
    struct save_job *j = (struct save_job *)vj;
    const size_t need = (size_t)(j->r1 - j->r0) * (size_t)j->cols * 21 + 1;
    if (need > j->cap) {
        free(j->buf);
        j->buf = (char *)malloc(need);
        j->cap = j->buf ? need : 0;
    }
    j->len = 0;
    if (!j->buf)
        return NULL;
    char *o = j->buf;
    for (int64_t r = j->r0; r < j->r1; r++) {
        const T *row = j->arr + r * j->cols;
        for (int c = 0; c < j->cols; c++) {
            o = put_i64(o, (int64_t)row[c]);
            *o++ = c < j->cols - 1 ? ',' : '\n';
        }
    }
    j->len = (size_t)(o - j->buf);
    return NULL;
}

int smj_csv_save(const char *path, int col_num, int64_t row_num, const T *arr)
{
    const int nt = col_num > 0 ? csv_threads((size_t)row_num * (size_t)col_num, (size_t)1 << 18) : 1;
    if (nt == 1)
        return csv_save_serial(path, col_num, row_num, arr);
    FILE *f = fopen(path, "w");
    if (!f)
        return -1;
    for (int i = 1; i <= col_num; i++)
        fprintf(f, i < col_num ? "col%d," : "col%d", i);
    fputc('\n', f);
    struct save_job *jobs = (struct save_job *)calloc((size_t)nt, sizeof *jobs);
    pthread_t *th = (pthread_t *)calloc((size_t)nt, sizeof *th);
    int rc = jobs && th ? 0 : -1;
    const int64_t slice = (int64_t)1 << 18; /* rows per thread and round */
    for (int64_t r = 0; rc == 0 && r < row_num; r += slice * nt) {
        for (int t = 0; t < nt; t++) {
            jobs[t].arr = arr;
            jobs[t].cols = col_num;
            jobs[t].r0 = r + slice * t < row_num ? r + slice * t : row_num;
            jobs[t].r1 = r + slice * (t + 1) < row_num ? r + slice * (t + 1) : row_num;
            pthread_create(&th[t], NULL, save_fmt, &jobs[t]);
        }
        for (int t = 0; t < nt; t++) {
            pthread_join(th[t], NULL);
            if (jobs[t].r1 > jobs[t].r0 && !jobs[t].buf)
                rc = -1;
        }
        for (int t = 0; rc == 0 && t < nt; t++)
            if (jobs[t].len && fwrite(jobs[t].buf, 1, jobs[t].len, f) != jobs[t].len)
                rc = -1;
    }
    if (jobs)
        for (int t = 0; t < nt; t++)
            free(jobs[t].buf);
    free(jobs);
    free(th);
    if (fclose(f) != 0)
        rc = -1;
    return rc;
}
