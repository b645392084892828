// cpu_mt.cpp -- CPU BASELINE / TEST INFRASTRUCTURE ONLY (bench.py's
// cpu_baseline leg and tests/; never the product path).
//
// A multi-core port of cpu_app.c's pipeline with the same semantics (SURVEY
// 8(d): "the build-owned multi-core std::stable_sort baseline with the same
// semantics, with core count stated"):
//   select_in_cpu (cpu_app.c:81-112)   stable compaction row[sc] > sv, per table
//   insertion_sort_in_cpu (:172-202)   stable ascending sort on row[key]
//   join_in_cpu (:204-266)             1:1 zip join, R columns then S columns
//                                      without key2 (:236-256)
// The sort orders (key, input index) pairs -- a total order equal to the
// stable order -- with chunk-parallel std::sort and pairwise parallel
// std::merge rounds; rows are then gathered in parallel.  The zip join is a
// serial O(n) walk.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct KI {
    int64_t key;
    int64_t idx;
};
inline bool ki_less(const KI &a, const KI &b) { return a.key < b.key || (a.key == b.key && a.idx < b.idx); }

template <class F>
void parallel_for(int threads, int64_t n, F f) {  // f(t, begin, end)
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        const int64_t b = n * t / threads, e = n * (t + 1) / threads;
        th.emplace_back([=] { f(t, b, e); });
    }
    for (auto &x : th) x.join();
}

// stable select + sort of one table into `out` (rows); returns the kept rows
int64_t select_sort(const int64_t *in, int64_t n, int cols, int use_sel, int sc, int64_t sv, int key, int threads,
                    int64_t *out) {
    std::vector<int64_t> cnt(threads + 1, 0);
    parallel_for(threads, n, [&](int t, int64_t b, int64_t e) {
        int64_t c = 0;
        for (int64_t i = b; i < e; i++) c += !use_sel || in[i * cols + sc] > sv;
        cnt[t + 1] = c;
    });
    for (int t = 0; t < threads; t++) cnt[t + 1] += cnt[t];
    const int64_t m = cnt[threads];
    std::vector<KI> a(m), tmp(m);
    parallel_for(threads, n, [&](int t, int64_t b, int64_t e) {
        int64_t o = cnt[t];
        for (int64_t i = b; i < e; i++)
            if (!use_sel || in[i * cols + sc] > sv) a[o++] = KI{in[i * cols + key], i};
    });
    // chunk sorts, then pairwise merge rounds (runs double each round)
    const int runs = threads;
    std::vector<int64_t> edge(runs + 1);
    for (int r = 0; r <= runs; r++) edge[r] = m * r / runs;
    parallel_for(runs, runs, [&](int, int64_t b, int64_t e) {
        for (int64_t r = b; r < e; r++) std::sort(a.begin() + edge[r], a.begin() + edge[r + 1], ki_less);
    });
    KI *src = a.data(), *dst = tmp.data();
    for (int w = 1; w < runs; w *= 2) {
        std::vector<std::thread> th;
        for (int r = 0; r < runs; r += 2 * w) {
            const int64_t lo = edge[r], mid = edge[std::min(r + w, runs)], hi = edge[std::min(r + 2 * w, runs)];
            th.emplace_back([=] { std::merge(src + lo, src + mid, src + mid, src + hi, dst + lo, ki_less); });
        }
        for (auto &x : th) x.join();
        std::swap(src, dst);
    }
    parallel_for(threads, m, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; i++) std::memcpy(out + i * cols, in + src[i].idx * cols, sizeof(int64_t) * cols);
    });
    return m;
}

}  // namespace

extern "C" {

// The pipeline on host tables.  R_sorted / S_sorted (capacity nr / ns rows)
// receive the sorted selected rows; out (capacity min(nr, ns) rows of
// c1 + c2 - 1 columns; NULL: count only) the joined rows.  rows[3] =
// {m_R, m_S, J}; *seconds = wall time of the three phases.  Returns 0, or -1
// on bad arguments.
int smj_mt_pipeline(const int64_t *R, int64_t nr, int c1, const int64_t *S, int64_t ns, int c2, int use_sel1,
                    int sc1, int64_t sv1, int use_sel2, int sc2, int64_t sv2, int key1, int key2, int threads,
                    int64_t *R_sorted, int64_t *S_sorted, int64_t *out, int64_t *rows, double *seconds) {
    if (threads < 1 || c1 < 1 || c2 < 1 || !R_sorted || !S_sorted || !rows) return -1;
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t mr = select_sort(R, nr, c1, use_sel1, sc1, sv1, key1, threads, R_sorted);
    const int64_t ms = select_sort(S, ns, c2, use_sel2, sc2, sv2, key2, threads, S_sorted);
    const int tc = c1 + c2 - 1;
    int64_t i = 0, j = 0, J = 0;
    while (i < mr && j < ms) {  // join_in_cpu: equal keys advance both cursors
        const int64_t a = R_sorted[i * c1 + key1], b = S_sorted[j * c2 + key2];
        if (a == b) {
            if (out) {
                int64_t *o = out + J * tc;
                std::memcpy(o, R_sorted + i * c1, sizeof(int64_t) * c1);
                for (int c = 0, k = c1; c < c2; c++)
                    if (c != key2) o[k++] = S_sorted[j * c2 + c];
            }
            J++;
            i++;
            j++;
        } else if (a < b) {
            i++;
        } else {
            j++;
        }
    }
    const auto t1 = std::chrono::steady_clock::now();
    rows[0] = mr;
    rows[1] = ms;
    rows[2] = J;
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    return 0;
}

}  // extern "C"
