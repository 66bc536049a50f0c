/*
 * rsp_oracle.c — TEST INFRASTRUCTURE ONLY (see rsp_oracle.h). CPU
 * restatement of the reference hot path; never linked into the product.
 *
 * Build flags matter: -ffp-contract=off so `s += v * x` is a rounded
 * product then a rounded sum (the order the GPU tiles reproduce), and fma()
 * is called explicitly where the restated algorithm fuses (ILU updates and
 * triangular solves), which the GPU kernels mirror with v_fma_f64 / v_fma_f32 (fma_t).
 */
#include "rsp_oracle.h"

#include <limits.h>
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>
#include <xmmintrin.h>

static unsigned ftz_enter(int on) {
    unsigned old = _mm_getcsr();
    if (on) _mm_setcsr(old | 0x8040u); /* test_pardiso.c:19-24 */
    return old;
}
static void ftz_leave(unsigned old) { _mm_setcsr(old); }

/* ------------------------------------------------------------------ SpMV */

void oracle_spmv_f64(int m, const int *rp, const int *ci, const double *v, const double *x,
                     double *y) {
    for (int i = 0; i < m; i++) {
        double s = 0.0;
        for (int k = rp[i]; k < rp[i + 1]; k++) s += v[k] * x[ci[k]];
        y[i] = s;
    }
}

void oracle_spmv_f32(int m, const int *rp, const int *ci, const float *v, const float *x,
                     float *y) {
    for (int i = 0; i < m; i++) {
        float s = 0.0f;
        for (int k = rp[i]; k < rp[i + 1]; k++) s += v[k] * x[ci[k]];
        y[i] = s;
    }
}

void oracle_spmv_f32_ftz(int m, const int *rp, const int *ci, const float *v, const float *x,
                         float *y) {
    unsigned old = ftz_enter(1);
    oracle_spmv_f32(m, rp, ci, v, x, y);
    ftz_leave(old);
}

void oracle_spmv_f64_omp(int m, const int *rp, const int *ci, const double *v, const double *x,
                         double *y) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < m; i++) {
        double s = 0.0;
        for (int k = rp[i]; k < rp[i + 1]; k++) s += v[k] * x[ci[k]];
        y[i] = s;
    }
}

void oracle_spmv_f32_omp(int m, const int *rp, const int *ci, const float *v, const float *x,
                         float *y) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < m; i++) {
        float s = 0.0f;
        for (int k = rp[i]; k < rp[i + 1]; k++) s += v[k] * x[ci[k]];
        y[i] = s;
    }
}

int oracle_num_threads(void) { return omp_get_max_threads(); }
void oracle_set_threads(int t) { omp_set_num_threads(t > 0 ? t : 1); }

/* Canonical summation order of the GPU SpMV (spmv.hip), a function of the
 * row alone (independent of tiling, lanes per row and row partition):
 *  - rows of <= 256 products: partial p_j sums the products e = j, j+8, ...
 *    (e counted from the row start) in order; y = ((p0+p4)+(p2+p6)) +
 *    ((p1+p5)+(p3+p7));
 *  - longer rows: cut into chunks of `cap` products from the row start
 *    (cap = 2047 fp64 / 4093 fp32, the tile capacity); in a chunk, q_t sums
 *    products t, t+256, ... in order (t < 256), each group of 64 q's is
 *    combined by a xor-butterfly tree (stride 32, 16, ..., 1) and the four
 *    results as (w0+w1)+(w2+w3); the chunks are added in order from 0. */
#define ORACLE_CANON(T, NAME)                                                                  \
    void NAME(int m, const int *rp, const int *ci, const T *v, const T *x, T *y, int cap) {    \
        for (int i = 0; i < m; i++) {                                                          \
            const int a = rp[i], len = rp[i + 1] - rp[i];                                      \
            if (len <= 256) {                                                                  \
                T p[8] = {0, 0, 0, 0, 0, 0, 0, 0};                                             \
                for (int k = a; k < a + len; k++) p[(k - a) & 7] += v[k] * x[ci[k]];           \
                for (int h = 4; h >= 1; h >>= 1)                                               \
                    for (int t = 0; t < h; t++) p[t] = p[t] + p[t + h];                        \
                y[i] = p[0];                                                                   \
                continue;                                                                      \
            }                                                                                  \
            T row = 0;                                                                         \
            for (int c0 = 0; c0 < len; c0 += cap) {                                            \
                const int c1 = c0 + cap < len ? c0 + cap : len;                                \
                T q[256];                                                                      \
                for (int t = 0; t < 256; t++) q[t] = 0;                                        \
                for (int e = c0; e < c1; e++) q[(e - c0) & 255] += v[a + e] * x[ci[a + e]];     \
                T w[4];                                                                        \
                for (int g = 0; g < 4; g++) {                                                  \
                    T *qq = q + 64 * g;                                                        \
                    for (int o = 32; o >= 1; o >>= 1)                                          \
                        for (int l = 0; l < o; l++) qq[l] = qq[l] + qq[l + o];                 \
                    w[g] = qq[0];                                                              \
                }                                                                              \
                row += (w[0] + w[1]) + (w[2] + w[3]);                                          \
            }                                                                                  \
            y[i] = row;                                                                        \
        }                                                                                      \
    }
ORACLE_CANON(double, oracle_spmv_canon_f64)
ORACLE_CANON(float, oracle_spmv_canon_f32)

void oracle_spmv_canon_f32_ftz(int m, const int *rp, const int *ci, const float *v, const float *x,
                               float *y, int cap) {
    unsigned old = ftz_enter(1);
    oracle_spmv_canon_f32(m, rp, ci, v, x, y, cap);
    ftz_leave(old);
}

/* ---------------------------------------------------------------- ILU(0) */

/* first position in row i with column >= i */
static int diag_pos(const int *rp, const int *ci, int i) {
    int lo = rp[i], hi = rp[i + 1];
    while (lo < hi) {
        int mid = lo + (hi - lo) / 2;
        if (ci[mid] < i)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

#define ORACLE_ILU0(T, NAME, FMA)                                                              \
    static int NAME(int n, const int *rp, const int *ci, T *v, int *zero_pivot) {              \
        int *dp = (int *)malloc(sizeof(int) * (size_t)(n ? n : 1));                            \
        int *hd = (int *)malloc(sizeof(int) * (size_t)(n ? n : 1));                            \
        int *iw = (int *)malloc(sizeof(int) * (size_t)(n ? n : 1));                            \
        int structural = -1;                                                                   \
        for (int i = 0; i < n; i++) {                                                          \
            dp[i] = diag_pos(rp, ci, i);                                                       \
            hd[i] = dp[i] < rp[i + 1] && ci[dp[i]] == i;                                       \
            if (!hd[i] && structural < 0) structural = i;                                      \
            iw[i] = -1;                                                                        \
        }                                                                                      \
        *zero_pivot = -1;                                                                      \
        if (structural >= 0) {                                                                 \
            free(dp);                                                                          \
            free(hd);                                                                          \
            free(iw);                                                                          \
            return structural;                                                                 \
        }                                                                                      \
        for (int i = 0; i < n; i++) {                                                          \
            for (int p = rp[i]; p < rp[i + 1]; p++) iw[ci[p]] = p;                             \
            for (int p = rp[i]; p < dp[i]; p++) {                                              \
                int k = ci[p];                                                                 \
                T lik = v[p] / v[dp[k]];                                                       \
                v[p] = lik;                                                                    \
                for (int q = dp[k] + 1; q < rp[k + 1]; q++) {                                  \
                    int w = iw[ci[q]];                                                         \
                    if (w > p) v[w] = FMA(-lik, v[q], v[w]);                                   \
                }                                                                              \
            }                                                                                  \
            if (v[dp[i]] == (T)0 && *zero_pivot < 0) *zero_pivot = i;                          \
            for (int p = rp[i]; p < rp[i + 1]; p++) iw[ci[p]] = -1;                            \
        }                                                                                      \
        free(dp);                                                                              \
        free(hd);                                                                              \
        free(iw);                                                                              \
        return -1;                                                                             \
    }

ORACLE_ILU0(double, ilu0_d, fma)
ORACLE_ILU0(float, ilu0_s, fmaf)

int oracle_ilu0_f64(int n, const int *rp, const int *ci, double *v, int *zero_pivot) {
    return ilu0_d(n, rp, ci, v, zero_pivot);
}

int oracle_ilu0_f32(int n, const int *rp, const int *ci, float *v, int *zero_pivot, int ftz) {
    unsigned old = ftz_enter(ftz);
    int r = ilu0_s(n, rp, ci, v, zero_pivot);
    ftz_leave(old);
    return r;
}

/* ------------------------------------------------------------------ trsv */

#define ORACLE_TRSV(T, SUF, FMA)                                                               \
    static void lower_n_##SUF(int n, const int *rp, const int *ci, const T *v, T alpha,        \
                              const T *x, T *y) {                                              \
        for (int i = 0; i < n; i++) {                                                          \
            T s = alpha * x[i];                                                                \
            for (int p = rp[i]; p < rp[i + 1] && ci[p] < i; p++) s = FMA(-v[p], y[ci[p]], s);  \
            y[i] = s;                                                                          \
        }                                                                                      \
    }                                                                                          \
    static void lower_t_##SUF(int n, const int *rp, const int *ci, const T *v, T alpha,        \
                              const T *x, T *y) {                                              \
        for (int i = 0; i < n; i++) y[i] = alpha * x[i];                                       \
        for (int j = n - 1; j >= 0; j--) {                                                     \
            const T yj = y[j];                                                                 \
            for (int p = rp[j]; p < rp[j + 1] && ci[p] < j; p++)                               \
                y[ci[p]] = FMA(-v[p], yj, y[ci[p]]);                                           \
        }                                                                                      \
    }                                                                                          \
    static void upper_##SUF(int n, const int *rp, const int *ci, const T *v, T alpha,          \
                            const T *x, T *y) {                                                \
        for (int i = n - 1; i >= 0; i--) {                                                     \
            T s = alpha * x[i];                                                                \
            int d = diag_pos(rp, ci, i);                                                       \
            int hd = d < rp[i + 1] && ci[d] == i;                                              \
            for (int p = d + hd; p < rp[i + 1]; p++) s = FMA(-v[p], y[ci[p]], s);              \
            y[i] = s / (hd ? v[d] : (T)0);                                                     \
        }                                                                                      \
    }

ORACLE_TRSV(double, d, fma)
ORACLE_TRSV(float, s, fmaf)

/* The solves in the SPLIT term order of the MI355X plans (round 4): the
 * terms of row i whose producer lies exactly one level below i in the
 * solve's DAG ("late": the level is the longest dependency path, so every
 * row of level > 0 has at least one) are applied after all its other terms
 * ("early"); each part keeps the reference's order (L: column ascending, as
 * the csrsv2 NON_TRANSPOSE sweep; L^T: j descending, as the TRANSPOSE column
 * sweep). Same terms, same fma per term; only the order of the sum differs,
 * within SURVEY 8c's solve tolerance (tests/test_oracle.py). The GPU can
 * then sum a row's early terms while the level just below it is still
 * running. */
static int *levels_l(int n, const int *rp, const int *ci) {
    int *lv = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int i = 0; i < n; i++) {
        int l = 0;
        for (int p = rp[i]; p < rp[i + 1] && ci[p] < i; p++)
            if (lv[ci[p]] + 1 > l) l = lv[ci[p]] + 1;
        lv[i] = l;
    }
    return lv;
}
/* the strict lower part by columns: for column k, the rows j > k with
 * l_jk != 0 in j-descending order (tp: CSR positions, tr: rows) */
static void lower_by_cols(int n, const int *rp, const int *ci, int **cp_, int **tp_, int **tr_) {
    int *cp = (int *)calloc((size_t)n + 1, sizeof(int));
    for (int j = 0; j < n; j++)
        for (int p = rp[j]; p < rp[j + 1] && ci[p] < j; p++) cp[ci[p] + 1]++;
    for (int k = 0; k < n; k++) cp[k + 1] += cp[k];
    int m = cp[n] > 0 ? cp[n] : 1;
    int *tp = (int *)malloc((size_t)m * sizeof(int)), *tr = (int *)malloc((size_t)m * sizeof(int));
    int *fill = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int k = 0; k < n; k++) fill[k] = cp[k];
    for (int j = n - 1; j >= 0; j--)
        for (int p = rp[j]; p < rp[j + 1] && ci[p] < j; p++) {
            tp[fill[ci[p]]] = p;
            tr[fill[ci[p]]++] = j;
        }
    free(fill);
    *cp_ = cp;
    *tp_ = tp;
    *tr_ = tr;
}

#define ORACLE_TRSV_SPLIT(T, SUF, FMA)                                                         \
    static void lower_n_split_##SUF(int n, const int *rp, const int *ci, const T *v, T alpha,  \
                                    const T *x, T *y) {                                        \
        int *lv = levels_l(n, rp, ci);                                                         \
        for (int i = 0; i < n; i++) {                                                          \
            T s = alpha * x[i];                                                                \
            for (int late = 0; late < 2; late++)                                               \
                for (int p = rp[i]; p < rp[i + 1] && ci[p] < i; p++)                           \
                    if ((lv[ci[p]] == lv[i] - 1) == late) s = FMA(-v[p], y[ci[p]], s);         \
            y[i] = s;                                                                          \
        }                                                                                      \
        free(lv);                                                                              \
    }                                                                                          \
    static void lower_t_split_##SUF(int n, const int *rp, const int *ci, const T *v, T alpha,  \
                                    const T *x, T *y) {                                        \
        int *cp, *tp, *tr;                                                                     \
        lower_by_cols(n, rp, ci, &cp, &tp, &tr);                                               \
        int *lv = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));                        \
        for (int k = n - 1; k >= 0; k--) { /* L^T levels: longest path from above */         \
            int l = 0;                                                                         \
            for (int q = cp[k]; q < cp[k + 1]; q++)                                            \
                if (lv[tr[q]] + 1 > l) l = lv[tr[q]] + 1;                                      \
            lv[k] = l;                                                                         \
        }                                                                                      \
        for (int k = n - 1; k >= 0; k--) {                                                     \
            T s = alpha * x[k];                                                                \
            for (int late = 0; late < 2; late++)                                               \
                for (int q = cp[k]; q < cp[k + 1]; q++)                                        \
                    if ((lv[tr[q]] == lv[k] - 1) == late) s = FMA(-v[tp[q]], y[tr[q]], s);     \
            y[k] = s;                                                                          \
        }                                                                                      \
        free(lv);                                                                              \
        free(cp);                                                                              \
        free(tp);                                                                              \
        free(tr);                                                                              \
    }

ORACLE_TRSV_SPLIT(double, d, fma)
ORACLE_TRSV_SPLIT(float, s, fmaf)

/* ---------------------------------------------- block-inverse solve order
 * (round 6, the deep-DAG solve of the MI355X plans; rsp_oracle.h). Every
 * step restated from the definition, independently of the product's planner
 * (respasol_amd/csrc/ilu_blocks.cpp):
 *  1. dependencies of row i in their order: kind 0 (L): (column j, position)
 *     of row i's strict lower part, j ascending; kind 1 (L^T): the rows j > i
 *     with l_ji != 0, j descending (the TRANSPOSE column sweep's order);
 *  2. levels (longest dependency path) and the level order: by level, rows
 *     ascending inside a level; "position" = index in that order;
 *  3. CHUNKS, one pass over the positions: a chunk starts at 0, at a
 *     position ch after its chunk's start, and at a position whose row has
 *     more than lcap dependencies at or after its chunk's start (that row
 *     starts a new chunk); no block crosses a chunk. Blocks, greedily over
 *     the positions: row p joins the current block (first position s) if the
 *     block has < bs rows, p does not start a chunk, and p's pattern with the
 *     block (below) has <= ymax y terms of which <= near are NEAR (position
 *     >= max(chunk start, s - nw));
 *     otherwise the block is closed and p starts a new block with its own
 *     dependencies as pattern; if that pattern breaks the same caps, p is a
 *     LONG block of its own (the next row starts a new block);
 *  4. pattern of p in block b (first position s): x sources = {p} and the x
 *     sources of its in-block dependencies; y sources = the y sources of its
 *     in-block dependencies and the positions of its dependencies before s;
 *     ordered x ascending, then y ascending;
 *  5. coefficients E (one per pattern entry, the block's partitioned
 *     inverse): start at 1 for x source p, 0 elsewhere; then, dependency by
 *     dependency in the order of 1. with value l: an in-block dependency q
 *     adds E_p[u] = fma(-l, E_q[u], E_p[u]) for every source u of q's
 *     pattern; one before the block adds E_p[q] = fma(-l, 1, E_p[q]);
 *  6. the solve, positions in order: a normal row is s = 0, then
 *     s = fma(E_k, v_k, s) over its pattern in order, v = alpha x_node for an
 *     x source (alpha x rounded first) and y of the source's position for a y
 *     source; a long row sums its pattern's entries k into 64 partials
 *     (k mod 64, each in order, from 0) combined by a xor butterfly
 *     (stride 32, 16, ..., 1: p_l = p_l + p_(l xor stride)), partial 0. */
#define BLK_DEFAULTS {64, 32, 12, 1 << 30, 16384, 768}
typedef struct {
    int *dp, *dj, *dv;  /* row i's dependencies [dp[i], dp[i+1]): source row, value position */
} BlkDeps;
static void blk_deps(int kind, int n, const int *rp, const int *ci, BlkDeps *d) {
    d->dp = (int *)calloc((size_t)n + 1, sizeof(int));
    if (kind == 0) {
        for (int i = 0; i < n; i++) {
            int c = 0;
            for (int p = rp[i]; p < rp[i + 1] && ci[p] < i; p++) c++;
            d->dp[i + 1] = d->dp[i] + c;
        }
        int m = d->dp[n] > 0 ? d->dp[n] : 1;
        d->dj = (int *)malloc((size_t)m * sizeof(int));
        d->dv = (int *)malloc((size_t)m * sizeof(int));
        for (int i = 0; i < n; i++) {
            int o = d->dp[i];
            for (int p = rp[i]; p < rp[i + 1] && ci[p] < i; p++, o++) {
                d->dj[o] = ci[p];
                d->dv[o] = p;
            }
        }
    } else {
        int *cp, *tp, *tr;
        lower_by_cols(n, rp, ci, &cp, &tp, &tr);
        memcpy(d->dp, cp, ((size_t)n + 1) * sizeof(int));
        d->dj = tr;
        d->dv = tp;
        free(cp);
    }
}
/* position -> row: level order, rows ascending inside a level */
static int *blk_order(int kind, int n, const BlkDeps *d) {
    int *lv = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    int nl = 0;
    for (int k = 0; k < n; k++) {
        int i = kind == 0 ? k : n - 1 - k, l = 0;
        for (int o = d->dp[i]; o < d->dp[i + 1]; o++)
            if (lv[d->dj[o]] + 1 > l) l = lv[d->dj[o]] + 1;
        lv[i] = l;
        if (l + 1 > nl) nl = l + 1;
    }
    int *cnt = (int *)calloc((size_t)nl + 1, sizeof(int));
    for (int i = 0; i < n; i++) cnt[lv[i] + 1]++;
    for (int l = 0; l < nl; l++) cnt[l + 1] += cnt[l];
    int *ord = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int i = 0; i < n; i++) ord[cnt[lv[i]]++] = i;
    free(cnt);
    free(lv);
    return ord;
}
typedef struct {
    int *v;
    long long n, cap;
} BlkVec;
static void bv_push(BlkVec *b, int x) {
    if (b->n == b->cap) {
        b->cap = b->cap ? 2 * b->cap : 1024;
        b->v = (int *)realloc(b->v, (size_t)b->cap * sizeof(int));
    }
    b->v[b->n++] = x;
}
static int cmp_int(const void *a, const void *b) {
    int x = *(const int *)a, y = *(const int *)b;
    return x < y ? -1 : x > y;
}
/* the plan: blocks, patterns (per position: sources at pool[po[p] ..], nx x
 * sources first), long blocks */
typedef struct {
    int nb;
    int *blk, *bstart, *islong; /* per position; per block (bstart[nb] = n) */
    long long *po;              /* per position: pattern offset, po[n] = total */
    int *nx;                    /* per position: x sources */
    int *pool;
} BlkPlan;
static void blk_plan(int n, const int *ord, const BlkDeps *d, const int *prm, BlkPlan *P) {
    const int bs = prm[0], ymax = prm[1], nmax = prm[2], nw = prm[3], ch = prm[4], lcap = prm[5];
    int *pos = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int p = 0; p < n; p++) pos[ord[p]] = p;
    /* chunk starts: cst[p] = the first position of p's chunk */
    int *cst = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int p = 0, c0 = 0; p < n; p++) {
        if (p - c0 == ch) c0 = p;
        else if (p > c0) {
            const int r = ord[p];
            int m = 0;
            for (int o = d->dp[r]; o < d->dp[r + 1]; o++) m += pos[d->dj[o]] >= c0;
            if (m > lcap) c0 = p;
        }
        cst[p] = c0;
    }
    int *stamp = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int p = 0; p < n; p++) stamp[p] = -1;
    P->blk = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    P->bstart = (int *)malloc(((size_t)n + 2) * sizeof(int));
    P->islong = (int *)calloc((size_t)n + 2, sizeof(int));
    P->po = (long long *)malloc(((size_t)n + 1) * sizeof(long long));
    P->nx = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    BlkVec pool = {0, 0, 0}, xs = {0, 0, 0}, ys = {0, 0, 0};
    int tag = 0, b = 0, bsize = 0, bst = 0, near = 0;
    /* the candidate pattern of position p in a block starting at s (s == p:
     * no block rows before p) */
#define BLK_CAND(S)                                                                         \
    do {                                                                                    \
        const int s_ = (S), lo_ = cst[p] > s_ - nw ? cst[p] : s_ - nw;                      \
        xs.n = ys.n = 0;                                                                    \
        near = 0;                                                                           \
        tag++;                                                                              \
        bv_push(&xs, p);                                                                    \
        stamp[p] = tag;                                                                     \
        for (int o = d->dp[r]; o < d->dp[r + 1]; o++) {                                     \
            const int q = pos[d->dj[o]];                                                    \
            if (q >= s_) {                                                                  \
                for (long long k = P->po[q]; k < P->po[q + 1]; k++) {                       \
                    const int u = pool.v[k];                                                \
                    if (stamp[u] == tag) continue;                                          \
                    stamp[u] = tag;                                                         \
                    bv_push(k - P->po[q] < P->nx[q] ? &xs : &ys, u);                        \
                }                                                                           \
            } else if (stamp[q] != tag) {                                                   \
                stamp[q] = tag;                                                             \
                bv_push(&ys, q);                                                            \
            }                                                                               \
        }                                                                                   \
        for (long long k = 0; k < ys.n; k++) near += ys.v[k] >= lo_;                        \
    } while (0)
    for (int p = 0; p < n; p++) {
        const int r = ord[p];
        int ok = 0;
        P->po[p] = pool.n; /* (the end of p - 1's pattern) */
        if (bsize > 0) {
            if (cst[p] != p) {
                BLK_CAND(bst);
                ok = bsize < bs && ys.n <= ymax && near <= nmax;
            }
            if (!ok) {
                P->bstart[b] = bst;
                b++;
                bsize = 0;
                bst = p;
            }
        }
        if (!ok) {
            BLK_CAND(p);
        }
        qsort(xs.v, (size_t)xs.n, sizeof(int), cmp_int);
        qsort(ys.v, (size_t)ys.n, sizeof(int), cmp_int);
        P->po[p] = pool.n;
        P->nx[p] = (int)xs.n;
        for (long long k = 0; k < xs.n; k++) bv_push(&pool, xs.v[k]);
        for (long long k = 0; k < ys.n; k++) bv_push(&pool, ys.v[k]);
        P->blk[p] = b;
        if (bsize == 0) bst = p;
        bsize++;
        if (!ok && (ys.n > ymax || near > nmax)) { /* a long row: a block of its own */
            P->islong[b] = 1;
            P->bstart[b] = bst;
            b++;
            bsize = 0;
            bst = p + 1;
        }
    }
#undef BLK_CAND
    if (bsize > 0) {
        P->bstart[b] = bst;
        b++;
    }
    P->po[n] = pool.n;
    P->bstart[b] = n;
    P->nb = b;
    P->pool = pool.v;
    free(xs.v);
    free(ys.v);
    free(stamp);
    free(pos);
    free(cst);
}
static void blk_free(BlkPlan *P, BlkDeps *d, int *ord) {
    free(P->blk);
    free(P->bstart);
    free(P->islong);
    free(P->po);
    free(P->nx);
    free(P->pool);
    free(d->dp);
    free(d->dj);
    free(d->dv);
    free(ord);
}
#define ORACLE_BLOCKS(T, SUF, FMA)                                                             \
    static int blocks_##SUF(int kind, int n, const int *rp, const int *ci, const T *v, T alpha, \
                            const T *x, T *y, const int *params) {                            \
        static const int dflt[6] = BLK_DEFAULTS;                                               \
        const int *prm = params ? params : dflt;                                               \
        if (n < 0 || kind < 0 || kind > 1 || prm[0] < 1 || prm[0] > 64 || prm[4] < 1) return -1; \
        if (n == 0) return 0;                                                                  \
        BlkDeps d;                                                                             \
        blk_deps(kind, n, rp, ci, &d);                                                         \
        int *ord = blk_order(kind, n, &d);                                                     \
        BlkPlan P;                                                                             \
        blk_plan(n, ord, &d, prm, &P);                                                         \
        int *pos = (int *)malloc((size_t)n * sizeof(int));                                     \
        for (int p = 0; p < n; p++) pos[ord[p]] = p;                                           \
        T *E = (T *)malloc((size_t)(P.po[n] > 0 ? P.po[n] : 1) * sizeof(T));                   \
        T *acc = (T *)calloc((size_t)n, sizeof(T));                                            \
        for (int p = 0; p < n; p++) { /* 5. coefficients */                                    \
            const int r = ord[p], s0 = P.bstart[P.blk[p]];                                     \
            for (long long k = P.po[p]; k < P.po[p + 1]; k++) acc[P.pool[k]] = (T)0;          \
            acc[p] = (T)1;                                                                     \
            for (int o = d.dp[r]; o < d.dp[r + 1]; o++) {                                      \
                const T l = v[d.dv[o]];                                                        \
                const int q = pos[d.dj[o]];                                                    \
                if (q >= s0)                                                                   \
                    for (long long k = P.po[q]; k < P.po[q + 1]; k++)                          \
                        acc[P.pool[k]] = FMA(-l, E[k], acc[P.pool[k]]);                        \
                else                                                                           \
                    acc[q] = FMA(-l, (T)1, acc[q]);                                            \
            }                                                                                  \
            for (long long k = P.po[p]; k < P.po[p + 1]; k++) E[k] = acc[P.pool[k]];          \
        }                                                                                      \
        T *yp = acc; /* 6. the solve (acc reused: positions' y) */                             \
        for (int p = 0; p < n; p++) {                                                          \
            const long long k0 = P.po[p], k1 = P.po[p + 1];                                    \
            T s = 0;                                                                           \
            if (!P.islong[P.blk[p]]) {                                                         \
                for (long long k = k0; k < k1; k++) {                                          \
                    const int u = P.pool[k];                                                   \
                    const T val = k - k0 < P.nx[p] ? (T)(alpha * x[ord[u]]) : yp[u];           \
                    s = FMA(E[k], val, s);                                                     \
                }                                                                              \
            } else {                                                                           \
                T part[64], tmp[64];                                                           \
                for (int l = 0; l < 64; l++) part[l] = 0;                                      \
                for (long long k = k0; k < k1; k++) {                                          \
                    const int u = P.pool[k];                                                   \
                    const T val = k - k0 < P.nx[p] ? (T)(alpha * x[ord[u]]) : yp[u];           \
                    part[(k - k0) & 63] = FMA(E[k], val, part[(k - k0) & 63]);                 \
                }                                                                              \
                for (int off = 32; off >= 1; off >>= 1) {                                      \
                    for (int l = 0; l < 64; l++) tmp[l] = part[l] + part[l ^ off];             \
                    memcpy(part, tmp, sizeof(part));                                           \
                }                                                                              \
                s = part[0];                                                                   \
            }                                                                                  \
            yp[p] = s;                                                                         \
        }                                                                                      \
        for (int p = 0; p < n; p++) y[ord[p]] = yp[p];                                         \
        const int nb = P.nb;                                                                   \
        free(E);                                                                               \
        free(acc);                                                                             \
        free(pos);                                                                             \
        blk_free(&P, &d, ord);                                                                 \
        return nb;                                                                             \
    }
ORACLE_BLOCKS(double, d, fma)
ORACLE_BLOCKS(float, s, fmaf)

int oracle_dag_levels(int kind, int n, const int *rp, const int *ci) {
    if (n <= 0 || kind < 0 || kind > 1) return 0;
    BlkDeps d;
    blk_deps(kind, n, rp, ci, &d);
    int *lv = (int *)malloc((size_t)n * sizeof(int)), nl = 0;
    for (int k = 0; k < n; k++) {
        int i = kind == 0 ? k : n - 1 - k, l = 0;
        for (int o = d.dp[i]; o < d.dp[i + 1]; o++)
            if (lv[d.dj[o]] + 1 > l) l = lv[d.dj[o]] + 1;
        lv[i] = l;
        if (l + 1 > nl) nl = l + 1;
    }
    free(lv);
    free(d.dp);
    free(d.dj);
    free(d.dv);
    return nl;
}

int oracle_trsv_blocks_f64(int kind, int n, const int *rp, const int *ci, const double *v, double alpha,
                           const double *x, double *y, const int *params) {
    return blocks_d(kind, n, rp, ci, v, alpha, x, y, params);
}
int oracle_trsv_blocks_f32(int kind, int n, const int *rp, const int *ci, const float *v, float alpha,
                           const float *x, float *y, const int *params, int ftz) {
    unsigned old = ftz_enter(ftz);
    const int r = blocks_s(kind, n, rp, ci, v, alpha, x, y, params);
    ftz_leave(old);
    return r;
}

void oracle_trsv_lower_n_split_f64(int n, const int *rp, const int *ci, const double *v, double alpha,
                                   const double *x, double *y) {
    lower_n_split_d(n, rp, ci, v, alpha, x, y);
}
void oracle_trsv_lower_n_split_f32(int n, const int *rp, const int *ci, const float *v, float alpha,
                                   const float *x, float *y, int ftz) {
    unsigned old = ftz_enter(ftz);
    lower_n_split_s(n, rp, ci, v, alpha, x, y);
    ftz_leave(old);
}
void oracle_trsv_lower_t_split_f64(int n, const int *rp, const int *ci, const double *v, double alpha,
                                   const double *x, double *y) {
    lower_t_split_d(n, rp, ci, v, alpha, x, y);
}
void oracle_trsv_lower_t_split_f32(int n, const int *rp, const int *ci, const float *v, float alpha,
                                   const float *x, float *y, int ftz) {
    unsigned old = ftz_enter(ftz);
    lower_t_split_s(n, rp, ci, v, alpha, x, y);
    ftz_leave(old);
}

void oracle_trsv_lower_n_f64(int n, const int *rp, const int *ci, const double *v, double alpha,
                             const double *x, double *y) {
    lower_n_d(n, rp, ci, v, alpha, x, y);
}
void oracle_trsv_lower_n_f32(int n, const int *rp, const int *ci, const float *v, float alpha,
                             const float *x, float *y, int ftz) {
    unsigned old = ftz_enter(ftz);
    lower_n_s(n, rp, ci, v, alpha, x, y);
    ftz_leave(old);
}
void oracle_trsv_lower_t_f64(int n, const int *rp, const int *ci, const double *v, double alpha,
                             const double *x, double *y) {
    lower_t_d(n, rp, ci, v, alpha, x, y);
}
void oracle_trsv_lower_t_f32(int n, const int *rp, const int *ci, const float *v, float alpha,
                             const float *x, float *y, int ftz) {
    unsigned old = ftz_enter(ftz);
    lower_t_s(n, rp, ci, v, alpha, x, y);
    ftz_leave(old);
}
void oracle_trsv_upper_f64(int n, const int *rp, const int *ci, const double *v, double alpha,
                           const double *x, double *y) {
    upper_d(n, rp, ci, v, alpha, x, y);
}
void oracle_trsv_upper_f32(int n, const int *rp, const int *ci, const float *v, float alpha,
                           const float *x, float *y, int ftz) {
    unsigned old = ftz_enter(ftz);
    upper_s(n, rp, ci, v, alpha, x, y);
    ftz_leave(old);
}

/* ---------------------------------------------------------------- dlarnv */

/* seed * mult mod 2^48 in 12-bit limbs, exactly as DLARUV's IT1..IT4 chain. */
static void limb_mul(const int s[4], const int mm[4], int out[4]) {
    const int P = 4096;
    int it4 = s[3] * mm[3];
    int it3 = it4 / P;
    it4 -= P * it3;
    it3 += s[2] * mm[3] + s[3] * mm[2];
    int it2 = it3 / P;
    it3 -= P * it2;
    it2 += s[1] * mm[3] + s[2] * mm[2] + s[3] * mm[1];
    int it1 = it2 / P;
    it2 -= P * it1;
    it1 += s[0] * mm[3] + s[1] * mm[2] + s[2] * mm[1] + s[3] * mm[0];
    it1 %= P;
    out[0] = it1;
    out[1] = it2;
    out[2] = it3;
    out[3] = it4;
}

int oracle_dlarnv(int idist, int *iseed, int n, double *x) {
    if (idist != 1 && idist != 2) return -1;
    static const int a1[4] = {494, 322, 2508, 2549}; /* DLARUV MM(1,:) */
    int mm[128][4];
    memcpy(mm[0], a1, sizeof(a1));
    for (int i = 1; i < 128; i++) limb_mul(mm[i - 1], a1, mm[i]);
    const double r = 1.0 / 4096.0;
    int seed[4] = {iseed[0], iseed[1], iseed[2], iseed[3]};
    for (int iv = 0; iv < n; iv += 64) { /* DLARNV: LV/2 = 64 per DLARUV call */
        int il = n - iv < 64 ? n - iv : 64;
        int last[4] = {seed[0], seed[1], seed[2], seed[3]};
        for (int i = 0; i < il; i++) {
            int it[4];
            limb_mul(seed, mm[i], it);
            double u = r * ((double)it[0] + r * ((double)it[1] + r * ((double)it[2] + r * (double)it[3])));
            x[iv + i] = idist == 1 ? u : 2.0 * u - 1.0;
            memcpy(last, it, sizeof(it));
        }
        memcpy(seed, last, sizeof(seed));
    }
    memcpy(iseed, seed, sizeof(seed));
    return 0;
}
