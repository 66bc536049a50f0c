/*
 * surrogate.c — seeded stand-ins for the 36 SuiteSparse matrices the
 * reference sweeps (GPU/run_spmv.sh:3-5, run_spmv.sh:3-40). No .mtx data is
 * present in the reference snapshot (matrices/ holds names + wget scripts only)
 * and there is no network, so every benchmark and most tests run on these
 * surrogates; a real file, when available, goes through the loader instead.
 *
 * Keyed by SURVEY Appendix A: same m, ~same stored nnz (nnz_s = rowptr[m];
 * symmetric matrices are stored as lower triangle + diagonal, which is what
 * the reference loader hands to every kernel), and a structural
 * family per matrix:
 *   stencil3d  — FEM/CFD: a 3-D grid, neighbours taken shell by shell
 *                (|d|^2 order) until the row length reaches the target, then
 *                a symmetric hash-drop trims to the exact expected count;
 *   stencil2d  — same on a 2-D grid (ecology2 = 5-point, ML_Laplace ~ 73);
 *   circuit    — power-law row lengths (density ~ x^-2 for 0.2% hub rows,
 *                capped at 5% of n), 70% of columns in a +-32 band, 30% far;
 *   randband   — uniform-ish row lengths, columns uniform in a wide band.
 * Values: off-diagonals uniform in [-1,1) from a counter hash of (i,j)
 * (of (min,max) for symmetric storage), diagonal = 1 + sum |off-diagonals of
 * the full row| (strict row diagonal dominance: an H-matrix, so ILU(0) has
 * non-zero pivots). Row i is a pure function of (name, scale, flags, i), so
 * any row range can be generated on its own (multi-GPU ranks build only
 * their slice) and the result is identical for every thread count.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rsp_host.h"

enum { FAM_S3D = 0, FAM_S2D = 1, FAM_CIRCUIT = 2, FAM_RANDBAND = 3 };

typedef struct {
    const char *name;
    int m;
    long long nnz_s; /* stored entries the reference kernels see */
    char sym;        /* 'S' symmetric storage (lower + diag), 'G' general */
    char set;        /* 0 moderate, 1 big */
    char family;
} surr_entry;

/* SURVEY Appendix A (sizes from public SuiteSparse metadata; approximate). */
static const surr_entry CATALOG[] = {
    {"2cubes_sphere", 101492, 874378, 'S', 0, FAM_S3D},
    {"ASIC_320ks", 321671, 1316085, 'G', 0, FAM_CIRCUIT},
    {"Baumann", 112211, 748331, 'G', 0, FAM_S3D},
    {"cfd2", 123440, 1604423, 'S', 0, FAM_S3D},
    {"crashbasis", 160000, 1750416, 'G', 0, FAM_S2D},
    {"ct20stif", 52329, 1326312, 'S', 0, FAM_S3D},
    {"dc1", 116835, 766396, 'G', 0, FAM_CIRCUIT},
    {"Dubcova3", 146689, 1891666, 'S', 0, FAM_S2D},
    {"ecology2", 999999, 2997995, 'S', 0, FAM_S2D},
    {"FEM_3D_thermal2", 147900, 3489300, 'G', 0, FAM_S3D},
    {"G2_circuit", 150102, 438388, 'S', 0, FAM_CIRCUIT},
    {"Goodwin_095", 100037, 3226066, 'G', 0, FAM_S3D},
    {"matrix-new_3", 125329, 893984, 'G', 0, FAM_CIRCUIT},
    {"offshore", 259789, 2251231, 'S', 0, FAM_S3D},
    {"para-10", 155924, 2094873, 'G', 0, FAM_RANDBAND},
    {"parabolic_fem", 525825, 2100225, 'S', 0, FAM_S2D},
    {"ss1", 205282, 845089, 'G', 0, FAM_CIRCUIT},
    {"stomach", 213360, 3021648, 'G', 0, FAM_S3D},
    {"thermomech_TK", 102158, 406858, 'S', 0, FAM_S2D},
    {"tmt_unsym", 917825, 4584801, 'G', 0, FAM_S2D},
    {"xenon2", 157464, 3866688, 'G', 0, FAM_S3D},
    {"af_shell10", 1508065, 26883975, 'S', 1, FAM_S3D},
    {"af_shell2", 504855, 9033453, 'S', 1, FAM_S3D},
    {"atmosmodd", 1270432, 8814880, 'G', 1, FAM_S3D},
    {"atmosmodl", 1489752, 10319760, 'G', 1, FAM_S3D},
    {"cage13", 445315, 7479343, 'G', 1, FAM_RANDBAND},
    {"CurlCurl_2", 806529, 4864159, 'S', 1, FAM_S3D},
    {"dielFilterV2real", 1157456, 24848204, 'S', 1, FAM_S3D},
    {"Geo_1438", 1437960, 30837141, 'S', 1, FAM_S3D},
    {"Hook_1498", 1498023, 30436237, 'S', 1, FAM_S3D},
    {"ML_Laplace", 377002, 27582698, 'G', 1, FAM_S2D},
    {"nlpkkt80", 1062400, 14352336, 'S', 1, FAM_S3D},
    {"Serena", 1391349, 32761660, 'S', 1, FAM_S3D},
    {"Si87H76", 240369, 5451000, 'S', 1, FAM_RANDBAND},
    {"StocF-1465", 1465137, 11235263, 'S', 1, FAM_S3D},
    {"Transport", 1602111, 23487281, 'G', 1, FAM_S3D},
};
#define NCAT ((int)(sizeof(CATALOG) / sizeof(CATALOG[0])))

int rsp_surrogate_count(void) { return NCAT; }

const char *rsp_surrogate_name(int i) { return (i >= 0 && i < NCAT) ? CATALOG[i].name : NULL; }

/* ------------------------------------------------------------- hashing */

static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint64_t h3(uint64_t seed, uint64_t a, uint64_t b) {
    return mix64(seed ^ mix64(a ^ mix64(b + 0x632BE59BD9B4E019ULL)));
}
static inline double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }
static inline double uval(uint64_t h) { return 2.0 * u01(h) - 1.0; }

static uint64_t fnv1a(const char *s) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (; *s; ++s) {
        h ^= (unsigned char)*s;
        h *= 0x100000001b3ULL;
    }
    return h;
}

/* ------------------------------------------------------------- context */

#define MAXOFF 512

typedef struct {
    int family, m, sym, flags;
    uint64_t seed_pat, seed_val, seed_len, seed_ftz;
    /* stencils */
    int nx, ny, nz, noff;
    int ox[MAXOFF], oy[MAXOFF], oz[MAXOFF];
    long long olin[MAXOFF]; /* sorted ascending */
    uint64_t drop_thresh;   /* off-diagonal (i,j) kept iff h >= drop_thresh */
    /* circuit / randband */
    double base;
    int cap, band, lmin;
    double hub_frac;
} gen_ctx;

static void calibrate_random(gen_ctx *c, double avg);

static int find_entry(const char *name) {
    for (int i = 0; i < NCAT; i++)
        if (strcmp(CATALOG[i].name, name) == 0) return i;
    return -1;
}

/* Custom spec "stencil3d:ROWS:NNZS:S" / "stencil2d:..." / "circuit:..." /
 * "randband:...". */
static int parse_custom(const char *name, surr_entry *e) {
    char fam[32];
    long long rows = 0, nnz = 0;
    char sym = 'G';
    if (sscanf(name, "%31[^:]:%lld:%lld:%c", fam, &rows, &nnz, &sym) != 4) return -1;
    if (rows <= 0 || nnz < rows || (sym != 'S' && sym != 'G')) return -1;
    if (strcmp(fam, "stencil3d") == 0)
        e->family = FAM_S3D;
    else if (strcmp(fam, "stencil2d") == 0)
        e->family = FAM_S2D;
    else if (strcmp(fam, "circuit") == 0)
        e->family = FAM_CIRCUIT;
    else if (strcmp(fam, "randband") == 0)
        e->family = FAM_RANDBAND;
    else
        return -1;
    e->name = name;
    e->m = (int)rows;
    e->nnz_s = nnz;
    e->sym = sym;
    e->set = 2;
    return 0;
}

static int lookup(const char *name, surr_entry *e) {
    int idx = find_entry(name);
    if (idx >= 0) {
        *e = CATALOG[idx];
        return 0;
    }
    return parse_custom(name, e);
}

int rsp_surrogate_info(const char *name, int *m, int64_t *nnz_target, int *symmetric, int *set,
                       int *family) {
    surr_entry e;
    if (!name || lookup(name, &e) != 0) return -1;
    if (m) *m = e.m;
    if (nnz_target) *nnz_target = e.nnz_s;
    if (symmetric) *symmetric = e.sym == 'S';
    if (set) *set = e.set;
    if (family) *family = e.family;
    return 0;
}

static int scaled_rows(const surr_entry *e, double scale) {
    if (!(scale > 0.0) || scale >= 1.0) return e->m;
    double r = floor((double)e->m * scale + 0.5);
    if (r < 64) r = 64;
    if (r > e->m) r = e->m;
    return (int)r;
}

/* Number of grid points i < m whose neighbour at offset (dx,dy,dz) is in the
 * grid and has linear index < m. */
static long long offset_count(const gen_ctx *c, int dx, int dy, int dz) {
    long long off = (long long)dx + (long long)c->nx * (dy + (long long)c->ny * dz);
    long long total = 0;
    int x0 = dx < 0 ? -dx : 0, x1 = dx > 0 ? c->nx - dx : c->nx;
    if (x1 <= x0) return 0;
    for (int z = 0; z < c->nz; z++) {
        if (z + dz < 0 || z + dz >= c->nz) continue;
        for (int y = 0; y < c->ny; y++) {
            if (y + dy < 0 || y + dy >= c->ny) continue;
            long long rowbase = (long long)c->nx * (y + (long long)c->ny * z);
            long long hi = x1;
            long long lim = (long long)c->m - rowbase; /* x < lim       */
            if (lim < hi) hi = lim;
            long long lim2 = (long long)c->m - rowbase - off; /* x + off < m */
            if (lim2 < hi) hi = lim2;
            if (hi > x0) total += hi - x0;
        }
    }
    return total;
}

typedef struct {
    int dx, dy, dz;
    long long d2;
} pair_t;

static int cmp_pair(const void *a, const void *b) {
    const pair_t *p = (const pair_t *)a, *q = (const pair_t *)b;
    if (p->d2 != q->d2) return p->d2 < q->d2 ? -1 : 1;
    if (p->dz != q->dz) return p->dz < q->dz ? -1 : 1;
    if (p->dy != q->dy) return p->dy < q->dy ? -1 : 1;
    return (p->dx > q->dx) - (p->dx < q->dx);
}

static int cmp_ll(const void *a, const void *b) {
    long long x = *(const long long *)a, y = *(const long long *)b;
    return (x > y) - (x < y);
}

static int setup_stencil(gen_ctx *c, long long target_s, int dim) {
    int m = c->m;
    if (dim == 3) {
        int s = (int)ceil(cbrt((double)m));
        c->nx = s;
        c->ny = s;
        c->nz = (int)((m + (long long)s * s - 1) / ((long long)s * s));
    } else {
        int s = (int)ceil(sqrt((double)m));
        c->nx = s;
        c->ny = (m + s - 1) / s;
        c->nz = 1;
    }
    int R = dim == 3 ? 3 : 6;
    /* canonical representatives of +-d pairs (first non-zero of dz,dy,dx > 0) */
    pair_t pairs[MAXOFF];
    int np = 0;
    for (int dz = (dim == 3 ? -R : 0); dz <= (dim == 3 ? R : 0); dz++)
        for (int dy = -R; dy <= R; dy++)
            for (int dx = -R; dx <= R; dx++) {
                int canon = dz > 0 || (dz == 0 && (dy > 0 || (dy == 0 && dx > 0)));
                if (!canon) continue;
                pairs[np].dx = dx;
                pairs[np].dy = dy;
                pairs[np].dz = dz;
                pairs[np].d2 = (long long)dx * dx + (long long)dy * dy + (long long)dz * dz;
                np++;
            }
    qsort(pairs, (size_t)np, sizeof(pair_t), cmp_pair);
    /* stored count with no drop = m + sum over chosen pairs of
     * count(+d) [+ count(-d) for general storage]. */
    long long need = target_s - m;
    long long have = 0;
    int chosen = 0;
    while (chosen < np && have < need) {
        pair_t *p = &pairs[chosen];
        long long cp = offset_count(c, p->dx, p->dy, p->dz);
        long long cn = offset_count(c, -p->dx, -p->dy, -p->dz);
        have += c->sym ? cn : (cp + cn);
        chosen++;
    }
    if (chosen == 0) chosen = 1, have = 1; /* always at least a 3-point stencil */
    double keep = (need <= 0) ? 0.0 : (double)need / (double)have;
    if (keep > 1.0) keep = 1.0;
    double drop = 1.0 - keep;
    c->drop_thresh = drop <= 0.0 ? 0 : (uint64_t)(drop * 18446744073709551615.0);
    /* offsets: centre + both signs of the chosen pairs, sorted by linear off */
    int no = 0;
    c->ox[no] = c->oy[no] = c->oz[no] = 0;
    no++;
    for (int k = 0; k < chosen; k++) {
        for (int sgn = -1; sgn <= 1; sgn += 2) {
            c->ox[no] = sgn * pairs[k].dx;
            c->oy[no] = sgn * pairs[k].dy;
            c->oz[no] = sgn * pairs[k].dz;
            no++;
        }
    }
    c->noff = no;
    /* sort all arrays by linear offset */
    long long key[MAXOFF];
    for (int k = 0; k < no; k++) {
        long long lin = (long long)c->ox[k] + (long long)c->nx * (c->oy[k] + (long long)c->ny * c->oz[k]);
        key[k] = lin * (1LL << 20) + k; /* = (lin << 20) | k without shifting a negative; |lin| < 2^42 */
    }
    qsort(key, (size_t)no, sizeof(long long), cmp_ll);
    int tx[MAXOFF], ty[MAXOFF], tz[MAXOFF];
    for (int k = 0; k < no; k++) {
        int src = (int)(key[k] & 0xFFFFF);
        tx[k] = c->ox[src];
        ty[k] = c->oy[src];
        tz[k] = c->oz[src];
    }
    for (int k = 0; k < no; k++) {
        c->ox[k] = tx[k];
        c->oy[k] = ty[k];
        c->oz[k] = tz[k];
        c->olin[k] = (long long)tx[k] + (long long)c->nx * (ty[k] + (long long)c->ny * tz[k]);
    }
    return 0;
}

static int setup(const char *name, double scale, int flags, gen_ctx *c) {
    surr_entry e;
    if (!name || lookup(name, &e) != 0) return -1;
    memset(c, 0, sizeof(*c));
    c->family = e.family;
    c->m = scaled_rows(&e, scale);
    c->sym = e.sym == 'S';
    c->flags = flags;
    uint64_t s = fnv1a(name);
    c->seed_pat = mix64(s ^ 0x1111);
    c->seed_val = mix64(s ^ 0x2222);
    c->seed_len = mix64(s ^ 0x3333);
    c->seed_ftz = mix64(s ^ 0x4444);
    double avg = (double)e.nnz_s / (double)e.m; /* stored per row */
    long long target = (long long)llround(avg * c->m);
    if (target < c->m) target = c->m;
    switch (e.family) {
        case FAM_S3D:
            return setup_stencil(c, target, 3);
        case FAM_S2D:
            return setup_stencil(c, target, 2);
        case FAM_CIRCUIT: {
            c->band = 32;
            c->cap = (int)(0.05 * c->m);
            if (c->cap < 8) c->cap = 8;
            c->hub_frac = 0.002;
            c->lmin = (int)ceil(4.0 * avg);
            if (c->lmin > c->cap) c->lmin = c->cap;
            double ehub = c->lmin * (1.0 + log((double)c->cap / c->lmin));
            double reg = (avg - c->hub_frac * ehub) / (1.0 - c->hub_frac);
            if (reg < 1.0) reg = 1.0;
            c->base = reg;
            calibrate_random(c, avg);
            return 0;
        }
        case FAM_RANDBAND: {
            c->band = c->m / 32;
            if (c->band < 128) c->band = 128;
            c->base = avg;
            c->cap = c->m;
            calibrate_random(c, avg);
            return 0;
        }
    }
    return -1;
}

static int row_length_random(const gen_ctx *c, int i);

/* Random families: nudge `base` until the mean row length of an evenly
 * spaced sample of rows matches the target (deterministic, so row i stays a
 * pure function of the spec). */
static void calibrate_random(gen_ctx *c, double avg) {
    const int samples = c->m < 2000000 ? c->m : 2000000;
    const double stride = (double)c->m / samples;
    for (int iter = 0; iter < 8; iter++) {
        double sum = 0.0;
        for (int s = 0; s < samples; s++) sum += row_length_random(c, (int)(s * stride));
        double mean = sum / samples;
        if (mean <= 0.0) return;
        double gap = avg - mean;
        if (fabs(gap) < 1e-4 * avg) return;
        double reg_share = c->family == FAM_CIRCUIT ? (1.0 - c->hub_frac) : 1.0;
        c->base += gap / reg_share;
        if (c->base < 1.0) c->base = 1.0;
    }
}

int rsp_surrogate_rows(const char *name, double scale, int *m) {
    surr_entry e;
    if (!name || !m || lookup(name, &e) != 0) return -1;
    *m = scaled_rows(&e, scale);
    return 0;
}

/* -------------------------------------------------------- stencil rows */

static inline int stencil_nbr(const gen_ctx *c, int i, int k, int x, int y, int z) {
    int xx = x + c->ox[k], yy = y + c->oy[k], zz = z + c->oz[k];
    if (xx < 0 || xx >= c->nx || yy < 0 || yy >= c->ny || zz < 0 || zz >= c->nz) return -1;
    long long j = (long long)i + c->olin[k];
    if (j < 0 || j >= c->m) return -1;
    return (int)j;
}

static inline int stencil_keep(const gen_ctx *c, int i, int j) {
    if (i == j || c->drop_thresh == 0) return 1;
    int a = i < j ? i : j, b = i < j ? j : i;
    return h3(c->seed_pat, (uint64_t)a, (uint64_t)b) >= c->drop_thresh;
}

static inline double offdiag_value(const gen_ctx *c, int i, int j) {
    int a = i, b = j;
    if (c->sym && a > b) {
        a = j;
        b = i;
    }
    double v = uval(h3(c->seed_val, (uint64_t)a, (uint64_t)b));
    if ((c->flags & RSP_SURR_FTZ_STRESS) && u01(h3(c->seed_ftz, (uint64_t)a, (uint64_t)b)) < 0.01)
        v *= 1e-40;
    return v;
}

/* Row i of a stencil surrogate. Returns the stored length; when cols/vals
 * are non-NULL writes the sorted stored entries. */
static int stencil_row(const gen_ctx *c, int i, int *cols, double *vals) {
    int x = i % c->nx;
    int y = (i / c->nx) % c->ny;
    int z = (int)(i / ((long long)c->nx * c->ny));
    int len = 0;
    double diag_sum = 1.0;
    int diag_slot = -1;
    for (int k = 0; k < c->noff; k++) {
        int j = stencil_nbr(c, i, k, x, y, z);
        if (j < 0 || !stencil_keep(c, i, j)) continue;
        int stored = !c->sym || j <= i;
        if (j == i) {
            if (cols) {
                diag_slot = len;
                cols[len] = j;
            }
            len++;
            continue;
        }
        if (vals) {
            double v = offdiag_value(c, i, j);
            diag_sum += fabs(v);
            if (stored) vals[len] = v;
        }
        if (stored) {
            if (cols) cols[len] = j;
            len++;
        }
    }
    if (vals && diag_slot >= 0) vals[diag_slot] = diag_sum;
    return len;
}

/* ------------------------------------------------ circuit / randband rows */

static int row_length_random(const gen_ctx *c, int i) {
    double u = u01(h3(c->seed_len, (uint64_t)i, 1));
    int len;
    if (c->family == FAM_CIRCUIT) {
        double uh = u01(h3(c->seed_len, (uint64_t)i, 2));
        if (uh < c->hub_frac) {
            double v = u < 1e-12 ? 1e-12 : u;
            double l = c->lmin / v;
            len = l > c->cap ? c->cap : (int)l;
        } else {
            /* 1 + uniform on [0, 2(base-1)], rounded: mean ~ base */
            len = 1 + (int)floor(u * 2.0 * (c->base - 1.0) + 0.5);
        }
    } else {
        /* uniform on [base/2, 3base/2], rounded: mean ~ base */
        len = (int)floor(0.5 * c->base + u * c->base + 0.5);
    }
    if (len < 1) len = 1;
    int maxlen = c->sym ? i + 1 : c->m;
    if (len > maxlen) len = maxlen;
    return len;
}

static int cmp_int_asc(const void *a, const void *b) {
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

static int uniq_sorted(int *a, int n) {
    if (n == 0) return 0;
    int w = 1;
    for (int r = 1; r < n; r++)
        if (a[r] != a[w - 1]) a[w++] = a[r];
    return w;
}

/* Columns of row i (sorted, unique, includes i). scratch holds >= 2*len. */
static int random_row(const gen_ctx *c, int i, int *cols, double *vals, int *scratch) {
    int len = row_length_random(c, i);
    int need = len - 1; /* off-diagonals */
    int have = 0;
    uint64_t t = 0;
    int hi = c->sym ? i : c->m; /* candidates in [0, hi) \ {i} */
    while (have < need) {
        int batch = need - have;
        for (int b = 0; b < batch; b++, t++) {
            uint64_t h = h3(c->seed_pat, (uint64_t)i, t);
            long long j;
            if (c->family == FAM_CIRCUIT && (h & 0xff) >= 77) { /* ~70% band */
                long long off = (long long)((h >> 8) % (uint64_t)c->band) + 1;
                j = c->sym ? i - off : ((h >> 40) & 1 ? i + off : i - off);
            } else if (c->family == FAM_RANDBAND) {
                long long off = (long long)((h >> 8) % (uint64_t)c->band) + 1;
                j = c->sym ? i - off : ((h >> 40) & 1 ? i + off : i - off);
            } else {
                j = (long long)((h >> 8) % (uint64_t)(hi > 0 ? hi : 1));
            }
            if (j < 0 || j >= hi || j == i) {
                b--; /* redraw with the next counter */
                if (t > (uint64_t)64 * (uint64_t)(need + 16) * 8ULL) goto done;
                continue;
            }
            scratch[have + b] = (int)j;
        }
        have += batch;
        qsort(scratch, (size_t)have, sizeof(int), cmp_int_asc);
        have = uniq_sorted(scratch, have);
        if (t > (uint64_t)64 * (uint64_t)(need + 16) * 8ULL) break;
    }
done:
    if (have > need) have = need;
    /* merge diagonal */
    int len_out = 0;
    double diag_sum = 1.0;
    int placed = 0, diag_slot = 0;
    for (int k = 0; k <= have; k++) {
        if (!placed && (k == have || scratch[k] > i)) {
            diag_slot = len_out;
            if (cols) cols[len_out] = i;
            len_out++;
            placed = 1;
        }
        if (k == have) break;
        int j = scratch[k];
        if (cols) cols[len_out] = j;
        if (vals) {
            double v = offdiag_value(c, i, j);
            vals[len_out] = v;
            diag_sum += fabs(v);
        }
        len_out++;
    }
    if (vals) vals[diag_slot] = diag_sum;
    return len_out;
}

static int row_scratch_size(const gen_ctx *c) {
    if (c->family == FAM_S3D || c->family == FAM_S2D) return 1;
    int cap = c->family == FAM_CIRCUIT ? c->cap : (int)(c->base * 2 + 8);
    if (cap > c->m) cap = c->m;
    return 2 * cap + 64;
}

static int gen_row(const gen_ctx *c, int i, int *cols, double *vals, int *scratch) {
    if (c->family == FAM_S3D || c->family == FAM_S2D) return stencil_row(c, i, cols, vals);
    return random_row(c, i, cols, vals, scratch);
}

int rsp_surrogate_rowlens(const char *name, double scale, int flags, int r0, int r1, int *rowlen) {
    gen_ctx c;
    if (setup(name, scale, flags, &c) != 0) return -1;
    if (r0 < 0 || r1 > c.m || r0 > r1 || !rowlen) return -1;
    int ss = row_scratch_size(&c);
    int err = 0;
#pragma omp parallel
    {
        int *scratch = (int *)malloc((size_t)ss * sizeof(int));
        if (!scratch) {
#pragma omp atomic write
            err = 1;
        } else {
#pragma omp for schedule(dynamic, 1024)
            for (int i = r0; i < r1; i++) {
                if (c.family == FAM_S3D || c.family == FAM_S2D)
                    rowlen[i - r0] = stencil_row(&c, i, NULL, NULL);
                else
                    rowlen[i - r0] = random_row(&c, i, NULL, NULL, scratch);
            }
            free(scratch);
        }
    }
    return err ? -1 : 0;
}

int rsp_surrogate_fill(const char *name, double scale, int flags, int r0, int r1, int *rowptr_local,
                       int *colidx, double *values) {
    gen_ctx c;
    if (setup(name, scale, flags, &c) != 0) return -1;
    if (r0 < 0 || r1 > c.m || r0 > r1 || !rowptr_local || !colidx || !values) return -1;
    int n = r1 - r0;
    if (rsp_surrogate_rowlens(name, scale, flags, r0, r1, rowptr_local + 1) != 0) return -1;
    rowptr_local[0] = 0;
    for (int i = 0; i < n; i++) rowptr_local[i + 1] += rowptr_local[i];
    int ss = row_scratch_size(&c);
    int err = 0;
#pragma omp parallel
    {
        int *scratch = (int *)malloc((size_t)ss * sizeof(int));
        if (!scratch) {
#pragma omp atomic write
            err = 1;
        } else {
#pragma omp for schedule(dynamic, 1024)
            for (int i = r0; i < r1; i++) {
                int off = rowptr_local[i - r0];
                int len = gen_row(&c, i, colidx + off, values + off, scratch);
                if (len != rowptr_local[i - r0 + 1] - off) {
#pragma omp atomic write
                    err = 1;
                }
            }
            free(scratch);
        }
    }
    return err ? -1 : 0;
}

int rsp_surrogate_csr(const char *name, double scale, int flags, CSR *A) {
    int m;
    memset(A, 0, sizeof(*A));
    if (rsp_surrogate_rows(name, scale, &m) != 0) return -1;
    int *rp = NULL;
    if (posix_memalign((void **)&rp, 64, ((size_t)m + 1) * sizeof(int)) != 0) return -1;
    if (rsp_surrogate_rowlens(name, scale, flags, 0, m, rp + 1) != 0) {
        free(rp);
        return -1;
    }
    rp[0] = 0;
    long long total = 0;
    for (int i = 0; i < m; i++) {
        total += rp[i + 1];
        if (total > 2147483647LL) {
            free(rp);
            return -1;
        }
        rp[i + 1] = (int)total;
    }
    int *ci = NULL;
    double *va = NULL;
    if (posix_memalign((void **)&ci, 64, (size_t)(total ? total : 1) * sizeof(int)) != 0 ||
        posix_memalign((void **)&va, 64, (size_t)(total ? total : 1) * sizeof(double)) != 0) {
        free(rp);
        free(ci);
        return -1;
    }
    if (rsp_surrogate_fill(name, scale, flags, 0, m, rp, ci, va) != 0) {
        free(rp);
        free(ci);
        free(va);
        return -1;
    }
    surr_entry e;
    lookup(name, &e);
    A->isSymmetric = e.sym == 'S';
    A->m = m;
    A->n = m;
    A->nnz = (int)total;
    A->rowptr = rp;
    A->colidx = ci;
    A->values = va;
    return 0;
}
