/*
 * mm_loader.c — Matrix-Market -> CSR/COO loader with the exact semantics of
 * ReSpaSol's ReadMatrixMarket library (the input side of the drop-in
 * boundary).
 *
 * Reference behaviour restated here (file:line in /root/reference):
 *   banner parse, lower-casing, type checks     ReadMatrixMarket/mm_io.cpp:54-158
 *   mm_is_valid                                 ReadMatrixMarket/mm_io.cpp:11-52
 *   size line (comment skip, sscanf/fscanf)     ReadMatrixMarket/mm_io.cpp:404-468
 *   entry parse ("%d %d %lg\n", pattern,
 *     integer via %lld, complex -> real part)   ReadMatrixMarket/mm_io.cpp:357-401
 *   open failure -> exit(-1)                    ReadMatrixMarket/loadMatrixMarket.cpp:49-53
 *   range check x > m || y > n                  loadMatrixMarket.cpp:126-130
 *   pattern -> 1.0, 0-based auto-detect         loadMatrixMarket.cpp:134-135,144-154
 *   lines != nnz -> failure                     loadMatrixMarket.cpp:156-160
 *   symmetric mirror count (binary_search in
 *     the sorted stored row)                    loadMatrixMarket.cpp:162-200
 *   COO->CSR over the HEADER nnz only, so the
 *     mirrored entries never reach the CSR      loadMatrixMarket.cpp:216-235
 *   per-row co-sort by column (qsort)           loadMatrixMarket.cpp:5-26,237-242
 *   matrix->nnz = expanded count                loadMatrixMarket.cpp:244-246
 *
 * Differences by design (documented in DESIGN.md): the whole file is read
 * into memory and parsed with strtol/strtod (the conversions scanf's %d/%lg
 * perform) instead of one fscanf per entry; rowptr is allocated m+1 (the
 * reference allocates `count`, loadMatrixMarket.cpp:206, which is short when
 * count < m+1); the value/index tails past rowptr[m] are zero-filled rather
 * than uninitialised. 0-based symmetric files: the reference's mirror count
 * reads uninitialised scratch (rowcnt[0] is never reset after the base shift,
 * loadMatrixMarket.cpp:149-153,166-168); here A.nnz is the well-defined count.
 */
#include <ctype.h>
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rsp_host.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#define MM_LINE_MAX 1025 /* MM_MAX_LINE_LENGTH, mm_io.h:12 */
#define MM_TOKEN_MAX 64  /* MM_MAX_TOKEN_LENGTH, mm_io.h:14 */

typedef struct {
    char object;   /* 'M' */
    char layout;   /* 'C' coordinate / 'A' array */
    char field;    /* 'R' real, 'C' complex, 'P' pattern, 'I' integer */
    char symmetry; /* 'G', 'S', 'H', 'K' */
} mm_code;

static void *aligned_alloc64(size_t bytes) {
    void *p = NULL;
    if (bytes == 0) bytes = 64;
    if (posix_memalign(&p, 64, bytes) != 0) return NULL;
    return p;
}

/* ------------------------------------------------------------- cursor */

typedef struct {
    const char *p;
    const char *end;
} cursor;

/* fgets(line, MM_LINE_MAX, f): copy up to MM_LINE_MAX-1 chars, stopping
 * after a newline. Returns 0 at EOF (nothing read). */
static int cur_fgets(cursor *c, char *line) {
    if (c->p >= c->end) return 0;
    size_t n = 0;
    while (c->p < c->end && n < MM_LINE_MAX - 1) {
        char ch = *c->p++;
        line[n++] = ch;
        if (ch == '\n') break;
    }
    line[n] = '\0';
    return 1;
}

static void cur_skip_ws(cursor *c) {
    while (c->p < c->end && isspace((unsigned char)*c->p)) c->p++;
}

/* scanf "%d" / "%lld": skip white space, then an optional sign and decimal
 * digits (strtol semantics). Returns 1 on success, 0 on a matching failure,
 * -1 at end of input. */
static int cur_int(cursor *c, long long *out) {
    cur_skip_ws(c);
    if (c->p >= c->end) return -1;
    const char *s = c->p;
    const char *q = s;
    if (q < c->end && (*q == '+' || *q == '-')) q++;
    if (q >= c->end || !isdigit((unsigned char)*q)) return 0;
    long long v = 0;
    int neg = (*s == '-');
    while (q < c->end && isdigit((unsigned char)*q)) {
        v = v * 10 + (*q - '0');
        q++;
    }
    *out = neg ? -v : v;
    c->p = q;
    return 1;
}

/* scanf "%lg": strtod on the token. The token (up to white space or `end`)
 * is copied into a NUL-terminated scratch first: rsp_mm_load_buffer does not
 * require its input to be terminated, and strtod must not read past `end`. */
static int cur_double(cursor *c, double *out) {
    cur_skip_ws(c);
    if (c->p >= c->end) return -1;
    const char *q = c->p;
    while (q < c->end && !isspace((unsigned char)*q)) q++;
    const size_t len = (size_t)(q - c->p);
    char small[256];
    char *tok = len < sizeof(small) ? small : (char *)malloc(len + 1);
    if (!tok) return 0;
    memcpy(tok, c->p, len);
    tok[len] = '\0';
    char *stop = NULL;
    double v = strtod(tok, &stop);
    const size_t used = (size_t)(stop - tok);
    if (tok != small) free(tok);
    if (used == 0) return 0;
    *out = v;
    c->p += used;
    return 1;
}

/* ------------------------------------------------------------- banner */

static void lower(char *s) {
    for (; *s; ++s) *s = (char)tolower((unsigned char)*s);
}

static int parse_banner(cursor *c, mm_code *code) {
    char line[MM_LINE_MAX];
    char banner[MM_LINE_MAX], mtx[MM_LINE_MAX], crd[MM_LINE_MAX], dtype[MM_LINE_MAX],
        storage[MM_LINE_MAX];
    code->object = ' ';
    code->layout = ' ';
    code->field = ' ';
    code->symmetry = 'G';
    if (!cur_fgets(c, line)) return -1;
    if (sscanf(line, "%1024s %1024s %1024s %1024s %1024s", banner, mtx, crd, dtype, storage) != 5)
        return -1;
    lower(mtx);
    lower(crd);
    lower(dtype);
    lower(storage);
    if (strncmp(banner, "%%MatrixMarket", strlen("%%MatrixMarket")) != 0) return -1;
    if (strcmp(mtx, "matrix") != 0) return -1;
    code->object = 'M';
    if (strcmp(crd, "coordinate") == 0)
        code->layout = 'C';
    else if (strcmp(crd, "array") == 0)
        code->layout = 'A';
    else
        return -1;
    if (strcmp(dtype, "real") == 0)
        code->field = 'R';
    else if (strcmp(dtype, "complex") == 0)
        code->field = 'C';
    else if (strcmp(dtype, "pattern") == 0)
        code->field = 'P';
    else if (strcmp(dtype, "integer") == 0)
        code->field = 'I';
    else
        return -1;
    if (strcmp(storage, "general") == 0)
        code->symmetry = 'G';
    else if (strcmp(storage, "symmetric") == 0)
        code->symmetry = 'S';
    else if (strcmp(storage, "hermitian") == 0)
        code->symmetry = 'H';
    else if (strcmp(storage, "skew-symmetric") == 0)
        code->symmetry = 'K';
    else
        return -1;
    return 0;
}

/* mm_is_valid (mm_io.cpp:11-52). */
static int code_valid(const mm_code *k) {
    if (k->object != 'M') return 0;
    if (k->layout == 'A' && k->field == 'P') return 0;
    if (k->field == 'R' && k->symmetry == 'H') return 0;
    if (k->field == 'P' && (k->symmetry == 'H' || k->symmetry == 'K')) return 0;
    return 1;
}

/* mm_read_mtx_crd_size (mm_io.cpp:404-468). */
static int parse_size(cursor *c, int *m, int *n, int *nz) {
    char line[MM_LINE_MAX];
    *m = *n = *nz = 0;
    do {
        if (!cur_fgets(c, line)) return -1;
    } while (line[0] == '%');
    if (sscanf(line, "%d %d %d", m, n, nz) == 3) return 0;
    /* fscanf(f, "%d %d %d") retried until three items are read. */
    long long a, b, d;
    if (cur_int(c, &a) != 1 || cur_int(c, &b) != 1 || cur_int(c, &d) != 1) return -1;
    *m = (int)a;
    *n = (int)b;
    *nz = (int)d;
    return 0;
}

/* mm_read_mtx_crd_entry (mm_io.cpp:357-401). Returns 1 on an entry. */
static int parse_entry(cursor *c, const mm_code *k, int *x, int *y, double *val) {
    long long a, b;
    if (cur_int(c, &a) != 1) return 0;
    if (cur_int(c, &b) != 1) return 0;
    *x = (int)a;
    *y = (int)b;
    if (k->field == 'P') {
        *val = 0.0;
        return 1;
    }
    if (k->field == 'I') {
        long long v;
        if (cur_int(c, &v) != 1) return 0;
        *val = (double)v;
        return 1;
    }
    double re;
    if (cur_double(c, &re) != 1) return 0;
    if (k->field == 'C') {
        double im;
        if (cur_double(c, &im) != 1) return 0;
    }
    *val = re;
    return 1;
}

/* --------------------------------------------------------------- sort */

/* loadMatrixMarket.cpp:5-26: quicksort of idx[left..right] carrying w,
 * pivot = middle element swapped to `left`, Lomuto partition on strict <.
 * The smaller side recurses and the larger side loops, which visits the same
 * disjoint sub-ranges with the same partitions, so the resulting order
 * (including the order of duplicate columns) is identical. */
void rsp_row_qsort(int *idx, double *w, int left, int right) {
    while (left < right) {
        int mid = left + (right - left) / 2;
        int ti = idx[left];
        idx[left] = idx[mid];
        idx[mid] = ti;
        double tw = w[left];
        w[left] = w[mid];
        w[mid] = tw;
        int last = left;
        for (int i = left + 1; i <= right; i++) {
            if (idx[i] < idx[left]) {
                ++last;
                ti = idx[last];
                idx[last] = idx[i];
                idx[i] = ti;
                tw = w[last];
                w[last] = w[i];
                w[i] = tw;
            }
        }
        ti = idx[left];
        idx[left] = idx[last];
        idx[last] = ti;
        tw = w[left];
        w[left] = w[last];
        w[last] = tw;
        if (last - left < right - last) {
            rsp_row_qsort(idx, w, left, last - 1);
            left = last + 1;
        } else {
            rsp_row_qsort(idx, w, last + 1, right);
            right = last - 1;
        }
    }
}

static int cmp_int(const void *a, const void *b) {
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

/* std::binary_search over a sorted [lo, hi) range. */
static int contains_sorted(const int *a, int lo, int hi, int key) {
    int l = lo, h = hi;
    while (l < h) {
        int mid = l + (h - l) / 2;
        if (a[mid] < key)
            l = mid + 1;
        else
            h = mid;
    }
    return l < hi && a[l] == key;
}

/* ------------------------------------------------------------- loader */

typedef struct {
    int m, n, nnz_header, symmetric, lines;
    int *row; /* 1-based after base fix-up */
    int *col;
    double *val;
    size_t cap;
} coo_tmp;

static void coo_tmp_free(coo_tmp *t) {
    free(t->row);
    free(t->col);
    free(t->val);
    t->row = t->col = NULL;
    t->val = NULL;
}

/* Parallel entry parse (the reference's fscanf loop is the
 * sweep's bottleneck). The entry text is cut at newlines into one piece per
 * thread; each piece is parsed with the same token rules (parse_entry). It is
 * accepted only if every piece parses to its end — then no entry straddles a
 * cut (a cut at a newline never splits a token, and a piece ending inside an
 * entry would fail), so the concatenated entries are exactly the sequential
 * parse's. Any failure (malformed text, a cut inside an entry) returns -1 and
 * the caller parses sequentially, which reproduces the reference's error
 * behaviour. Returns the entry count; the arrays are malloc'ed into px, py, pv. */
#define MM_PAR_MIN_BYTES (8u << 20)

static long parse_entries_parallel(const char *p, const char *end, const mm_code *k, int **px,
                                   int **py, double **pv) {
    int nt = 1;
#ifdef _OPENMP
    nt = omp_get_max_threads();
#endif
    if (nt < 2 || (size_t)(end - p) < MM_PAR_MIN_BYTES) return -1;
    if (nt > 256) nt = 256;
    const char *cut[257];
    cut[0] = p;
    for (int t = 1; t < nt; t++) {
        const char *q = p + (size_t)(end - p) * (size_t)t / (size_t)nt;
        if (q < cut[t - 1]) q = cut[t - 1];
        while (q < end && *q != '\n') q++;
        cut[t] = q < end ? q + 1 : end;
    }
    cut[nt] = end;
    long cnt[256];
    int *bx[256];
    int *by[256];
    double *bv[256];
    int ok = 1;
#pragma omp parallel for num_threads(nt) schedule(static, 1) reduction(&& : ok)
    for (int t = 0; t < nt; t++) {
        cursor c = {cut[t], cut[t + 1]};
        size_t cap = (size_t)(cut[t + 1] - cut[t]) / 4 + 16; /* an entry takes >= 4 bytes */
        bx[t] = (int *)malloc(cap * sizeof(int));
        by[t] = (int *)malloc(cap * sizeof(int));
        bv[t] = (double *)malloc(cap * sizeof(double));
        cnt[t] = 0;
        if (!bx[t] || !by[t] || !bv[t]) {
            ok = 0;
            continue;
        }
        int x, y;
        double v;
        while ((size_t)cnt[t] < cap && parse_entry(&c, k, &x, &y, &v)) {
            bx[t][cnt[t]] = x;
            by[t][cnt[t]] = y;
            bv[t][cnt[t]] = v;
            cnt[t]++;
        }
        cur_skip_ws(&c);
        if (c.p < c.end) ok = 0; /* stopped early: malformed or a straddling entry */
    }
    long total = 0;
    for (int t = 0; t < nt; t++) total += cnt[t];
    int *X = NULL, *Y = NULL;
    double *V = NULL;
    if (ok) {
        X = (int *)malloc((total ? total : 1) * sizeof(int));
        Y = (int *)malloc((total ? total : 1) * sizeof(int));
        V = (double *)malloc((total ? total : 1) * sizeof(double));
        ok = X && Y && V;
    }
    if (ok) {
        long off[257];
        off[0] = 0;
        for (int t = 0; t < nt; t++) off[t + 1] = off[t] + cnt[t];
#pragma omp parallel for num_threads(nt) schedule(static, 1)
        for (int t = 0; t < nt; t++) {
            memcpy(X + off[t], bx[t], (size_t)cnt[t] * sizeof(int));
            memcpy(Y + off[t], by[t], (size_t)cnt[t] * sizeof(int));
            memcpy(V + off[t], bv[t], (size_t)cnt[t] * sizeof(double));
        }
    }
    for (int t = 0; t < nt; t++) {
        free(bx[t]);
        free(by[t]);
        free(bv[t]);
    }
    if (!ok) {
        free(X);
        free(Y);
        free(V);
        return -1;
    }
    *px = X;
    *py = Y;
    *pv = V;
    return total;
}

static const char *status_msg_open = "Failed to open file %s\n";

/* Banner + size + entries + base fix-up + nnz check, shared by the CSR and
 * COO entry points. Entries are stored in file order with room for the
 * symmetric mirror (2*nnz), exactly like loadMatrixMarket.cpp:79-141. */
static int read_coo(const char *buf, size_t len, int transpose, int quiet, const char *fname,
                    coo_tmp *t, int serial) {
    cursor c = {buf, buf + len};
    mm_code code;
    memset(t, 0, sizeof(*t));
    if (parse_banner(&c, &code) != 0) {
        if (!quiet) fprintf(stderr, "Error: could not process Matrix Market banner.\n");
        return RSP_MM_BAD_BANNER;
    }
    if (!code_valid(&code) || code.layout == 'A') {
        if (!quiet) fprintf(stderr, "Error: only support sparse and real matrices.\n");
        return RSP_MM_UNSUPPORTED;
    }
    int pattern = code.field == 'P';
    int m, n, nz;
    if (parse_size(&c, &m, &n, &nz) != 0) {
        if (!quiet) fprintf(stderr, "Error: could not read matrix size.\n");
        return RSP_MM_BAD_SIZE;
    }
    if (transpose) {
        int s = m;
        m = n;
        n = s;
    }
    if (m < 0 || n < 0 || nz < 0) {
        if (!quiet) fprintf(stderr, "Error: could not read matrix size.\n");
        return RSP_MM_BAD_SIZE;
    }
    t->m = m;
    t->n = n;
    t->nnz_header = nz;
    t->symmetric = code.symmetry == 'S';
    size_t cap = t->symmetric ? 2 * (size_t)nz : (size_t)nz;
    t->cap = cap;
    t->row = (int *)malloc((cap ? cap : 1) * sizeof(int));
    t->col = (int *)malloc((cap ? cap : 1) * sizeof(int));
    t->val = (double *)malloc((cap ? cap : 1) * sizeof(double));
    if (!t->row || !t->col || !t->val) {
        coo_tmp_free(t);
        if (!quiet) fprintf(stderr, "Failed to allocate memory\n");
        return RSP_MM_ALLOC_FAILED;
    }
    int base = 1;
    long lines = 0;
    int x, y;
    double v;
    /* entries: parsed in parallel when the text is large (same result), else
     * one by one; the per-entry checks below run in file order either way */
    int *px = NULL, *py = NULL;
    double *pv = NULL;
    const long npar = serial ? -1 : parse_entries_parallel(c.p, c.end, &code, &px, &py, &pv);
    long ip = 0;
    for (;;) {
        if (npar >= 0) {
            if (ip >= npar) break;
            x = px[ip];
            y = py[ip];
            v = pv[ip];
            ip++;
        } else if (!parse_entry(&c, &code, &x, &y, &v)) {
            break;
        }
        if (transpose) {
            int s = x;
            x = y;
            y = s;
        }
        if (x > m || y > n || x < 0 || y < 0) {
            if (!quiet) fprintf(stderr, "Error: (%d %d) coordinate is out of range.\n", x, y);
            coo_tmp_free(t);
            free(px);
            free(py);
            free(pv);
            return RSP_MM_OUT_OF_RANGE;
        }
        if ((size_t)lines >= cap) { /* more entries than the header: the
                                       reference overruns; we stop and fail */
            lines++;
            break;
        }
        t->row[lines] = x;
        t->col[lines] = y;
        t->val[lines] = pattern ? 1.0 : v;
        if (x == 0 || y == 0) base = 0;
        lines++;
    }
    free(px);
    free(py);
    free(pv);
    if (lines != nz) {
        if (!quiet)
            fprintf(stderr,
                    "Error: nnz (%d) specified in the header doesn't match with # of lines (%ld) "
                    "in file %s\n",
                    nz, lines, fname ? fname : "<buffer>");
        coo_tmp_free(t);
        return RSP_MM_NNZ_MISMATCH;
    }
    if (base == 0) {
        for (long i = 0; i < lines; i++) {
            t->row[i]++;
            t->col[i]++;
        }
    }
    /* 1-based rows/cols must now be in [1, m] x [1, n]. A 0-based file with a
     * coordinate equal to m passes the reference's range check and writes
     * past rowptr; reject it instead. */
    for (long i = 0; i < lines; i++) {
        if (t->row[i] < 1 || t->row[i] > m || t->col[i] < 1 || t->col[i] > n) {
            if (!quiet)
                fprintf(stderr, "Error: (%d %d) coordinate is out of range.\n", t->row[i],
                        t->col[i]);
            coo_tmp_free(t);
            return RSP_MM_OUT_OF_RANGE;
        }
    }
    t->lines = (int)lines;
    return RSP_MM_OK;
}

/* Mirror pass of loadMatrixMarket.cpp:162-200: for every stored off-diagonal
 * (x,y) whose transpose is absent from row y's stored columns, append (y,x).
 * Returns the expanded count. Appends into t (capacity 2*nnz). */
static int mirror_symmetric(coo_tmp *t, int append) {
    int m = t->m, cnt = t->lines;
    int *start = (int *)calloc((size_t)m + 2, sizeof(int));
    int *cols = (int *)malloc((cnt ? (size_t)cnt : 1) * sizeof(int));
    if (!start || !cols) {
        free(start);
        free(cols);
        return -1;
    }
    for (int i = 0; i < cnt; i++) start[t->row[i]]++; /* row r (1-based) counted at r */
    for (int r = 0; r < m; r++) start[r + 1] += start[r]; /* start[r] = first of 0-based row r */
    int *fill = (int *)malloc(((size_t)m + 1) * sizeof(int));
    if (!fill) {
        free(start);
        free(cols);
        return -1;
    }
    memcpy(fill, start, ((size_t)m + 1) * sizeof(int));
    for (int i = 0; i < cnt; i++) cols[fill[t->row[i] - 1]++] = t->col[i];
    free(fill);
    for (int r = 0; r < m; r++)
        if (start[r + 1] - start[r] > 1)
            qsort(cols + start[r], (size_t)(start[r + 1] - start[r]), sizeof(int), cmp_int);
    int real_count = cnt;
    for (int i = 0; i < cnt; i++) {
        int x = t->row[i], yy = t->col[i];
        if (x == yy) continue;
        /* row yy may exceed m for non-square "symmetric" files: no such row. */
        int present = (yy <= m) ? contains_sorted(cols, start[yy - 1], start[yy], x) : 0;
        if (!present) {
            if (append) {
                t->row[real_count] = yy;
                t->col[real_count] = x;
                t->val[real_count] = t->val[i];
            }
            real_count++;
        }
    }
    free(start);
    free(cols);
    return real_count;
}

static int build_csr(coo_tmp *t, CSR *A, int outBase, int flags) {
    int m = t->m;
    int expanded = t->lines;
    if (t->symmetric) {
        expanded = mirror_symmetric(t, 1);
        if (expanded < 0) return RSP_MM_ALLOC_FAILED;
    }
    /* Entries that reach the CSR: the header nnz (loadMatrixMarket.cpp:220,225),
     * unless the full-symmetric extension is requested. */
    int used = (flags & RSP_MM_FULL_SYMMETRIC) ? expanded : t->lines;
    size_t alloc = (size_t)(expanded > used ? expanded : used);
    A->values = (double *)aligned_alloc64(alloc * sizeof(double));
    A->colidx = (int *)aligned_alloc64(alloc * sizeof(int));
    A->rowptr = (int *)aligned_alloc64(((size_t)m + 1) * sizeof(int));
    if (!A->values || !A->colidx || !A->rowptr) {
        free(A->values);
        free(A->colidx);
        free(A->rowptr);
        A->values = NULL;
        A->colidx = A->rowptr = NULL;
        return RSP_MM_ALLOC_FAILED;
    }
    memset(A->values, 0, alloc * sizeof(double));
    memset(A->colidx, 0, alloc * sizeof(int));
    int *rp = A->rowptr;
    memset(rp, 0, ((size_t)m + 1) * sizeof(int));
    for (int i = 0; i < used; i++) rp[t->row[i]]++;
    for (int i = 0; i < m; i++) rp[i + 1] += rp[i];
    /* rp[r] now = first slot of 0-based row r ... shifted by one row; fill in
     * file order (stable counting sort), then restore. */
    for (int l = 0; l < used; l++) {
        int slot = rp[t->row[l] - 1]++;
        A->values[slot] = t->val[l];
        A->colidx[slot] = t->col[l] - 1 + outBase;
    }
    for (int i = m; i > 0; i--) rp[i] = rp[i - 1] + outBase;
    rp[0] = outBase;
#pragma omp parallel for schedule(dynamic, 4096)
    for (int i = 0; i < m; i++)
        rsp_row_qsort(A->colidx, A->values, rp[i] - outBase, rp[i + 1] - 1 - outBase);
    A->isSymmetric = t->symmetric;
    A->m = m;
    A->n = t->n;
    A->nnz = expanded;
    return RSP_MM_OK;
}

int rsp_mm_load_buffer(const char *buf, size_t len, CSR *A, int outputBase, int transpose,
                       int flags) {
    coo_tmp t;
    memset(A, 0, sizeof(*A));
    int st = read_coo(buf, len, transpose, flags & RSP_MM_QUIET, NULL, &t, flags & RSP_MM_SERIAL);
    if (st != RSP_MM_OK) return st;
    st = build_csr(&t, A, outputBase, flags);
    coo_tmp_free(&t);
    return st;
}

static char *slurp(const char *file, size_t *len) {
    FILE *fp = fopen(file, "rb");
    if (!fp) return NULL;
    if (fseek(fp, 0, SEEK_END) != 0) {
        fclose(fp);
        return NULL;
    }
    long sz = ftell(fp);
    if (sz < 0) {
        fclose(fp);
        return NULL;
    }
    rewind(fp);
    char *buf = (char *)malloc((size_t)sz + 1);
    if (!buf) {
        fclose(fp);
        return NULL;
    }
    size_t got = fread(buf, 1, (size_t)sz, fp);
    fclose(fp);
    buf[got] = '\0';
    *len = got;
    return buf;
}

int rsp_mm_load(const char *file, CSR *A, int outputBase, int transpose, int flags) {
    size_t len = 0;
    memset(A, 0, sizeof(*A));
    char *buf = slurp(file, &len);
    if (!buf) {
        if (!(flags & RSP_MM_QUIET)) fprintf(stderr, status_msg_open, file);
        return RSP_MM_OPEN_FAILED;
    }
    coo_tmp t;
    int st = read_coo(buf, len, transpose, flags & RSP_MM_QUIET, file, &t, flags & RSP_MM_SERIAL);
    free(buf);
    if (st != RSP_MM_OK) return st;
    st = build_csr(&t, A, outputBase, flags);
    coo_tmp_free(&t);
    return st;
}

int loadMatrixMarket(const char *file, CSR *matrix, int outputBase, int transpose) {
    int st = rsp_mm_load(file, matrix, outputBase, transpose, 0);
    if (st == RSP_MM_OPEN_FAILED) exit(-1);
    return st == RSP_MM_OK;
}

int loadCooMatrix(const char *file, COO *matrix, int outputbase, int transpose) {
    size_t len = 0;
    memset(matrix, 0, sizeof(*matrix));
    char *buf = slurp(file, &len);
    if (!buf) {
        fprintf(stderr, status_msg_open, file);
        exit(-1);
    }
    coo_tmp t;
    int st = read_coo(buf, len, transpose, 0, file, &t, 0);
    free(buf);
    if (st != RSP_MM_OK) return 0;
    int count = t.lines;
    if (t.symmetric) {
        count = mirror_symmetric(&t, 1);
        if (count < 0) {
            coo_tmp_free(&t);
            return 0;
        }
    }
    /* loadCooMatrix keeps 1-based file coordinates (it never applies
     * outputbase, loadMatrixMarket.cpp:362-372,432-434). */
    (void)outputbase;
    size_t alloc = t.cap ? t.cap : 1;
    matrix->values = (double *)aligned_alloc64(alloc * sizeof(double));
    matrix->Colidx = (int *)aligned_alloc64(alloc * sizeof(int));
    matrix->Rowidx = (int *)aligned_alloc64(alloc * sizeof(int));
    if (!matrix->values || !matrix->Colidx || !matrix->Rowidx) {
        coo_tmp_free(&t);
        return 0;
    }
    memcpy(matrix->values, t.val, (size_t)count * sizeof(double));
    memcpy(matrix->Colidx, t.col, (size_t)count * sizeof(int));
    memcpy(matrix->Rowidx, t.row, (size_t)count * sizeof(int));
    matrix->isSymmetric = t.symmetric;
    matrix->m = t.m;
    matrix->n = t.n;
    matrix->nnz = count;
    coo_tmp_free(&t);
    return 1;
}

void rsp_csr_free(CSR *A) {
    if (!A) return;
    free(A->rowptr);
    free(A->colidx);
    free(A->values);
    A->rowptr = A->colidx = NULL;
    A->values = NULL;
}

void rsp_coo_free(COO *A) {
    if (!A) return;
    free(A->Rowidx);
    free(A->Colidx);
    free(A->values);
    A->Rowidx = A->Colidx = NULL;
    A->values = NULL;
}

/* ----------------------------------------------------- binary cache */

#define RSP_CSR_MAGIC 0x52535043u /* "RSPC" */

int rsp_csr_save(const char *path, const CSR *A) {
    FILE *fp = fopen(path, "wb");
    if (!fp) return -1;
    int base = A->rowptr ? A->rowptr[0] : 0;
    int stored = A->rowptr ? A->rowptr[A->m] - base : 0;
    uint32_t hdr[8] = {RSP_CSR_MAGIC, 1u, (uint32_t)A->isSymmetric, (uint32_t)A->m,
                       (uint32_t)A->n, (uint32_t)A->nnz, (uint32_t)stored, 0u};
    int ok = fwrite(hdr, sizeof(hdr), 1, fp) == 1;
    ok = ok && fwrite(A->rowptr, sizeof(int), (size_t)A->m + 1, fp) == (size_t)A->m + 1;
    size_t alloc = (size_t)(A->nnz > stored ? A->nnz : stored);
    ok = ok && fwrite(A->colidx, sizeof(int), alloc, fp) == alloc;
    ok = ok && fwrite(A->values, sizeof(double), alloc, fp) == alloc;
    ok = (fclose(fp) == 0) && ok;
    return ok ? 0 : -1;
}

int rsp_csr_load(const char *path, CSR *A) {
    memset(A, 0, sizeof(*A));
    FILE *fp = fopen(path, "rb");
    if (!fp) return -1;
    uint32_t hdr[8];
    if (fread(hdr, sizeof(hdr), 1, fp) != 1 || hdr[0] != RSP_CSR_MAGIC || hdr[1] != 1u) {
        fclose(fp);
        return -1;
    }
    A->isSymmetric = (int)hdr[2];
    A->m = (int)hdr[3];
    A->n = (int)hdr[4];
    A->nnz = (int)hdr[5];
    int stored = (int)hdr[6];
    size_t alloc = (size_t)(A->nnz > stored ? A->nnz : stored);
    A->rowptr = (int *)aligned_alloc64(((size_t)A->m + 1) * sizeof(int));
    A->colidx = (int *)aligned_alloc64(alloc * sizeof(int));
    A->values = (double *)aligned_alloc64(alloc * sizeof(double));
    int ok = A->rowptr && A->colidx && A->values;
    ok = ok && fread(A->rowptr, sizeof(int), (size_t)A->m + 1, fp) == (size_t)A->m + 1;
    ok = ok && fread(A->colidx, sizeof(int), alloc, fp) == alloc;
    ok = ok && fread(A->values, sizeof(double), alloc, fp) == alloc;
    fclose(fp);
    if (!ok) {
        rsp_csr_free(A);
        return -1;
    }
    return 0;
}
