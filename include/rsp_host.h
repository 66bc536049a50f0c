/*
 * rsp_host.h — C-ABI of the host-side library `librsp_host.so`: the input
 * side of the drop-in boundary (Matrix-Market -> CSR loader with the
 * reference's exact semantics), the LAPACK dlarnv generator the CPU driver
 * uses for x, the seeded SuiteSparse surrogate generator and the nnz-balanced
 * row partitioner used by the multi-GPU SpMV.
 *
 * Reference interface replaced:
 *   CSR / COO structs        ReadMatrixMarket/loadMatrixMarket.h:17-36
 *   loadMatrixMarket()       ReadMatrixMarket/loadMatrixMarket.h:41, .cpp:47-253
 *   loadCooMatrix()          ReadMatrixMarket/loadMatrixMarket.h:42, .cpp:277-436
 *   LAPACKE_dlarnv()         test_spmv.c:75-76 (MKL; LAPACK dlarnv/dlaruv algorithm)
 *
 * The reference loader has C++ linkage; this library exports the same names
 * and struct layouts with C linkage (the boundary is a C ABI). Arrays are
 * 64-byte aligned (posix_memalign) and owned by the caller, who releases them
 * with free() exactly as the drivers do (GPU/spmv.cu:265-267).
 */
#ifndef RSP_HOST_H
#define RSP_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field order and types as loadMatrixMarket.h:17-25. */
typedef struct {
    int isSymmetric;
    int m;
    int n;
    int nnz;      /* reference semantics: EXPANDED count for symmetric files */
    int *rowptr;  /* m+1 entries, base = outputBase */
    int *colidx;  /* nnz entries allocated; rowptr[m]-base are meaningful */
    double *values;
} CSR;

/* Same field order and types as loadMatrixMarket.h:28-36. */
typedef struct {
    int isSymmetric;
    int m;
    int n;
    int nnz;
    int *Colidx;
    int *Rowidx;
    double *values;
} COO;

/* Status codes of rsp_mm_load (the reference returns true/false and exits on
 * a missing file; this extended entry point reports why instead). */
typedef enum {
    RSP_MM_OK = 0,
    RSP_MM_OPEN_FAILED = 1,    /* "Failed to open file %s"                 (.cpp:49-53)   */
    RSP_MM_BAD_BANNER = 2,     /* "could not process Matrix Market banner" (.cpp:56-60)   */
    RSP_MM_UNSUPPORTED = 3,    /* "only support sparse and real matrices"  (.cpp:63-67)   */
    RSP_MM_BAD_SIZE = 4,       /* "could not read matrix size"             (.cpp:70-76)   */
    RSP_MM_OUT_OF_RANGE = 5,   /* "(%d %d) coordinate is out of range"     (.cpp:122-126) */
    RSP_MM_NNZ_MISMATCH = 6,   /* "nnz (%d) specified in the header ..."   (.cpp:156-160) */
    RSP_MM_ALLOC_FAILED = 7
} rsp_mm_status_t;

/* Load options beyond the reference's (outputBase, transpose). */
#define RSP_MM_FULL_SYMMETRIC 0x1 /* keep the mirrored entries in the CSR */
#define RSP_MM_QUIET 0x2          /* do not print the reference's stderr messages */
#define RSP_MM_SERIAL 0x4         /* parse entries on one thread (default: OpenMP for large files) */

/* Reference-compatible loader: loadMatrixMarket.cpp:47-253. Returns 1 on
 * success and 0 on failure; prints the reference's messages on stderr and
 * calls exit(-1) if the file cannot be opened (.cpp:49-53). For symmetric
 * files the CSR holds the STORED triangle only while nnz is the expanded
 * count. */
int loadMatrixMarket(const char *file, CSR *matrix, int outputBase, int transpose);
/* loadMatrixMarket.cpp:277-436: COO incl. mirrored entries. Same conventions. */
int loadCooMatrix(const char *file, COO *matrix, int outputBase, int transpose);
/* Same algorithm, returns an rsp_mm_status_t and never exits. */
int rsp_mm_load(const char *file, CSR *matrix, int outputBase, int transpose, int flags);
/* Parse from an in-memory buffer (same semantics as rsp_mm_load). */
int rsp_mm_load_buffer(const char *buf, size_t len, CSR *matrix, int outputBase, int transpose,
                       int flags);
/* The reference's per-row co-sort (loadMatrixMarket.cpp:5-26): recursive,
 * middle pivot, unstable. Exposed so tests can pin duplicate ordering. */
void rsp_row_qsort(int *idx, double *w, int left, int right);
void rsp_csr_free(CSR *matrix);
void rsp_coo_free(COO *matrix);

/* Binary CSR cache: a fixed little-endian image of the
 * CSR struct and arrays so a sweep parses each .mtx once. Returns 0 on
 * success. */
int rsp_csr_save(const char *path, const CSR *matrix);
int rsp_csr_load(const char *path, CSR *matrix);

/* LAPACK dlarnv (LAPACKE_dlarnv(idist, iseed, n, x), test_spmv.c:75-76):
 * idist 1 = uniform(0,1), 2 = uniform(-1,1), 3 = normal(0,1). iseed[4] is a
 * 48-bit seed in 12-bit limbs (iseed[3] odd) and is advanced on return. */
int rsp_dlarnv(int idist, int *iseed, int64_t n, double *x);

/* x86 MXCSR FTZ|DAZ (test_pardiso.c:19-24 `set_ftz`, README.md:79-80). */
void rsp_set_cpu_ftz(int enable);

/* ------------------------------------------------ surrogate generator
 * Seeded stand-ins for the SuiteSparse matrices the reference sweeps
 * (GPU/run_spmv.sh:3-5): same m, ~same stored nnz, same
 * symmetric-storage convention (lower triangle + diagonal), a structural
 * family per matrix. Row i is a pure function of (name, i), so any row range
 * can be generated independently (multi-GPU ranks generate only their rows). */
#define RSP_SURR_FTZ_STRESS 0x1 /* scale ~1% of off-diagonals into fp32-subnormal range */

/* Number of catalogued names and the i-th name (NULL past the end). */
int rsp_surrogate_count(void);
const char *rsp_surrogate_name(int i);
/* set: 0 = moderate, 1 = big. family: 0 stencil3d, 1 stencil2d, 2 circuit, 3 randband. */
int rsp_surrogate_info(const char *name, int *m, int64_t *nnz_target, int *symmetric, int *set,
                       int *family);
/* A spec selects a catalogued name, optionally scaled down (scale in (0,1],
 * rows = max(64, m*scale)) for tests. Generic custom spec: name "stencil3d:ROWS:NNZ_PER_ROW:SYM"
 * etc. is also accepted (see surrogate.c). */
/* Row lengths of rows [r0, r1) into rowlen[0..r1-r0). Returns 0 on success. */
int rsp_surrogate_rowlens(const char *name, double scale, int flags, int r0, int r1, int *rowlen);
/* Rows of the surrogate: m (rows == cols). */
int rsp_surrogate_rows(const char *name, double scale, int *m);
/* Fill rows [r0, r1): rowptr_local[0..r1-r0] (base 0, starting at 0),
 * colidx/values sized rowptr_local[r1-r0]. Columns are global, sorted, unique. */
int rsp_surrogate_fill(const char *name, double scale, int flags, int r0, int r1, int *rowptr_local,
                       int *colidx, double *values);
/* Convenience: the whole matrix as a reference-style CSR (isSymmetric set,
 * nnz = stored count; base 0). */
int rsp_surrogate_csr(const char *name, double scale, int flags, CSR *matrix);

/* ---------------------------------------------------------- partition
 * nnz-balanced contiguous row ranges: bounds[p] =
 * lower_bound(rowptr, rowptr[0] + p*nnz/P), bounds[0] = 0, bounds[P] = m. */
int rsp_partition_rows(const int *rowptr, int m, int parts, int *bounds);
/* Padded all-gather layout of a row-partitioned x: slice p's entries sit at
 * x_pad[p*chunk ..) with chunk = max_p (bounds[p+1] - bounds[p]) (returned;
 * -1 on bad arguments), so one equal-count ncclAllGather reassembles x. */
int rsp_padded_chunk(const int *bounds, int parts);
/* colidx_out[k] = p*chunk + (c - bounds[p]) for c = colidx_in[k] in slice p
 * (in place allowed). -1 if a column lies outside [0, bounds[parts]). */
int rsp_remap_cols_padded(int64_t nnz, const int *colidx_in, const int *bounds, int parts, int chunk,
                          int *colidx_out);

/* Host CSR SpMV used by the drivers' verification step (the role MKL's
 * sequential mkl_sparse_?_mv plays in GPU/spmv.cu:221-260). Row-parallel. */
void rsp_host_spmv_f64(int m, const int *rowptr, const int *colidx, const double *vals,
                       const double *x, double *y);
void rsp_host_spmv_f32(int m, const int *rowptr, const int *colidx, const float *vals,
                       const float *x, float *y);

#ifdef __cplusplus
}
#endif

#endif /* RSP_HOST_H */
