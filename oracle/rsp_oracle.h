/*
 * rsp_oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of ReSpaSol's
 * hot-path arithmetic, used as the parity checker by tests/, by
 * __graft_entry__.smoke() and as bench.py's cpu_baseline ("kind": "port").
 * Nothing in the product (respasol_amd/) links, loads or calls this code.
 *
 * Parity pins (see DESIGN.md "Oracle"):
 *   - loader: the product loader is checked byte-for-byte against the
 *     reference loader itself, compiled from /root/reference by
 *     oracle/Makefile into oracle/_ref/ (this container only), and against
 *     committed dumps of it (tests/golden/);
 *   - SpMV / ILU(0) / trsv: restated from the cuSPARSE semantics the drivers
 *     request (GPU/spmv.cu:148-186, GPU/ilu0.cu:122-310) and pinned by the
 *     known-answer tests of SURVEY §8c (bcspwr01 integer-exact ILU solve,
 *     b1_ss structural zero, identity); cuSPARSE itself is closed source and
 *     unavailable, so bitwise parity with it is unpinned (its summation order
 *     is unspecified) and the stated tolerances apply.
 *   - dlarnv: restated from LAPACK DLARUV's 12-bit-limb arithmetic and pinned
 *     by the MKL values recorded in SURVEY §0.7.
 */
#ifndef RSP_ORACLE_H
#define RSP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* y = A x, row by row, sequential column order, product rounded then added
 * (GPU/spmv.cu:184-186 with alpha = 1, beta = 0; test_spmv.c:169). */
void oracle_spmv_f64(int m, const int *rowptr, const int *colidx, const double *vals,
                     const double *x, double *y);
/* fp32 storage and accumulation (GPU/spmv.cu:179-181; test_spmv.c:178-179). */
void oracle_spmv_f32(int m, const int *rowptr, const int *colidx, const float *vals,
                     const float *x, float *y);
/* fp32 with MXCSR FTZ|DAZ (test_pardiso.c:19-24) around the arithmetic only. */
void oracle_spmv_f32_ftz(int m, const int *rowptr, const int *colidx, const float *vals,
                         const float *x, float *y);
/* Row-parallel OpenMP versions (same per-row arithmetic => identical y):
 * the CPU baseline the reference's test_spmv.c times (MKL gnu_thread). */
void oracle_spmv_f64_omp(int m, const int *rowptr, const int *colidx, const double *vals,
                         const double *x, double *y);
void oracle_spmv_f32_omp(int m, const int *rowptr, const int *colidx, const float *vals,
                         const float *x, float *y);
int oracle_num_threads(void);
void oracle_set_threads(int threads); /* OpenMP threads of the _omp kernels */
/* Same products in the CANONICAL summation order of the GPU SpMV (see
 * rsp_oracle.c): 8-way interleave + fixed tree for rows of <= 256 products,
 * chunked (cap = tile capacity: 2047 fp64 / 4093 fp32) 256-way interleave +
 * wave butterflies for longer rows. The GPU result equals this bit for bit. */
void oracle_spmv_canon_f64(int m, const int *rowptr, const int *colidx, const double *vals,
                           const double *x, double *y, int cap);
void oracle_spmv_canon_f32(int m, const int *rowptr, const int *colidx, const float *vals,
                           const float *x, float *y, int cap);
void oracle_spmv_canon_f32_ftz(int m, const int *rowptr, const int *colidx, const float *vals,
                               const float *x, float *y, int cap);

/* In-place ILU(0), IKJ, fma updates (cusparse?csrilu02, GPU/ilu0.cu:264-268).
 * Returns the first structurally missing diagonal (>= 0) without factoring,
 * else -1; *zero_pivot = smallest i with u_ii == 0 after the factor, or -1. */
int oracle_ilu0_f64(int n, const int *rowptr, const int *colidx, double *vals, int *zero_pivot);
int oracle_ilu0_f32(int n, const int *rowptr, const int *colidx, float *vals, int *zero_pivot,
                    int ftz);

/* L y = alpha x (unit lower, strictly-lower entries), GPU/ilu0.cu:296-298. */
void oracle_trsv_lower_n_f64(int n, const int *rowptr, const int *colidx, const double *vals,
                             double alpha, const double *x, double *y);
void oracle_trsv_lower_n_f32(int n, const int *rowptr, const int *colidx, const float *vals,
                             float alpha, const float *x, float *y, int ftz);
/* L^T y = alpha x, column sweep j = n-1 .. 0 (GPU/ilu0.cu:300-302). */
void oracle_trsv_lower_t_f64(int n, const int *rowptr, const int *colidx, const double *vals,
                             double alpha, const double *x, double *y);
void oracle_trsv_lower_t_f32(int n, const int *rowptr, const int *colidx, const float *vals,
                             float alpha, const float *x, float *y, int ftz);
/* The same two solves in the split term order of the MI355X plans: a row's
 * terms from the level just below its own (in the solve's DAG) applied
 * last, each part in the order above (rsp_oracle.c ORACLE_TRSV_SPLIT). */
void oracle_trsv_lower_n_split_f64(int n, const int *rowptr, const int *colidx, const double *vals,
                                   double alpha, const double *x, double *y);
void oracle_trsv_lower_n_split_f32(int n, const int *rowptr, const int *colidx, const float *vals,
                                   float alpha, const float *x, float *y, int ftz);
void oracle_trsv_lower_t_split_f64(int n, const int *rowptr, const int *colidx, const double *vals,
                                   double alpha, const double *x, double *y);
void oracle_trsv_lower_t_split_f32(int n, const int *rowptr, const int *colidx, const float *vals,
                                   float alpha, const float *x, float *y, int ftz);
/* The two unit-lower solves (kind 0: L y = alpha x; kind 1: L^T y = alpha x)
 * in the BLOCK-INVERSE order of the MI355X deep-DAG solve (round 6; the
 * product's planner is ilu_blocks.cpp, restated here independently):
 * rows in level order, cut greedily into blocks of <= bs rows; inside a
 * block every row's unknown is written as a combination of the block's
 * right-hand sides (alpha x) and of y values of earlier blocks (the
 * block's explicit partitioned inverse), so a block is one dependent step.
 * Same unknowns, different rounding from the reference order: within
 * SURVEY 8c's solve tolerance (tests/test_oracle.py), and the GPU equals
 * THIS restatement bit for bit. params = {bs, ymax, near, nw, ch, lcap}
 * (rows per block, y terms of a row, near terms of a row, near window in
 * positions, chunk length, a row with more dependencies in its chunk starts
 * a new one; see rsp_oracle.c); null = the product's defaults. Returns the number of blocks (< 0: bad
 * arguments). */
/* Levels (longest dependency path + 1) of the L (kind 0) or L^T (kind 1) DAG. */
int oracle_dag_levels(int kind, int n, const int *rowptr, const int *colidx);
int oracle_trsv_blocks_f64(int kind, int n, const int *rowptr, const int *colidx, const double *vals,
                           double alpha, const double *x, double *y, const int *params);
int oracle_trsv_blocks_f32(int kind, int n, const int *rowptr, const int *colidx, const float *vals,
                           float alpha, const float *x, float *y, const int *params, int ftz);

/* U y = alpha x (upper incl. diagonal) — the desc_U extension. */
void oracle_trsv_upper_f64(int n, const int *rowptr, const int *colidx, const double *vals,
                           double alpha, const double *x, double *y);
void oracle_trsv_upper_f32(int n, const int *rowptr, const int *colidx, const float *vals,
                           float alpha, const float *x, float *y, int ftz);

/* LAPACK DLARNV via DLARUV's 12-bit limb arithmetic (independent of the
 * product's 64-bit implementation). idist 1/2 only. */
int oracle_dlarnv(int idist, int *iseed, int n, double *x);

#ifdef __cplusplus
}
#endif

#endif
