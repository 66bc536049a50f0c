/*
 * rsp.h — C-ABI of the MI355X (gfx950) sparse operator library `librsp.so`.
 *
 * This is the drop-in boundary for the vendor-math layer of ReSpaSol's GPU
 * drivers: every entry point below replaces one cuSPARSE call (or call family)
 * made by /root/reference/GPU/spmv.cu or /root/reference/GPU/ilu0.cu, with the
 * same argument meaning, the same lifecycle (create -> bufferSize ->
 * analysis -> compute -> zeroPivot -> destroy) and status codes numbered like
 * cusparseStatus_t so that the drivers' error printing is unchanged.
 *
 * Conventions
 *   - Plain C types only: device pointers are `void*`/typed pointers obtained
 *     from hipMalloc (or any HIP allocator), sizes are int64_t / size_t, the
 *     stream is an opaque `void*` holding a hipStream_t (NULL = default stream).
 *   - CSR with int32 row offsets / column indices, index base 0 (the only form
 *     the reference uses: GPU/spmv.cu:132-151, GPU/ilu0.cu:122-126).
 *   - alpha / beta are HOST pointers of the compute type (cuSPARSE default
 *     pointer mode, GPU/spmv.cu:61-62,77-78).
 *   - Every call is stream-ordered on the handle's stream; only the calls
 *     marked "host-blocking" synchronise (as their cuSPARSE counterparts do).
 *   - No call aborts or exits: failures return a status code.
 *
 * Precision: RSP_R_64F / RSP_R_32F select fp64 or fp32 storage AND
 * accumulation (GPU/spmv.cu:131-162 with and without `#define FLOAT`).
 * Flush-to-zero is an EXTENSION, not reference parity: the reference's nvcc
 * flag is commented out (`CFLAGS = -arch=sm_70 -O3  #-ftz=true`,
 * GPU/Makefile:5) and would not reach cuSPARSE's precompiled kernels anyway.
 * It is a handle mode here (rsp_set_ftz) selecting kernels compiled with fp32
 * denormal flushing, for the "fp32+FTZ" experiment the README describes
 * (README.md:79-80). The parity configuration is fp32 without FTZ.
 */
#ifndef RSP_H
#define RSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSP_VERSION_MAJOR 0
#define RSP_VERSION_MINOR 1

/* Numbered exactly like cusparseStatus_t (GPU/spmv.cu:24-29 prints the
 * integer), so drivers print identical codes. */
typedef enum {
    RSP_STATUS_SUCCESS = 0,
    RSP_STATUS_NOT_INITIALIZED = 1,
    RSP_STATUS_ALLOC_FAILED = 2,
    RSP_STATUS_INVALID_VALUE = 3,
    RSP_STATUS_ARCH_MISMATCH = 4,
    RSP_STATUS_EXECUTION_FAILED = 6,
    RSP_STATUS_INTERNAL_ERROR = 7,
    RSP_STATUS_MATRIX_TYPE_NOT_SUPPORTED = 8,
    RSP_STATUS_ZERO_PIVOT = 9,
    RSP_STATUS_NOT_SUPPORTED = 10
} rsp_status_t;

/* CUDA_R_64F / CUDA_R_32F (GPU/spmv.cu:135,151). */
typedef enum { RSP_R_64F = 0, RSP_R_32F = 1 } rsp_datatype_t;

/* CUSPARSE_OPERATION_NON_TRANSPOSE / _TRANSPOSE (GPU/ilu0.cu:296,300). */
typedef enum { RSP_OPERATION_NON_TRANSPOSE = 0, RSP_OPERATION_TRANSPOSE = 1 } rsp_operation_t;

typedef struct rsp_context *rsp_handle_t;       /* cusparseHandle_t       */
typedef struct rsp_spmat *rsp_spmat_t;          /* cusparseSpMatDescr_t   */
typedef struct rsp_ilu0_info *rsp_ilu0_info_t;  /* csrilu02Info_t + both csrsv2Info_t */
typedef struct rsp_spmv_batch *rsp_spmv_batch_t; /* no cuSPARSE counterpart (below) */

/* ---------------------------------------------------------------- handle */

/* cusparseCreate (GPU/spmv.cu:128, GPU/ilu0.cu:85). Binds the current HIP
 * device; fails with ARCH_MISMATCH if it is not gfx950. */
rsp_status_t rsp_create(rsp_handle_t *handle);
/* cusparseDestroy (GPU/spmv.cu:282, GPU/ilu0.cu:340). */
rsp_status_t rsp_destroy(rsp_handle_t handle);
/* cusparseSetStream. `stream` is a hipStream_t (NULL = default stream). */
rsp_status_t rsp_set_stream(rsp_handle_t handle, void *stream);
rsp_status_t rsp_get_stream(rsp_handle_t handle, void **stream);
/* Extension (the reference's `-ftz=true` at GPU/Makefile:5 is commented
 * out): fp32 kernels flush denormal inputs and results to zero when enabled.
 * fp64 is never flushed (as with nvcc -ftz). Default off = parity mode. */
rsp_status_t rsp_set_ftz(rsp_handle_t handle, int enable);
rsp_status_t rsp_get_ftz(rsp_handle_t handle, int *enable);
/* cusparseGetErrorString analogue. Never NULL. */
const char *rsp_get_error_string(rsp_status_t status);
/* Library version: major*1000 + minor. */
int rsp_get_version(void);

/* ------------------------------------------------------- CSR descriptor */

/* cusparseCreateCsr(&matA, rows, cols, nnz, offsets, columns, values,
 * CUSPARSE_INDEX_32I, CUSPARSE_INDEX_32I, CUSPARSE_INDEX_BASE_ZERO, dtype)
 * (GPU/spmv.cu:132-135,148-151). `nnz` is the caller's count; like cuSPARSE
 * the kernels use offsets[rows] (the reference passes A.nnz, which exceeds
 * offsets[rows] for symmetric inputs: SURVEY §0.3). Host-side object only. */
rsp_status_t rsp_create_csr(rsp_spmat_t *mat, int64_t rows, int64_t cols, int64_t nnz,
                            void *d_row_offsets, void *d_col_ind, void *d_values,
                            rsp_datatype_t value_type);
/* Re-point the values array (e.g. fp64 -> fp32 copy) keeping the analysis. */
rsp_status_t rsp_csr_set_values(rsp_spmat_t mat, void *d_values, rsp_datatype_t value_type);
rsp_status_t rsp_destroy_spmat(rsp_spmat_t mat); /* cusparseDestroySpMat (GPU/spmv.cu:279) */

/* ------------------------------------------------------------------ SpMV */

/* cusparseSpMV_bufferSize (GPU/spmv.cu:143-145,159-161). Host-blocking: builds
 * the row-block schedule of `mat` for `compute_type` (reads the row offsets and
 * column indices once, validates them — INVALID_VALUE for a malformed
 * pattern — and keeps a 16-bit copy of the column indices, relative to each
 * tile's first column, for tiles spanning < 65536 columns) in device memory
 * owned by `mat` (freed by rsp_destroy_spmat), so that the reference's call
 * sequence create_csr -> bufferSize -> malloc -> SpMV x50 (GPU/spmv.cu:143-195)
 * plans nothing inside a timed call. *buffer_size is 0: rsp_spmv needs no
 * caller workspace (any pointer, NULL included, is accepted), and several
 * matrices may share one. The schedule is reused while it is valid; as with
 * cuSPARSE, the sparsity pattern must not change afterwards without a new
 * rsp_spmv_preprocess (values may: they are read on every call). */
rsp_status_t rsp_spmv_buffer_size(rsp_handle_t handle, rsp_operation_t op, const void *alpha,
                                  rsp_spmat_t mat, const void *beta, rsp_datatype_t compute_type,
                                  size_t *buffer_size);
/* cusparseSpMV_preprocess analogue (cuSPARSE 12; the reference has no such
 * call): rebuilds the schedule of `mat` (host-blocking, as bufferSize). Only
 * needed after the pattern changed; rsp_spmv plans lazily if neither call was
 * made. `d_buffer` is unused. */
rsp_status_t rsp_spmv_preprocess(rsp_handle_t handle, rsp_operation_t op, const void *alpha,
                                 rsp_spmat_t mat, const void *d_x, const void *beta, void *d_y,
                                 rsp_datatype_t compute_type, void *d_buffer);
/* cusparseSpMV (GPU/spmv.cu:179-186): y = alpha * A * x + beta * y.
 * op must be NON_TRANSPOSE (the only form the reference uses). If *beta == 0,
 * y is write-only. compute_type must equal the matrix value type. Deterministic:
 * the same inputs give bitwise identical y on every call. `d_buffer` is
 * accepted for signature parity and unused. Calls on one matrix must be
 * stream-ordered (its long-row tickets live in its schedule). */
rsp_status_t rsp_spmv(rsp_handle_t handle, rsp_operation_t op, const void *alpha, rsp_spmat_t mat,
                      const void *d_x, const void *beta, void *d_y, rsp_datatype_t compute_type,
                      void *d_buffer);

/* --------------------------------------------------------- ILU(0) + trsv */

/* cusparseCreateCsrilu02Info + 2x cusparseCreateCsrsv2Info (GPU/ilu0.cu:143-150). */
rsp_status_t rsp_create_ilu0_info(rsp_ilu0_info_t *info);
rsp_status_t rsp_destroy_ilu0_info(rsp_ilu0_info_t info);

/* cusparse?csrilu02_bufferSize / csrsv2_bufferSize (GPU/ilu0.cu:166-186).
 * The schedule lives in `info` (library-owned), so the external buffer size
 * is 0; kept for lifecycle parity. */
rsp_status_t rsp_ilu0_buffer_size(rsp_handle_t handle, int n, int nnz, rsp_datatype_t value_type,
                                  rsp_ilu0_info_t info, size_t *buffer_size);

/* cusparse?csrilu02_analysis (GPU/ilu0.cu:203-217, the reference's timed
 * "Symbolic"): diagonal positions, structural-zero detection, the symbolic
 * factor, level sets of the lower triangle (factor + L-solve) and of its
 * transpose (L^T-solve), and the factor plan. The two solve plans (the
 * csrsv2_analysis half, rsp_trsv_analysis below) are started on a worker
 * thread as soon as the levels exist and left running when this call
 * returns. `nnz` may exceed offsets[n] (the
 * reference passes A.nnz, GPU/ilu0.cu:166); offsets[n] is what is analysed.
 * Each row's column indices must be strictly increasing (sorted, no
 * duplicates — as csrilu02 requires); otherwise INVALID_VALUE. The reference
 * loader sorts rows but keeps duplicate entries of a file, so a file with
 * repeated coordinates is rejected here rather than factored as undefined.
 * Host-blocking (reads the pattern once). */
rsp_status_t rsp_ilu0_analysis(rsp_handle_t handle, int n, int nnz, const int *d_row_offsets,
                               const int *d_col_ind, rsp_ilu0_info_t info);

/* cusparse?csrsv2_analysis for the L (op NON_TRANSPOSE) or L^T (op
 * TRANSPOSE) solve of an analysed info (GPU/ilu0.cu:228-252, untimed there):
 * waits for the solve plans rsp_ilu0_analysis started and uploads them (the
 * first call does both kinds; later calls return at once). Optional — the
 * first solve does it if it was not called. Host-blocking. */
rsp_status_t rsp_trsv_analysis(rsp_handle_t handle, rsp_operation_t op, rsp_ilu0_info_t info);

/* cusparseXcsrilu02_zeroPivot (GPU/ilu0.cu:222,278). Host-blocking. Returns
 * RSP_STATUS_ZERO_PIVOT and *position = j (0-based) when A(j,j) is
 * structurally missing (after analysis) or U(j,j) == 0 (after the numeric
 * factorisation); the smallest such j is reported. Otherwise SUCCESS, -1. */
rsp_status_t rsp_ilu0_zero_pivot(rsp_handle_t handle, rsp_ilu0_info_t info, int *position);
/* Flow launches (one launch over a run of fat levels) take their work items by
 * start tickets (the default since round 6): a workgroup owns the items of the
 * ticket it claimed when it started, and a workgroup that has waited long
 * while some tickets are still unclaimed (their workgroups have not started:
 * another kernel holds the CUs) claims those too, so progress never depends on
 * other kernels leaving CUs free and no wait gives up in normal operation. The
 * bounded wait (RSP_ILU_FLOW_TIMEOUT_US, default 0.2 s) stays as a backstop,
 * and it is what the older static item walk (RSP_ILU_FLOW_MODE=0) needs: a
 * factor whose flow wait gave up is RECOVERED here — its input values (kept
 * by the factor call) are restored, the factor runs again without flow
 * launches, and so does every solve made after it — and the call reports as
 * usual. The buffers of the recorded calls (values, x) must then be unchanged
 * since those calls; a later recorded solve that wrote its y over one of them
 * (e.g. L: r -> z, then L^T: z -> r) makes the recovery impossible and the
 * call returns RSP_STATUS_EXECUTION_FAILED, as it does when recovery is off
 * (RSP_ILU_FLOW_RECOVER=0). About the LAST factor call only. */

/* cusparseXcsrsv2_zeroPivot (the csrsv2 infos of GPU/ilu0.cu:143-150) for
 * the solves below; which = RSP_TRSV_L (op N), RSP_TRSV_LT (op T) or
 * RSP_TRSV_U (rsp_trsv_upper). Host-blocking. Reports on the LAST solve of
 * that kind. If its flow launch gave up a wait, the solve (its x is
 * unchanged: x != y) and every solve made after it are run again without
 * flow launches first (their x and values must be unchanged, as above);
 * RSP_STATUS_EXECUTION_FAILED with RSP_ILU_FLOW_RECOVER=0 or when a later
 * recorded solve overwrote one of those inputs. For RSP_TRSV_U, ZERO_PIVOT + *position as
 * rsp_ilu0_zero_pivot (U divides by u_jj); else SUCCESS, -1. */
#define RSP_TRSV_L 0
#define RSP_TRSV_LT 1
#define RSP_TRSV_U 2
rsp_status_t rsp_trsv_zero_pivot(rsp_handle_t handle, rsp_ilu0_info_t info, int which, int *position);

/* cusparse?csrilu02 (GPU/ilu0.cu:264-268): in-place ILU(0) on the CSR
 * pattern, IKJ order: for each row i, for each k < i in the pattern
 * (ascending): a_ik /= u_kk; a_ij -= a_ik * u_kj for j > k in both rows.
 * value_type selects fp64 or fp32 arithmetic (FTZ per handle mode). */
rsp_status_t rsp_ilu0_factor(rsp_handle_t handle, rsp_ilu0_info_t info, rsp_datatype_t value_type,
                             void *d_values);

/* cusparse?csrsv2_solve with desc_L = {LOWER, UNIT} (GPU/ilu0.cu:129-134):
 *   op == NON_TRANSPOSE: solve L   y = alpha x   (GPU/ilu0.cu:296-298)
 *   op == TRANSPOSE:     solve L^T y = alpha x   (GPU/ilu0.cu:300-302)
 * where L is the unit-diagonal strictly-lower part of `d_values` on the
 * analysed pattern. x and y must not alias. */
rsp_status_t rsp_trsv_lower_unit(rsp_handle_t handle, rsp_operation_t op, const void *alpha,
                                 rsp_ilu0_info_t info, rsp_datatype_t value_type,
                                 const void *d_values, const void *d_x, void *d_y);

/* Extension (off by default): solve with the upper factor
 * U (non-unit diagonal, upper part incl. diagonal), i.e. the true ILU(0)
 * apply that the reference's unused desc_U describes (GPU/ilu0.cu:136-141). */
rsp_status_t rsp_trsv_upper(rsp_handle_t handle, const void *alpha, rsp_ilu0_info_t info,
                            rsp_datatype_t value_type, const void *d_values, const void *d_x,
                            void *d_y);

/* ------------------------------------------------ multi-GPU halo exchange */

/* Indexed gather dst[i] = src[idx[i]] for i < n (value_type elements). The
 * pack / unpack step of the row-partitioned SpMV's halo exchange (SURVEY
 * §8e-f): pack the x entries peers need into an RCCL send buffer, and unpack
 * the received halo into each slice's extended x. idx must be in range. */
rsp_status_t rsp_gather(rsp_handle_t handle, rsp_datatype_t value_type, int64_t n,
                        const int64_t *d_idx, const void *d_src, void *d_dst);
/* Indexed scatter dst[idx[i]] = src[i] for i < n (idx without duplicates). */
rsp_status_t rsp_scatter(rsp_handle_t handle, rsp_datatype_t value_type, int64_t n,
                         const int64_t *d_idx, const void *d_src, void *d_dst);

/* Schedule facts of the current schedule of `mat` (no cuSPARSE
 * counterpart; for byte accounting): its tile count, and how many stored
 * entries it reads through 16-bit column offsets (2 B each instead of the
 * 4-B colidx: tiles whose columns span < 65536; the rest read colidx).
 * NOT_INITIALIZED before the first bufferSize / preprocess / SpMV. */
rsp_status_t rsp_spmv_plan_info(rsp_spmat_t mat, int64_t *tiles, int64_t *entries_16bit);

/* Overlap of the halo exchange with the SpMV. Columns [0, ncols_local) of
 * `mat` are the rank's own x entries, the others arrive with the exchange.
 * Invalidates the schedule (the next bufferSize / preprocess / SpMV re-plans
 * it, and batches holding the old one become stale): the schedule then
 * puts the tiles that read own columns only first. rsp_spmv_part runs
 * part 1 = those interior tiles (launch it while the exchange is in flight),
 * part 2 = the remaining tiles, long rows included; part 0 = everything
 * (== rsp_spmv). Part 1 followed by part 2 gives y bit for bit equal to
 * rsp_spmv. beta must be 0 for parts 1 and 2. */
rsp_status_t rsp_spmat_set_local_cols(rsp_spmat_t mat, int64_t ncols_local);
rsp_status_t rsp_spmv_part(rsp_handle_t handle, const void *alpha, rsp_spmat_t mat,
                           const void *d_x, const void *beta, void *d_y,
                           rsp_datatype_t compute_type, void *d_buffer, int part);

/* Batched SpMV: y_j = alpha*A_j*x_j + beta*y_j for `count` independent
 * matrices of one compute type, as ONE kernel launch per 32 matrices (rows
 * longer than a tile are finished inside it by their last-arriving chunk).
 * No cuSPARSE counterpart: the reference calls cusparseSpMV once per matrix
 * (GPU/spmv.cu:179-186); this is the same product per matrix, bit for bit
 * equal to rsp_spmv / rsp_spmv_part on each, without the per-launch ramp and
 * drain. `part` selects the schedule part of every matrix as rsp_spmv_part
 * (0 = whole product). Create records the pointers (x_j, y_j stay valid
 * until destroy) and plans the batch's own tiling of every matrix (full tiles
 * once the launch fills the chip; a matrix without a schedule is planned
 * first, its long-row partials stay in its schedule, so a matrix may appear
 * once per batch: INVALID_VALUE otherwise). d_buffers is unused (may be
 * NULL). Run fails with INVALID_VALUE if a matrix has been re-planned or
 * given other values (rsp_csr_set_values) since. Create and destroy are
 * host-blocking. */
rsp_status_t rsp_spmv_batch_create(rsp_handle_t handle, int count, const rsp_spmat_t *mats,
                                   const void *const *d_x, void *const *d_y,
                                   void *const *d_buffers, rsp_datatype_t compute_type,
                                   int part, rsp_spmv_batch_t *batch);
rsp_status_t rsp_spmv_batch_run(rsp_handle_t handle, rsp_spmv_batch_t batch, const void *alpha,
                                const void *beta);
rsp_status_t rsp_spmv_batch_destroy(rsp_spmv_batch_t batch);
/* rsp_spmv_plan_info of a batch's own schedule (its part of every matrix):
 * tiles of all its launches, and the entries they read through 16-bit
 * column offsets. */
rsp_status_t rsp_spmv_batch_info(rsp_spmv_batch_t batch, int64_t *tiles, int64_t *entries_16bit);

/* Number of dependency levels found by the analysis (L DAG, L^T DAG). */
rsp_status_t rsp_ilu0_levels(rsp_ilu0_info_t info, int *levels_lower, int *levels_upper);
/* Extension (round 6): the blocks of the block-inverse solve the analysis
 * planned for the L and L^T solves (0: that solve is level-scheduled). Deep
 * DAGs (<= 32 rows per level on average; RSP_ILU_BLOCKS=1 / 0 at analysis
 * time forces it on / off) are solved block by block, each row's unknown
 * written as a combination of its block's right-hand sides and of earlier
 * blocks' unknowns: same unknowns, rounding of that order (restated in the
 * oracle), within SURVEY 8c's tolerance of the reference's order. */
rsp_status_t rsp_ilu0_solve_blocks(rsp_ilu0_info_t info, int *blocks_lower, int *blocks_upper);

/* Tests and profiling (no cuSPARSE counterpart, no device needed): the host
 * phases of rsp_ilu0_analysis on HOST arrays (base 0) — validation, levels,
 * symbolic factor, factor and solve plans. Returns the level counts, a 64-bit
 * digest of every array built (equal to rsp_ilu0_plan_digest of a device
 * analysis of the same pattern, whatever runs where) and, if phase_ms is not
 * NULL, the wall time of its 6 phases in ms. Same status codes as the
 * analysis (INVALID_VALUE for a malformed or unsorted pattern). */
rsp_status_t rsp_ilu0_analysis_host(int n, const int *row_offsets, const int *col_ind,
                                    int *levels_lower, int *levels_upper, uint64_t *digest,
                                    double *phase_ms);
/* Tests (no cuSPARSE counterpart, no device needed): the SpMV schedule
 * rsp_spmv_buffer_size builds (tiles, 16-bit column offsets, staged tiles'
 * column runs) for HOST arrays (base 0, m rows, compute type fp64 / fp32),
 * checked for consistency: every entry of a 16-bit tile decodes to its own
 * column (cbase + offset, or the staged tile's runs at its slot index), every
 * staged tile's runs are ascending and within its slot and run caps. Returns
 * the tile count, the entries read through 16-bit values and, of those, the
 * entries of staged tiles; INTERNAL_ERROR if a check fails. */
rsp_status_t rsp_spmv_plan_host(int m, const int *row_offsets, const int *col_ind, int64_t nnz,
                                rsp_datatype_t compute_type, int64_t *tiles, int64_t *entries_16bit,
                                int64_t *entries_staged);
/* The digest of the plan an rsp_ilu0_analysis built (see above); computed
 * only when the environment sets RSP_ILU_DIGEST=1 at analysis time
 * (INVALID_VALUE otherwise). */
rsp_status_t rsp_ilu0_plan_digest(rsp_ilu0_info_t info, uint64_t *digest);

#ifdef __cplusplus
}
#endif

#endif /* RSP_H */
