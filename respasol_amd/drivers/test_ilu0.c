/*
 * test_ilu0.c — GPU ILU(0) factor + triangular-solve driver, drop-in for
 * ReSpaSol's GPU/ilu0.cu (built as `test_ilu0`, also installed as `ilu0`,
 * the name GPU/run_ilu0.sh:12,21 calls).
 *
 *   test_ilu0 <A.mtx | surrogate:NAME[@scale]> [--prec=fp64|fp32] [--ftz]
 *             [--dump=FILE] [--true-lu] [--full-symmetric]
 *
 * Flow (GPU/ilu0.cu:29-342): load with outputbase 0 (:42-44); fp32 demotion
 * under --prec=fp32 (`#define FLOAT`, :55-63); x = 1 (:63,74); H2D;
 * bufferSize x3 (:165-194); [timed "Symbolic"] ILU analysis (:196-217);
 * structural zero pivot -> "A(%d,%d) is missing" and exit 0 (:221-226);
 * the two trsv analyses, untimed (:228-252);
 * [timed "Numeric"] factorisation (:257-275); numerical zero pivot ->
 * "L(%d,%d) is zero" and exit 0 (:278-282); [timed "Solve"] L z = x then
 * L^T y = z with the unit-lower descriptor (:284-310 — the reference never
 * applies U); the 5-line report of :312-317.
 * Symbolic is wall-clock (the analysis here is host-side and blocking);
 * Numeric and Solve are event pairs on the stream, as in the reference.
 * Extensions: --dump writes y (binary, value type) for verification;
 * --true-lu solves U y = z instead of L^T y = z (desc_U, :136-141).
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "drv_common.h"
#include "rsp.h"
#include "rsp_host.h"

#define hipErrCheck(stat)                                                                       \
    do {                                                                                        \
        hipError_t s_ = (stat);                                                                 \
        if (s_ != hipSuccess)                                                                   \
            fprintf(stderr, "HIP Error: %s %s %d\n", hipGetErrorString(s_), __FILE__, __LINE__); \
    } while (0)
#define rspErrCheck(stat)                                                                       \
    do {                                                                                        \
        rsp_status_t s_ = (stat);                                                               \
        if (s_ != RSP_STATUS_SUCCESS && s_ != RSP_STATUS_ZERO_PIVOT)                            \
            fprintf(stderr, "RSP Error: %d %s %d\n", (int)s_, __FILE__, __LINE__);              \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr,
                "-- Usage examples --\n"
                "  %s inline_1.mtx type: run with inline_1 matrix in matrix market format\n",
                argv[0]);
        return -1;
    }
    const char *prec = drv_flag(argc, argv, 2, "prec");
    const char *dump = drv_flag(argc, argv, 2, "dump");
    int fp32 = prec && strcmp(prec, "fp32") == 0;
    int ftz = drv_flag(argc, argv, 2, "ftz") != NULL;
    int true_lu = drv_flag(argc, argv, 2, "true-lu") != NULL;
    int fullsym = drv_flag(argc, argv, 2, "full-symmetric") != NULL;

    CSR A;
    if (!drv_load(argv[1], &A, 0, fullsym)) {
        fprintf(stderr, "Error: failed to load %s\n", argv[1]);
        return 1;
    }
    const int n = A.n, nnz_s = A.rowptr[A.m];
    const size_t vsz = fp32 ? sizeof(float) : sizeof(double);
    const rsp_datatype_t dt = fp32 ? RSP_R_32F : RSP_R_64F;
    void *hv = malloc((size_t)(nnz_s ? nnz_s : 1) * vsz);
    void *hx = malloc((size_t)(n ? n : 1) * vsz);
    for (int k = 0; k < nnz_s; k++) {
        if (fp32)
            ((float *)hv)[k] = (float)A.values[k];
        else
            ((double *)hv)[k] = A.values[k];
    }
    for (int i = 0; i < n; i++) {
        if (fp32)
            ((float *)hx)[i] = 1.0f;
        else
            ((double *)hx)[i] = 1.0;
    }
    double alpha64 = 1.0;
    float alpha32 = 1.0f;
    const void *alpha = fp32 ? (const void *)&alpha32 : (const void *)&alpha64;

    rsp_handle_t handle = NULL;
    rspErrCheck(rsp_create(&handle));
    rspErrCheck(rsp_set_ftz(handle, ftz));

    int *d_rp = NULL, *d_ci = NULL;
    void *d_v = NULL, *d_x = NULL, *d_y = NULL, *d_z = NULL;
    hipErrCheck(hipMalloc((void **)&d_rp, ((size_t)n + 1) * sizeof(int)));
    hipErrCheck(hipMalloc((void **)&d_ci, (size_t)(nnz_s ? nnz_s : 1) * sizeof(int)));
    hipErrCheck(hipMalloc(&d_v, (size_t)(nnz_s ? nnz_s : 1) * vsz));
    hipErrCheck(hipMalloc(&d_x, (size_t)(n ? n : 1) * vsz));
    hipErrCheck(hipMalloc(&d_y, (size_t)(n ? n : 1) * vsz));
    hipErrCheck(hipMalloc(&d_z, (size_t)(n ? n : 1) * vsz));
    hipErrCheck(hipMemcpy(d_rp, A.rowptr, ((size_t)n + 1) * sizeof(int), hipMemcpyHostToDevice));
    hipErrCheck(hipMemcpy(d_ci, A.colidx, (size_t)nnz_s * sizeof(int), hipMemcpyHostToDevice));
    hipErrCheck(hipMemcpy(d_v, hv, (size_t)nnz_s * vsz, hipMemcpyHostToDevice));
    hipErrCheck(hipMemcpy(d_x, hx, (size_t)n * vsz, hipMemcpyHostToDevice));

    rsp_ilu0_info_t info = NULL;
    rspErrCheck(rsp_create_ilu0_info(&info));
    size_t bufsz = 0;
    rspErrCheck(rsp_ilu0_buffer_size(handle, n, A.nnz, dt, info, &bufsz));

    hipEvent_t start, stop;
    hipErrCheck(hipEventCreate(&start));
    hipErrCheck(hipEventCreate(&stop));

    double t0 = drv_wtime();
    rspErrCheck(rsp_ilu0_analysis(handle, n, A.nnz, d_rp, d_ci, info));
    float time_symbolic = (float)((drv_wtime() - t0) * 1e3);

    int structural_zero = -1;
    if (rsp_ilu0_zero_pivot(handle, info, &structural_zero) == RSP_STATUS_ZERO_PIVOT) {
        printf("A(%d,%d) is missing\n", structural_zero, structural_zero);
        return 0;
    }
    /* the two csrsv2_analysis calls (:228-252), untimed as there */
    rspErrCheck(rsp_trsv_analysis(handle, RSP_OPERATION_NON_TRANSPOSE, info));
    rspErrCheck(rsp_trsv_analysis(handle, RSP_OPERATION_TRANSPOSE, info));

    hipEventRecord(start, NULL);
    rspErrCheck(rsp_ilu0_factor(handle, info, dt, d_v));
    hipEventRecord(stop, NULL);
    hipEventSynchronize(stop);
    float time_numeric = 0.0f;
    hipEventElapsedTime(&time_numeric, start, stop);

    int numerical_zero = -1;
    rsp_status_t st = rsp_ilu0_zero_pivot(handle, info, &numerical_zero);
    if (st == RSP_STATUS_ZERO_PIVOT) {
        printf("L(%d,%d) is zero\n", numerical_zero, numerical_zero);
        return 0;
    }
    if (st != RSP_STATUS_SUCCESS) {  /* e.g. EXECUTION_FAILED: the factor is not valid */
        fprintf(stderr, "Error: ILU(0) factorisation failed (%s)\n", rsp_get_error_string(st));
        return 1;
    }

    hipEventRecord(start, NULL);
    rspErrCheck(rsp_trsv_lower_unit(handle, RSP_OPERATION_NON_TRANSPOSE, alpha, info, dt, d_v, d_x, d_z));
    if (true_lu)
        rspErrCheck(rsp_trsv_upper(handle, alpha, info, dt, d_v, d_z, d_y));
    else
        rspErrCheck(rsp_trsv_lower_unit(handle, RSP_OPERATION_TRANSPOSE, alpha, info, dt, d_v, d_z, d_y));
    hipEventRecord(stop, NULL);
    hipEventSynchronize(stop);
    float time_solve = 0.0f;
    hipEventElapsedTime(&time_solve, start, stop);
    /* the solves' status (csrsv2_zeroPivot), outside the timed region */
    const int kinds[2] = {RSP_TRSV_L, true_lu ? RSP_TRSV_U : RSP_TRSV_LT};
    for (int q = 0; q < 2; q++) {
        int pos = -1;
        st = rsp_trsv_zero_pivot(handle, info, kinds[q], &pos);
        if (st != RSP_STATUS_SUCCESS) {
            fprintf(stderr, "Error: triangular solve %d failed (%s)\n", kinds[q], rsp_get_error_string(st));
            return 1;
        }
    }

    printf(fp32 ? "SINGLE PRECISION SOLVE IN  MILLISECONDS\n " : "DOUBLE PRECISION SOLVE IN  MILLISECONDS\n ");
    printf("Symbolic = %f\n Numeric = %f \n Symbolic+ Numeric = %f\n Solve = %f\n", time_symbolic,
           time_numeric, time_symbolic + time_numeric, time_solve);

    if (dump && *dump) {
        void *hy = malloc((size_t)(n ? n : 1) * vsz);
        hipErrCheck(hipMemcpy(hy, d_y, (size_t)n * vsz, hipMemcpyDeviceToHost));
        FILE *fp = fopen(dump, "wb");
        if (fp) {
            fwrite(hy, vsz, (size_t)n, fp);
            fclose(fp);
        }
        free(hy);
    }

    hipEventDestroy(start);
    hipEventDestroy(stop);
    rsp_destroy_ilu0_info(info);
    rsp_destroy(handle);
    hipFree(d_rp);
    hipFree(d_ci);
    hipFree(d_v);
    hipFree(d_x);
    hipFree(d_y);
    hipFree(d_z);
    free(hv);
    free(hx);
    rsp_csr_free(&A);
    return 0;
}
