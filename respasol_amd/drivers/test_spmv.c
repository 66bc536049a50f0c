/*
 * test_spmv.c — GPU CSR SpMV driver, drop-in for ReSpaSol's GPU/spmv.cu
 * (built as `test_spmv`, also installed as `spmv`, the name the sweep scripts
 * call: GPU/run_spmv.sh:12,21).
 *
 *   test_spmv <A.mtx | surrogate:NAME[@scale]> [--prec=fp64|fp32|both] [--ftz]
 *             [--x=ones|dlarnv] [--reps=50] [--batched] [--stats] [--full-symmetric]
 *
 * Default output is the reference's, byte for byte in format
 * (GPU/spmv.cu:202-207,260):
 *   DOUBLE PRECISION SPMV solve time (microseconds) = %f
 *   Error= %e
 * Flow (GPU/spmv.cu:32-284): load with outputbase 0 (:45-47); fp32 demotion
 * on the host under --prec=fp32 (the reference's `#define FLOAT`, :60-71);
 * x = 1 (:71,83); H2D; rsp_create/create_csr/spmv_buffer_size
 * (cusparseCreate/CreateCsr/SpMV_bufferSize, :122-164); 50 calls each
 * bracketed by an event pair and synchronised (:174-195), mean in
 * microseconds; D2H; host CSR SpMV in the same precision as the check
 * (MKL's role, :221-254); Error = sum|ref - y| / n (:256-260).
 * Deliberate differences: a loader failure exits non-zero instead of running
 * on garbage; rows = A.m (the reference uses A.n for both dimensions, :50-51,
 * identical for the square matrices it targets); --batched also reports one
 * event pair around all calls; --stats prints GFLOP/s and algorithmic GB/s.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
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
        if (s_ != RSP_STATUS_SUCCESS) fprintf(stderr, "RSP Error: %d %s %d\n", (int)s_, __FILE__, __LINE__); \
    } while (0)

static int run(const CSR *A, int fp32, int ftz, int use_dlarnv, int reps, int batched, int stats) {
    const int m = A->m, n = A->n;
    const int nnz_s = A->rowptr[m];
    const size_t vsz = fp32 ? sizeof(float) : sizeof(double);
    /* host values / vectors in the run's precision */
    void *hv = malloc((size_t)(nnz_s ? nnz_s : 1) * vsz);
    void *hx = malloc((size_t)(n ? n : 1) * vsz);
    void *hy = malloc((size_t)(m ? m : 1) * vsz);
    void *href = malloc((size_t)(m ? m : 1) * vsz);
    double *x64 = (double *)malloc((size_t)(n ? n : 1) * sizeof(double));
    if (!hv || !hx || !hy || !href || !x64) {
        fprintf(stderr, "Failed to allocate memory\n");
        return 1;
    }
    if (use_dlarnv) {
        int seed[4] = {0, 0, 0, 1};
        rsp_dlarnv(1, seed, n, x64);
    } else {
        for (int i = 0; i < n; i++) x64[i] = 1.0;
    }
    for (int k = 0; k < nnz_s; k++) {
        if (fp32)
            ((float *)hv)[k] = (float)A->values[k];
        else
            ((double *)hv)[k] = A->values[k];
    }
    for (int i = 0; i < n; i++) {
        if (fp32)
            ((float *)hx)[i] = (float)x64[i];
        else
            ((double *)hx)[i] = x64[i];
    }

    int *d_rp = NULL, *d_ci = NULL;
    void *d_v = NULL, *d_x = NULL, *d_y = NULL, *d_buf = NULL;
    hipErrCheck(hipMalloc((void **)&d_rp, ((size_t)m + 1) * sizeof(int)));
    hipErrCheck(hipMalloc((void **)&d_ci, (size_t)(nnz_s ? nnz_s : 1) * sizeof(int)));
    hipErrCheck(hipMalloc(&d_v, (size_t)(nnz_s ? nnz_s : 1) * vsz));
    hipErrCheck(hipMalloc(&d_x, (size_t)(n ? n : 1) * vsz));
    hipErrCheck(hipMalloc(&d_y, (size_t)(m ? m : 1) * vsz));
    hipErrCheck(hipMemcpy(d_rp, A->rowptr, ((size_t)m + 1) * sizeof(int), hipMemcpyHostToDevice));
    hipErrCheck(hipMemcpy(d_ci, A->colidx, (size_t)nnz_s * sizeof(int), hipMemcpyHostToDevice));
    hipErrCheck(hipMemcpy(d_v, hv, (size_t)nnz_s * vsz, hipMemcpyHostToDevice));
    hipErrCheck(hipMemcpy(d_x, hx, (size_t)n * vsz, hipMemcpyHostToDevice));

    rsp_handle_t handle = NULL;
    rsp_spmat_t matA = NULL;
    const rsp_datatype_t dt = fp32 ? RSP_R_32F : RSP_R_64F;
    double alpha64 = 1.0, beta64 = 0.0;
    float alpha32 = 1.0f, beta32 = 0.0f;
    const void *alpha = fp32 ? (const void *)&alpha32 : (const void *)&alpha64;
    const void *beta = fp32 ? (const void *)&beta32 : (const void *)&beta64;
    size_t bufsz = 0;
    rspErrCheck(rsp_create(&handle));
    rspErrCheck(rsp_set_ftz(handle, ftz));
    /* the reference hands A.nnz (expanded for symmetric files) to CreateCsr */
    rspErrCheck(rsp_create_csr(&matA, m, n, A->nnz > nnz_s ? A->nnz : nnz_s, d_rp, d_ci, d_v, dt));
    rspErrCheck(rsp_spmv_buffer_size(handle, RSP_OPERATION_NON_TRANSPOSE, alpha, matA, beta, dt, &bufsz));
    hipErrCheck(hipMalloc(&d_buf, bufsz ? bufsz : 1));
    rspErrCheck(rsp_spmv_preprocess(handle, RSP_OPERATION_NON_TRANSPOSE, alpha, matA, d_x, beta,
                                    d_y, dt, d_buf));

    hipEvent_t start, stop;
    hipErrCheck(hipEventCreate(&start));
    hipErrCheck(hipEventCreate(&stop));
    float sum_ms = 0.0f;
    for (int r = 0; r < reps; r++) {
        hipEventRecord(start, NULL);
        rspErrCheck(rsp_spmv(handle, RSP_OPERATION_NON_TRANSPOSE, alpha, matA, d_x, beta, d_y, dt, d_buf));
        hipEventRecord(stop, NULL);
        hipEventSynchronize(stop);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, start, stop);
        sum_ms += ms;
    }
    printf(fp32 ? "SINGLE PRECISION SPMV " : "DOUBLE PRECISION SPMV ");
    printf("solve time (microseconds) = %f\n", (sum_ms / reps) * 1000);
    float batched_ms = 0.0f;
    if (batched) {
        hipEventRecord(start, NULL);
        for (int r = 0; r < reps; r++)
            rsp_spmv(handle, RSP_OPERATION_NON_TRANSPOSE, alpha, matA, d_x, beta, d_y, dt, d_buf);
        hipEventRecord(stop, NULL);
        hipEventSynchronize(stop);
        hipEventElapsedTime(&batched_ms, start, stop);
        printf(fp32 ? "SINGLE PRECISION SPMV " : "DOUBLE PRECISION SPMV ");
        printf("batched time (microseconds) = %f\n", (batched_ms / reps) * 1000);
    }

    hipErrCheck(hipMemcpy(hy, d_y, (size_t)m * vsz, hipMemcpyDeviceToHost));
    double error = 0.0;
    if (fp32) {
        rsp_host_spmv_f32(m, A->rowptr, A->colidx, (const float *)hv, (const float *)hx, (float *)href);
        for (int i = 0; i < m; i++) error += fabs((double)((float *)href)[i] - (double)((float *)hy)[i]);
    } else {
        rsp_host_spmv_f64(m, A->rowptr, A->colidx, (const double *)hv, (const double *)hx, (double *)href);
        for (int i = 0; i < m; i++) error += fabs(((double *)href)[i] - ((double *)hy)[i]);
    }
    printf("Error= %e\n", n ? error / n : 0.0);
    if (stats) {
        double us = batched ? (batched_ms / reps) * 1000 : (sum_ms / reps) * 1000;
        double bytes = (double)(vsz + 4) * nnz_s + 4.0 * (m + 1) + (double)vsz * (n + m);
        printf("STATS m=%d n=%d nnz_s=%d A.nnz=%d us=%f GFLOPs=%f GBs=%f\n", m, n, nnz_s, A->nnz, us,
               2.0 * nnz_s / (us * 1e3), bytes / (us * 1e3));
    }

    hipEventDestroy(start);
    hipEventDestroy(stop);
    rsp_destroy_spmat(matA);
    rsp_destroy(handle);
    hipFree(d_rp);
    hipFree(d_ci);
    hipFree(d_v);
    hipFree(d_x);
    hipFree(d_y);
    hipFree(d_buf);
    free(hv);
    free(hx);
    free(hy);
    free(href);
    free(x64);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr,
                "-- Usage examples --\n"
                "  %s inline_1.mtx type: run with inline_1 matrix in matrix market format\n",
                argv[0]);
        return -1;
    }
    const char *prec = drv_flag(argc, argv, 2, "prec");
    const char *xs = drv_flag(argc, argv, 2, "x");
    const char *reps_s = drv_flag(argc, argv, 2, "reps");
    int ftz = drv_flag(argc, argv, 2, "ftz") != NULL;
    int batched = drv_flag(argc, argv, 2, "batched") != NULL;
    int stats = drv_flag(argc, argv, 2, "stats") != NULL;
    int fullsym = drv_flag(argc, argv, 2, "full-symmetric") != NULL;
    int reps = reps_s && *reps_s ? atoi(reps_s) : 50;
    if (reps < 1) reps = 1;
    int use_dlarnv = xs && strcmp(xs, "dlarnv") == 0;
    int do64 = 1, do32 = 0;
    if (prec && strcmp(prec, "fp32") == 0) do64 = 0, do32 = 1;
    if (prec && strcmp(prec, "both") == 0) do64 = 1, do32 = 1;

    CSR A;
    if (!drv_load(argv[1], &A, 0, fullsym)) {
        fprintf(stderr, "Error: failed to load %s\n", argv[1]);
        return 1;
    }
    int rc = 0;
    if (do64) rc |= run(&A, 0, 0, use_dlarnv, reps, batched, stats);
    if (do32) rc |= run(&A, 1, ftz, use_dlarnv, reps, batched, stats);
    rsp_csr_free(&A);
    return rc;
}
