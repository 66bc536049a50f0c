/*
 * test_spmv.c — GPU CSR SpMV driver, drop-in for ReSpaSol's GPU/spmv.cu
 * (built as `test_spmv`, also installed as `spmv`, the name the sweep scripts
 * call: GPU/run_spmv.sh:12,21).
 *
 *   test_spmv <A.mtx | surrogate:NAME[@scale]> [--prec=fp64|fp32|both] [--ftz]
 *             [--x=ones|dlarnv] [--reps=50] [--batched] [--stats] [--full-symmetric]
 *             [--ref-sequence | --preprocess] [--rep-times] [--ngpu=N]
 *
 * Default output is the reference's, byte for byte in format
 * (GPU/spmv.cu:202-207,260):
 *   DOUBLE PRECISION SPMV solve time (microseconds) = %f
 *   Error= %e
 * Flow (GPU/spmv.cu:32-284): load with outputbase 0 (:45-47); fp32 demotion
 * on the host under --prec=fp32 (the reference's `#define FLOAT`, :60-71);
 * x = 1 (:71,83); H2D; rsp_create/create_csr/spmv_buffer_size
 * (cusparseCreate/CreateCsr/SpMV_bufferSize, :122-164) and the workspace
 * malloc, with no other call before the timed loop (--ref-sequence, the
 * default: the library builds its schedule at bufferSize time, so timed call
 * 0 plans nothing; --preprocess adds an explicit rsp_spmv_preprocess, the
 * cuSPARSE-12 SpMV_preprocess step the reference does not have); 50 calls each
 * bracketed by an event pair and synchronised (:174-195), mean in
 * microseconds; D2H; host CSR SpMV in the same precision as the check
 * (MKL's role, :221-254); Error = sum|ref - y| / n (:256-260).
 * Deliberate differences: a loader failure exits non-zero instead of running
 * on garbage; rows = A.m (the reference uses A.n for both dimensions, :50-51,
 * identical for the square matrices it targets); --batched also reports one
 * event pair around all calls; --stats prints GFLOP/s and algorithmic GB/s.
 *
 * --ngpu=N (the reference is single-GPU): the rows are split
 * into N nnz-balanced contiguous slices (rsp_partition_rows), one per GPU of
 * this node, driven from this one host thread over an RCCL clique
 * (ncclCommInitAll: no extra processes, no re-exec). x lives on every GPU in
 * the padded all-gather layout (slice p at [p*chunk, p*chunk + m_p),
 * rsp_padded_chunk / rsp_remap_cols_padded remap each slice's columns once),
 * so one timed call is: ncclAllGather of the x slices over xGMI (in place,
 * grouped over the GPUs), then y_p = A_p x on each GPU. Reported: the
 * reference's line with the max-over-GPUs mean call time, an NGPU line with
 * the exchange-only and SpMV-only times, and Error= over the reassembled y.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <rccl/rccl.h>
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

static int cmp_float(const void *a, const void *b) {
    const float x = *(const float *)a, y = *(const float *)b;
    return (x > y) - (x < y);
}

static int run(const CSR *A, int fp32, int ftz, int use_dlarnv, int reps, int batched, int stats,
               int preprocess, int rep_times) {
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
    if (preprocess)
        rspErrCheck(rsp_spmv_preprocess(handle, RSP_OPERATION_NON_TRANSPOSE, alpha, matA, d_x, beta,
                                        d_y, dt, d_buf));
    float *rep_ms = (float *)malloc((size_t)reps * sizeof(float));

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
        if (rep_ms) rep_ms[r] = ms;
    }
    printf(fp32 ? "SINGLE PRECISION SPMV " : "DOUBLE PRECISION SPMV ");
    printf("solve time (microseconds) = %f\n", (sum_ms / reps) * 1000);
    if (rep_times && rep_ms) {  /* rep 0 against the steady state */
        const float first = rep_ms[0];
        qsort(rep_ms, (size_t)reps, sizeof(float), cmp_float);
        printf("REPS first_us=%f median_us=%f mean_us=%f max_us=%f\n", first * 1000,
               rep_ms[reps / 2] * 1000, (sum_ms / reps) * 1000, rep_ms[reps - 1] * 1000);
    }
    free(rep_ms);
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

#define ncclErrCheck(stat)                                                                      \
    do {                                                                                        \
        ncclResult_t s_ = (stat);                                                               \
        if (s_ != ncclSuccess) {                                                                \
            fprintf(stderr, "RCCL Error: %s %s %d\n", ncclGetErrorString(s_), __FILE__, __LINE__); \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

#define RSP_MAX_GPUS 64

/* Row-partitioned SpMV over `ngpu` GPUs of this node (see the header). */
static int run_multi(const CSR *A, int fp32, int ftz, int use_dlarnv, int reps, int ngpu) {
    const int m = A->m, n = A->n;
    const size_t vsz = fp32 ? sizeof(float) : sizeof(double);
    int ndev = 0;
    hipErrCheck(hipGetDeviceCount(&ndev));
    if (ngpu < 1 || ngpu > RSP_MAX_GPUS || ngpu > ndev) {
        fprintf(stderr, "Error: --ngpu=%d but %d GPU(s) visible\n", ngpu, ndev);
        return 1;
    }
    if (m != n) {
        fprintf(stderr, "Error: --ngpu needs a square matrix (x is partitioned like the rows)\n");
        return 1;
    }
    int bounds[RSP_MAX_GPUS + 1];
    if (rsp_partition_rows(A->rowptr, m, ngpu, bounds) != 0) return 1;
    const int chunk = rsp_padded_chunk(bounds, ngpu);
    const int nnz_s = A->rowptr[m];
    int *ci_pad = (int *)malloc((size_t)(nnz_s ? nnz_s : 1) * sizeof(int));
    double *x64 = (double *)malloc((size_t)(n ? n : 1) * sizeof(double));
    void *hv = malloc((size_t)(nnz_s ? nnz_s : 1) * vsz);
    void *hxp = calloc((size_t)ngpu * (chunk ? chunk : 1), vsz);
    void *hy = malloc((size_t)(m ? m : 1) * vsz);
    void *href = malloc((size_t)(m ? m : 1) * vsz);
    void *hx = malloc((size_t)(n ? n : 1) * vsz);
    if (!ci_pad || !x64 || !hv || !hxp || !hy || !href || !hx) {
        fprintf(stderr, "Failed to allocate memory\n");
        return 1;
    }
    if (chunk < 0 || rsp_remap_cols_padded(nnz_s, A->colidx, bounds, ngpu, chunk, ci_pad) != 0) {
        fprintf(stderr, "Error: column index out of range\n");
        return 1;
    }
    if (use_dlarnv) {
        int seed[4] = {0, 0, 0, 1};
        rsp_dlarnv(1, seed, n, x64);
    } else {
        for (int i = 0; i < n; i++) x64[i] = 1.0;
    }
    for (int k = 0; k < nnz_s; k++) {
        if (fp32) ((float *)hv)[k] = (float)A->values[k];
        else ((double *)hv)[k] = A->values[k];
    }
    for (int p = 0; p < ngpu; p++)  /* every GPU starts from its own slice of x only */
        for (int i = bounds[p]; i < bounds[p + 1]; i++) {
            const size_t at = (size_t)p * chunk + (size_t)(i - bounds[p]);
            if (fp32) ((float *)hxp)[at] = (float)x64[i], ((float *)hx)[i] = (float)x64[i];
            else ((double *)hxp)[at] = x64[i], ((double *)hx)[i] = x64[i];
        }

    const rsp_datatype_t dt = fp32 ? RSP_R_32F : RSP_R_64F;
    const ncclDataType_t nt = fp32 ? ncclFloat : ncclDouble;
    double alpha64 = 1.0, beta64 = 0.0;
    float alpha32 = 1.0f, beta32 = 0.0f;
    const void *alpha = fp32 ? (const void *)&alpha32 : (const void *)&alpha64;
    const void *beta = fp32 ? (const void *)&beta32 : (const void *)&beta64;
    int devs[RSP_MAX_GPUS];
    ncclComm_t comms[RSP_MAX_GPUS];
    hipStream_t streams[RSP_MAX_GPUS];
    rsp_handle_t handles[RSP_MAX_GPUS];
    rsp_spmat_t mats[RSP_MAX_GPUS];
    int *d_rp[RSP_MAX_GPUS], *d_ci[RSP_MAX_GPUS];
    void *d_v[RSP_MAX_GPUS], *d_x[RSP_MAX_GPUS], *d_y[RSP_MAX_GPUS], *d_buf[RSP_MAX_GPUS];
    hipEvent_t ev0[RSP_MAX_GPUS], ev1[RSP_MAX_GPUS], ev2[RSP_MAX_GPUS];
    for (int p = 0; p < ngpu; p++) {
        devs[p] = p;
        const int r0 = bounds[p], mp = bounds[p + 1] - r0;
        const int k0 = A->rowptr[r0], np_ = A->rowptr[bounds[p + 1]] - k0;
        int *rp = (int *)malloc(((size_t)mp + 1) * sizeof(int));
        if (!rp) return 1;
        for (int i = 0; i <= mp; i++) rp[i] = A->rowptr[r0 + i] - k0;  /* rebased slice */
        hipErrCheck(hipSetDevice(p));
        hipErrCheck(hipStreamCreateWithFlags(&streams[p], hipStreamNonBlocking));
        hipErrCheck(hipMalloc((void **)&d_rp[p], ((size_t)mp + 1) * sizeof(int)));
        hipErrCheck(hipMalloc((void **)&d_ci[p], (size_t)(np_ ? np_ : 1) * sizeof(int)));
        hipErrCheck(hipMalloc(&d_v[p], (size_t)(np_ ? np_ : 1) * vsz));
        hipErrCheck(hipMalloc(&d_x[p], (size_t)ngpu * (chunk ? chunk : 1) * vsz));
        hipErrCheck(hipMalloc(&d_y[p], (size_t)(mp ? mp : 1) * vsz));
        hipErrCheck(hipMemcpy(d_rp[p], rp, ((size_t)mp + 1) * sizeof(int), hipMemcpyHostToDevice));
        hipErrCheck(hipMemcpy(d_ci[p], ci_pad + k0, (size_t)np_ * sizeof(int), hipMemcpyHostToDevice));
        hipErrCheck(hipMemcpy(d_v[p], (char *)hv + (size_t)k0 * vsz, (size_t)np_ * vsz, hipMemcpyHostToDevice));
        /* only this GPU's own slice is valid before the first exchange */
        hipErrCheck(hipMemset(d_x[p], 0xff, (size_t)ngpu * (chunk ? chunk : 1) * vsz));
        hipErrCheck(hipMemcpy((char *)d_x[p] + (size_t)p * chunk * vsz, (char *)hxp + (size_t)p * chunk * vsz,
                              (size_t)mp * vsz, hipMemcpyHostToDevice));
        free(rp);
        rspErrCheck(rsp_create(&handles[p]));
        rspErrCheck(rsp_set_stream(handles[p], streams[p]));
        rspErrCheck(rsp_set_ftz(handles[p], ftz));
        rspErrCheck(rsp_create_csr(&mats[p], mp, (int64_t)ngpu * chunk, np_, d_rp[p], d_ci[p], d_v[p], dt));
        size_t bufsz = 0;
        rspErrCheck(rsp_spmv_buffer_size(handles[p], RSP_OPERATION_NON_TRANSPOSE, alpha, mats[p], beta, dt,
                                         &bufsz));
        hipErrCheck(hipMalloc(&d_buf[p], bufsz ? bufsz : 1));
        hipErrCheck(hipEventCreate(&ev0[p]));
        hipErrCheck(hipEventCreate(&ev1[p]));
        hipErrCheck(hipEventCreate(&ev2[p]));
        hipErrCheck(hipDeviceSynchronize());
    }
    ncclErrCheck(ncclCommInitAll(comms, ngpu, devs));

    /* one call: all-gather x (grouped: one host thread drives every GPU),
     * then the local SpMVs; event pairs per GPU, synchronised per call like
     * the reference's loop (GPU/spmv.cu:174-195), max over GPUs */
    double sum_ms = 0.0, sum_ex = 0.0, sum_mv = 0.0;
    for (int r = -1; r < reps; r++) {  /* r = -1: untimed warm-up (RCCL connection setup) */
        for (int p = 0; p < ngpu; p++) {
            hipErrCheck(hipSetDevice(p));
            hipErrCheck(hipEventRecord(ev0[p], streams[p]));
        }
        ncclErrCheck(ncclGroupStart());
        for (int p = 0; p < ngpu; p++)
            ncclErrCheck(ncclAllGather((char *)d_x[p] + (size_t)p * chunk * vsz, d_x[p], (size_t)chunk, nt,
                                       comms[p], streams[p]));
        ncclErrCheck(ncclGroupEnd());
        for (int p = 0; p < ngpu; p++) {
            hipErrCheck(hipSetDevice(p));
            hipErrCheck(hipEventRecord(ev1[p], streams[p]));
            rspErrCheck(rsp_spmv(handles[p], RSP_OPERATION_NON_TRANSPOSE, alpha, mats[p], d_x[p], beta, d_y[p],
                                 dt, d_buf[p]));
            hipErrCheck(hipEventRecord(ev2[p], streams[p]));
        }
        float tot = 0.0f, ex = 0.0f, mv = 0.0f;
        for (int p = 0; p < ngpu; p++) {
            hipErrCheck(hipSetDevice(p));
            hipErrCheck(hipEventSynchronize(ev2[p]));
            float a = 0.0f, b = 0.0f, c = 0.0f;
            hipEventElapsedTime(&a, ev0[p], ev2[p]);
            hipEventElapsedTime(&b, ev0[p], ev1[p]);
            hipEventElapsedTime(&c, ev1[p], ev2[p]);
            if (a > tot) tot = a;
            if (b > ex) ex = b;
            if (c > mv) mv = c;
        }
        if (r >= 0) sum_ms += tot, sum_ex += ex, sum_mv += mv;
    }
    printf(fp32 ? "SINGLE PRECISION SPMV " : "DOUBLE PRECISION SPMV ");
    printf("solve time (microseconds) = %f\n", (sum_ms / reps) * 1000);
    {
        const double us = (sum_ms / reps) * 1000;
        printf("NGPU=%d exchange=allgather chunk=%d allgather_us=%f spmv_us=%f GFLOPs=%f\n", ngpu, chunk,
               (sum_ex / reps) * 1000, (sum_mv / reps) * 1000, 2.0 * nnz_s / (us * 1e3));
    }
    for (int p = 0; p < ngpu; p++) {  /* reassemble y in global row order */
        hipErrCheck(hipSetDevice(p));
        hipErrCheck(hipMemcpy((char *)hy + (size_t)bounds[p] * vsz, d_y[p],
                              (size_t)(bounds[p + 1] - bounds[p]) * vsz, hipMemcpyDeviceToHost));
    }
    double error = 0.0;
    if (fp32) {
        rsp_host_spmv_f32(m, A->rowptr, A->colidx, (const float *)hv, (const float *)hx, (float *)href);
        for (int i = 0; i < m; i++) error += fabs((double)((float *)href)[i] - (double)((float *)hy)[i]);
    } else {
        rsp_host_spmv_f64(m, A->rowptr, A->colidx, (const double *)hv, (const double *)hx, (double *)href);
        for (int i = 0; i < m; i++) error += fabs(((double *)href)[i] - ((double *)hy)[i]);
    }
    printf("Error= %e\n", n ? error / n : 0.0);
    for (int p = 0; p < ngpu; p++) {
        hipErrCheck(hipSetDevice(p));
        ncclCommDestroy(comms[p]);
        rsp_destroy_spmat(mats[p]);
        rsp_destroy(handles[p]);
        hipEventDestroy(ev0[p]);
        hipEventDestroy(ev1[p]);
        hipEventDestroy(ev2[p]);
        hipFree(d_rp[p]);
        hipFree(d_ci[p]);
        hipFree(d_v[p]);
        hipFree(d_x[p]);
        hipFree(d_y[p]);
        hipFree(d_buf[p]);
        hipStreamDestroy(streams[p]);
    }
    hipSetDevice(0);
    free(ci_pad);
    free(x64);
    free(hv);
    free(hxp);
    free(hy);
    free(href);
    free(hx);
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
    int preprocess = drv_flag(argc, argv, 2, "preprocess") != NULL;
    int rep_times = drv_flag(argc, argv, 2, "rep-times") != NULL;
    const char *ngpu_s = drv_flag(argc, argv, 2, "ngpu");
    int ngpu = ngpu_s && *ngpu_s ? atoi(ngpu_s) : 0;
    if (drv_flag(argc, argv, 2, "ref-sequence")) preprocess = 0; /* GPU/spmv.cu:143-195 verbatim */
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
    if (ngpu > 0) { /* row-partitioned over RCCL */
        if (do64) rc |= run_multi(&A, 0, 0, use_dlarnv, reps, ngpu);
        if (do32) rc |= run_multi(&A, 1, ftz, use_dlarnv, reps, ngpu);
    } else {
        if (do64) rc |= run(&A, 0, 0, use_dlarnv, reps, batched, stats, preprocess, rep_times);
        if (do32) rc |= run(&A, 1, ftz, use_dlarnv, reps, batched, stats, preprocess, rep_times);
    }
    rsp_csr_free(&A);
    return rc;
}
