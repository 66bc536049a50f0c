/*
 * host_util.c — nnz-balanced row partitioning for the multi-GPU SpMV
 *  and the host CSR SpMV the drivers use for their "Error ="
 * verification line (the role of MKL's sequential mkl_sparse_?_mv in
 * GPU/spmv.cu:221-260; the MKL library itself is not part of this build).
 */
#include "rsp_host.h"

/* bounds[p] = lower_bound(rowptr[0..m], rowptr[0] + p*nnz/P): rows are split
 * where the running nnz crosses each 1/P quantile; empty tail ranges are
 * allowed (P > m). */
int rsp_partition_rows(const int *rowptr, int m, int parts, int *bounds) {
    if (!rowptr || !bounds || m < 0 || parts < 1) return -1;
    long long base = rowptr[0];
    long long nnz = (long long)rowptr[m] - base;
    bounds[0] = 0;
    for (int p = 1; p < parts; p++) {
        long long target = base + (nnz * p) / parts;
        int lo = bounds[p - 1], hi = m;
        while (lo < hi) {
            int mid = lo + (hi - lo) / 2;
            if ((long long)rowptr[mid] < target)
                lo = mid + 1;
            else
                hi = mid;
        }
        bounds[p] = lo;
    }
    bounds[parts] = m;
    return 0;
}

void rsp_host_spmv_f64(int m, const int *rowptr, const int *colidx, const double *vals,
                       const double *x, double *y) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < m; i++) {
        double s = 0.0;
        for (int k = rowptr[i]; k < rowptr[i + 1]; k++) s += vals[k] * x[colidx[k]];
        y[i] = s;
    }
}

void rsp_host_spmv_f32(int m, const int *rowptr, const int *colidx, const float *vals,
                       const float *x, float *y) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < m; i++) {
        float s = 0.0f;
        for (int k = rowptr[i]; k < rowptr[i + 1]; k++) s += vals[k] * x[colidx[k]];
        y[i] = s;
    }
}
