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

/* Padded all-gather layout of a row-partitioned x: slice p's
 * entries x[bounds[p] .. bounds[p+1]) sit at x_pad[p*chunk ..), chunk = the
 * largest slice, so one equal-count all-gather (ncclAllGather, sendcount =
 * chunk) reassembles x on every rank. */
int rsp_padded_chunk(const int *bounds, int parts) {
    if (!bounds || parts < 1) return -1;
    int chunk = 0;
    for (int p = 0; p < parts; p++) {
        const int len = bounds[p + 1] - bounds[p];
        if (len < 0) return -1;
        if (len > chunk) chunk = len;
    }
    return chunk;
}

/* colidx_out[k] = padded position of global column colidx_in[k]: the slice
 * p owning it (bounds[p] <= c < bounds[p+1], by binary search) gives
 * p*chunk + (c - bounds[p]). In place allowed. */
int rsp_remap_cols_padded(int64_t nnz, const int *colidx_in, const int *bounds, int parts, int chunk,
                          int *colidx_out) {
    if (nnz < 0 || (nnz > 0 && (!colidx_in || !colidx_out)) || !bounds || parts < 1 || chunk < 0)
        return -1;
    if ((int64_t)parts * chunk > 2147483647LL) return -1;
    const int n = bounds[parts];
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int64_t k = 0; k < nnz; k++) {
        const int c = colidx_in[k];
        if (c < 0 || c >= n) {
            bad = 1;
            continue;
        }
        int lo = 0, hi = parts - 1;  /* last p with bounds[p] <= c */
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (bounds[mid] <= c)
                lo = mid;
            else
                hi = mid - 1;
        }
        colidx_out[k] = lo * chunk + (c - bounds[lo]);
    }
    return bad ? -1 : 0;
}
