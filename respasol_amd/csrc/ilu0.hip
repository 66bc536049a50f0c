// ilu0.hip — level-scheduled ILU(0) factorisation and unit-lower triangular
// solves for gfx950, replacing cusparse?csrilu02 and cusparse?csrsv2_solve
// (GPU/ilu0.cu:257-310).
//
// The analysis (rsp_ilu0_analysis, host) groups rows into dependency levels:
// row i depends on every row k < i with a_ik in the pattern (factor and
// L-solve), and for L^T on every row j > i with l_ji in the pattern. Rows of
// one level are independent; one kernel launch per level (the kernel
// boundary is the inter-level barrier).
//
// Arithmetic (identical in the CPU oracle, so results are bitwise equal):
//   factor, row i, k ascending over its lower entries:
//       l_ik = a_ik / u_kk;  a_ij = fma(-l_ik, u_kj, a_ij) for j > k in row k ∩ row i
//   L   y = alpha x : y_i = fma(-l_ij, y_j, ...) over j ascending, from alpha*x_i
//   L^T y = alpha x : y_i = fma(-l_ji, y_j, ...) over j DESCENDING, from alpha*x_i
//   U   y = alpha x : y_i = (alpha*x_i - sum_j>i u_ij y_j) / u_ii, j ascending
// Zero pivots: the smallest i with u_ii == 0 after the factor (atomicMin),
// structural zeros (missing a_ii) are reported by the analysis.
//
// Compiled twice like spmv.hip (rsp_k / rsp_k_ftz).

#include <hip/hip_runtime.h>
#include <limits.h>

#include "rsp_kernels.h"

#ifndef RSP_KNS
#define RSP_KNS rsp_k
#endif

namespace RSP_KNS {

using rsp::IluArgs;
using rsp::TrsvArgs;

constexpr int kIluWaves = 4;  // rows per 256-thread workgroup (one wave each)

// position of column j in the sorted range cols[lo, hi), or -1
__device__ __forceinline__ int find_col(const int *__restrict__ cols, int lo, int hi, int j) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const int c = cols[mid];
        if (c == j) return mid;
        if (c < j)
            lo = mid + 1;
        else
            hi = mid;
    }
    return -1;
}

template <typename T>
__global__ __launch_bounds__(64 * kIluWaves) void ilu0_level(
    const int *__restrict__ rowptr, const int *__restrict__ colidx, const int *__restrict__ dpos,
    const int *__restrict__ hasdiag, T *vals, int *zero_pivot, const int *__restrict__ rows,
    int nrows) {
    const int w = blockIdx.x * kIluWaves + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= nrows) return;
    const int i = rows[w];
    const int rs = rowptr[i], re = rowptr[i + 1], di = dpos[i];
    for (int p = rs; p < di; ++p) {
        const int k = colidx[p];
        const T ukk = hasdiag[k] ? vals[dpos[k]] : T(0);
        const T lik = vals[p] / ukk;
        // row k's upper part, lanes in parallel; each j hits a distinct a_ij
        const int q0 = dpos[k] + hasdiag[k], q1 = rowptr[k + 1];
        for (int q = q0 + lane; q < q1; q += 64) {
            const int pos = find_col(colidx, p + 1, re, colidx[q]);
            if (pos >= 0) vals[pos] = __builtin_fma(-lik, vals[q], vals[pos]);
        }
        if (lane == 0) vals[p] = lik;
        // make this step's stores visible to the wave's next loads
        __threadfence_block();
    }
    if (lane == 0 && hasdiag[i] && vals[di] == T(0)) atomicMin(zero_pivot, i);
}

// L y = alpha x, unit diagonal, strictly-lower entries [rowptr[i], dpos[i]).
template <typename T>
__global__ __launch_bounds__(256) void trsv_lower_n_level(
    const int *__restrict__ rowptr, const int *__restrict__ colidx, const int *__restrict__ dpos,
    const T *__restrict__ vals, const T *__restrict__ x, T *y, T alpha,
    const int *__restrict__ rows, int nrows) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nrows) return;
    const int i = rows[t];
    T s = alpha * x[i];
    const int e = dpos[i];
    for (int p = rowptr[i]; p < e; ++p) s = __builtin_fma(-vals[p], y[colidx[p]], s);
    y[i] = s;
}

// L^T y = alpha x: row i of L^T holds l_ji (j > i), stored j-descending.
template <typename T>
__global__ __launch_bounds__(256) void trsv_lower_t_level(
    const int *__restrict__ lt_ptr, const int *__restrict__ lt_src, const int *__restrict__ lt_col,
    const T *__restrict__ vals, const T *__restrict__ x, T *y, T alpha,
    const int *__restrict__ rows, int nrows) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nrows) return;
    const int i = rows[t];
    T s = alpha * x[i];
    for (int q = lt_ptr[i]; q < lt_ptr[i + 1]; ++q) s = __builtin_fma(-vals[lt_src[q]], y[lt_col[q]], s);
    y[i] = s;
}

// U y = alpha x: upper entries (dpos+1, rowend), diagonal at dpos.
template <typename T>
__global__ __launch_bounds__(256) void trsv_upper_level(
    const int *__restrict__ rowptr, const int *__restrict__ colidx, const int *__restrict__ dpos,
    const int *__restrict__ hasdiag, const T *__restrict__ vals, const T *__restrict__ x, T *y,
    T alpha, const int *__restrict__ rows, int nrows) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nrows) return;
    const int i = rows[t];
    T s = alpha * x[i];
    const int d = dpos[i], hd = hasdiag[i];
    for (int p = d + hd; p < rowptr[i + 1]; ++p) s = __builtin_fma(-vals[p], y[colidx[p]], s);
    y[i] = s / (hd ? vals[d] : T(0));
}

template <typename T>
static hipError_t launch_factor(const IluArgs &a, hipStream_t s) {
    for (int l = 0; l < a.nlev; ++l) {
        const int off = a.level_ptr_host[l], cnt = a.level_ptr_host[l + 1] - off;
        if (cnt <= 0) continue;
        hipLaunchKernelGGL((ilu0_level<T>), dim3((cnt + kIluWaves - 1) / kIluWaves),
                           dim3(64 * kIluWaves), 0, s, a.rowptr, a.colidx, a.dpos, a.hasdiag,
                           (T *)a.vals, a.zero_pivot, a.level_rows + off, cnt);
    }
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_lower_n(const TrsvArgs &a, hipStream_t s) {
    for (int l = 0; l < a.nlev; ++l) {
        const int off = a.level_ptr_host[l], cnt = a.level_ptr_host[l + 1] - off;
        if (cnt <= 0) continue;
        hipLaunchKernelGGL((trsv_lower_n_level<T>), dim3((cnt + 255) / 256), dim3(256), 0, s,
                           a.rowptr, a.colidx, a.dpos, (const T *)a.vals, (const T *)a.x,
                           (T *)a.y, (T)a.alpha, a.level_rows + off, cnt);
    }
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_lower_t(const TrsvArgs &a, hipStream_t s) {
    for (int l = 0; l < a.nlev; ++l) {
        const int off = a.level_ptr_host[l], cnt = a.level_ptr_host[l + 1] - off;
        if (cnt <= 0) continue;
        hipLaunchKernelGGL((trsv_lower_t_level<T>), dim3((cnt + 255) / 256), dim3(256), 0, s,
                           a.lt_ptr, a.lt_src, a.lt_col, (const T *)a.vals, (const T *)a.x,
                           (T *)a.y, (T)a.alpha, a.level_rows + off, cnt);
    }
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_upper(const TrsvArgs &a, hipStream_t s) {
    for (int l = 0; l < a.nlev; ++l) {
        const int off = a.level_ptr_host[l], cnt = a.level_ptr_host[l + 1] - off;
        if (cnt <= 0) continue;
        hipLaunchKernelGGL((trsv_upper_level<T>), dim3((cnt + 255) / 256), dim3(256), 0, s,
                           a.rowptr, a.colidx, a.dpos, a.hasdiag, (const T *)a.vals,
                           (const T *)a.x, (T *)a.y, (T)a.alpha, a.level_rows + off, cnt);
    }
    return hipGetLastError();
}

hipError_t ilu0_factor_f32(const IluArgs &a, hipStream_t s) { return launch_factor<float>(a, s); }
hipError_t trsv_lower_n_f32(const TrsvArgs &a, hipStream_t s) { return launch_lower_n<float>(a, s); }
hipError_t trsv_lower_t_f32(const TrsvArgs &a, hipStream_t s) { return launch_lower_t<float>(a, s); }
hipError_t trsv_upper_f32(const TrsvArgs &a, hipStream_t s) { return launch_upper<float>(a, s); }
#ifndef RSP_FTZ_BUILD
hipError_t ilu0_factor_f64(const IluArgs &a, hipStream_t s) { return launch_factor<double>(a, s); }
hipError_t trsv_lower_n_f64(const TrsvArgs &a, hipStream_t s) { return launch_lower_n<double>(a, s); }
hipError_t trsv_lower_t_f64(const TrsvArgs &a, hipStream_t s) { return launch_lower_t<double>(a, s); }
hipError_t trsv_upper_f64(const TrsvArgs &a, hipStream_t s) { return launch_upper<double>(a, s); }
#endif

}  // namespace RSP_KNS
