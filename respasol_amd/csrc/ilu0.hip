// ilu0.hip — level-scheduled ILU(0) factorisation and unit-lower triangular
// solves for gfx950, replacing cusparse?csrilu02 and cusparse?csrsv2_solve
// (GPU/ilu0.cu:257-310).
//
// The analysis (rsp_ilu0_analysis, host) groups rows into dependency levels:
// row i depends on every row k < i with a_ik in the pattern (factor and
// L-solve), and for L^T on every row j > i with l_ji in the pattern. Rows of
// one level are independent. Execution follows the level plan's segments:
//   * fat level  -> one launch over its rows (the kernel boundary is the
//                   inter-level barrier);
//   * thin run   -> ONE launch of a single 1024-thread workgroup that walks a
//                   run of consecutive small levels with __syncthreads()
//                   between them (every row of the run is produced and
//                   consumed inside one CU, so the workgroup barrier orders
//                   it; rows of earlier fat levels come from earlier launches).
// Deep level sets (circuits: ~10^4 levels of ~10 rows) thus cost one launch
// per run instead of one per level.
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
using rsp::kIluWaves;
using rsp::kThinThreads;
using rsp::LevelPlan;
using rsp::TrsvArgs;

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

// ------------------------------------------------------------ per-row work

// ILU(0) of row i by one wave (lane = 0..63).
template <typename T>
__device__ __forceinline__ void factor_row(int i, int lane, const int *__restrict__ rowptr,
                                           const int *__restrict__ colidx,
                                           const int *__restrict__ dpos,
                                           const int *__restrict__ hasdiag, T *vals,
                                           int *zero_pivot) {
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

template <typename T>
__device__ __forceinline__ void lower_n_row(int i, const int *__restrict__ rowptr,
                                            const int *__restrict__ colidx,
                                            const int *__restrict__ dpos,
                                            const T *__restrict__ vals, const T *__restrict__ x,
                                            T *y, T alpha) {
    T s = alpha * x[i];
    const int e = dpos[i];
    for (int p = rowptr[i]; p < e; ++p) s = __builtin_fma(-vals[p], y[colidx[p]], s);
    y[i] = s;
}

template <typename T>
__device__ __forceinline__ void lower_t_row(int i, const int *__restrict__ lt_ptr,
                                            const int *__restrict__ lt_src,
                                            const int *__restrict__ lt_col,
                                            const T *__restrict__ vals, const T *__restrict__ x,
                                            T *y, T alpha) {
    T s = alpha * x[i];
    for (int q = lt_ptr[i]; q < lt_ptr[i + 1]; ++q)
        s = __builtin_fma(-vals[lt_src[q]], y[lt_col[q]], s);
    y[i] = s;
}

template <typename T>
__device__ __forceinline__ void upper_row(int i, const int *__restrict__ rowptr,
                                          const int *__restrict__ colidx,
                                          const int *__restrict__ dpos,
                                          const int *__restrict__ hasdiag,
                                          const T *__restrict__ vals, const T *__restrict__ x, T *y,
                                          T alpha) {
    T s = alpha * x[i];
    const int d = dpos[i], hd = hasdiag[i];
    for (int p = d + hd; p < rowptr[i + 1]; ++p) s = __builtin_fma(-vals[p], y[colidx[p]], s);
    y[i] = s / (hd ? vals[d] : T(0));
}

// --------------------------------------------------------------- kernels

// Fat level: one wave per row.
template <typename T>
__global__ __launch_bounds__(64 * kIluWaves) void ilu0_level(
    const int *__restrict__ rowptr, const int *__restrict__ colidx, const int *__restrict__ dpos,
    const int *__restrict__ hasdiag, T *vals, int *zero_pivot, const int *__restrict__ rows,
    int nrows) {
    const int w = blockIdx.x * kIluWaves + (threadIdx.x >> 6);
    if (w >= nrows) return;
    factor_row<T>(rows[w], threadIdx.x & 63, rowptr, colidx, dpos, hasdiag, vals, zero_pivot);
}

// Thin run of levels [lb, le): one workgroup, 16 waves, one row per wave per pass.
template <typename T>
__global__ __launch_bounds__(kThinThreads) void ilu0_thin(
    const int *__restrict__ rowptr, const int *__restrict__ colidx, const int *__restrict__ dpos,
    const int *__restrict__ hasdiag, T *vals, int *zero_pivot, const int *__restrict__ rows,
    const int *__restrict__ ptr, int lb, int le) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int l = lb; l < le; ++l) {
        const int off = ptr[l], cnt = ptr[l + 1] - off;
        for (int r = wave; r < cnt; r += kThinThreads / 64)
            factor_row<T>(rows[off + r], lane, rowptr, colidx, dpos, hasdiag, vals, zero_pivot);
        __syncthreads();
    }
}

// kind: 0 = L (op N), 1 = L^T (op T), 2 = U
template <typename T, int KIND>
__device__ __forceinline__ void solve_row(const TrsvArgs &a, int i, T alpha) {
    if constexpr (KIND == 0)
        lower_n_row<T>(i, a.rowptr, a.colidx, a.dpos, (const T *)a.vals, (const T *)a.x, (T *)a.y,
                       alpha);
    else if constexpr (KIND == 1)
        lower_t_row<T>(i, a.lt_ptr, a.lt_src, a.lt_col, (const T *)a.vals, (const T *)a.x,
                       (T *)a.y, alpha);
    else
        upper_row<T>(i, a.rowptr, a.colidx, a.dpos, a.hasdiag, (const T *)a.vals, (const T *)a.x,
                     (T *)a.y, alpha);
}

template <typename T, int KIND>
__global__ __launch_bounds__(256) void trsv_level(TrsvArgs a, T alpha, int off, int nrows) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nrows) return;
    solve_row<T, KIND>(a, a.plan.rows[off + t], alpha);
}

template <typename T, int KIND>
__global__ __launch_bounds__(kThinThreads) void trsv_thin(TrsvArgs a, T alpha, int lb, int le) {
    for (int l = lb; l < le; ++l) {
        const int off = a.plan.ptr_dev[l], cnt = a.plan.ptr_dev[l + 1] - off;
        for (int t = threadIdx.x; t < cnt; t += kThinThreads) solve_row<T, KIND>(a, a.plan.rows[off + t], alpha);
        __syncthreads();
    }
}

// --------------------------------------------------------------- launchers

template <typename T>
static hipError_t launch_factor(const IluArgs &a, hipStream_t s) {
    const LevelPlan &P = a.plan;
    for (int g = 0; g < P.nseg; ++g) {
        const rsp::LevelSeg sg = P.segs[g];
        if (sg.thin) {
            hipLaunchKernelGGL((ilu0_thin<T>), dim3(1), dim3(kThinThreads), 0, s, a.rowptr,
                               a.colidx, a.dpos, a.hasdiag, (T *)a.vals, a.zero_pivot, P.rows,
                               P.ptr_dev, sg.lb, sg.le);
            continue;
        }
        for (int l = sg.lb; l < sg.le; ++l) {
            const int off = P.ptr_host[l], cnt = P.ptr_host[l + 1] - off;
            if (cnt <= 0) continue;
            hipLaunchKernelGGL((ilu0_level<T>), dim3((cnt + kIluWaves - 1) / kIluWaves),
                               dim3(64 * kIluWaves), 0, s, a.rowptr, a.colidx, a.dpos, a.hasdiag,
                               (T *)a.vals, a.zero_pivot, P.rows + off, cnt);
        }
    }
    return hipGetLastError();
}

template <typename T, int KIND>
static hipError_t launch_solve(const TrsvArgs &a, hipStream_t s) {
    const LevelPlan &P = a.plan;
    const T alpha = (T)a.alpha;
    for (int g = 0; g < P.nseg; ++g) {
        const rsp::LevelSeg sg = P.segs[g];
        if (sg.thin) {
            hipLaunchKernelGGL((trsv_thin<T, KIND>), dim3(1), dim3(kThinThreads), 0, s, a, alpha,
                               sg.lb, sg.le);
            continue;
        }
        for (int l = sg.lb; l < sg.le; ++l) {
            const int off = P.ptr_host[l], cnt = P.ptr_host[l + 1] - off;
            if (cnt <= 0) continue;
            hipLaunchKernelGGL((trsv_level<T, KIND>), dim3((cnt + 255) / 256), dim3(256), 0, s, a,
                               alpha, off, cnt);
        }
    }
    return hipGetLastError();
}

hipError_t ilu0_factor_f32(const IluArgs &a, hipStream_t s) { return launch_factor<float>(a, s); }
hipError_t trsv_lower_n_f32(const TrsvArgs &a, hipStream_t s) { return launch_solve<float, 0>(a, s); }
hipError_t trsv_lower_t_f32(const TrsvArgs &a, hipStream_t s) { return launch_solve<float, 1>(a, s); }
hipError_t trsv_upper_f32(const TrsvArgs &a, hipStream_t s) { return launch_solve<float, 2>(a, s); }
#ifndef RSP_FTZ_BUILD
hipError_t ilu0_factor_f64(const IluArgs &a, hipStream_t s) { return launch_factor<double>(a, s); }
hipError_t trsv_lower_n_f64(const TrsvArgs &a, hipStream_t s) { return launch_solve<double, 0>(a, s); }
hipError_t trsv_lower_t_f64(const TrsvArgs &a, hipStream_t s) { return launch_solve<double, 1>(a, s); }
hipError_t trsv_upper_f64(const TrsvArgs &a, hipStream_t s) { return launch_solve<double, 2>(a, s); }
#endif

}  // namespace RSP_KNS
