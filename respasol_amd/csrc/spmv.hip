// spmv.hip — CSR SpMV y = alpha*A*x + beta*y for gfx950 (MI355X), fp64 and
// fp32 (fp32 storage AND accumulation, as cusparseSpMV with CUDA_R_32F,
// GPU/spmv.cu:131-145,179-181). Replaces cusparseSpMV (GPU/spmv.cu:148-186).
//
// Schedule ("row-block" tiles, built on the host by rsp_spmv_preprocess):
// consecutive rows are packed into tiles of at most SpmvTile<T>::kMaxNnz
// entries (<= kSpmvMaxRows rows); one 256-thread workgroup per tile.
//   1. stream: every thread issues kSpmvIter 16-byte loads of colidx and vals
//      (fully coalesced, 1 KiB per wave-instruction for vals), gathers
//      x[col] and writes the products into LDS (16 KiB per tile);
//   2. reduce: L = 1..64 lanes per row (power of two chosen from the tile's
//      rows and average row length) sum the row's products from LDS and
//      combine with wave shuffles; lane 0 writes y.
// Rows longer than a tile are split into tile-sized chunks whose partial sums
// a tiny fixup kernel adds in chunk order. Every summation order is fixed, so
// results are bitwise reproducible run to run (cuSPARSE ALG_DEFAULT is not).
// With L == 1 (the common case for short rows) each row is summed
// sequentially in column order, i.e. bit-identical to the CPU oracle.
//
// Roofline: HBM-bound, no MFMA (no dense contraction). Algorithmic bytes per
// call: (sizeof(T)+4)*nnz_s + 4*(m+1) + sizeof(T)*(n + m) (+ sizeof(T)*m if
// beta != 0); see DESIGN.md.
//
// Compiled twice: namespace rsp_k (fp64 + fp32) and rsp_k_ftz (fp32 only,
// -fgpu-flush-denormals-to-zero), see rsp_kernels.h.

#include <hip/hip_runtime.h>

#include "rsp_kernels.h"

#ifndef RSP_KNS
#define RSP_KNS rsp_k
#endif

namespace RSP_KNS {

using rsp::SpmvArgs;
using rsp::SpmvBlock;
using rsp::SpmvLongRow;
using rsp::SpmvTile;
using rsp::kSpmvIter;
using rsp::kSpmvThreads;

template <typename T, int N>
struct VecT;
template <>
struct VecT<double, 2> {
    typedef double __attribute__((ext_vector_type(2))) V;
    typedef int __attribute__((ext_vector_type(2))) I;
};
template <>
struct VecT<float, 4> {
    typedef float __attribute__((ext_vector_type(4))) V;
    typedef int __attribute__((ext_vector_type(4))) I;
};
template <typename T>
struct VecT<T, 1> {
    typedef T V;
    typedef int I;
};

// Logical tile for workgroup `bid`: each of the 8 XCDs (round-robin dispatch)
// gets a contiguous run of tiles, so neighbouring row blocks — which gather
// overlapping parts of x — share one L2 (guide T1, bijective form).
__device__ __forceinline__ int xcd_swizzle(int bid, int nwg) {
    const int q = nwg >> 3, r = nwg & 7;
    const int xcd = bid & 7, idx = bid >> 3;
    const int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return start + idx;
}

template <typename T>
__device__ __forceinline__ T wave_sum_group(T v, int width) {
    // butterfly over the low log2(width) lane bits (width <= 64, power of 2)
    for (int off = width >> 1; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Stream the tile's [k0, k1) entries with 16-B loads starting at the aligned
// element kb = k0 & ~(VW-1); products land in lds[e - kb]. Returns this
// thread's running sum of its products in element order (used by long-row
// chunks; ignored by normal tiles).
template <typename T, int VW, bool kStore>
__device__ __forceinline__ T stream_tile(const int *__restrict__ colidx,
                                         const T *__restrict__ vals, const T *__restrict__ x,
                                         int k0, int k1, T *lds) {
    typedef typename VecT<T, VW>::V V;
    typedef typename VecT<T, VW>::I I;
    const int tid = threadIdx.x;
    const int kb = k0 & ~(VW - 1);
    int c[kSpmvIter][VW];
    T v[kSpmvIter][VW];
#pragma unroll
    for (int it = 0; it < kSpmvIter; ++it) {
        const int e = kb + (it * kSpmvThreads + tid) * VW;
        if (e >= k0 && e + VW <= k1) {
            if constexpr (VW == 1) {
                c[it][0] = colidx[e];
                v[it][0] = vals[e];
            } else {
                const I ci = *reinterpret_cast<const I *>(colidx + e);
                const V vi = *reinterpret_cast<const V *>(vals + e);
#pragma unroll
                for (int j = 0; j < VW; ++j) {
                    c[it][j] = ci[j];
                    v[it][j] = vi[j];
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                const int ej = e + j;
                const bool ok = ej >= k0 && ej < k1;
                c[it][j] = ok ? colidx[ej] : -1;
                v[it][j] = ok ? vals[ej] : T(0);
            }
        }
    }
    T acc = T(0);
#pragma unroll
    for (int it = 0; it < kSpmvIter; ++it) {
        const int e = kb + (it * kSpmvThreads + tid) * VW;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            if (c[it][j] >= 0) {
                const T p = v[it][j] * x[c[it][j]];
                if constexpr (kStore)
                    lds[e + j - kb] = p;
                else
                    acc += p;
            }
        }
    }
    return acc;
}

template <typename T, int VW>
__global__ __launch_bounds__(kSpmvThreads) void spmv_tiles(
    const int *__restrict__ rowptr, const int *__restrict__ colidx, const T *__restrict__ vals,
    const T *__restrict__ x, T *__restrict__ y, const SpmvBlock *__restrict__ blocks, int nblocks,
    T *__restrict__ partials, T alpha, T beta, int beta_nonzero) {
    __shared__ T lds[SpmvTile<T>::kSlots];
    __shared__ T wsum[kSpmvThreads / 64];
    const int b = xcd_swizzle(blockIdx.x, nblocks);
    const SpmvBlock blk = blocks[b];
    const int tid = threadIdx.x;

    if (blk.r1 < 0) {
        // chunk of a long row: per-thread sums -> wave butterfly -> LDS -> slot
        T s = stream_tile<T, VW, false>(colidx, vals, x, blk.k0, blk.k1, lds);
        s = wave_sum_group(s, 64);
        if ((tid & 63) == 0) wsum[tid >> 6] = s;
        __syncthreads();
        if (tid == 0) {
            T t = T(0);
#pragma unroll
            for (int w = 0; w < kSpmvThreads / 64; ++w) t += wsum[w];
            partials[-(blk.r1 + 1)] = t;
        }
        return;
    }

    stream_tile<T, VW, true>(colidx, vals, x, blk.k0, blk.k1, lds);
    __syncthreads();

    const int r0 = blk.r0, nrows = blk.r1 - blk.r0;
    const int kb = blk.k0 & ~(VW - 1);
    const int nnz = blk.k1 - blk.k0;
    // lanes per row: power of two <= 64 such that every lane still sums >= 4
    // products of an average row and the groups fit the workgroup. Tiles of
    // short rows (avg < 8) keep L = 1: sequential column order per row, i.e.
    // bit-identical to the CPU oracle.
    int L = 1;
    while (L < 64 && 2 * L * nrows <= kSpmvThreads && 8 * L * nrows <= nnz) L <<= 1;
    const int g = tid / L, lane = tid & (L - 1), ngroups = kSpmvThreads / L;
    // groups of one wave share a trip count within +-1, and all lanes of a
    // group stay convergent for the shuffles.
    for (int rr = g; rr - g < nrows; rr += ngroups) {
        const bool active = rr < nrows;
        T s = T(0);
        if (active) {
            const int a = rowptr[r0 + rr] - kb, e = rowptr[r0 + rr + 1] - kb;
            for (int k = a + lane; k < e; k += L) s += lds[k];
        }
        if (L > 1) s = wave_sum_group(s, L);
        if (active && lane == 0) {
            T out = alpha * s;
            if (beta_nonzero) out += beta * y[r0 + rr];
            y[r0 + rr] = out;
        }
    }
}

// y[row] = alpha * sum(partials of the row, chunk order) (+ beta*y[row]).
template <typename T>
__global__ __launch_bounds__(64) void spmv_longrow_fixup(const SpmvLongRow *__restrict__ lr,
                                                          int nlong, const T *__restrict__ partials,
                                                          T *__restrict__ y, T alpha, T beta,
                                                          int beta_nonzero) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= nlong) return;
    const SpmvLongRow r = lr[i];
    T s = T(0);
    for (int c = 0; c < r.nchunks; ++c) s += partials[r.first + c];
    T out = alpha * s;
    if (beta_nonzero) out += beta * y[r.row];
    y[r.row] = out;
}

template <typename T>
static hipError_t launch_spmv(const SpmvArgs &a, hipStream_t s) {
    if (a.nblocks > 0) {
        const T alpha = (T)a.alpha, beta = (T)a.beta;
        const int bnz = a.beta != 0.0;
        if (a.vector_ok)
            hipLaunchKernelGGL((spmv_tiles<T, SpmvTile<T>::kVec>), dim3(a.nblocks),
                               dim3(kSpmvThreads), 0, s, a.rowptr, a.colidx, (const T *)a.vals,
                               (const T *)a.x, (T *)a.y, a.blocks, a.nblocks, (T *)a.partials,
                               alpha, beta, bnz);
        else
            hipLaunchKernelGGL((spmv_tiles<T, 1>), dim3(a.nblocks), dim3(kSpmvThreads), 0, s,
                               a.rowptr, a.colidx, (const T *)a.vals, (const T *)a.x, (T *)a.y,
                               a.blocks, a.nblocks, (T *)a.partials, alpha, beta, bnz);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (a.nlong > 0) {
            hipLaunchKernelGGL((spmv_longrow_fixup<T>), dim3((a.nlong + 63) / 64), dim3(64), 0, s,
                               a.longrows, a.nlong, (const T *)a.partials, (T *)a.y, alpha, beta,
                               bnz);
            e = hipGetLastError();
        }
        return e;
    }
    return hipSuccess;
}

hipError_t spmv_f32(const SpmvArgs &a, hipStream_t s) { return launch_spmv<float>(a, s); }
#ifndef RSP_FTZ_BUILD
hipError_t spmv_f64(const SpmvArgs &a, hipStream_t s) { return launch_spmv<double>(a, s); }
#endif

}  // namespace RSP_KNS
