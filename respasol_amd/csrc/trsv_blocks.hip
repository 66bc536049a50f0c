// trsv_blocks.hip — block-inverse solve of deep-DAG unit-lower triangles for
// gfx950 (round 6): the L and L^T solves of cusparse?csrsv2_solve
// (GPU/ilu0.cu:284-310) on DAGs of ~10^4 levels of ~10 rows (the circuits),
// where the level-scheduled kernels of ilu0.hip pay one dependent hand-off
// per level (~190 ns) and lose to one CPU core.
//
// Plan (ilu_blocks.cpp, rsp::BlkDesc): the rows in level order ("positions")
// are cut into chunks of kBlkWin positions and, inside a chunk, into blocks
// of <= 64 rows; every row's unknown is a combination of its block's
// right-hand sides and of earlier blocks' unknowns (the block's partitioned
// inverse), so a block is ONE dependent step instead of several levels. The
// arithmetic is restated in oracle/rsp_oracle.c (oracle_trsv_blocks_*): the
// results here equal it bit for bit; against the reference's order they
// differ by rounding only (SURVEY §8c tolerance).
//
// A row's pattern is summed in order: x terms, y terms of EARLIER chunks,
// y terms of its own chunk (<= kBlkNear for a normal row, <= kBlkNear rounds
// of 64 for a long one). One solve is:
//   trsv_blk_coef  one wave per block: the coefficients E from the values
//                  the solve is given (a changed value array is always
//                  honoured), intra-block level by level in LDS;
//   per chunk g:
//     trsv_blk_pro  one wave per block of the chunk, all in parallel: the x
//                  terms and the earlier chunks' y terms (known: earlier
//                  launches wrote them) summed into c, and the block's RECORD
//                  written: c and its in-chunk terms (coefficient, window
//                  slot) lane-interleaved, fixed size per block;
//     trsv_blk_seg  ONE wave walks the chunk's blocks in order: records
//                  prefetched kBlkPre blocks ahead into registers, then per
//                  block the in-chunk y gathered from the LDS window (the
//                  chunk's y), a <= kBlkNear fma chain, y into the window and
//                  out to HBM. No hand-off between waves, no atomics: the
//                  only dependency chain is the wave's own LDS order;
//   trsv_blk_out   y[row] = y by position.
// Compiled twice like ilu0.hip (rsp_k / rsp_k_ftz).

#include <hip/hip_runtime.h>

#include "rsp_kernels.h"

#ifndef RSP_KNS
#define RSP_KNS rsp_k
#endif

namespace RSP_KNS {

using rsp::BlkArgs;
using rsp::BlkDesc;
using rsp::BlkRow;

namespace {

[[maybe_unused]] __device__ __forceinline__ double fmab(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fmab(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

constexpr int KR = rsp::kBlkNear;  // in-chunk terms per lane in a record
// A record slot past a lane's terms: coefficient -0 times the window's zero
// cell (kBlkWin, +0): fma(-0, +0, s) = s exactly for every s (-0 + s is s,
// also for s = -0 and +0; under FTZ s is never subnormal, being an fma
// result itself), so pads need no select.
constexpr unsigned short kZeroCell = rsp::kBlkWin, kDumpCell = rsp::kBlkWin + 1;

// ---------------------------------------------------------- coefficients
// One wave per block. A normal block's coefficients are built in LDS, its
// intra-block levels in order (an entry of a row reads entries of rows of
// lower levels only; one wave, so LDS order needs no barrier): entry value =
// init (1 for the row's own right-hand side, else 0), then per recipe item
// (dependency order) v = fma(-l, E_source, v), the source the constant 1 for
// a dependency before the block (rsp_oracle.c step 5). Everything the levels
// read is staged in LDS first (its dependency values, the slot order, the
// recipe items: two memory round trips in all, not three per level). A long
// block has no in-block dependencies: every entry is independent, straight
// from HBM.
template <typename T>
__global__ __launch_bounds__(64) void trsv_blk_coef(BlkArgs a) {
    extern __shared__ __align__(16) unsigned char blk_sm[];
    const int lane = threadIdx.x;
    const BlkDesc d = a.desc[blockIdx.x];
    const T *vals = (const T *)a.vals;
    T *ev = (T *)a.ev;
    if (d.kind) {
        for (int k = lane; k < d.ne; k += 64) {
            const unsigned w = a.eord[d.eoff + k];
            T v = (w >> 31) ? T(1) : T(0);
            for (int q = a.rptr[d.eoff + k]; q < a.rptr[d.eoff + k + 1]; ++q)
                v = fmab(-vals[a.vpos[d.doff + (int)a.rit[q]]], T(1), v);
            ev[d.eoff + (int)(w & 0x7fffffffu)] = v;
        }
        return;
    }
    // LDS: lv[nd] | el[1 + ne] (el[0] = 1) | ew[ne] | rp[ne + 1] | lb[nlev + 1] | it[items]
    T *lv = reinterpret_cast<T *>(blk_sm);
    T *el = lv + d.nd;
    unsigned *ew = reinterpret_cast<unsigned *>(blk_sm + (size_t)a.lds_elems * sizeof(T));
    int *rp = reinterpret_cast<int *>(ew + d.ne);
    int *lb = rp + d.ne + 1;
    unsigned *it = reinterpret_cast<unsigned *>(lb + d.nlev + 1);
    const int r0 = a.rptr[d.eoff], r1 = a.rptr[d.eoff + d.ne];
    for (int k = lane; k < d.nd; k += 64) lv[k] = vals[a.vpos[d.doff + k]];
    for (int k = lane; k < d.ne; k += 64) {
        ew[k] = a.eord[d.eoff + k];
        rp[k] = a.rptr[d.eoff + k] - r0;
    }
    for (int k = lane; k <= d.nlev; k += 64) lb[k] = a.lptr[d.loff + k] - d.eoff;
    for (int q = lane; q < r1 - r0; q += 64) it[q] = a.rit[r0 + q];
    if (lane == 0) {
        el[0] = T(1);
        rp[d.ne] = r1 - r0;
    }
    for (int l = 0; l < d.nlev; ++l) {
        const int k1 = lb[l + 1];
        for (int k = lb[l] + lane; k < k1; k += 64) {
            const unsigned w = ew[k];
            T v = (w >> 31) ? T(1) : T(0);
            const int q1 = rp[k + 1];
            for (int q = rp[k]; q < q1; ++q) {
                const unsigned i = it[q];
                v = fmab(-lv[i >> 16], el[i & 0xffffu], v);
            }
            el[1 + (int)(w & 0x7fffffffu)] = v;
        }
    }
    for (int k = lane; k < d.ne; k += 64) ev[d.eoff + k] = el[1 + k];
}

// ----------------------------------------------------- block records
// A lane's record: its sum so far (x terms, earlier chunks' y terms), its
// in-chunk terms' coefficients and window slots (pads: -0 x the zero cell), the
// position its y goes to (-1: no row) and the block's in-chunk terms (rounds
// for a long row) | long << 16. 144 B (fp64) / 96 B (fp32): read as 16-B
// vectors, 9 / 6 per lane — per-lane data, so vector loads counted in
// order (a block-uniform header would become a scalar load, whose counter
// is shared with LDS and waited on whole) and few memory instructions per
// record (the wave's counter of outstanding vector memory instructions
// stops at 63).
template <typename T>
struct alignas(16) BlkLane {
    T c;
    T cf[KR];
    unsigned short sl[KR];
    int pos, meta;
};
static_assert(sizeof(BlkLane<double>) == 144 && sizeof(BlkLane<float>) == 96, "record layout");
template <typename T>
constexpr int kLaneVec = sizeof(BlkLane<T>) / 16;

// ----------------------------------------------------- chunk prologue
// One wave per block of the chunk starting at position p0: the sum of each
// row's x terms and earlier chunks' y terms (in pattern order), and the
// block's record. A normal block: lane = row; a long block: lane l holds the
// partial of the row's terms k = l, l + 64, ... (rsp_oracle.c step 6), its
// in-chunk terms in rounds (<= kBlkNear rounds: a row with more starts a
// chunk, ilu_blocks.cpp).
template <typename T>
__global__ __launch_bounds__(64) void trsv_blk_pro(BlkArgs a, int b0, int p0) {
    const int lane = threadIdx.x, b = b0 + (int)blockIdx.x;
    const BlkDesc d = a.desc[b];
    const T al = (T)a.alpha;
    const T *ev = (const T *)a.ev, *x = (const T *)a.x, *yp = (const T *)a.yp;
    BlkLane<T> L;
    T s = T(0);
    if (d.kind == 0) {
        const bool ok = lane < d.np;
        const BlkRow r = a.rows[d.p0 + (ok ? lane : 0)];
        const int nx = ok ? r.nx : 0, nh = ok ? r.nx + r.nfar : 0, nn = ok ? r.ny - r.nfar : 0;
        for (int t0 = 0; __ballot(t0 < nh); t0 += 4) {
            T e[4], v[4];
            int q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = r.off + min(t0 + u, max(r.nx + r.nfar - 1, 0));
                e[u] = ev[k];
                q[u] = a.ref[k];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = t0 + u < nx ? al * x[q[u]] : yp[q[u]];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (t0 + u < nh) s = fmab(e[u], v[u], s);
        }
        const int kb = r.off + r.nx + r.nfar;
#pragma unroll
        for (int t = 0; t < KR; ++t) {
            const int k = kb + min(t, max(r.ny - r.nfar - 1, 0));
            const T e = ev[k];
            const int q = a.ref[k];
            L.cf[t] = t < nn ? e : T(-0.0);
            L.sl[t] = t < nn ? (unsigned short)(q - p0) : kZeroCell;
        }
        L.pos = ok ? d.p0 + lane : -1;
        L.meta = d.kn;
    } else {
        const BlkRow r = a.rows[d.p0];
        const int ne = r.nx + r.ny, kp = r.nx + r.nfar;
        for (int k0 = 0; k0 < kp; k0 += 256) {
            T e[4], v[4];
            int q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = r.off + min(k0 + lane + 64 * u, ne - 1);
                e[u] = ev[k];
                q[u] = a.ref[k];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = k0 + lane + 64 * u < r.nx ? al * x[q[u]] : yp[q[u]];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (k0 + lane + 64 * u < kp) s = fmab(e[u], v[u], s);
        }
        // in-chunk terms: lane l's t-th is k = f + 64 t, f its first k >= kp
        const int f = kp + ((lane - kp % 64) & 63);
#pragma unroll
        for (int t = 0; t < KR; ++t) {
            const int k = f + 64 * t;
            const int kk = r.off + min(k, ne - 1);
            const T e = ev[kk];
            const int q = a.ref[kk];
            L.cf[t] = k < ne ? e : T(-0.0);
            L.sl[t] = k < ne ? (unsigned short)(q - p0) : kZeroCell;
        }
        L.pos = lane == 0 ? d.p0 : -1;
        L.meta = (ne - kp + 63) / 64 | 1 << 16;
    }
    L.c = s;
    uint4 w[kLaneVec<T>];
    __builtin_memcpy(w, &L, sizeof(L));
    uint4 *dst = reinterpret_cast<uint4 *>((BlkLane<T> *)a.rc + (size_t)b * 64 + lane);
#pragma unroll
    for (int i = 0; i < kLaneVec<T>; ++i) dst[i] = w[i];
}

// ------------------------------------------------------------ one chunk
// The records of D blocks are in registers at once (a ring indexed by
// compile-time slots: the block loop is unrolled by D), each loaded D
// blocks before its use; D x (8 or 5 loads + a store) stays under the
// wave's 63 outstanding vector memory instructions.
template <typename T>
struct BlkRec {
    BlkLane<T> L;
};

template <typename T>
__device__ __forceinline__ void blk_load(BlkRec<T> &R, const BlkArgs &a, int b, int lane) {
    const uint4 *src = reinterpret_cast<const uint4 *>((const BlkLane<T> *)a.rc + (size_t)b * 64 + lane);
    uint4 w[kLaneVec<T>];
#pragma unroll
    for (int i = 0; i < kLaneVec<T>; ++i) w[i] = src[i];
    __builtin_memcpy(&R.L, w, sizeof(R.L));
}

// One block of the chunk walk. Its in-chunk terms in groups of four, a group
// skipped when the block has no term in it (a uniform branch around LDS and
// VALU work only: no vector memory instruction is conditional, so the
// compiler's counters stay exact across the unrolled walk and a block waits
// only for its own record); pads are exact no-ops (kZeroCell). The y of a
// lane without a row goes to the dump cell and to HBM's spare cell.
template <typename T>
__device__ __forceinline__ void blk_step(const BlkRec<T> &R, T *win, T *yp, int n, int p0) {
    const int meta = __builtin_amdgcn_readfirstlane(R.L.meta);
    const bool lng = (meta >> 16) != 0;
    const int kr = meta & 0xffff;
    T s = R.L.c;
#pragma unroll
    for (int g = 0; g < KR; g += 4) {
        if (g < kr) {
            T yv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) yv[u] = win[R.L.sl[g + u]];
#pragma unroll
            for (int u = 0; u < 4; ++u) s = fmab(R.L.cf[g + u], yv[u], s);
        }
    }
    if (lng) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s = s + __shfl_xor(s, off, 64);
    }
    const bool in = R.L.pos >= 0;
    win[in ? R.L.pos - p0 : (int)kDumpCell] = s;
    yp[in ? R.L.pos : n] = s;
}

template <typename T, int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void trsv_blk_seg(BlkArgs a, int b0, int b1,
                                                                                        int p0) {
    __shared__ T win[rsp::kBlkWin + 2];  // y of the chunk's positions, the zero cell, the dump cell
    const int lane = threadIdx.x;
    T *yp = (T *)a.yp;
    if (lane == 0) win[kZeroCell] = T(0);
    BlkRec<T> R[D];
#pragma unroll
    for (int j = 0; j < D; ++j) blk_load(R[j], a, min(b0 + j, b1 - 1), lane);
    int b = b0;
    for (; b + D <= b1; b += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            blk_step(R[j], win, yp, a.n, p0);
            blk_load(R[j], a, min(b + j + D, b1 - 1), lane);  // (unconditional: exact counters)
        }
    }
#pragma unroll
    for (int j = 0; j < D; ++j)
        if (b + j < b1) blk_step(R[j], win, yp, a.n, p0);
}

template <typename T>
__global__ __launch_bounds__(256) void trsv_blk_out(BlkArgs a) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p < a.n) ((T *)a.y)[a.order[p]] = ((const T *)a.yp)[p];
}

template <typename T>
hipError_t blocks_run(const BlkArgs &a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    const size_t lds = (size_t)a.lds_elems * sizeof(T) + (size_t)a.lds_words * 4;
    if (lds > 65536) {
        static bool set = false;  // per instantiation
        if (!set) {
            const hipError_t e = hipFuncSetAttribute((const void *)trsv_blk_coef<T>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            set = true;
        }
    }
    hipLaunchKernelGGL(trsv_blk_coef<T>, dim3(a.nb), dim3(64), lds, s, a);
    for (int g = 0; g < a.nseg; ++g) {
        const rsp::BlkSeg sg = a.segs[g];
        if (sg.b1 <= sg.b0) continue;
        hipLaunchKernelGGL(trsv_blk_pro<T>, dim3(sg.b1 - sg.b0), dim3(64), 0, s, a, sg.b0, sg.p0);
        hipLaunchKernelGGL((trsv_blk_seg<T, sizeof(T) == 8 ? rsp::kBlkPre : rsp::kBlkPre + 2>), dim3(1), dim3(64), 0,
                           s, a, sg.b0, sg.b1, sg.p0);
    }
    hipLaunchKernelGGL(trsv_blk_out<T>, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace

hipError_t trsv_blocks_f32(const BlkArgs &a, hipStream_t s) { return blocks_run<float>(a, s); }
#ifndef RSP_FTZ_BUILD
hipError_t trsv_blocks_f64(const BlkArgs &a, hipStream_t s) { return blocks_run<double>(a, s); }
#endif

}  // namespace RSP_KNS
