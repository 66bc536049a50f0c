// spmv_probe.h — diagnostic-only pieces of the SpMV tile kernel, compiled
// into probe builds of librsp.so (`make probe PROBE_NAME=loadsonly
// PROBE_DEFS=-DRSP_SPMV_PROBE_LOADS`, scripts/spmv_probe.py), never into the
// shipped library. Included by spmv.hip inside its kernel namespace.
#pragma once

// The tile's colidx / vals stream alone (no gathers, no LDS, no reduce):
// the loads-only ceiling of the tile structure. Every load is
// kept live by a never-taken store.
template <typename T, bool NT>
__device__ __forceinline__ void probe_tile_loads(const int *__restrict__ colidx, const T *__restrict__ vals,
                                                 T *__restrict__ y, const SpmvBlock blk, int kb, int k1, int rp0) {
    constexpr int VW = 16 / sizeof(T);
    typedef typename VecT<T, VW>::V V;
    typedef typename VecT<T, VW>::I I;
    constexpr int IT = SpmvTile<T>::kSlots / (kSpmvThreads * VW);
    const int tid = threadIdx.x;
    const int last = (k1 - 1) & ~(VW - 1);
    T acc = T(0);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = min(kb + (it * kSpmvThreads + tid) * VW, last);
        const I c = ld<NT>(reinterpret_cast<const I *>(colidx + e));
        const V v = ld<NT>(reinterpret_cast<const V *>(vals + e));
#pragma unroll
        for (int j = 0; j < VW; ++j) acc += v[j] + T(c[j]);
    }
    if (acc == T(-12345.0)) y[blk.r0] = acc + T(rp0);
}
