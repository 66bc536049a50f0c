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
//   evaluated in pull form: every position applies its own precomputed update
//   list in k order (same fma sequence per position), so the positions of a
//   row run in parallel lanes except where l_ij needs an l_ik of its own row.
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

// ------------------------------------------------------------ per-row work

// s - sum_p v_p y_p as a serial fma chain over p = p0 .. p1-1, ascending.
// The operands of B consecutive terms are loaded together (clamped,
// unpredicated) so the loads of a batch overlap instead of serialising
// behind each fma; B is picked per DAG from its mean chain length so short
// rows do not pay for dead loads.
template <typename T, int B, typename FV, typename FY>
__device__ __forceinline__ T fma_chain(T s, int p0, int p1, FV vat, FY yat) {
    const int n = p1 - p0;
    for (int b0 = 0; b0 < n; b0 += B) {
        T v[B], y[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int p = p0 + min(b0 + b, n - 1);
            v[b] = vat(p);
            y[b] = yat(p);
        }
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (b0 + b < n) s = __builtin_fma(-v[b], y[b], s);
    }
    return s;
}

// The same serial fma chain for one long row, by a whole wave: lanes load 64
// terms at once, then the chain runs over them in order on wave-uniform
// registers (readlane), so a hub row pays one load round trip per 64 terms.
__device__ __forceinline__ double wave_read(double v, int j) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, j), hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float wave_read(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

template <typename T, typename FV, typename FY>
__device__ __forceinline__ T wave_chain(T s, int k0, int k1, int lane, FV vat, FY yat) {
    for (int base = k0; base < k1; base += 64) {
        const int k = min(base + lane, k1 - 1);
        const T v = vat(k), yv = yat(k);
        const int cnt = min(64, k1 - base);
        for (int j = 0; j < cnt; ++j) s = __builtin_fma(-wave_read(v, j), wave_read(yv, j), s);
    }
    return s;
}

// One position of the factor, pull form: v = a_p - sum_k l_ik u_kj over the
// position's update list (k ascending, one fma each — the same sequence of
// roundings as the IKJ loop).
template <typename T, int B>
__device__ __forceinline__ T factor_entry(const IluArgs &a, const T *vals, int p) {
    const int *ul = a.upd_l, *uu = a.upd_u;
    return fma_chain<T, B>(vals[p], a.upd_ptr[p], a.upd_ptr[p + 1],
                           [&](int u) { return vals[ul[u]]; },
                           [&](int u) { return vals[uu[u]]; });
}

// ILU(0) of row i by the 64 lanes of a wave: lower positions stage by stage
// (a stage's positions depend only on earlier stages of the row and on
// earlier rows), l_ij = v / u_jj, then every upper position at once.
template <typename T, int B>
__device__ __forceinline__ void factor_row(const IluArgs &a, int i, int lane) {
    T *vals = (T *)a.vals;
    const int rs = a.rowptr[i], re = a.rowptr[i + 1], di = a.dpos[i];
    for (int s = rs; s < di;) {
        const int e = a.lend[s];
        for (int x = s + lane; x < e; x += 64) {
            const int p = a.lord[x];
            const int k = a.colidx[p];
            const T ukk = a.hasdiag[k] ? vals[a.dpos[k]] : T(0);
            vals[p] = factor_entry<T, B>(a, vals, p) / ukk;
        }
        // this stage's l_ik visible to the next stage's lanes
        __threadfence_block();
        s = e;
    }
    for (int p = di + lane; p < re; p += 64) {
        const T v = factor_entry<T, B>(a, vals, p);
        vals[p] = v;
        if (p == di && a.hasdiag[i] && v == T(0)) atomicMin(a.zero_pivot, i);
    }
}

// LDS-only workgroup barrier (no vmcnt drain).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// --------------------------------------------------------------- kernels

// Fat level: one wave per row.
template <typename T, int B>
__global__ __launch_bounds__(64 * kIluWaves) void ilu0_level(IluArgs a, int off, int nrows) {
    const int w = blockIdx.x * kIluWaves + (threadIdx.x >> 6);
    if (w >= nrows) return;
    factor_row<T, B>(a, a.plan.rows[off + w], threadIdx.x & 63);
}

// Thin run of the factor, chunk by chunk (rsp::FacChunk), one 1024-thread
// workgroup. Per chunk: a full barrier (every earlier factor value is in
// global memory and visible), then all threads stage in LDS the values of
// the chunk's rows (cv, one slot per item), the item / update-pair index
// lists, and the values of every u_kk / u_kj that comes from a row before the
// chunk; the chunk's levels then run on LDS alone: wave w takes rows w, w+16,
// ... of a level, each row stage by stage exactly as factor_row (same fma
// order), writing every finished value to its LDS slot and to vals; an
// LDS-only barrier separates the levels.
template <typename T>
__global__ __launch_bounds__(kThinThreads) void ilu0_chunked(IluArgs a, int c0, int c1) {
    __shared__ T cv[rsp::kFacItems];
    __shared__ T dpre[rsp::kFacItems];
    __shared__ int lpos[rsp::kFacItems], lu0[rsp::kFacItems + 1], lsend[rsp::kFacItems], ld[rsp::kFacItems];
    __shared__ T upre[rsp::kFacPairs];
    __shared__ int lpl[rsp::kFacPairs], lpu[rsp::kFacPairs];
    __shared__ rsp::FacRow lrow[rsp::kFacRows];
    __shared__ int lptr[rsp::kFacRows + 1];  // a chunk has <= kFacRows levels
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    T *vals = (T *)a.vals;
    const int *ptr = a.plan.ptr_dev;
    for (int c = c0; c < c1; ++c) {
        const rsp::FacChunk ch = a.fchunks[c];
        const int ni = ch.item1 - ch.item0, np = ch.pair1 - ch.pair0;
        __syncthreads();  // earlier chunks' values visible, LDS free
        for (int x = tid; x < ni; x += kThinThreads) {
            const int g = ch.item0 + x;
            const int pos = a.fpos[g], d = a.fd[g];
            lpos[x] = pos;
            cv[x] = vals[pos];
            lu0[x] = a.fu0[g];
            lsend[x] = a.fsend[g];
            ld[x] = d;
            dpre[x] = (d < 0 && d != INT_MIN) ? vals[-d - 1] : T(0);
        }
        if (tid == 0) lu0[ni] = np;
        const int x0 = ptr[ch.l0], nr = ptr[ch.l1] - x0;
        for (int r = tid; r < nr; r += kThinThreads) lrow[r] = a.frows[x0 + r];
        for (int q = tid; q <= ch.l1 - ch.l0; q += kThinThreads) lptr[q] = ptr[ch.l0 + q];
        for (int u = tid; u < np; u += kThinThreads) {
            const int g = ch.pair0 + u;
            const int pu = a.fpu[g];
            lpl[u] = a.fpl[g];
            lpu[u] = pu;
            upre[u] = pu < 0 ? vals[-pu - 1] : T(0);
        }
        __syncthreads();
        for (int l = ch.l0; l < ch.l1; ++l) {
            const int xe = lptr[l - ch.l0 + 1];
            for (int x = lptr[l - ch.l0] + wave; x < xe; x += kThinThreads / 64) {
                const rsp::FacRow r = lrow[x - x0];
                const int nitem = r.nitem_hd & ((1 << 30) - 1), hd = r.nitem_hd >> 30;
                const int lo_end = r.item0 + r.nlow, end = r.item0 + nitem;
                auto item = [&](int it) {
                    T v = cv[it];
                    for (int u = lu0[it]; u < lu0[it + 1]; ++u) {
                        const int pu = lpu[u];
                        v = __builtin_fma(-cv[lpl[u]], pu >= 0 ? cv[pu] : upre[u], v);
                    }
                    return v;
                };
                for (int st = r.item0; st < lo_end;) {
                    const int e = lsend[st];
                    for (int it = st + lane; it < e; it += 64) {
                        const int d = ld[it];
                        const T v = item(it) / (d >= 0 ? cv[d] : dpre[it]);
                        cv[it] = v;
                        vals[lpos[it]] = v;
                    }
                    // this stage's l_ik visible to the wave's next stage
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
                    st = e;
                }
                for (int it = lo_end + lane; it < end; it += 64) {
                    const T v = item(it);
                    cv[it] = v;
                    vals[lpos[it]] = v;
                    if (it == lo_end && hd && v == T(0)) atomicMin(a.zero_pivot, r.i);
                }
            }
            lds_barrier();
        }
    }
}

// Triangular solves (kind 0 = L op N, 1 = L^T op T, 2 = U) over the DAG's
// flat terms: y_i = (alpha x_i - sum_k vals[tpos[k]] * y[src[k]]) (/ u_ii),
// one fma per term in the term order (for L^T: j descending).

// Fat level, terms straight from global memory: blocks [0, nb) one thread
// per short row (the level's first nshort rows), the blocks after them one
// wave per long row.
template <typename T, int KIND, int B>
__global__ __launch_bounds__(256) void trsv_level(TrsvArgs a, T alpha, int off, int nrows,
                                                  int nshort, int nb) {
    const T *vals = (const T *)a.vals;
    T *y = (T *)a.y;
    const int *tpos = a.plan.tpos, *src = a.plan.src;
    auto vat = [&](int k) { return vals[tpos[k]]; };
    auto yat = [&](int k) { return y[src[k]]; };
    T s;
    rsp::RowTask t;
    if ((int)blockIdx.x < nb) {
        const int r = blockIdx.x * 256 + threadIdx.x;
        if (r >= nshort) return;
        t = a.plan.tasks[off + r];
        s = fma_chain<T, B>(alpha * ((const T *)a.x)[t.i], t.t0, t.t1, vat, yat);
    } else {
        const int r = nshort + (blockIdx.x - nb) * 4 + (threadIdx.x >> 6);
        if (r >= nrows) return;
        t = a.plan.tasks[off + r];
        s = wave_chain<T>(alpha * ((const T *)a.x)[t.i], t.t0, t.t1, threadIdx.x & 63, vat, yat);
        if ((threadIdx.x & 63) != 0) return;
    }
    if constexpr (KIND == 2) s = s / (t.d >= 0 ? vals[t.d] : T(0));
    y[t.i] = s;
}

// Thin run (levels [lb, le) cut into chunks [c0, c1)), one 1024-thread
// workgroup. Per chunk: a full barrier (every earlier y store visible), then
// the chunk's tasks, x_i, u_ii, term values and — for terms whose y was
// produced before the chunk and has left the LDS window — those y values are
// staged in LDS by all threads at once (one memory round trip per chunk);
// then the chunk's levels run on LDS alone: thread r computes row r of the
// level, reading each y from the LDS window (src < 0: produced earlier in the
// run, slot = run index mod kYWin) or from the staged copy, writes y to
// global memory and to its window slot, and an LDS-only barrier separates
// the levels. Same operation order as trsv_level.
template <typename T, int KIND, int B, int NTH>
__global__ __launch_bounds__(NTH) void trsv_thin(TrsvArgs a, T alpha, int c0, int c1, int base) {
    __shared__ T ywin[rsp::kYWin];
    __shared__ T lval[rsp::kChunkTerms], lyv[rsp::kChunkTerms];
    __shared__ int lsrc[rsp::kChunkTerms];
    __shared__ rsp::RowTask ltask[rsp::kChunkRows];
    __shared__ T lx[rsp::kChunkRows], ldg[KIND == 2 ? rsp::kChunkRows : 1];  // u_ii: U solve only
    __shared__ int lptr[rsp::kChunkRows + 1], lns[rsp::kChunkRows];  // a chunk has <= kChunkRows levels
    const int tid = threadIdx.x;
    const T *vals = (const T *)a.vals, *x = (const T *)a.x;
    T *y = (T *)a.y;
    const int *ptr = a.plan.ptr_dev;
    for (int c = c0; c < c1; ++c) {
        const rsp::LevelChunk ch = a.plan.chunks[c];
        const int x0 = ch.x0, x1 = ch.x1, k0 = ch.k0, k1 = ch.k1;
        __syncthreads();  // the previous chunk's y stores are visible, LDS is free
        for (int r = tid; r < x1 - x0; r += NTH) {
            const rsp::RowTask t = a.plan.tasks[x0 + r];
            ltask[r] = t;
            lx[r] = alpha * x[t.i];
            if constexpr (KIND == 2) ldg[r] = t.d >= 0 ? vals[t.d] : T(0);
        }
        for (int k = tid; k < k1 - k0; k += NTH) {
            const int sc = a.plan.src[k0 + k];
            lsrc[k] = sc;
            lval[k] = vals[a.plan.tpos[k0 + k]];
            lyv[k] = sc >= 0 ? y[sc] : T(0);
        }
        for (int q = tid; q <= ch.l1 - ch.l0; q += NTH) {
            lptr[q] = ptr[ch.l0 + q];
            if (q < ch.l1 - ch.l0) lns[q] = a.plan.nshort[ch.l0 + q];
        }
        __syncthreads();
        for (int l = ch.l0; l < ch.l1; ++l) {
            const int lp = lptr[l - ch.l0], off = lp - x0, cnt = lptr[l - ch.l0 + 1] - lp,
                      ns = lns[l - ch.l0];
            auto vat = [&](int k) { return lval[k]; };
            auto yat = [&](int k) {
                const int sc = lsrc[k];
                return sc < 0 ? ywin[-sc - 1] : lyv[k];
            };
            for (int r = tid; r < ns; r += NTH) {
                const rsp::RowTask t = ltask[off + r];
                T s = fma_chain<T, B>(lx[off + r], t.t0 - k0, t.t1 - k0, vat, yat);
                if constexpr (KIND == 2) s = s / ldg[off + r];
                y[t.i] = s;
                ywin[(lp + r - base) & (rsp::kYWin - 1)] = s;
            }
            for (int r = ns + (tid >> 6); r < cnt; r += NTH / 64) {  // long rows: a wave each
                const rsp::RowTask t = ltask[off + r];
                T s = wave_chain<T>(lx[off + r], t.t0 - k0, t.t1 - k0, tid & 63, vat, yat);
                if constexpr (KIND == 2) s = s / ldg[off + r];
                if ((tid & 63) == 0) {
                    y[t.i] = s;
                    ywin[(lp + r - base) & (rsp::kYWin - 1)] = s;
                }
            }
            lds_barrier();
        }
    }
}

// Prefetching form of trsv_thin for 1024-thread runs. A chunk holds <= 1024
// rows and <= 2048 terms: one row and two terms per thread. Its staging data
// comes in two dependent loads — the plan (task, sources, term positions,
// level offsets), then the gathers that need it (alpha*x_i, u_ii, term
// values, staged y) — so the prefetch is two chunks deep: while chunk c's
// levels run on LDS, the gathers of chunk c+1 (whose plan arrived during
// chunk c-1) and the plan of chunk c+2 are in flight, and a chunk switch
// costs two barriers and LDS writes instead of a chain of global round
// trips. Every prefetch load is unpredicated (indices clamped into range,
// unused values never stored), so nothing waits for them before the next
// chunk switch. A term that stages y (src >= 0) has its producer > kYWin
// rows before its level ends, i.e. before chunk c began (chunks have
// <= kChunkRows << kYWin rows): that y is final, and its store is visible
// since chunk c's first barrier.
template <typename T, int KIND, int B>
__global__ __launch_bounds__(rsp::kThinThreads) void trsv_thin_pf(TrsvArgs a, T alpha, int c0,
                                                                  int c1, int base) {
    constexpr int NTH = rsp::kThinThreads;
    constexpr int TPT = (rsp::kChunkTerms + NTH - 1) / NTH;  // terms of a chunk per thread
    static_assert(rsp::kChunkRows <= NTH, "one row of a chunk per thread");
    __shared__ T ywin[rsp::kYWin];
    __shared__ T lval[rsp::kChunkTerms], lyv[rsp::kChunkTerms];
    __shared__ int lsrc[rsp::kChunkTerms];
    __shared__ rsp::RowTask ltask[rsp::kChunkRows];
    __shared__ T lx[rsp::kChunkRows], ldg[KIND == 2 ? rsp::kChunkRows : 1];  // u_ii: U solve only
    __shared__ int lptr[rsp::kChunkRows + 1], lns[rsp::kChunkRows];
    const int tid = threadIdx.x;
    const T *vals = (const T *)a.vals, *x = (const T *)a.x;
    T *y = (T *)a.y;
    const int *ptr = a.plan.ptr_dev;
    struct Plan {  // this thread's share of a chunk's plan
        rsp::RowTask t;
        int sc[TPT], tp[TPT];
        int lp, ln, lpe;
    };
    struct Vals {  // ... and of its gathers
        T xv, dg, v[TPT], y[TPT];
    };
    auto load_plan = [&](const rsp::LevelChunk ch) {
        Plan p;
        const int kl = max(ch.k1 - 1, 0), nl = ch.l1 - ch.l0;
        p.t = a.plan.tasks[min(ch.x0 + tid, max(ch.x1 - 1, 0))];
#pragma unroll
        for (int j = 0; j < TPT; ++j) {
            p.sc[j] = a.plan.src[min(ch.k0 + tid + j * NTH, kl)];
            p.tp[j] = a.plan.tpos[min(ch.k0 + tid + j * NTH, kl)];
        }
        p.lp = ptr[ch.l0 + min(tid, nl)];
        p.ln = a.plan.nshort[ch.l0 + min(tid, max(nl - 1, 0))];
        p.lpe = ptr[ch.l1];
        return p;
    };
    auto load_vals = [&](const Plan &p) {
        Vals v;
        v.xv = x[p.t.i];  // alpha applied when staged: no arithmetic on a pending load
        v.dg = KIND == 2 ? vals[max(p.t.d, 0)] : T(0);
#pragma unroll
        for (int j = 0; j < TPT; ++j) {
            v.v[j] = vals[p.tp[j]];
            v.y[j] = y[max(p.sc[j], 0)];
        }
        return v;
    };
    // Chunk switch. The levels write y to the LDS window only; the previous
    // chunk's rows go to global y here, one store per thread, so no global
    // store is pending while levels run and the wait below only ever finds
    // operations issued a whole chunk ago (this chunk's prefetch, the flush
    // before). After it and the barrier, every flush up to the previous switch
    // is complete — the staged y a prefetch reads (producer > kYWin rows back,
    // i.e. in a chunk flushed at least one switch before) is in memory.
    auto mark = [&](int c, int j) {  // diagnostics only (RSP_ILU_TRACE)
        if (a.trace && tid == 0 && 4 * c + j < a.trace_cap) a.trace[4 * c + j] = wall_clock64();
    };
    auto stage = [&](int c, int px0, int px1, const rsp::LevelChunk &ch, const Plan &p,
                     const Vals &v) {
        const int nk = ch.k1 - ch.k0, nl = ch.l1 - ch.l0;
        mark(c, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();  // the previous chunk's levels are done with LDS
        mark(c, 1);
        const bool flush = tid < px1 - px0;
        const int fi = ltask[tid].i;  // read before this thread restages its slot
        const T fv = ywin[(px0 + tid - base) & (rsp::kYWin - 1)];
        if (tid < ch.x1 - ch.x0) {
            ltask[tid] = p.t;
            lx[tid] = alpha * v.xv;
            if constexpr (KIND == 2) ldg[tid] = p.t.d >= 0 ? v.dg : T(0);
        }
#pragma unroll
        for (int j = 0; j < TPT; ++j)
            if (tid + j * NTH < nk) {
                lsrc[tid + j * NTH] = p.sc[j];
                lval[tid + j * NTH] = v.v[j];
                lyv[tid + j * NTH] = p.sc[j] >= 0 ? v.y[j] : T(0);
            }
        if (tid <= nl) lptr[tid] = p.lp;
        if (tid < nl) lns[tid] = p.ln;
        if (tid == 0 && nl == NTH) lptr[NTH] = p.lpe;
        if (flush) y[fi] = fv;  // after the last use of the prefetched registers
        lds_barrier();
        mark(c, 2);
    };
    auto levels = [&](const rsp::LevelChunk &ch) {
        const int x0 = ch.x0, k0 = ch.k0;
        for (int l = ch.l0; l < ch.l1; ++l) {
            const int lp = lptr[l - ch.l0], off = lp - x0, cnt = lptr[l - ch.l0 + 1] - lp,
                      ns = lns[l - ch.l0];
            auto vat = [&](int k) { return lval[k]; };
            auto yat = [&](int k) {
                const int sc = lsrc[k];
                return sc < 0 ? ywin[-sc - 1] : lyv[k];
            };
            if (tid < ns) {
                const rsp::RowTask t = ltask[off + tid];
                T s = fma_chain<T, B>(lx[off + tid], t.t0 - k0, t.t1 - k0, vat, yat);
                if constexpr (KIND == 2) s = s / ldg[off + tid];
                ywin[(lp + tid - base) & (rsp::kYWin - 1)] = s;
            }
            for (int r = ns + (tid >> 6); r < cnt; r += NTH / 64) {  // long rows: a wave each
                const rsp::RowTask t = ltask[off + r];
                T s = wave_chain<T>(lx[off + r], t.t0 - k0, t.t1 - k0, tid & 63, vat, yat);
                if constexpr (KIND == 2) s = s / ldg[off + r];
                if ((tid & 63) == 0) ywin[(lp + r - base) & (rsp::kYWin - 1)] = s;
            }
            lds_barrier();
            if (a.trace && tid == 0 && l < a.trace_cap / 2)  // diagnostics: level end stamps
                a.trace[a.trace_cap / 2 + l] = wall_clock64();
        }
    };
    // two register sets, A and B, alternate between even and odd chunks (no
    // copies of pending loads); chunk indices past the run are clamped, so
    // every prefetch is unconditional
    const int cl = c1 - 1;
    // chunk records through the constant address space: scalar loads, which
    // the y stores cannot alias and which leave vmcnt to the prefetch; each is
    // fetched one chunk before its plan is
    typedef const __attribute__((address_space(4))) int *ChunkPtr;
    const ChunkPtr chunks = (ChunkPtr)a.plan.chunks;
    auto chunk = [&](int c) {
        const ChunkPtr q = chunks + (size_t)c * (sizeof(rsp::LevelChunk) / sizeof(int));
        rsp::LevelChunk r;
        r.l0 = q[0];
        r.l1 = q[1];
        r.x0 = q[2];
        r.x1 = q[3];
        r.k0 = q[4];
        r.k1 = q[5];
        return r;
    };
    rsp::LevelChunk ra = chunk(c0), rb = chunk(min(c0 + 1, cl)), rn = chunk(min(c0 + 2, cl));
    Plan pa = load_plan(ra), pb = load_plan(rb);
    Vals va = load_vals(pa), vb;
    int px0 = 0, px1 = 0;  // the chunk to flush at the next switch
    for (int c = c0; c < c1; c += 2) {
        const rsp::LevelChunk ca = ra;
        stage(c, px0, px1, ca, pa, va);
        vb = load_vals(pb);  // chunk c+1's gathers
        pa = load_plan(rn);  // chunk c+2's plan
        ra = rn;
        rn = chunk(min(c + 3, cl));
        levels(ca);
        mark(c, 3);
        px0 = ca.x0;
        px1 = ca.x1;
        if (c + 1 >= c1) break;
        const rsp::LevelChunk cb = rb;
        stage(c + 1, px0, px1, cb, pb, vb);
        va = load_vals(pa);  // chunk c+2's gathers
        pb = load_plan(rn);  // chunk c+3's plan
        rb = rn;
        rn = chunk(min(c + 4, cl));
        levels(cb);
        mark(c + 1, 3);
        px0 = cb.x0;
        px1 = cb.x1;
    }
    // the last chunk's rows (its levels ended with a barrier)
    if (tid < px1 - px0) y[ltask[tid].i] = ywin[(px0 + tid - base) & (rsp::kYWin - 1)];
}

// --------------------------------------------------------------- launchers

template <typename T, int B>
static hipError_t launch_factor(const IluArgs &a, hipStream_t s) {
    const LevelPlan &P = a.plan;
    for (int g = 0; g < P.nseg; ++g) {
        const rsp::LevelSeg sg = P.segs[g];
        if (sg.thin) {
            hipLaunchKernelGGL((ilu0_chunked<T>), dim3(1), dim3(kThinThreads), 0, s, a, sg.c0, sg.c1);
            continue;
        }
        for (int l = sg.lb; l < sg.le; ++l) {
            const int off = P.ptr_host[l], cnt = P.ptr_host[l + 1] - off;
            if (cnt <= 0) continue;
            hipLaunchKernelGGL((ilu0_level<T, B>), dim3((cnt + kIluWaves - 1) / kIluWaves),
                               dim3(64 * kIluWaves), 0, s, a, off, cnt);
        }
    }
    return hipGetLastError();
}

template <typename T, int KIND, int B>
static hipError_t launch_solve(const TrsvArgs &a, hipStream_t s) {
    const LevelPlan &P = a.plan;
    const T alpha = (T)a.alpha;
    for (int g = 0; g < P.nseg; ++g) {
        const rsp::LevelSeg sg = P.segs[g];
        if (sg.thin) {
            const int base = P.ptr_host[sg.lb];
            if (sg.nth <= 64)
                hipLaunchKernelGGL((trsv_thin<T, KIND, B, 64>), dim3(1), dim3(64), 0, s, a, alpha,
                                   sg.c0, sg.c1, base);
            else if (sg.nth <= 256)
                hipLaunchKernelGGL((trsv_thin<T, KIND, B, 256>), dim3(1), dim3(256), 0, s, a, alpha,
                                   sg.c0, sg.c1, base);
            else if (a.thin_prefetch)
                hipLaunchKernelGGL((trsv_thin_pf<T, KIND, B>), dim3(1), dim3(kThinThreads), 0, s, a,
                                   alpha, sg.c0, sg.c1, base);
            else
                hipLaunchKernelGGL((trsv_thin<T, KIND, B, kThinThreads>), dim3(1), dim3(kThinThreads),
                                   0, s, a, alpha, sg.c0, sg.c1, base);
            continue;
        }
        for (int l = sg.lb; l < sg.le; ++l) {
            const int off = P.ptr_host[l], cnt = P.ptr_host[l + 1] - off;
            if (cnt <= 0) continue;
            const int ns = P.nshort_host[l], nb = (ns + 255) / 256;
            hipLaunchKernelGGL((trsv_level<T, KIND, B>), dim3(nb + (cnt - ns + 3) / 4), dim3(256), 0,
                               s, a, alpha, off, cnt, ns, nb);
        }
    }
    return hipGetLastError();
}

// batch width from the plan (2, 4 or 8)
template <typename T>
static hipError_t factor_dispatch(const IluArgs &a, hipStream_t s) {
    switch (a.plan.batch) {
        case 2: return launch_factor<T, 2>(a, s);
        case 4: return launch_factor<T, 4>(a, s);
        default: return launch_factor<T, 8>(a, s);
    }
}

template <typename T, int KIND>
static hipError_t solve_dispatch(const TrsvArgs &a, hipStream_t s) {
    switch (a.plan.batch) {
        case 2: return launch_solve<T, KIND, 2>(a, s);
        case 4: return launch_solve<T, KIND, 4>(a, s);
        default: return launch_solve<T, KIND, 8>(a, s);
    }
}

hipError_t ilu0_factor_f32(const IluArgs &a, hipStream_t s) { return factor_dispatch<float>(a, s); }
hipError_t trsv_lower_n_f32(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<float, 0>(a, s); }
hipError_t trsv_lower_t_f32(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<float, 1>(a, s); }
hipError_t trsv_upper_f32(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<float, 2>(a, s); }
#ifndef RSP_FTZ_BUILD
hipError_t ilu0_factor_f64(const IluArgs &a, hipStream_t s) { return factor_dispatch<double>(a, s); }
hipError_t trsv_lower_n_f64(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<double, 0>(a, s); }
hipError_t trsv_lower_t_f64(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<double, 1>(a, s); }
hipError_t trsv_upper_f64(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<double, 2>(a, s); }
#endif

}  // namespace RSP_KNS
