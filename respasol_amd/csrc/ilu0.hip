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

#include <type_traits>
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

// Fused multiply-add in the working precision: v_fma_f64 / v_fma_f32 (one
// rounding), as the oracle's fma / fmaf. (__builtin_fma on float operands
// would compute in double and round twice.)
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// x / d, the IEEE quotient rounded to T. The FTZ build's float division
// switches the denormal mode on and off around its Newton steps (two
// s_setreg per division: the only difference between ilu0_rounds<float> in
// rsp_k and rsp_k_ftz, found in their ISA), serialising the wave on every
// l_ik = a_ik / u_kk. Here the FTZ build takes a float quotient in double,
// rounded once to float: double has >= 2 * 24 + 2 bits, so that is the
// correctly rounded float quotient for every operand, with fp32 denormals
// flushed by the mode as the oracle's DAZ/FTZ (same bits as the float
// division). Measured on dc1, matrix-new_3, xenon2, ASIC_320ks, crashbasis
// (FTZ factor, ms): float division 25.32, this 24.89; the float Newton
// sequence without the mode switch is 24.06 but loses the correct rounding
// when a residual is denormal (numerators near 2^-103, divisors >= 2^126),
// and guarding it (range checks + rescaling, 26.33; a fallback branch,
// 27.88) costs more than it saves: the division is on the factor's
// dependency chain (profiles/r06_ftz_division_ab.txt).
template <typename T>
__device__ __forceinline__ T qdiv(T x, T d) {
#ifdef RSP_FTZ_BUILD
    if constexpr (sizeof(T) == 4) {
        // (the empty asm keeps the optimiser from folding the widened
        // division back into a float one, a legal rewrite it makes)
        double xd = x, dd = d;
        asm volatile("" : "+v"(xd), "+v"(dd));
        return (float)(xd / dd);
    }
#endif
    return x / d;
}


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
            if (b0 + b < n) s = fma_t(-v[b], y[b], s);
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
        for (int j = 0; j < cnt; ++j) s = fma_t(-wave_read(v, j), wave_read(yv, j), s);
    }
    return s;
}

// The same chain for one fat-level row by a wave, on LDS broadcast operands:
// each group of 64 terms is gathered by the lanes (values, then y; the next
// group's loads are issued before this group's chain), parked in the wave's
// LDS rows, and every lane runs the in-order fma chain reading them (reads
// independent of the sum, so they issue ahead of it) — instead of four
// readlanes per term. One fma per term in order: the same bits.
template <typename T>
__device__ __forceinline__ T wave_chain_lds(T s, int k0, int k1, int lane, T *wv, T *wy, const T *sval,
                                           const int *src, const T *y) {
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    };
    int k = min(k0 + lane, k1 - 1);
    T v = sval[k];
    int id = src[k];
    T yv = y[id];
    for (int base = k0; base < k1; base += 64) {
        wv[lane] = v;
        wy[lane] = yv;
        wave_sync();
        const int cnt = min(64, k1 - base);
        const bool more = base + 64 < k1;
        if (more) {  // the next group's values and y indices in flight under this chain
            k = min(base + 64 + lane, k1 - 1);
            v = sval[k];
            id = src[k];
        }
        int j = 0;
        for (; j + 4 <= cnt; j += 4) {
            T p[4], q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                p[u] = wv[j + u];
                q[u] = wy[j + u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) s = fma_t(-p[u], q[u], s);
        }
        for (; j < cnt; ++j) s = fma_t(-wv[j], wy[j], s);
        wave_sync();  // this group's reads before the next group's stores
        if (more) yv = y[id];
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
            vals[p] = qdiv<T>(factor_entry<T, B>(a, vals, p), ukk);
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

// Wait until the LDS counter *p >= want (wave-uniform value; bounded: a plan
// bug gives wrong bits in the tests, never a hung GPU). RSP_POLL_MODE (A/B):
// 0 (shipped) = read -> wait -> compare; 1 = two reads in flight, each step
// waiting for the older one only; 2 = s_sleep(RSP_POLL_SLEEP) between reads;
// 3 = s_sleep only while the counter is below `near` (the wave is not next in
// line). Config 3, same box, interleaved x2: fp64 factor / solve 58.5-58.8 /
// 43.5-43.7 ms (mode 0), 59.6-59.7 / 46.7 (mode 1), 59.8 / 45.8 (mode 2,
// sleep 1), 60.2 / 47.3 (sleep 2), 59.0 / 47.3 (mode 3, sleep 1; dc1 solve
// 4.88 -> 6.23 ms), 58.9 / 48.8 (sleep 3). Also measured slower: reading the
// counter and the level's y values together in every poll, so a level pays
// one LDS round trip after its producer instead of two (solve 43.5 -> 45.4
// ms; dc1 4.86 -> 5.62). A narrow level is ~425 cycles (160 ns, dc1,
// RSP_ILU_TRACE_CLK) and any extra LDS traffic or wake-up delay lands on it.
// (Mode 1 was removed in round 4 with the other inline-asm ordering.)
// 4 (round 5) = s_sleep between reads, ended early by the publishing wave's
// s_wakeup: dc1 fp32 solve 4.16 -> 4.71 ms, the factor slower too
// (profiles/r05_poll_wakeup_ab.txt).
// The counter is published by lds_publish (release) and read here with an
// acquire fence after the last poll: the HIP memory model orders a wave's y
// stores before the counter and the waiting wave's y loads after it.
#ifndef RSP_POLL_MODE
#define RSP_POLL_MODE 0
#endif
#ifndef RSP_POLL_SLEEP
#define RSP_POLL_SLEEP 1
#endif
__device__ __forceinline__ void lds_wait_geq(int *p, int want, int near) {
#if RSP_POLL_MODE == 4
    // sleep between polls; the publishing wave's s_wakeup (lds_publish) ends
    // the sleep at once, so a waiting wave neither polls the LDS continuously
    // (its reads queue beside the working wave's) nor sleeps past the hand-off
    for (int it = 0; it < (1 << 26) && __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want;
         ++it)
        __builtin_amdgcn_s_sleep(RSP_POLL_SLEEP);
#elif RSP_POLL_MODE == 3
    for (int it = 0; it < (1 << 26); ++it) {
        const int c = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (c >= want) break;
        if (c < near) __builtin_amdgcn_s_sleep(RSP_POLL_SLEEP);  // not next in line: poll less
    }
#else
    for (int it = 0; it < (1 << 26) && __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want;
         ++it) {
#if RSP_POLL_MODE == 2
        __builtin_amdgcn_s_sleep(RSP_POLL_SLEEP);
#endif
    }
#endif
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Publish an LDS counter of completed levels / rounds (lane 0 of the wave
// that completed them): a workgroup-scope release store, so every LDS store
// of the wave before it (its y / values) is visible to a wave whose
// lds_wait_geq has seen the new value. RSP_LDS_RELAXED (A/B builds only): the
// round-3 form, a relaxed store behind a compiler-only fence, which relied on
// one wave's LDS operations being performed in order.
#ifndef RSP_LDS_RELAXED
#define RSP_LDS_RELAXED 0
#endif
__device__ __forceinline__ void lds_publish(int *p, int v, bool leader) {
#if RSP_LDS_RELAXED
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (leader) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
    if (leader) __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
#if RSP_POLL_MODE == 4
    asm volatile("s_wakeup" ::: "memory");  // the waves sleeping in lds_wait_geq
#endif
}

// --------------------------------------------------------------- kernels

// Fat level, global-memory path: one wave per row.
template <typename T, int B>
__global__ __launch_bounds__(64 * kIluWaves) void ilu0_level(IluArgs a, int off, int nrows) {
    const int w = blockIdx.x * kIluWaves + (threadIdx.x >> 6);
    if (w >= nrows) return;
    factor_row<T, B>(a, a.plan.rows[off + w], threadIdx.x & 63);
}

// The stages of one fat-level row on LDS operands (ilu0_level_lds and
// ilu0_level_slot): lower positions stage by stage, l_ij = v / u_jj, then the
// upper positions; rv holds the row's values on entry and its factor on exit.
template <typename T>
__device__ __forceinline__ void row_lds_factor(T *rv, const T *dv, const T *pu, const int *up,
                                               const int *lo, const int *le, const unsigned short *pl,
                                               int nlo, int nr, int lane, int hasdiag, int i,
                                               int *zero_pivot) {
    auto wave_sync = [] {  // order this wave's LDS stores before its later loads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    };
    wave_sync();
    auto entry = [&](int x) {  // a_ij - sum l_ik u_kj over its pairs, k ascending
        T v = rv[x];
        const int u0 = up[x], u1 = up[x + 1];
        auto batch = [&](int u) {
            T l[4], w[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int uu = min(u + b, u1 - 1);
                l[b] = rv[pl[uu]];
                w[b] = pu[uu];
            }
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (u + b < u1) v = fma_t(-l[b], w[b], v);
        };
        if (u1 > u0) {  // the first batch straight-line
            batch(u0);
            for (int u = u0 + 4; u < u1; u += 4) batch(u);
        }
        return v;
    };
    for (int s = 0; s < nlo;) {  // lower positions, stage by stage
        const int e = le[s];
        for (int x = s + lane; x < e; x += 64) {
            const int r = lo[x];
            const T d = dv[r];  // read before the chain, not after it
            rv[r] = qdiv<T>(entry(r), d);
        }
        wave_sync();
        s = e;
    }
    for (int x = nlo + lane; x < nr; x += 64) {  // upper positions (never operands of this row)
        const T v = entry(x);
        rv[x] = v;
        if (x == nlo && hasdiag && v == T(0)) atomicMin(zero_pivot, i);
    }
    wave_sync();
}

// Fat level, one wave (workgroup) per row with the row staged in LDS. Every
// operand that does not come from the row itself is final before the level
// starts: the u_kj of all the row's update pairs (rows of earlier levels)
// and its divisors u_kk. So they, the row's values and its stage structure
// are loaded up front in a few independent memory round trips; the stages
// then run on LDS operands only (an l_ik of an earlier stage is the row's own
// LDS value; one wave's LDS accesses are in order), and the row is written
// back once. Same per-position fma sequence and division as factor_row, so
// bitwise equal to it. Rows beyond kFacRow entries or kFacPairs pairs take
// the global path (factor_row).
template <typename T, int B>
__global__ __launch_bounds__(64) void ilu0_level_lds(IluArgs a, int off) {
    constexpr int R = rsp::kFacRow, Q = rsp::kFacPairs;
    __shared__ T rv[R], dv[R], pu[Q];
    __shared__ int up[R + 1], lo[R], le[R];
    __shared__ unsigned short pl[Q];
    const int lane = threadIdx.x;
    const rsp::FacRow fr = a.frow[off + blockIdx.x];
    T *vals = (T *)a.vals;
    const int i = fr.i, rs = fr.rs, re = fr.re, q0 = fr.q0;
    const int nr = re - rs, nq = fr.q1 - q0, nlo = fr.di - rs;
    if (nr > R || nq > Q) {
        factor_row<T, B>(a, i, lane);
        return;
    }
    for (int x = lane; x < nr; x += 64) {
        const bool lower = x < nlo;
        const int d = lower ? a.udiv[rs + x] : -1;
        rv[x] = vals[rs + x];
        dv[x] = d >= 0 ? vals[d] : T(0);
        up[x] = a.upd_ptr[rs + x] - q0;
        if (lower) {
            lo[x] = a.lord[rs + x] - rs;
            le[x] = a.lend[rs + x] - rs;
        }
    }
    if (lane == 0) up[nr] = nq;
    for (int u = lane; u < nq; u += 64) {
        pl[u] = (unsigned short)(a.upd_l[q0 + u] - rs);
        pu[u] = vals[a.upd_u[q0 + u]];
    }
    row_lds_factor<T>(rv, dv, pu, up, lo, le, pl, nlo, nr, lane, fr.hasdiag, i, a.zero_pivot);
    for (int x = lane; x < nr; x += 64) vals[rs + x] = rv[x];
}

// ------------------------------------------------- flow hand-offs (helpers)
// Words handed between workgroups of one persistent launch (trsv_flow,
// ilu0_flow): written once by a 4- / 8-byte device-scope (sc1) store, read by
// device-scope (sc1) loads, which bypass the reader's L1 — MI355X_MICROARCH.md
// (inter-workgroup visibility; price list, handoff-1to1 / handoff-flag).
template <typename T>
struct FlowWord;
template <>
struct FlowWord<double> {
    typedef unsigned long long U;
    static constexpr U kNotYet = 0x7ff5eed15eed1001ull;
};
template <>
struct FlowWord<float> {
    typedef unsigned int U;
    static constexpr U kNotYet = 0x7fa5eed1u;
};
// A flow wait gives up after fc.ticks of the 100 MHz wall clock (default
// 0.2 s, RSP_ILU_FLOW_TIMEOUT_US) and records the call's generation in
// *fc.status (rsp::FlowCtl).
__device__ __forceinline__ void flow_give_up(const rsp::FlowCtl &fc) {
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(fc.status, fc.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Work-item claims of a flow launch (rsp::FlowCtl): lane 0 takes the next
// item with an agent-scope fetch_add, issued one item ahead (its return is
// read at the top of the next item, so the atomic's latency overlaps the
// current item); flow_item() turns the claim into the item index.
__device__ __forceinline__ unsigned long long flow_claim(const rsp::FlowCtl &fc) {
    return (threadIdx.x & 63) == 0
               ? __hip_atomic_fetch_add(fc.claim, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
               : 0ull;
}
__device__ __forceinline__ int flow_item(unsigned long long c, unsigned long long base, int it0, int it1) {
    // the difference fits an int (claims of this launch); lane 0's is the one
    const long long d = (long long)(c - base);
    return __builtin_amdgcn_readfirstlane((int)min(d, (long long)(it1 - it0))) + it0;
}

// One wave's walk over the items [it0, it1) of a flow launch (rsp::FlowCtl):
//   for (fq.first(); fq.more(); fq.next()) { const int it = fq.item(); ... }
// A wait inside an item that returns true (fq.expire(), tickets only) makes
// the item yield: it runs through on what it has but stores nothing, and
// fq.item_end(it, true) has next() run it again or walk a grown ticket list.
// Static (RSP_ILU_FLOW_MODE=0): w, w + W, ... (the whole grid must be resident).
// Claimed (kFlowClaims): in start order, TWO items ahead — the claim for item
// j + 2 is issued during item j, behind its first loads (claim_ahead), and
// read when item j + 1 ends, so the atomic's latency hides under a whole
// item. A wave makes 2 + (items it processes) claims, so a launch advances
// the counter by exactly items + 2 W (flow_claims on the host). The lowest
// unfinished item is always some running wave's CURRENT item (a wave's
// claimed items are above its current one), so progress needs no
// co-residency.
// Start tickets (kFlowTickets, the default): thread 0 takes the workgroup's
// ticket t — from one of eight counters (blockIdx % 8; counter q hands out
// q, q + 8, ..., so the G start claims do not queue on one address) of the
// launch's counter slot (base & 1; block 0 zeroes the other slot for the
// next launch, the previous launch's, which has ended) — and each wave walks
// the static items of t, it0 + 4 t + wave + k W: a resident grid runs
// exactly the static walk. A workgroup whose counter is spent owns nothing.
// Steals: a wait past kFlowStealUs (2 us once its workgroup has stolen)
// asks expire(): with every counter spent and the owned list unchanged
// (calm) it waits on; else the item yields — it runs through on what it
// has, stores nothing — and next() claims another ticket for the workgroup
// (under an LDS lock, inserted so that own[] stays ascending) unless none
// is left, then runs the item again — unless the list has grown (by this
// steal or another wave's): then the wave walks again from the start:
// rounds k = 0, 1, ..., in each the owned tickets in list order — the
// merged index order of its items — skipping the items it has finished
// (those of the start ticket below the round it had reached, and those
// marked with the call's epoch in fc.done since).
// A wave out of items waits in the workgroup until all four are (the list
// could still grow), counted with the list length in one LDS word.
// Progress: let u be the lowest unfinished item. If its ticket is owned,
// its owner's wave for u has walked every owned item below u (finished) and
// is at u, or waits on a higher item or for its siblings and sees the list
// grow once u's ticket joined it: it comes to u, whose operands are lower
// items, finished. If u's ticket is unclaimed, every started wave that
// cannot go on waits, and either steals (a ticket is claimed) or its
// workgroup ends (a new one starts and claims). Every wait is bounded by
// fc.ticks; nothing needs co-residency.
struct FlowTicketLds {
    int own[rsp::kFlowOwnMax];  // the workgroup's tickets, ascending (own[0] the start ticket until a steal)
    int state;                  // tickets owned | waves out of items << 16
    int lock;                   // a steal is in progress
    int dry;                    // every counter is spent: no ticket left to steal
};
template <bool TK>  // TK: start tickets (kFlowTickets); else static or claimed (fc.mode)
struct FlowClaims {
    const rsp::FlowCtl &fc;
    unsigned long long base, c1 = 0, c2 = 0;
    int it0, it1, cur, stride, wv;
    int mode;  // 0 static, 1 claims, 2 tickets (TK)
    FlowTicketLds *L;
    // tickets: the owned list as this wave last read it, its position
    // (round k, list index j), the round its fast walk reached (start ticket
    // items below it are finished), whether it walks with done checks
    int nseen = 0, k = 0, j = 0, fast_k = 0, t0 = 0;
    // a wait this long (100 MHz ticks) may steal: kFlowStealUs, 2 us after a steal
    unsigned long long steal_at = 100ull * rsp::kFlowStealUs;
    bool scan = false, redo = false, over = false;
    __device__ FlowClaims(const rsp::FlowCtl &f, unsigned long long b, int i0, int i1, int w, int W,
                          FlowTicketLds *l)
        : fc(f), base(b), it0(i0), it1(i1), cur(i0 + w), stride(W), wv(w & 3),
          mode(TK ? 2 : (f.mode & rsp::kFlowClaims) ? 1 : 0), L(l) {}
    // tickets: counter q of this launch's slot hands out q, q + 8, q + 16, ...
    // (eight counters, so the G start claims do not queue on one address)
    __device__ unsigned *ctr() const { return fc.tickets + rsp::kFlowTicketCtrs * (int)(base & 1); }
    __device__ int take(int q) const {
        return q + rsp::kFlowTicketCtrs * (int)__hip_atomic_fetch_add(ctr() + q, 1u, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ bool spent(int q) const {  // counter q has no ticket < G left
        return q + rsp::kFlowTicketCtrs * (long long)__hip_atomic_load(ctr() + q, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT) >= (long long)gridDim.x;
    }
    __device__ static int lds_ld(const int *p) {
        return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    }
    // LDS-only acquire (the "local" address-space fence): a workgroup-scope
    // acquire on a plain atomic would also wait for the wave's outstanding
    // GLOBAL accesses (s_waitcnt vmcnt(0))
    __device__ static int lds_acq(const int *p) {
        const int v = lds_ld(p);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        return v;
    }
    __device__ void first() {
        if constexpr (!TK) {
            if (mode == 1) {
                const unsigned long long c0 = flow_claim(fc);
                c1 = flow_claim(fc);
                cur = flow_item(c0, base, it0, it1);
            }
            return;
        }
        if (threadIdx.x == 0) {
            if (blockIdx.x == 0)  // the next launch's slot (the previous launch's: it has ended)
                for (int q = 0; q < rsp::kFlowTicketCtrs; ++q)
                    __hip_atomic_store(fc.tickets + rsp::kFlowTicketCtrs * (int)((base + 1) & 1) + q, 0u,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int t = take(blockIdx.x % rsp::kFlowTicketCtrs);
            L->own[0] = t;
            L->state = t < (int)gridDim.x ? 1 : 0;
            L->lock = 0;
            L->dry = t >= (int)gridDim.x;
        }
        __syncthreads();  // (once, at the start)
        nseen = lds_ld(&L->state) & 0xffff;
        t0 = lds_ld(&L->own[0]);
        settle();
    }
    __device__ bool more() const { return TK ? !over : cur < it1; }
    __device__ int item() const { return cur; }
    __device__ void claim_ahead() {
        __builtin_amdgcn_sched_barrier(0);
        if (mode == 1) c2 = flow_claim(fc);
        __builtin_amdgcn_sched_barrier(0);
    }
    // tickets: from position (k, j), the next item of this wave to run
    // (cur), or none left in the workgroup (over)
    __device__ void settle() {
        if (!scan && nseen == 1) {  // the start ticket alone: the static walk
            const int it = it0 + 4 * t0 + wv + k * stride;
            if (it < it1) {
                cur = it;
                return;
            }
        }
        for (;;) {
            if (j >= nseen && nseen > 0) {
                ++k;
                j = 0;
            }
            if (nseen > 0) {
                const int tj = lds_ld(&L->own[j]);
                const int it = it0 + 4 * tj + wv + k * stride;
                if (it < it1) {
                    const bool fin = scan && ((tj == t0 && k < fast_k) ||
                                              __hip_atomic_load(fc.done + it, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_WAVEFRONT) == (int)fc.epoch);
                    if (!fin) {
                        cur = it;
                        return;
                    }
                    ++j;
                    continue;
                }
                if (j > 0) {  // the rest of round k is past it1 too
                    ++k;
                    j = 0;
                    continue;
                }
            }
            const int s = idle();  // out of items
            if (s < 0) {
                over = true;
                cur = it1;
                return;
            }
            rescan(s);
        }
    }
    // walk again from the start over an owned list of s tickets
    __device__ void rescan(int s) {
        if (!scan) fast_k = k;  // (the fast walk was at round k of the start ticket)
        scan = true;
        steal_at = 200;
        nseen = s;
        k = j = 0;
    }
    // out of items: wait until the owned list grows (its new length) or all
    // four waves are out (-1)
    __device__ int idle() {
        const int me = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63));
        int r = -1;
        if ((int)(threadIdx.x & 63) == me) {
            int s = __hip_atomic_fetch_add(&L->state, 1 << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) +
                    (1 << 16);
            for (;;) {
                if ((s & 0xffff) != nseen) {
                    __hip_atomic_fetch_add(&L->state, -(1 << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    r = s & 0xffff;
                    break;
                }
                if ((s >> 16) == 4) break;
                __builtin_amdgcn_s_sleep(2);
                s = __hip_atomic_load(&L->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        r = __builtin_amdgcn_readfirstlane(r);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");  // own[] entries up to r
        return r;
    }
    // a wait that began at wall clock t0 runs until this deadline, then
    // expire() tells it to give up or (tickets) to yield the item to next(),
    // which may steal, then runs the item again or walks a grown list; the
    // give-up bound counts from the wait's start (one compare per poll, as
    // without tickets; nothing written, so a wait of one lane is fine). An
    // item yields only while a steal can follow (not calm), fewer than G + 1
    // times per wave, so no item escapes the bound by yielding.
    __device__ unsigned long long deadline(unsigned long long t0) const {
        if constexpr (!TK) return t0 + fc.ticks;
        return t0 + min(fc.ticks, steal_at);
    }
    // a wait past its deadline: 0 give up, 1 yield, 2 wait on until the new
    // deadline dl (tickets: nothing to steal and the owned list as this wave
    // knows it — every ticket is claimed, a grown list would have had a
    // steal succeed first)
    __device__ int expire(unsigned long long now, unsigned long long t0, unsigned long long &dl) const {
        if (TK && now <= t0 + fc.ticks) {
            if (!calm()) return 1;
            dl = t0 + fc.ticks;
            return 2;
        }
        flow_give_up(fc);
        return 0;
    }
    // tickets: no steal can succeed (LDS dry, set here once the counter
    // shows all G tickets claimed) and the owned list has not grown past nseen
    __device__ bool calm() const {
        if constexpr (!TK) return true;
        if (!__hip_atomic_load(&L->dry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            for (int q = 0; q < rsp::kFlowTicketCtrs; ++q)
                if (!spent(q)) return false;
            __hip_atomic_store(&L->dry, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return (__hip_atomic_load(&L->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & 0xffff) == nseen;
    }
    // next() after a yield: the owned list's length if it has grown past
    // nseen (maybe by a steal made here), else 0
    __device__ int steal() {
        const int me = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63));
        int r = 0;
        if ((int)(threadIdx.x & 63) == me) {
            const int s = __hip_atomic_load(&L->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((s & 0xffff) != nseen)
                r = s & 0xffff;
            else if (!__hip_atomic_load(&L->dry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                int z = 0;
                if (__hip_atomic_compare_exchange_strong(&L->lock, &z, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP)) {
                    const int n = __hip_atomic_load(&L->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) &
                                  0xffff;
                    if (n != nseen)
                        r = n;
                    else if (n < rsp::kFlowOwnMax) {
                        int t = (int)gridDim.x;
                        for (int d = 0; d < rsp::kFlowTicketCtrs && t >= (int)gridDim.x; ++d) {
                            const int q = (int)(blockIdx.x + d) % rsp::kFlowTicketCtrs;
                            if (!spent(q)) t = take(q);
                        }
                        if (t < (int)gridDim.x) {  // insert, keeping own[] ascending
                            int x = n;
                            for (; x > 0 && L->own[x - 1] > t; --x) L->own[x] = L->own[x - 1];
                            L->own[x] = t;
                            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                            __hip_atomic_fetch_add(&L->state, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            r = n + 1;
                        } else
                            __hip_atomic_store(&L->dry, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    __hip_atomic_store(&L->lock, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
        r = __builtin_amdgcn_readfirstlane(r);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");  // own[] entries up to r
        return r;
    }
    // the item is finished: after a steal its index is marked with the epoch
    __device__ void done(int it) const {
        if (TK && scan && (threadIdx.x & 63) == 0)
            __hip_atomic_store(fc.done + it, (int)fc.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    // the item ends: finished, or (yl) yielded — then next() runs it again
    // unless the owned list grows
    __device__ void item_end(int it, bool yl) {
        if constexpr (!TK) return;
        if (yl)
            redo = true;
        else
            done(it);
    }
    __device__ void next() {
        if constexpr (!TK) {
            if (mode == 0) {
                cur += stride;
            } else {
                cur = flow_item(c1, base, it0, it1);
                c1 = c2;
            }
            return;
        }
        if (__builtin_expect(!redo && !scan && nseen == 1, 1)) {  // the static walk of the start ticket
            cur += stride;
            ++k;
            if (cur < it1) return;
        } else if (redo) {  // the item yielded: it runs again unless the owned list grows
            redo = false;
            const int n = steal();
            if (n == 0) return;
            rescan(n);
        } else
            ++j;
        settle();
    }
};

template <typename T>
__device__ __forceinline__ typename FlowWord<T>::U flow_load(const T *p) {
    return __hip_atomic_load((typename FlowWord<T>::U *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void flow_store(T *p, T v) {
    typedef typename FlowWord<T>::U U;
    __hip_atomic_store((U *)p, __builtin_bit_cast(U, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Re-read this lane's operand words [0, n) that are still kNotYet until none
// of the wave's is (wave-uniform loop; the pause between polls doubles up to
// max_sleep s_sleep units of 64 clocks). True: the item yields (FlowClaims::expire).
template <typename T, int NB, typename FQ>
__device__ __forceinline__ bool flow_wait(typename FlowWord<T>::U (&w)[NB], const int (&id)[NB], int n,
                                          const T *y, FQ &fq, int max_sleep, bool skip = false) {
    constexpr auto kNot = FlowWord<T>::kNotYet;
    auto pending = [&] {
        bool p = false;
#pragma unroll
        for (int b = 0; b < NB; ++b) p |= b < n && w[b] == kNot;
        return p;
    };
    if (!__ballot(pending())) return false;
    const unsigned long long t0 = wall_clock64();
    unsigned long long dl = skip ? 0ull : fq.deadline(t0);  // (skip: the item has yielded)
    for (int sl = 1;; sl = min(2 * sl, max_sleep)) {
        for (int q = 0; q < sl; ++q) __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (b < n && w[b] == kNot) w[b] = flow_load(y + id[b]);
        if (!__ballot(pending())) return false;
        const unsigned long long now = wall_clock64();
        if (now > dl) {
            const int r = fq.expire(now, t0, dl);
            if (r != 2) return r != 0;
        }
    }
}

// An item's gate: before polling its own operands, a wave waits (one lane,
// one word) for the y of the last row of the level three below its own (plan:
// RSP_ILU_FLOW_GATE; 2 and 1 measured slower) — only
// a throttle, so that waves whose items are far ahead of the progress front
// poll one word instead of a word per operand (the operand polls alone, up to
// 8 per lane, slowed the loads on the critical path). Row g's item has a
// lower index, so the gate cannot deadlock.
template <typename T, typename FQ>
__device__ __forceinline__ bool flow_gate(int g, const T *y, FQ &fq, int max_sleep) {
    if (g < 0) return false;
    typename FlowWord<T>::U w[1] = {0};
    int id[1] = {g};
    if ((threadIdx.x & 63) == 0) w[0] = flow_load(y + g);
    return flow_wait<T, 1>(w, id, (threadIdx.x & 63) == 0 ? 1 : 0, y, fq, max_sleep);
}

// Fat level in the slot layout (rsp::FacSlotLevel): the row's structure is
// one fixed-stride slot, so its header, divisor positions, packed stage
// structure and update pairs are one memory round trip, issued together
// (KR / KQ = the level's entries / pairs per lane, compile-time, loads
// clamped and unpredicated); the values they point at (the row's a_ij, its
// divisors u_kk, the u_kj of its pairs) are the second. ilu0_level_lds reads
// a record first and then loops over its arrays, a dependent round trip per
// 64 pairs. Same LDS stages (row_lds_factor), so the same bits.
template <typename T, int KR, int KQ>
__global__ __launch_bounds__(64) void ilu0_level_slot(IluArgs a, const int *__restrict__ lvl, int stride,
                                                      int rm, int qm) {
    constexpr int R = rsp::kFacRow, Q = rsp::kFacPairs;
    static_assert(KR * 64 <= R && KQ * 64 <= Q, "slot kernel budgets");
    __shared__ T rv[R], dv[R], pu[Q];
    __shared__ int up[R + 1], lo[R], le[R];
    __shared__ unsigned short pl[Q];
    const int lane = threadIdx.x;
    const int *slot = lvl + (size_t)blockIdx.x * stride;
    const int pa = rsp::fac_pairs_at(rm);
    int dpos_[KR], bw[KR];
    int2 pr[KQ];
#pragma unroll
    for (int k = 0; k < KR; ++k) {  // clamped to the level's region sizes (rm, qm >= 1 here)
        const int x = min(lane + 64 * k, rm - 1);
        dpos_[k] = slot[8 + x];
        bw[k] = slot[8 + rm + x];
    }
#pragma unroll
    for (int k = 0; k < KQ; ++k)
        pr[k] = *reinterpret_cast<const int2 *>(slot + pa + 2 * min(lane + 64 * k, qm - 1));
    const int i = slot[0], rs = slot[1], nlo = slot[2], nr = slot[3], nq = slot[4];
    const int hasdiag = slot[5], global = slot[6];
    if (nr == 0) return;  // (an empty row has no lower entries: it is never in a slot level)
    if (global) {
        factor_row<T, 4>(a, i, lane);
        return;
    }
    T *vals = (T *)a.vals;
    T av[KR], dd[KR], uv[KQ];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const int x = min(lane + 64 * k, nr - 1);
        av[k] = vals[rs + x];
        dd[k] = vals[max(dpos_[k], 0)];
    }
#pragma unroll
    for (int k = 0; k < KQ; ++k) uv[k] = vals[pr[k].x];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const int x = lane + 64 * k;
        if (x < nr) {
            rv[x] = av[k];
            dv[x] = dpos_[k] >= 0 ? dd[k] : T(0);
            up[x] = bw[k] & 0x7ff;
            lo[x] = (bw[k] >> 11) & 0x1ff;
            le[x] = (bw[k] >> 20) & 0x1ff;
        }
    }
    if (lane == 0) up[nr] = nq;
#pragma unroll
    for (int k = 0; k < KQ; ++k) {
        const int u = lane + 64 * k;
        if (u < nq) {
            pl[u] = (unsigned short)pr[k].y;
            pu[u] = uv[k];
        }
    }
    row_lds_factor<T>(rv, dv, pu, up, lo, le, pl, nlo, nr, lane, hasdiag, i, a.zero_pivot);
    for (int x = lane; x < nr; x += 64) vals[rs + x] = rv[x];
}

// Re-read this lane's operand words that are still kNotYet (need[b] set)
// until none of the wave's is (wave-uniform loop, bounded like flow_wait).
template <typename T, int NB, typename FQ>
__device__ __forceinline__ bool tagged_wait(typename FlowWord<T>::U (&w)[NB], const int (&pos)[NB],
                                            const bool (&need)[NB], const T *vals, FQ &fq,
                                            int max_sleep, bool skip) {
    constexpr auto kNot = FlowWord<T>::kNotYet;
    auto pending = [&] {
        bool p = false;
#pragma unroll
        for (int b = 0; b < NB; ++b) p |= need[b] && w[b] == kNot;
        return p;
    };
    if (!__ballot(pending())) return false;
    const unsigned long long t0 = wall_clock64();
    unsigned long long dl = skip ? 0ull : fq.deadline(t0);  // (skip: the item has yielded)
    for (int sl = 1;; sl = min(2 * sl, max_sleep)) {
        for (int q = 0; q < sl; ++q) __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (need[b] && w[b] == kNot) w[b] = flow_load(vals + pos[b]);
        if (!__ballot(pending())) return false;
        const unsigned long long now = wall_clock64();
        if (now > dl) {
            const int r = fq.expire(now, t0, dl);
            if (r != 2) return r != 0;
        }
    }
}

// A finished factor value as it is published: a value whose bits are the
// kNotYet pattern (only an untouched input can be: arithmetic never makes a
// signalling NaN) is published as the quiet NaN of the same payload.
template <typename T>
__device__ __forceinline__ T flow_publishable(T v) {
    typedef typename FlowWord<T>::U U;
    constexpr U kQuiet = sizeof(T) == 8 ? (U)0x0008000000000000ull : (U)0x00400000u;
    const U b = __builtin_bit_cast(U, v);
    return b == FlowWord<T>::kNotYet ? __builtin_bit_cast(T, (U)(b | kQuiet)) : v;
}

// Before a factor call's flow runs (one launch over all their items): each
// flow row's upper part (diagonal included) — the values its consumers read
// as u_kk and u_kj — is saved to forig and replaced by kNotYet in vals, so
// that vals itself tells a consumer whether an operand is final (the
// data-tagged hand-off trsv_flow uses for y). A wave per item.
template <typename T>
__global__ __launch_bounds__(256) void ilu0_flow_prep(IluArgs a, int nitems) {
    const int lane = threadIdx.x & 63;
    const int it = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (it >= nitems) return;
    const int *slot = a.fslots + a.fitems[it].off;
    const int rs = slot[1], nlo = slot[2], nr = slot[3];
    T *vals = (T *)a.vals, *orig = (T *)a.forig;
    typedef typename FlowWord<T>::U U;
    for (int x = nlo + lane; x < nr; x += 64) {
        orig[rs + x] = vals[rs + x];
        reinterpret_cast<U *>(vals)[rs + x] = FlowWord<T>::kNotYet;
    }
}

// Flow run of the factor (rsp::FacFlowRun): ONE launch of a.flow_grid
// workgroups over the run's rows in level order instead of a launch per fat
// level; the waves walk the items statically or by claims (FlowClaims,
// rsp::FlowCtl). The hand-off is DATA-TAGGED, as trsv_flow's: the rows of
// flow runs start the call with their upper values (the u_kk and u_kj other
// rows read) set to kNotYet by ilu0_flow_prep (originals in forig); a row
// reads its operands (divisors and update-pair values) straight from vals
// with agent-scope atomic loads and re-reads those still kNotYet; the
// producer publishes each final value with one agent-scope atomic store.
// Every hand-off is a single location written once by an atomic and read by
// atomics (coherence alone orders it under the HIP memory model): no flag,
// no fence, no dependency lookup. Operands of rows outside flow runs are
// final in vals (earlier kernels) and never kNotYet. A gate row three levels
// back is polled first (lane 0, its first upper value) so that waves far
// ahead of the front poll one word. Progress as trsv_flow (an item waits
// for lower items only); a wait past fc.ticks gives up (rsp::FlowCtl).
// Config 3 against the round-3 flag hand-off (flags stored relaxed after an
// s_waitcnt, which the HIP memory model does not order): fp64 factor 58.6 ->
// 59.5 ms; the same flags with an agent-scope release / acquire pair (an L2
// write-back and an L2 invalidate per row) took 116 ms. Structure and
// arithmetic as ilu0_level_slot (the level's rm / qm at run time, budgets
// KR / KQ at their maximum): the same bits.
template <typename T, bool TK>
__global__ __launch_bounds__(256) void ilu0_flow(IluArgs a, int it0, int it1, unsigned long long base) {
    constexpr int R = rsp::kFacRow, Q = rsp::kFacPairs, KR = R / 64, KQ = Q / 64;
    typedef typename FlowWord<T>::U U;
    __shared__ T rv_[4][R], dv_[4][R], pu_[4][Q];
    __shared__ int up_[4][R + 1], lo_[4][R], le_[4][R];
    __shared__ unsigned short pl_[4][Q];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    T *rv = rv_[wv], *dv = dv_[wv], *pu = pu_[wv];
    int *up = up_[wv], *lo = lo_[wv], *le = le_[wv];
    unsigned short *pl = pl_[wv];
    T *vals = (T *)a.vals;
    const T *orig = (const T *)a.forig;
    __shared__ std::conditional_t<TK, FlowTicketLds, int> tl_;  // (tickets only)
    FlowClaims<TK> fq(a.fc, base, it0, it1, blockIdx.x * 4 + wv, (int)gridDim.x * 4, reinterpret_cast<FlowTicketLds *>(&tl_));
    for (fq.first(); fq.more(); fq.next()) {
        const int it = fq.item();
        if (it >= it1) continue;  // (tickets: a last round's spare waves)
        const rsp::FacFlowItem f = a.fitems[it];
        const int *slot = a.fslots + f.off;
        const int rm = f.rmqm & 0xffff, qm = f.rmqm >> 16, pa = rsp::fac_pairs_at(rm);
        int dpos_[KR], bw[KR];
        int2 pr[KQ];
#pragma unroll
        for (int k = 0; k < KR; ++k)
            if (64 * k < rm) {
                const int x = min(lane + 64 * k, rm - 1);
                dpos_[k] = slot[8 + x];
                bw[k] = slot[8 + rm + x];
            }
#pragma unroll
        for (int k = 0; k < KQ; ++k)
            if (64 * k < qm) pr[k] = *reinterpret_cast<const int2 *>(slot + pa + 2 * min(lane + 64 * k, qm - 1));
        const int i = slot[0], rs = slot[1], nlo = slot[2], nr = slot[3], nq = slot[4], hasdiag = slot[5];
        int gp = -1, ge = -1;  // the gate row's first upper position and its row end
        if (f.gate >= 0 && lane == 0) {
            gp = a.dpos[f.gate];
            ge = a.rowptr[f.gate + 1];
        }
        fq.claim_ahead();  // behind this item's structure loads
        // the row's own a_ij: lower part from vals, upper part from forig
        // (its vals entries hold kNotYet until this row publishes them)
        T av[KR];
#pragma unroll
        for (int k = 0; k < KR; ++k)
            if (64 * k < rm) {
                const int x = min(lane + 64 * k, max(nr - 1, 0));
                av[k] = x < nlo ? vals[rs + x] : orig[rs + x];
            }
        // yl: a wait yielded (tickets, FlowClaims::expire): the item still
        // runs through on what it has, but stores nothing and runs again
        // later — no branch out of the polling loops (the structured control
        // flow of such an exit cost the factor ~9 %, config-3 FEM subset)
        int gate_yl = 0;
        if (lane == 0 && gp >= 0 && gp < ge) {
            U gw[1] = {flow_load(vals + gp)};
            const int gpos[1] = {gp};
            const bool gn[1] = {true};
            gate_yl = tagged_wait<T, 1>(gw, gpos, gn, vals, fq, a.flow_sleep, false);
        }
        bool yl = __builtin_amdgcn_readfirstlane(gate_yl) != 0;
        // operands: divisors u_kk of the lower entries, u_kj of the update pairs
        U dw[KR], uw[KQ];
        int dp[KR], upos[KQ];
        bool dn[KR], un[KQ];
#pragma unroll
        for (int k = 0; k < KR; ++k) {
            dn[k] = 64 * k < rm && lane + 64 * k < nlo && dpos_[k] >= 0;
            dp[k] = 64 * k < rm ? max(dpos_[k], 0) : 0;
            dw[k] = 64 * k < rm ? flow_load(vals + dp[k]) : U(0);
        }
#pragma unroll
        for (int k = 0; k < KQ; ++k) {
            un[k] = 64 * k < qm && lane + 64 * k < nq;
            upos[k] = 64 * k < qm ? pr[k].x : 0;
            uw[k] = 64 * k < qm ? flow_load(vals + upos[k]) : U(0);
        }
        if (tagged_wait<T, KR>(dw, dp, dn, vals, fq, a.flow_sleep, yl)) yl = true;
        if (tagged_wait<T, KQ>(uw, upos, un, vals, fq, a.flow_sleep, yl)) yl = true;
        if (nr > 0) {
#pragma unroll
            for (int k = 0; k < KR; ++k) {
                const int x = lane + 64 * k;
                if (64 * k < rm && x < nr) {
                    rv[x] = av[k];
                    dv[x] = dpos_[k] >= 0 ? __builtin_bit_cast(T, dw[k]) : T(0);
                    up[x] = bw[k] & 0x7ff;
                    lo[x] = (bw[k] >> 11) & 0x1ff;
                    le[x] = (bw[k] >> 20) & 0x1ff;
                }
            }
            if (lane == 0) up[nr] = nq;
#pragma unroll
            for (int k = 0; k < KQ; ++k) {
                const int u = lane + 64 * k;
                if (64 * k < qm && u < nq) {
                    pl[u] = (unsigned short)pr[k].y;
                    pu[u] = __builtin_bit_cast(T, uw[k]);
                }
            }
            // (after a yield: a zero pivot found here is real — a pivot built
            // from a kNotYet operand is a NaN — and the rerun finds it again)
            row_lds_factor<T>(rv, dv, pu, up, lo, le, pl, nlo, nr, lane, hasdiag, i, a.zero_pivot);
            if (!yl)
                for (int x = lane; x < nr; x += 64) flow_store(vals + rs + x, flow_publishable(rv[x]));
        }
        fq.item_end(it, yl);
    }
}

// The whole factor of a pattern without update pairs (IluArgs::fac_one: a
// stored lower triangle): l_ik = a_ik / u_kk for every lower position, where
// u_kk = a_kk is never updated, and the zero-pivot check of each diagonal; a
// thread per row. Per position the division factor_row and row_lds_factor
// make (no fma: the update lists are empty), the divisor read as they read
// it (0 for a row without diagonal): the same bits. Diagonals are only read,
// so the rows are independent. One launch instead of the L DAG's levels
// (G2_circuit: 5 799) or of the one-level plan's per-row workgroups. A row
// with more than kScaleRow lower entries (a circuit's hub row: thousands, a
// serial chain of dependent gathers for one thread) is listed in LDS and
// done by the whole workgroup after its short rows.
template <typename T>
__global__ __launch_bounds__(256) void ilu0_scale_lower(IluArgs a) {
    constexpr int kScaleRow = 32;
    __shared__ int hub[256];
    __shared__ int nhub;
    if (threadIdx.x == 0) nhub = 0;
    __syncthreads();
    T *vals = (T *)a.vals;
    auto scale = [&](int p) {
        const int k = a.colidx[p];
        const T ukk = a.hasdiag[k] ? vals[a.dpos[k]] : T(0);
        vals[p] = qdiv<T>(vals[p], ukk);
    };
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < a.n) {
        const int rs = a.rowptr[i], di = a.dpos[i];
        if (di - rs <= kScaleRow)
            for (int p = rs; p < di; ++p) scale(p);
        else
            hub[atomicAdd(&nhub, 1)] = i;
        if (a.hasdiag[i] && vals[di] == T(0)) atomicMin(a.zero_pivot, i);
    }
    __syncthreads();
    for (int h = 0; h < nhub; ++h) {
        const int r = hub[h], di = a.dpos[r];
        for (int p = a.rowptr[r] + (int)threadIdx.x; p < di; p += 256) scale(p);
    }
}

// Thin run of the factor in ROUNDS (plan: build_factor_plan; rsp::RndChunk,
// rsp::RndItem), one 1024-thread workgroup. A round's items (positions) are
// independent: each is v = a_ij - sum_k l_ik u_kj over its update pairs (k
// ascending, one fma each — the oracle's rounding sequence), then / u_kk for
// a lower item; its operands are earlier rounds' values. Per chunk, LDS holds
// V = [chunk slots, buffer 0 | chunk slots, buffer 1 | staged | 0] (this
// chunk's and the previous chunk's values alternate buffers), the item
// records, the update pairs as operand indices, and the round starts.
// Staging is pipelined like the solve's: while chunk c's rounds run, the
// a_ij and staged values of chunk c+1 (gathers by the positions loaded a
// chunk earlier; staged producers are two or more chunks back, so their
// stores completed at this chunk's switch) and the records of chunk c+2 are
// in flight. Rounds of <= 64 items run on wave 0 alone, consecutive narrow
// rounds without workgroup barriers (in-order LDS of one wave); wider rounds
// use every thread and an LDS-only barrier.
#ifndef RSP_FAC_PRE3
#define RSP_FAC_PRE3 1
#endif
#ifndef RSP_FAC_PRE3C
#define RSP_FAC_PRE3C 1
#endif
template <typename T>
__global__ __launch_bounds__(kThinThreads) void ilu0_rounds(IluArgs a, int c0, int c1) {
    constexpr int NTH = kThinThreads, K = rsp::kRndItems, S = rsp::kRndStaged;
    constexpr int IPT = K / NTH, PPT = rsp::kRndPairs / NTH, SPT = S / NTH, RPT = rsp::kRndRounds / NTH;
    static_assert((K & (K - 1)) == 0 && IPT * NTH == K && PPT * NTH == rsp::kRndPairs &&
                      SPT * NTH == S && RPT * NTH == rsp::kRndRounds, "chunk budgets per thread");
    constexpr int kZero = 2 * K + S;
    __shared__ T V[2 * K + S + 1];
    __shared__ int4 litem[K];               // pos, pairs (start | count << 16), divisor index, zr
    __shared__ int lpair[rsp::kRndPairs];   // operand indices l_ik | u_kj << 16
    __shared__ int lrnd[rsp::kRndRounds + 1];
    __shared__ unsigned char lfirst[rsp::kRndRounds + 1];  // round opens a level (rsp::kRndLevelStart)
    __shared__ int lds_rdone;  // multi-wave narrow runs: absolute rounds completed
    const int tid = threadIdx.x, lane = tid & 63;
    T *vals = (T *)a.vals;
    if (tid == 0) {
        V[kZero] = T(0);
        lds_rdone = INT_MIN;  // ordered before any use by the first chunk's barriers
    }
    typedef const __attribute__((address_space(4))) int *ChunkPtr;  // scalar loads
    const ChunkPtr chunks = (ChunkPtr)a.rchunks;
    auto chunk = [&](int c) {
        const ChunkPtr q = chunks + (size_t)c * (sizeof(rsp::RndChunk) / sizeof(int));
        return rsp::RndChunk{q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]};
    };
    struct Recs {  // item records and staged positions of a chunk (this thread's share)
        rsp::RndItem it[IPT];
        int q[SPT];
    };
    struct Pre {  // ... its a_ij and staged values, pairs, round starts
        T aij[IPT], sv[SPT];
        int pr[PPT], rs[RPT];
    };
    auto load_recs = [&](const rsp::RndChunk &ch) {
        Recs R;
#pragma unroll
        for (int j = 0; j < IPT; ++j)
            if (ch.i0 + tid + j * NTH < ch.i1) R.it[j] = a.ritems[ch.i0 + tid + j * NTH];
#pragma unroll
        for (int j = 0; j < SPT; ++j)
            if (ch.s0 + tid + j * NTH < ch.s1) R.q[j] = a.rstaged[ch.s0 + tid + j * NTH];
        return R;
    };
    auto load_pre = [&](const rsp::RndChunk &ch, const Recs &R) {
        Pre P;
#pragma unroll
        for (int j = 0; j < IPT; ++j)
            if (ch.i0 + tid + j * NTH < ch.i1) P.aij[j] = vals[R.it[j].pos];
#pragma unroll
        for (int j = 0; j < SPT; ++j)
            if (ch.s0 + tid + j * NTH < ch.s1) P.sv[j] = vals[R.q[j]];
#pragma unroll
        for (int j = 0; j < PPT; ++j)
            if (ch.p0 + tid + j * NTH < ch.p1) P.pr[j] = a.rpairs[ch.p0 + tid + j * NTH];
#pragma unroll
        for (int j = 0; j < RPT; ++j)
            if (ch.r0 + tid + j * NTH < ch.r1) P.rs[j] = a.rrounds[ch.r0 + tid + j * NTH];
        return P;
    };
    // plan operand class -> LDS index for chunk parity par
    auto idx = [&](int x, int par) { return x < 2 * K ? (((x >= K) ^ par) * K + (x & (K - 1))) : x; };
    auto stage = [&](int c, const rsp::RndChunk &ch, const Recs &R, const Pre &P) {
        const int ni = ch.i1 - ch.i0, ns = ch.s1 - ch.s0, np = ch.p1 - ch.p0, nr = ch.r1 - ch.r0;
        const int par = c & 1, cb = par * K;
        __syncthreads();  // earlier chunks' values stored and visible (workgroup scope); LDS free
#pragma unroll
        for (int j = 0; j < IPT; ++j)
            if (tid + j * NTH < ni) {
                const rsp::RndItem r = R.it[j];
                litem[tid + j * NTH] = make_int4(r.pos, r.u, r.d >= 0 ? idx(r.d, par) : -1, r.zr);
                V[cb + tid + j * NTH] = P.aij[j];
            }
#pragma unroll
        for (int j = 0; j < SPT; ++j)
            if (tid + j * NTH < ns) V[2 * K + tid + j * NTH] = P.sv[j];
#pragma unroll
        for (int j = 0; j < PPT; ++j)
            if (tid + j * NTH < np)
                lpair[tid + j * NTH] = idx(P.pr[j] & 0xffff, par) | idx(P.pr[j] >> 16, par) << 16;
#pragma unroll
        for (int j = 0; j < RPT; ++j)
            if (tid + j * NTH < nr) {
                lrnd[tid + j * NTH] = P.rs[j] & (rsp::kRndLevelStart - 1);
                lfirst[tid + j * NTH] = (P.rs[j] & rsp::kRndLevelStart) != 0;
            }
        if (tid == 0) {
            lrnd[nr] = ni;
            lfirst[nr] = 1;
        }
        lds_barrier();
    };
    // An item: its value in the chunk's LDS slot and (wide rounds, STORE) in
    // vals. Narrow rounds skip the global store and the zero-pivot check: a
    // run's items go to vals in one flush by all threads after the run, so a
    // narrow round is LDS traffic and arithmetic only.
    auto process = [&](int it, int cb, auto store_tag) {
        constexpr bool STORE = decltype(store_tag)::value;
        const int4 r = litem[it];
        T v = V[cb + it];
        const T dv = V[r.z >= 0 ? r.z : kZero];  // the divisor, read with the pair indices
        const int u0 = r.y & 0xffff, u1 = u0 + (r.y >> 16);
        auto batch = [&](int u) {  // operands of 4 pairs loaded together (clamped)
            int pr[4];
            T l[4], w[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) pr[b] = lpair[min(u + b, u1 - 1)];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                l[b] = V[pr[b] & 0xffff];
                w[b] = V[pr[b] >> 16];
            }
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (u + b < u1) v = fma_t(-l[b], w[b], v);
        };
        if (u1 > u0) {  // the first batch straight-line (most items have <= 4 pairs)
            batch(u0);
            for (int u = u0 + 4; u < u1; u += 4) batch(u);
        }
        if (r.z >= 0) v = qdiv<T>(v, dv);
        V[cb + it] = v;
        if constexpr (STORE) {
            vals[r.x] = v;
            if (r.w >= 0 && v == T(0)) atomicMin(a.zero_pivot, r.w);
        }
    };
    auto flush = [&](int cb, int i0, int i1) {  // items [i0, i1) of a narrow run, after its barrier
        for (int i = i0 + tid; i < i1; i += NTH) {
            const int4 r = litem[i];
            const T v = V[cb + i];
            vals[r.x] = v;
            if (r.w >= 0 && v == T(0)) atomicMin(a.zero_pivot, r.w);
        }
    };
    auto narrow = [&](int q) { return lrnd[q + 1] - lrnd[q] <= 64; };
    auto run_end = [&](int q, int nr) {  // first round >= q that is not narrow, or nr
        for (int b = q;; b += 64) {
            const int qq = b + lane;
            const unsigned long long m = __ballot(!(qq < nr && narrow(qq)));
            if (m) return b + __builtin_ctzll(m);
        }
    };
    // Narrow run on KW waves (a.narrow_waves, deferred stores only): the run's
    // rounds are cut into segments at the rounds that open a level (a level's
    // rounds depend on each other through its rows' l_ik: one wave runs a
    // segment in order, its in-order LDS accesses ordering them, as in the
    // one-wave run), and wave w takes segments w, w + KW, ... Before waiting,
    // a wave loads what no value of the run feeds — the first two rounds'
    // item records, initial values a_ij and first four pair indices; then it
    // waits until the segment before its own is complete (an LDS counter of
    // absolute rounds done, published by each segment's wave with a release
    // store after its value stores, lds_publish), and only then reads operands (divisors, l_ik,
    // u_kj) and runs the fma chains and divisions. While one wave is on its
    // chain, the others have prepared their next levels. Same items, same
    // pairs in the same order, same divisions as the one-wave run: same bits.
    struct ItemPre {
        int4 r;
        T v;
        int pr[4];
    };
    auto item_pre = [&](int it, int cb) {
        ItemPre p;
        p.r = litem[it];
        p.v = V[cb + it];
        const int u0 = p.r.y & 0xffff, u1 = u0 + (p.r.y >> 16);
#pragma unroll
        for (int b = 0; b < 4; ++b) p.pr[b] = lpair[min(u0 + b, max(u1 - 1, 0))];
        return p;
    };
    // short: no item of the wave's round has more than two pairs (wave-
    // uniform), so only the first two pairs' operands are read and chained
    auto item_post = [&](int it, int cb, const ItemPre &p, bool short2) {
        const int4 r = p.r;
        T v = p.v;
        const T dv = V[r.z >= 0 ? r.z : kZero];
        const int u0 = r.y & 0xffff, u1 = u0 + (r.y >> 16);
        if (short2) {
            if (u1 > u0) {
                T l[2], w[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    l[b] = V[p.pr[b] & 0xffff];
                    w[b] = V[p.pr[b] >> 16];
                }
                v = fma_t(-l[0], w[0], v);
                if (u1 > u0 + 1) v = fma_t(-l[1], w[1], v);
            }
        } else if (u1 > u0) {
            T l[4], w[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                l[b] = V[p.pr[b] & 0xffff];
                w[b] = V[p.pr[b] >> 16];
            }
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (u0 + b < u1) v = fma_t(-l[b], w[b], v);
            for (int u = u0 + 4; u < u1; u += 4) {  // items of more than four pairs (rare)
                int pr[4];
#pragma unroll
                for (int b = 0; b < 4; ++b) pr[b] = lpair[min(u + b, u1 - 1)];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    l[b] = V[pr[b] & 0xffff];
                    w[b] = V[pr[b] >> 16];
                }
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (u + b < u1) v = fma_t(-l[b], w[b], v);
            }
        }
        if (r.z >= 0) v = qdiv<T>(v, dv);
        V[cb + it] = v;
    };
    auto wave_order = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    };
    auto run_mw = [&](const rsp::RndChunk &ch, int q, int qe, int cb, int KW) {
        const int w = tid >> 6;
        auto seg_end = [&](int s) {  // first round > s that opens a level, or qe (wave-uniform)
            for (int b = s + 1;; b += 64) {
                const int qq = b + lane;
                const unsigned long long m = __ballot(qq >= qe || lfirst[qq]);
                if (m) return min(b + (int)__builtin_ctzll(m), qe);
            }
        };
        int k = 0, sp = q;  // sp: the previous level's first round
        for (int s0 = q; s0 < qe; ++k) {
            const int s1 = seg_end(s0);
            if (k % KW == w) {
                const int b0 = lrnd[s0], n0 = lrnd[s0 + 1] - b0;
                const bool has1 = s0 + 1 < s1;
                const int b1 = has1 ? lrnd[s0 + 1] : b0, n1 = has1 ? lrnd[s0 + 2] - b1 : 0;
#if RSP_FAC_PRE3
                // (a third round's records too: levels of three rounds are
                // common on the deep circuits, dc1 2.7 rounds per level)
                const bool has2 = s0 + 2 < s1;
                const int b2 = has2 ? lrnd[s0 + 2] : b0, n2 = has2 ? lrnd[s0 + 3] - b2 : 0;
#endif
                const ItemPre p0 = item_pre(b0 + min(lane, n0 - 1), cb);
                const ItemPre p1 = item_pre(b1 + min(lane, max(n1 - 1, 0)), cb);
#if RSP_FAC_PRE3
#if RSP_FAC_PRE3C
                ItemPre p2{};
                if (has2) p2 = item_pre(b2 + min(lane, max(n2 - 1, 0)), cb);  // (wave-uniform: levels of >= 3 rounds)
#else
                const ItemPre p2 = item_pre(b2 + min(lane, max(n2 - 1, 0)), cb);
#endif
                const bool sh2 = !__ballot(lane < n2 && (p2.r.y >> 16) > 2);
#endif
                const bool sh0 = !__ballot(lane < n0 && (p0.r.y >> 16) > 2);
                const bool sh1 = !__ballot(lane < n1 && (p1.r.y >> 16) > 2);
                if (s0 > q) lds_wait_geq(&lds_rdone, ch.r0 + s0, ch.r0 + sp);
                if (lane < n0) item_post(b0 + lane, cb, p0, sh0);
                wave_order();
                if (has1) {
                    if (lane < n1) item_post(b1 + lane, cb, p1, sh1);
                    wave_order();
#if RSP_FAC_PRE3
                    if (has2) {
                        if (lane < n2) item_post(b2 + lane, cb, p2, sh2);
                        wave_order();
                    }
                    for (int qq = s0 + 3; qq < s1; ++qq) {  // levels of more than three rounds
#else
                    for (int qq = s0 + 2; qq < s1; ++qq) {  // levels of more than two rounds
#endif
                        const int bq = lrnd[qq];
                        if (bq + lane < lrnd[qq + 1]) process(bq + lane, cb, std::false_type());
                        wave_order();
                    }
                }
                lds_publish(&lds_rdone, ch.r0 + s1, lane == 0);  // after the value stores
            }
            sp = s0;
            s0 = s1;
        }
    };
    auto rounds = [&](int c, const rsp::RndChunk &ch) {
        const int nr = ch.r1 - ch.r0, cb = (c & 1) * K;
        for (int q = 0; q < nr;) {
            if (narrow(q)) {
                const int qe = run_end(q, nr);
                // long runs defer the global stores to one flush after the
                // run; short ones (between wide rounds) store as they go
                const bool defer = qe - q >= a.defer_rounds;
                auto run = [&](auto store_tag) {
                    for (int qq = q; qq < qe; ++qq) {
                        const int b0 = lrnd[qq];
                        if (b0 + lane < lrnd[qq + 1]) process(b0 + lane, cb, store_tag);
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
                    }
                };
                const int KW = min(a.narrow_waves, NTH / 64);
                if (defer && KW > 1) {
                    if (tid < 64 * KW) run_mw(ch, q, qe, cb, KW);
                } else if (tid < 64) {  // (a software-pipelined form of this loop measured slower)
                    if (defer)
                        run(std::false_type());
                    else
                        run(std::true_type());
                }
                lds_barrier();
                if (defer) flush(cb, lrnd[q], lrnd[qe]);
                q = qe;
                continue;
            }
            for (int it = lrnd[q] + tid; it < lrnd[q + 1]; it += NTH) process(it, cb, std::true_type());
            lds_barrier();
            ++q;
        }
    };
    const int cl = c1 - 1;
    rsp::RndChunk rc = chunk(c0), rn = chunk(min(c0 + 1, cl));
    Recs R = load_recs(rc);
    Pre P = load_pre(rc, R);
    Recs Rn = load_recs(rn);
    auto mark = [&](int c, int j, unsigned long long v) {  // diagnostics only (RSP_ILU_FTRACE)
        if (a.trace && tid == 0 && 4 * c + j < a.trace_cap) a.trace[4 * c + j] = v;
    };
    for (int c = c0; c < c1; ++c) {
        mark(c, 0, clock64());
        stage(c, rc, R, P);
        mark(c, 1, clock64());
        const rsp::RndChunk cur = rc;
        if (c + 1 < c1) {
            const rsp::RndChunk r2 = chunk(min(c + 2, cl));
            P = load_pre(rn, Rn);  // chunk c+1's gathers
            R = Rn;
            Rn = load_recs(r2);    // chunk c+2's records
            rc = rn;
            rn = r2;
        }
        rounds(c, cur);
        mark(c, 2, clock64());
        mark(c, 3, (unsigned long long)(cur.r1 - cur.r0) | (unsigned long long)(cur.i1 - cur.i0) << 32);
    }
}

// Triangular solves (kind 0 = L op N, 1 = L^T op T, 2 = U) over the DAG's
// flat terms: y_i = (alpha x_i - sum_k vals[tpos[k]] * y[src[k]]) (/ u_ii),
// one fma per term in the term order (for L^T: j descending).

// s - sum v_k y[src_k] over k = k0 .. k1-1 in order, from the solve streams
// (term values in flat order, no position indirection). The values and y
// indices of batch j+1 are loaded while batch j's y gather is in flight (the
// loads are clamped, unpredicated), so a batch costs one memory round trip.
template <typename T, int B>
__device__ __forceinline__ T stream_chain(T s, int k0, int k1, const T *sval, const int *src, const T *y) {
    const int n = k1 - k0;
    if (n <= 0) return s;
    T v[B];
    int id[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int k = k0 + min(b, n - 1);
        v[b] = sval[k];
        id[b] = src[k];
    }
    for (int b0 = 0; b0 < n; b0 += B) {
        T yv[B], vc[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            yv[b] = y[id[b]];
            vc[b] = v[b];
        }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int k = k0 + min(b0 + B + b, n - 1);
            v[b] = sval[k];
            id[b] = src[k];
        }
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (b0 + b < n) s = fma_t(-vc[b], yv[b], s);
    }
    return s;
}

// The serial chain of one hub row (thousands of terms) by a 256-thread
// workgroup: waves 1-3 gather the terms group by group (768 a group: value
// and y index, then the y) into an LDS double buffer while wave 0 runs the
// chain over the previous group on broadcast LDS operands, one fma per term
// in order. A wave alone paid two dependent global round trips per 64 terms.
// The result is valid in wave 0.
template <typename T>
__device__ __forceinline__ T block_chain(T s, int k0, int k1, const T *sval, const int *src, const T *y) {
    constexpr int NL = 192, PER = 4, GS = NL * PER;
    __shared__ T bv[2][GS], by[2][GS];
    const int tid = threadIdx.x, n = k1 - k0, ng = (n + GS - 1) / GS;
    auto gather = [&](int g) {  // loader waves: group g into buffer g & 1
        T v[PER], yv[PER];
        int id[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int k = min(g * GS + (tid - 64) + j * NL, n - 1);
            v[j] = sval[k0 + k];
            id[j] = src[k0 + k];
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) yv[j] = y[id[j]];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            bv[g & 1][(tid - 64) + j * NL] = v[j];
            by[g & 1][(tid - 64) + j * NL] = yv[j];
        }
    };
    if (tid >= 64) gather(0);
    __syncthreads();
    for (int g = 0; g < ng; ++g) {
        if (tid >= 64) {
            if (g + 1 < ng) gather(g + 1);
        } else {
            const T *pv = bv[g & 1], *py = by[g & 1];
            const int cnt = min(GS, n - g * GS);
#pragma unroll 8
            for (int j = 0; j < cnt; ++j) s = fma_t(-pv[j], py[j], s);
        }
        __syncthreads();
    }
    return s;
}

// Fat level, terms from the solve streams (trsv_stream): blocks [0, nb) one
// thread per short row (the level's first nshort rows), the next nwb blocks
// one wave per long row (rows up to nwave), the blocks after them one hub row
// each. Slot off + r of the level order: task, alpha x_i (and u_ii) at the
// same index, so the row's first loads are independent.
template <typename T, int KIND, int B>
__global__ __launch_bounds__(256) void trsv_level(TrsvArgs a, int off, int nrows, int nshort, int nb,
                                                  int nwave, int nwb, int sbase) {
    const T *sval = (const T *)a.sval;
    T *y = (T *)a.y;
    const int *src = a.plan.src;
    int x;
    T s;
    rsp::RowTask t;
    if ((int)blockIdx.x >= nb + nwb) {  // hub row: the whole workgroup (uniform branch)
        x = off + nwave + (blockIdx.x - nb - nwb);
        t = a.plan.tasks[x];
        s = block_chain<T>(((const T *)a.sx)[x], t.t0, t.t1, sval, src, y);
        if (threadIdx.x != 0) return;
    } else if ((int)blockIdx.x < nb) {
        const int r = blockIdx.x * 256 + threadIdx.x;
        if (r >= nshort) return;
        x = off + r;
        t = a.plan.tasks[x];
        if (sbase >= 0) {
            // padded short rows: the row's kFatLongTerms flat terms start at
            // sbase + 8 r, so the values and y indices load with the task
            // instead of after it; pads (beyond t1) are never used
            constexpr int F = rsp::kFatLongTerms;
            const int t0 = sbase + r * F;
            T v[F], yv[F];
            int id[F];
#pragma unroll
            for (int b = 0; b < F; ++b) {
                v[b] = sval[t0 + b];
                id[b] = src[t0 + b];
            }
            s = ((const T *)a.sx)[x];
            const int n = t.t1 - t0;
#pragma unroll
            for (int b = 0; b < F; ++b) yv[b] = y[b < n ? id[b] : 0];
#pragma unroll
            for (int b = 0; b < F; ++b)
                if (b < n) s = fma_t(-v[b], yv[b], s);
        } else {
            s = stream_chain<T, B>(((const T *)a.sx)[x], t.t0, t.t1, sval, src, y);
        }
    } else {
        const int r = nshort + (blockIdx.x - nb) * 4 + (threadIdx.x >> 6);
        if (r >= nwave) return;
        x = off + r;
        t = a.plan.tasks[x];
        if (a.wave_lds) {
            __shared__ T cwv[4][64], cwy[4][64];
            const int w = threadIdx.x >> 6;
            s = wave_chain_lds<T>(((const T *)a.sx)[x], t.t0, t.t1, threadIdx.x & 63, cwv[w], cwy[w], sval,
                                  src, y);
        } else {
            s = wave_chain<T>(((const T *)a.sx)[x], t.t0, t.t1, threadIdx.x & 63,
                              [&](int k) { return sval[k]; }, [&](int k) { return y[src[k]]; });
        }
        if ((threadIdx.x & 63) != 0) return;
    }
    if constexpr (KIND == 2) s = qdiv<T>(s, ((const T *)a.sdg)[x]);
    y[t.i] = s;
}

// Flow segments (a solve DAG's runs of two or more fat levels): ONE launch of
// a.flow_grid workgroups instead of a launch per level. The waves walk the
// segment's work items (rsp::FlowItem, level order) statically or by claims
// (FlowClaims, rsp::FlowCtl); an item starts as soon as the y values it reads
// exist, not when its whole previous level has ended. Existence is read from
// the value itself: trsv_stream sets every y to kNotYet, a signalling-NaN
// bit pattern that no y can have (every y is an arithmetic result — alpha x_i,
// an fma, a division — and arithmetic only produces quiet NaNs); a row's y is
// written once, by one 4- / 8-byte device-scope (sc1) store, and a consumer
// reads its operands with device-scope (sc1) loads, re-reading (after an
// s_sleep) those still kNotYet: the data-tagged hand-off of the price list
// in MI355X_MICROARCH.md (handoff-1to1) — no flag, no fence.
// Progress: an item waits only for items of lower index, and each wave runs
// its items in index order; with static items the grid is resident at once
// (the lowest unfinished item is some wave's current item), with claims any
// item waited on is held by a running wave. A wait beyond fc.ticks (never
// expected) gives up and records the call in *fc.status (rsp_trsv_zero_pivot
// then returns EXECUTION_FAILED) instead of hanging the GPU.
// Same terms, same order, same fma chain as trsv_level: the same bits.
template <typename T, int KIND, bool TK>
__global__ __launch_bounds__(256) void trsv_flow(TrsvArgs a, int it0, int it1, unsigned long long base) {
    typedef typename FlowWord<T>::U U;
    constexpr int F = rsp::kFatLongTerms;
    __shared__ T fwv[4][64], fwy[4][64];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const T *sval = (const T *)a.sval, *sx = (const T *)a.sx;
    T *y = (T *)a.y;
    const int *src = a.plan.src;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    };
    __shared__ std::conditional_t<TK, FlowTicketLds, int> tl_;  // (tickets only)
    FlowClaims<TK> fq(a.fc, base, it0, it1, blockIdx.x * 4 + wv, (int)gridDim.x * 4, reinterpret_cast<FlowTicketLds *>(&tl_));
    // claims are issued behind each item's first loads (task, term values and sources)
    for (fq.first(); fq.more(); fq.next()) {
        const int it = fq.item();
        if (it >= it1) continue;  // (tickets: a last round's spare waves)
        const rsp::FlowItem f = a.plan.fitems[it];
        if (f.n > 0) {  // short rows, a lane each (lanes past them repeat the last row)
            const int r = min(lane, f.n - 1), x = f.x0 + r;
            const rsp::RowTask t = a.plan.tasks[x];
            T v[F];
            int id[F], n;
            if (f.t0 >= 0) {  // padded: the terms load with the task
                const int t0 = f.t0 + r * F;
#pragma unroll
                for (int b = 0; b < F; ++b) {
                    v[b] = sval[t0 + b];
                    id[b] = src[t0 + b];
                }
                n = t.t1 - t0;
            } else {
                n = t.t1 - t.t0;
                const int kl = max(t.t1 - 1, 0);
#pragma unroll
                for (int b = 0; b < F; ++b) {
                    const int k = min(t.t0 + b, kl);
                    v[b] = sval[k];
                    id[b] = src[k];
                }
            }
            T s = sx[x];
            fq.claim_ahead();
            // yl: a wait yielded (as in ilu0_flow: the item runs through and stores nothing)
            bool yl = flow_gate<T>(f.gate, y, fq, a.flow_sleep);
            U w[F];
#pragma unroll
            for (int b = 0; b < F; ++b) w[b] = b < n ? flow_load(y + id[b]) : U(0);
            if (flow_wait<T, F>(w, id, n, y, fq, a.flow_sleep, yl)) yl = true;
#pragma unroll
            for (int b = 0; b < F; ++b)
                if (b < n) s = fma_t(-v[b], __builtin_bit_cast(T, w[b]), s);
            if constexpr (KIND == 2) s = qdiv<T>(s, ((const T *)a.sdg)[x]);
            if (lane < f.n && !yl) flow_store(y + t.i, s);
            fq.item_end(it, yl);
        } else {  // one row of more terms: a wave, 64 terms at a time on LDS broadcast operands
            const int x = f.x0;
            const rsp::RowTask t = a.plan.tasks[x];
            T s = sx[x];
            fq.claim_ahead();
            bool yl = flow_gate<T>(f.gate, y, fq, a.flow_sleep);
            for (int base = t.t0; base < t.t1; base += 64) {
                const int k = min(base + lane, t.t1 - 1);
                const T v = sval[k];
                int id[1] = {src[k]};
                U w[1] = {flow_load(y + id[0])};
                if (flow_wait<T, 1>(w, id, 1, y, fq, a.flow_sleep, yl)) yl = true;
                fwv[wv][lane] = v;
                fwy[wv][lane] = __builtin_bit_cast(T, w[0]);
                wave_sync();
                const int cnt = min(64, t.t1 - base);
                int j = 0;
                for (; j + 4 <= cnt; j += 4) {
                    T p[4], q[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        p[u] = fwv[wv][j + u];
                        q[u] = fwy[wv][j + u];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) s = fma_t(-p[u], q[u], s);
                }
                for (; j < cnt; ++j) s = fma_t(-fwv[wv][j], fwy[wv][j], s);
                wave_sync();  // this group's reads before the next group's stores
            }
            if constexpr (KIND == 2) s = qdiv<T>(s, ((const T *)a.sdg)[x]);
            if (lane == 0 && !yl) flow_store(y + t.i, s);
            fq.item_end(it, yl);
        }
    }
}

// Thin run (levels cut into LDS-staged chunks [c0, c1)), one 1024-thread
// workgroup. A chunk holds <= kChunkRows rows and <= kChunkTerms term slots;
// every row of a thin run has its terms padded to whole groups of G = 4 (or 2,
// for DAGs of short chains)
// (pads: a zero value times the zero slot of the y buffer, an exact no-op), so
// a row is read as groups of four terms with vector LDS loads and no length
// tests. LDS per chunk:
//   lrow[r]  = {alpha x_i, first group | groups << 16, y slot}  (one 16-B load)
//   lval[k], lidx[k] = term value, byte offset of its y in ybuf (row order)
//   ybuf     = [ y window (kYWin slots, run index mod kYWin) | 0 | y staged
//               for slot k at kYWin + 1 + k (producers before the run or
//               already out of the window) ]
// The chunk's data reaches LDS through registers, two chunks deep: while chunk
// c's levels run, the plan loads of chunk c+2 (task, term positions and
// sources, level offsets: one row and four slots per thread) and the gathers
// of chunk c+1 (x_i, term values, staged y) are in flight, unpredicated with
// clamped indices, so nothing waits on them before the switch; y is written to
// global memory only at chunk switches (one store per thread), so no store is
// pending under the levels. A staged y has its producer > kYWin rows back —
// at least two switches earlier — so it is in memory when prefetched.
//
// Levels: a narrow level (<= 64 rows, all short) is computed by wave 0 alone,
// and consecutive narrow levels are ordered by the wave's in-order LDS
// accesses instead of workgroup barriers; the wave runs them software-
// pipelined — while level q's y loads, fma chain and y store are on the
// critical path, the first term group of level q+1 and the row records of
// level q+2 are already loading — so a level costs about one LDS round trip.
// The other waves skip to the barrier after the run. (Deep-level circuits are
// ~10^4 levels of ~10 rows: nearly every level is narrow.) Wider levels use
// all waves, one row per thread, long rows (> kLongTerms terms) a wave each,
// and an LDS-only barrier after each level.
template <typename T>
struct alignas(16) ThinRow {  // LDS row record of a thin chunk
    T x;                      // alpha * x_i
    int g;                    // first group (chunk-relative) | groups << 16
    int out;                  // byte offset of the row's y window slot in ybuf
};
template <typename T, int G>
struct alignas(sizeof(T) * G) TermGroup {  // values of one group of terms
    T v[G];
};
template <int G>
struct alignas(4 * G) TermIds {  // byte offsets of their y in ybuf
    int v[G];
};

// Solve streams, one pass over the DAG before its thin runs: per flat term
// its value (0 for a pad), per level-order slot alpha x_i (and u_ii for the U
// solve) — so a thin run stages contiguous streams instead of gathering.
template <typename T, int KIND>
__global__ __launch_bounds__(256) void trsv_stream(TrsvArgs a, T alpha) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const T *vals = (const T *)a.vals;
    if (k < a.plan.nterms) {
        const int tp = a.plan.tpos[k];
        ((T *)a.sval)[k] = tp >= 0 ? vals[tp] : T(0);
    }
    if (k < a.n) {
        const rsp::RowTask t = a.plan.tasks[k];
        ((T *)a.sx)[k] = alpha * ((const T *)a.x)[t.i];
        if constexpr (KIND == 2) ((T *)a.sdg)[k] = t.d >= 0 ? vals[t.d] : T(0);
        // flow segments read "not produced yet" from y itself (trsv_flow);
        // every other row's y is written by its own segment before any reader
        if (a.flow && a.plan.has_flow) ((typename FlowWord<T>::U *)a.y)[t.i] = FlowWord<T>::kNotYet;
    }
}

// The LDS layout of trsv_thin_pf (byte offsets into its one LDS object).
template <typename T, int KIND, int G>
struct ThinLay {
    static constexpr int al(int v, int a) { return (v + a - 1) / a * a; }
    static constexpr int idx = 0;
    static constexpr int val = al(idx + (rsp::kChunkTerms / G + 1) * (int)sizeof(TermIds<G>), 32);
    static constexpr int yb = al(val + (rsp::kChunkTerms / G + 1) * (int)sizeof(TermGroup<T, G>), 16);
    static constexpr int row = al(yb + (rsp::kYWin + 1 + rsp::kChunkTerms) * (int)sizeof(T), 16);
    static constexpr int rowi = row + rsp::kChunkRows * (int)sizeof(ThinRow<T>);
    static constexpr int ptr = rowi + 4 * rsp::kChunkRows;
    static constexpr int ns = ptr + 4 * (rsp::kChunkRows + 1);
    static constexpr int dg = al(ns + 4 * rsp::kChunkRows, 8);
    static constexpr int done = dg + (int)sizeof(T) * (KIND == 2 ? rsp::kChunkRows : 1);
    static constexpr int egr = done + 4;
    static constexpr int bytes = al(egr + rsp::kChunkRows, 16);
};

// PAIRS: narrow runs (levels of <= 64 short rows) on a.narrow_waves waves
// with two consecutive levels per wave turn (narrow_run_mw2), else one level
// per turn (narrow_run_mw; one wave: narrow_run). Its own instantiation (the
// registers).
// LW (round 5): the first LW waves never load the next chunk; the loader
// threads are the other kThinThreads - 64 LW (a thread stages rows lt + r NL
// and terms lt + j NL). The narrow waves then hold none of the chunk
// prefetch's registers, which gives narrow_run_mw2 the room to prepare every
// term group of up to three per level before its wait (G = 2): config-3 deep
// set, same box, interleaved x2 (profiles/r05_ilu_loaders_ab.txt): dc1 solve
// 4.77 -> 4.46 ms, G2_circuit 2.58 -> 2.33, matrix-new_3 5.60 -> 5.24; the
// split alone (without the extra groups) measured equal, and on DAGs that do
// not take the pair loop it cost (thermomech_TK 1.01 -> 1.05): LW = 4 with
// PAIRS only.
template <typename T, int KIND, int G, bool PAIRS = false, int LW = 0>
__global__ __launch_bounds__(rsp::kThinThreads) void trsv_thin_pf(TrsvArgs a, int c0, int c1, int base) {
    constexpr int NTH = rsp::kThinThreads;
    constexpr int NL = NTH - 64 * LW;                     // loader threads: lt = tid - 64 LW >= 0
    constexpr int TPT = (rsp::kChunkTerms + NL - 1) / NL;  // terms of a chunk per loader: lt + j NL
    constexpr int RPT = (rsp::kChunkRows + NL - 1) / NL;   // rows (and level pointers) per loader: lt + r NL
    static_assert(NL > 0 && G <= rsp::kGroup, "chunk loaders");
    static_assert(NTH >= rsp::kChunkRows, "a thin level's short rows: one per thread");
    constexpr int kZero = rsp::kYWin, kStaged = rsp::kYWin + 1;
    // + one pad group (values 0, y from the zero slot) after the chunk's groups
    constexpr int kPadGroup = rsp::kChunkTerms / G;
    // The workgroup's LDS is ONE object with a fixed layout, so the arrays the
    // narrow loops index per term sit where an LDS instruction's 16-bit offset
    // field can add their base: the term groups' y indices (lidx) at 0, their
    // values (lval) next, the y buffer (ybuf: window | zero slot | staged y)
    // after them; then the row records and the per-level arrays.
    using Lay = ThinLay<T, KIND, G>;
    static_assert(Lay::yb < 65536 && Lay::val < 65536 && Lay::bytes <= 163840, "LDS layout");
    __shared__ __attribute__((aligned(32))) char lds_arena[Lay::bytes];
    T *const ybuf = (T *)(lds_arena + Lay::yb);
    TermGroup<T, G> *const lval = (TermGroup<T, G> *)(lds_arena + Lay::val);
    TermIds<G> *const lidx = (TermIds<G> *)(lds_arena + Lay::idx);
    ThinRow<T> *const lrow = (ThinRow<T> *)(lds_arena + Lay::row);
    int *const lrowi = (int *)(lds_arena + Lay::rowi);
    unsigned char *const legr = (unsigned char *)(lds_arena + Lay::egr);  // per row: its early term groups (split order)
    T *const ldg = (T *)(lds_arena + Lay::dg);  // u_ii: U solve only
    int *const lptr = (int *)(lds_arena + Lay::ptr);
    int *const lns = (int *)(lds_arena + Lay::ns);
    int &lds_done = *(int *)(lds_arena + Lay::done);  // multi-wave narrow runs: absolute levels completed
    const int tid = threadIdx.x;
    const int lt = tid - 64 * LW;  // loader index (< 0: a narrow-run wave that never loads)
    if (tid == 0) lds_done = INT_MIN;  // ordered before any use by the first chunk's barriers
    const T *sval = (const T *)a.sval, *sx = (const T *)a.sx, *sdg = (const T *)a.sdg;
    T *y = (T *)a.y;
    const int *ptr = a.plan.ptr_dev;
    if (tid == 0) ybuf[kZero] = T(0);
    if (tid < G) {  // the pad group: exact no-op terms, fma(-0, 0, s) == s
        lval[kPadGroup].v[tid] = T(0);
        lidx[kPadGroup].v[tid] = kZero * (int)sizeof(T);
    }
    struct Pre {  // this loader's share of a chunk: rows lt + r NL, terms lt + j NL (all streams)
        rsp::ThinRowPlan r[RPT];
        T xv[RPT], dg[RPT], v[TPT];
        int id[TPT];
        int lp[RPT], ln[RPT], lpe;
    };
    struct Stg {  // staged terms lt + j NL of a chunk
        int slot[TPT], j[TPT];
    };
    struct StgY {  // ... and their y
        int slot[TPT];
        T y[TPT];
    };
    // Loads past the chunk's rows / terms are predicated off (a whole wave
    // past them issues nothing): the staging is bound by this CU's load
    // bandwidth, and a chunk of short rows fills a fraction of its term slots.
    auto load_pre = [&](const rsp::LevelChunk &ch) {
        Pre p;
        const int nl = ch.l1 - ch.l0;
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) {
            const int x = ch.x0 + lt + rr * NL;
            if (lt >= 0 && x < ch.x1) {
                p.r[rr] = a.plan.trow[x];
                p.xv[rr] = sx[x];
                p.dg[rr] = KIND == 2 ? sdg[x] : T(0);
            }
        }
#pragma unroll
        for (int j = 0; j < TPT; ++j) {
            const int k = ch.k0 + lt + j * NL;
            if (lt >= 0 && k < ch.k1) {
                p.v[j] = sval[k];
                p.id[j] = a.plan.sid[k];
            }
        }
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr)
            if (lt >= 0) {
                p.lp[rr] = ptr[ch.l0 + min(lt + rr * NL, nl)];
                p.ln[rr] = a.plan.nshort[ch.l0 + min(lt + rr * NL, max(nl - 1, 0))];
            }
        p.lpe = ptr[ch.l1];
        return p;
    };
    auto load_stg = [&](const rsp::LevelChunk &ch) {
        Stg q;
        const int el = max(ch.st1 - 1, 0);
#pragma unroll
        for (int j = 0; j < TPT; ++j)
            if (lt >= 0) {
                const rsp::StagedTerm t = a.plan.stg[max(min(ch.st0 + lt + j * NL, el), 0)];
                q.slot[j] = t.slot;
                q.j[j] = t.j;
            }
        return q;
    };
    auto load_stgy = [&](const Stg &q) {
        StgY w;
#pragma unroll
        for (int j = 0; j < TPT; ++j)
            if (lt >= 0) {
                w.slot[j] = q.slot[j];
                w.y[j] = y[q.j[j]];
            }
        return w;
    };
    // Chunk switch. The levels write y to the LDS window only; the previous
    // chunk's rows go to global y here, one store per thread, so no global
    // store is pending while levels run and the wait below only ever finds
    // operations issued a whole chunk ago (this chunk's prefetch, the flush
    // before). After it and the barrier, every flush up to the previous switch
    // is complete — the staged y a prefetch reads (producer > kYWin rows back,
    // i.e. in a chunk flushed at least one switch before) is in memory.
    auto mark_by = [&](int c, int j, int t) {  // diagnostics only (RSP_ILU_TRACE)
        if (a.trace && tid == t && 8 * c + j < a.trace_cap / 2) a.trace[8 * c + j] = wall_clock64();
    };
    auto mark = [&](int c, int j) { mark_by(c, j, 0); };
    auto stage = [&](int c, int px0, int px1, const rsp::LevelChunk &ch, const Pre &p, const StgY &w) {
        const int nk = ch.k1 - ch.k0, nl = ch.l1 - ch.l0, ns = ch.st1 - ch.st0;
        mark(c, 0);
        // the previous chunk's levels are done with LDS, and the y flushed at
        // earlier switches (global stores of other threads) are ordered before
        // this chunk's prefetch loads: workgroup-scope release / acquire
        __syncthreads();
        mark(c, 1);
        int fi[RPT];
        T fv[RPT];
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) {  // read before this thread restages its slots
            const int t = min(max(lt, 0) + rr * NL, rsp::kChunkRows - 1);
            fi[rr] = lrowi[t];
            fv[rr] = ybuf[(px0 + t - base) & (rsp::kYWin - 1)];
        }
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) {
            const int t = lt + rr * NL;
            if (lt >= 0 && t < ch.x1 - ch.x0) {
                ThinRow<T> r;
                r.x = p.xv[rr];
                r.g = p.r[rr].g;
                r.out = (p.r[rr].out & 0xffff) * (int)sizeof(T);
                lrow[t] = r;
                legr[t] = (unsigned char)(p.r[rr].out >> 16);  // early groups (split order)
                lrowi[t] = p.r[rr].i;
                if constexpr (KIND == 2) ldg[t] = p.dg[rr];
            }
        }
#pragma unroll
        for (int j = 0; j < TPT; ++j)
            if (lt >= 0 && lt + j * NL < nk) {
                ((T *)lval)[lt + j * NL] = p.v[j];
                ((int *)lidx)[lt + j * NL] = p.id[j] * (int)sizeof(T);
            }
#pragma unroll
        for (int j = 0; j < TPT; ++j)
            if (lt >= 0 && lt + j * NL < ns) ybuf[kStaged + w.slot[j]] = w.y[j];
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) {
            const int t = lt + rr * NL;
            if (lt >= 0 && t <= nl) lptr[t] = p.lp[rr];
            if (lt >= 0 && t < nl) lns[t] = p.ln[rr];
        }
        if (lt == 0 && nl == rsp::kChunkRows) lptr[rsp::kChunkRows] = p.lpe;
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr)  // after the last use of the prefetched registers
            if (lt >= 0 && lt + rr * NL < px1 - px0) y[fi[rr]] = fv[rr];
        lds_barrier();
        mark(c, 2);
    };
    // s += -sum over the terms of one group (in order; pads are exact no-ops)
    auto yb = [&](int off) { return *(const T *)((const char *)ybuf + off); };
    auto put = [&](int off, T v) { *(T *)((char *)ybuf + off) = v; };
    auto group_fma = [&](T s, const TermGroup<T, G> &g, const TermIds<G> &id) {
        T yv[G];
#pragma unroll
        for (int j = 0; j < G; ++j) yv[j] = yb(id.v[j]);
#pragma unroll
        for (int j = 0; j < G; ++j) s = fma_t(-g.v[j], yv[j], s);
        return s;
    };
    // groups [g, ge) of a row after s, in order; group g+1's values, indices
    // and y are read under group g's fmas (the same fmas in the same order)
    auto groups_fma = [&](T s, int g, int ge) {
        TermGroup<T, G> vc = lval[g];
        T yc[G];
        {
            const TermIds<G> ic = lidx[g];
#pragma unroll
            for (int j = 0; j < G; ++j) yc[j] = yb(ic.v[j]);
        }
        for (; g < ge; ++g) {
            const int gn = min(g + 1, ge - 1);
            const TermGroup<T, G> vn = lval[gn];
            const TermIds<G> in = lidx[gn];
            T yn[G];
#pragma unroll
            for (int j = 0; j < G; ++j) yn[j] = yb(in.v[j]);
#pragma unroll
            for (int j = 0; j < G; ++j) s = fma_t(-vc.v[j], yc[j], s);
            vc = vn;
#pragma unroll
            for (int j = 0; j < G; ++j) yc[j] = yn[j];
        }
        return s;
    };
    // (groups_fma for every short row, and for the narrow rows' third group
    // on, measured 1.6 % slower on config 3: short chains gain nothing from
    // the lookahead and pay its loads; long rows gain 10 %)
    auto row_value = [&](const ThinRow<T> &r) {  // one short row, groups in order
        T s = r.x;
        const int g0 = r.g & 0xffff, ng = r.g >> 16;
        for (int g = 0; g < ng; ++g) s = group_fma(s, lval[g0 + g], lidx[g0 + g]);
        return s;
    };
    auto narrow = [&](int q) {
        const int cnt = lptr[q + 1] - lptr[q];
        return cnt <= 64 && lns[q] == cnt;
    };
    auto run_end = [&](int q, int nl) {  // first level >= q that is not narrow, or nl
        for (int b = q;; b += 64) {
            const int qq = b + (tid & 63);
            const unsigned long long m = __ballot(!(qq < nl && narrow(qq)));
            if (m) return b + __builtin_ctzll(m);
        }
    };
    // A lane past a narrow level's last row reads that last row's record (its
    // index is clamped) and so computes the same value into the same slot: no
    // store predicate (duplicate same-address LDS writes cost less than the
    // exec-mask branch of a predicate; measured). The prefetches for levels
    // q+1 / q+2 are unconditional (clamped indices: past the run they read
    // valid records that go unused), so a level is straight-line code; the
    // diagnostics stamp is a separate instantiation (TR), not a branch per level.
    auto narrow_run = [&](const rsp::LevelChunk &ch, int q0, int q1, auto trace_tag) {  // wave 0
        constexpr bool TR = decltype(trace_tag)::value;
        const int lane = tid, x0 = ch.x0, nl = ch.l1 - ch.l0;
        auto lpt = [&](int q) { return lptr[min(q, nl)]; };
        auto ld_row = [&](int p0, int p1) { return max(p0 - x0 + min(lane, p1 - p0 - 1), 0); };
        // level pointers p2, p3 = lptr[q+2], lptr[q+3] (clamped), rolling
        const int p1 = lpt(q0 + 1);
        int p2 = lpt(q0 + 2), p3 = lpt(q0 + 3);
        int cr = ld_row(lpt(q0), p1);
        ThinRow<T> cR = lrow[cr];
        TermIds<G> cI = lidx[cR.g & 0xffff];
        int nr = ld_row(p1, p2);
        ThinRow<T> nR = lrow[nr];
        // Drain the prologue's LDS loads here: the compiler merges the wait
        // state of the loop entry into the loop head, and with these loads
        // pending there it waits at the head of EVERY level — which in the
        // steady state is a wait for the previous level's y store.
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        for (int q = q0; q < q1; ++q) {
            // loads for later levels (none depends on a y): the y indices of
            // level q+1's first group, the row records of level q+2. Term
            // values are not carried: they load with the y, off the critical path.
            const int p4 = lpt(q + 4);
            const TermIds<G> nI = lidx[nR.g & 0xffff];
            const int mr = ld_row(p2, p3);
            const ThinRow<T> mR = lrow[mr];
            // level q: y loads -> fma chain -> y store (the critical path)
            T s;
            const int g0 = cR.g & 0xffff, ng = cR.g >> 16;
            if (__ballot(ng >= 2)) {
                // a row of the level has a second group: every lane loads one
                // (its own, or the pad group) together with the first group's
                // y, so its y loads overlap instead of following the first
                // group's fma chain (one LDS round trip instead of two)
                const int gi = ng >= 2 ? g0 + 1 : kPadGroup;
                const TermIds<G> i2 = lidx[gi];
                s = group_fma(cR.x, lval[g0], cI);
                s = group_fma(s, lval[gi], i2);
                if (__ballot(ng >= 3))
                    for (int g = 2; g < ng; ++g) s = group_fma(s, lval[g0 + g], lidx[g0 + g]);
            } else {
                s = group_fma(cR.x, lval[g0], cI);
            }
            if constexpr (KIND == 2) s = qdiv<T>(s, ldg[cr]);
            put(cR.out, s);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
            if constexpr (TR) {  // diagnostics: level end stamps
                if (lane == 0 && ch.l0 + q < a.trace_cap / 2)
                    a.trace[a.trace_cap / 2 + ch.l0 + q] = a.trace_clk ? clock64() : wall_clock64();
            }
            cR = nR;
            cr = nr;
            cI = nI;
            nR = mR;
            nr = mr;
            p2 = p3;
            p3 = p4;
        }
    };
    // Narrow run in the SPLIT term order (L / L^T: a row's terms from the
    // level just below it are its last groups, legr[] = the groups before
    // them), wave 0 alone, software-pipelined so that only the late part of a
    // level is on the critical path: after level q's y stores, the wave issues
    // the late y loads of level q+1 and, while they are in flight, finishes
    // level q+1's EARLY partial sum (its producers are two or more levels back,
    // done) and prefetches the records of the levels after; then it waits for
    // the late y, runs the late fmas from the early partial and stores. A
    // wave's LDS accesses are performed in order, so no counter and no barrier
    // orders consecutive levels. Lanes past a level's rows repeat its last row
    // (same value to the same slot); groups past a row's own read the pad
    // group (exact no-op fmas); past the run, records are clamped and unused.
    // Same terms, same order (early then late), same fma chain as every other
    // solve path in the split order: same bits.
    auto narrow_run_split = [&](const rsp::LevelChunk &ch, int q0, int q1) {  // wave 0
        const int lane = tid, x0 = ch.x0, nl = ch.l1 - ch.l0;
        auto lpt = [&](int q) { return lptr[min(q, nl)]; };
        struct Lev {
            ThinRow<T> R;
            int eg;  // early groups; late groups = (R.g >> 16) - eg
        };
        auto lev = [&](int q) {
            const int p0 = lpt(q), p1 = lpt(q + 1);
            const int cr = max(p0 - x0 + min(lane, p1 - p0 - 1), 0);
            Lev v;
            v.R = lrow[cr];
            v.eg = legr[cr];
            return v;
        };
        auto early_grp = [&](const Lev &v, int gi) { return gi < v.eg ? (v.R.g & 0xffff) + gi : kPadGroup; };
        auto late_grp = [&](const Lev &v, int gi) {
            return gi < (v.R.g >> 16) - v.eg ? (v.R.g & 0xffff) + v.eg + gi : kPadGroup;
        };
        auto fma_group = [&](T s, const TermGroup<T, G> &g, const T (&y)[G]) {
#pragma unroll
            for (int j = 0; j < G; ++j) s = fma_t(-g.v[j], y[j], s);
            return s;
        };
        auto ygroup = [&](T (&y)[G], const TermIds<G> &id) {
#pragma unroll
            for (int j = 0; j < G; ++j) y[j] = yb(id.v[j]);
        };
        auto nlate = [&](const Lev &v) { return (v.R.g >> 16) - v.eg; };
        Lev c = lev(q0), n = lev(q0 + 1);
        // early partial of level q0 (its early producers are done)
        T e = c.R.x;
        for (int gi = 0; __ballot(gi < c.eg); ++gi) {
            const int gg = early_grp(c, gi);
            e = group_fma(e, lval[gg], lidx[gg]);
        }
        // a level's first two late groups are read ahead (values and y
        // indices do not depend on any y), and their y are loaded together
        // right after the previous level's stores: one LDS round trip on the
        // critical path for rows of up to 2 G late terms
        bool c2 = __ballot(nlate(c) >= 2) != 0;
        TermGroup<T, G> cLV = lval[late_grp(c, 0)], cLV1 = lval[late_grp(c, 1)];
        TermIds<G> nEI = lidx[early_grp(n, 0)];
        TermGroup<T, G> nEV = lval[early_grp(n, 0)];
        T cy[G], cy1[G];
        {
            const TermIds<G> cLI = lidx[late_grp(c, 0)], cLI1 = lidx[late_grp(c, 1)];
            ygroup(cy, cLI);
            ygroup(cy1, cLI1);
        }
        for (int q = q0; q < q1; ++q) {
            // early y of level q+1 (producers two or more levels back)
            T ny[G];
            ygroup(ny, nEI);
            // records of level q+2, the late groups 0 and 1 of level q+1
            const Lev m = lev(q + 2);
            const bool n2 = __ballot(nlate(n) >= 2) != 0;
            const int nlg = late_grp(n, 0), nlg1 = late_grp(n, 1);
            const TermIds<G> nLI = lidx[nlg], nLI1 = lidx[nlg1];
            const TermGroup<T, G> nLV = lval[nlg], nLV1 = lval[nlg1];
            // level q: the late part (critical path)
            T s = fma_group(e, cLV, cy);
            if (c2) {
                s = fma_group(s, cLV1, cy1);
                for (int gi = 2; __ballot(gi < nlate(c)); ++gi) {
                    const int gg = late_grp(c, gi);
                    s = group_fma(s, lval[gg], lidx[gg]);
                }
            }
            put(c.R.out, s);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
            // late y of level q+1 (after level q's stores)
            ygroup(cy, nLI);
            if (n2) ygroup(cy1, nLI1);
            // level q+1's early partial, under those loads
            T e2 = fma_group(n.R.x, nEV, ny);
            for (int gi = 1; __ballot(gi < n.eg); ++gi) {
                const int gg = early_grp(n, gi);
                e2 = group_fma(e2, lval[gg], lidx[gg]);
            }
            // early group 0 of level q+2
            const int meg = early_grp(m, 0);
            nEI = lidx[meg];
            nEV = lval[meg];
            e = e2;
            c = n;
            n = m;
            c2 = n2;
            cLV = nLV;
            cLV1 = nLV1;
        }
    };
    // Narrow run on K waves (a.narrow_waves): wave w computes levels q0 + w,
    // q0 + w + K, ... A level reads its row records, term indices and values
    // first (nothing there depends on a y), then waits until the run's
    // earlier levels are complete — an LDS counter of absolute levels done,
    // advanced by each level's wave after its y stores — and only then does
    // the critical part: y loads -> fma chain -> y stores. While one wave is
    // on its critical part, the others prepare their next levels, so a level
    // costs about its critical part alone (one wave did all of it in line).
    // The counter is a release store after the wave's y stores (lds_publish)
    // and the waiting wave's poll ends in an acquire fence, so its y loads
    // see them (HIP memory model, workgroup scope).
    // Same terms, same order, same fma chain as narrow_run: same bits.
    auto narrow_run_mw = [&](const rsp::LevelChunk &ch, int q0, int q1, int K) {
        const int w = tid >> 6, lane = tid & 63, x0 = ch.x0;
        const int L0 = ch.l0 + q0;
        for (int q = q0 + w; q < q1; q += K) {
            const int p0 = lptr[q], p1 = lptr[q + 1];
            const int cr = max(p0 - x0 + min(lane, p1 - p0 - 1), 0);
            const ThinRow<T> R = lrow[cr];
            const int g0 = R.g & 0xffff, ng = R.g >> 16;
            const bool two = __ballot(ng >= 2) != 0;
            const int gi = ng >= 2 ? g0 + 1 : kPadGroup;
            const TermIds<G> i1 = lidx[g0];
            const TermGroup<T, G> v1 = lval[g0];
            TermIds<G> i2;
            TermGroup<T, G> v2;
            if (two) {
                i2 = lidx[gi];
                v2 = lval[gi];
            }
            const int L = ch.l0 + q;
            if (L > L0) lds_wait_geq(&lds_done, L, L - 1);
            T s = group_fma(R.x, v1, i1);
            if (two) {
                s = group_fma(s, v2, i2);
                if (__ballot(ng >= 3))
                    for (int g = 2; g < ng; ++g) s = group_fma(s, lval[g0 + g], lidx[g0 + g]);
            }
            if constexpr (KIND == 2) s = qdiv<T>(s, ldg[cr]);
            put(R.out, s);
            lds_publish(&lds_done, L + 1, lane == 0);  // after the y stores
            if (a.trace && lane == 0 && L < a.trace_cap / 2)  // diagnostics: level end stamps
                a.trace[a.trace_cap / 2 + L] = a.trace_clk ? clock64() : wall_clock64();
        }
    };
    // The same on K waves with TWO consecutive levels per turn (a.narrow_pairs,
    // RSP_ILU_NARROW_PAIRS; L / L^T of DAGs with small levels, see the
    // launcher): wave w takes levels (q0 + 2 (w + jK), + 1). (The same for the thin factor's narrow
    // rounds measured 21.2 -> 26.0 ms — the second level's item preparation
    // lands on the chain — and was removed.)
    // The second level of a pair reads the first's y from this wave's own
    // stores (in-order LDS of one wave, a wavefront fence between), so a
    // pair pays one counter wait and one release instead of two. Before the
    // wait the wave loads both levels' row records and the first level's
    // term groups; the second level's values load with its y. Same terms,
    // same order, same fma chain: same bits.
    auto narrow_run_mw2 = [&](const rsp::LevelChunk &ch, int q0, int q1, int K) {
        const int w = tid >> 6, lane = tid & 63, x0 = ch.x0;
        const int L0 = ch.l0 + q0;
        auto row_of = [&](int q) {
            const int p0 = lptr[q], p1 = lptr[q + 1];
            return max(p0 - x0 + min(lane, p1 - p0 - 1), 0);
        };
        for (int q = q0 + 2 * w; q < q1; q += 2 * K) {
            const bool has2 = q + 1 < q1;  // wave-uniform
            const int cr = row_of(q), cr2 = has2 ? row_of(q + 1) : cr;
            const ThinRow<T> R = lrow[cr], R2 = lrow[cr2];
            const int g0 = R.g & 0xffff, ng = R.g >> 16;
            const bool two = __ballot(ng >= 2) != 0;
            const int gi = ng >= 2 ? g0 + 1 : kPadGroup;
            const TermIds<G> i1 = lidx[g0];
            const TermGroup<T, G> v1 = lval[g0];
            const TermIds<G> j1 = lidx[R2.g & 0xffff];
            TermIds<G> i2;
            TermGroup<T, G> v2;
            if (two) {
                i2 = lidx[gi];
                v2 = lval[gi];
            }
            // LW > 0 (the narrow waves hold no chunk prefetch, so the registers
            // are there): the third group of the first level and the second and
            // third of the second are prepared before the wait as well, so those
            // groups' y loads join the level's first round trip
            const int h0 = R2.g & 0xffff, nh = R2.g >> 16;
            constexpr bool MORE = LW > 0 && G == 2;
            const bool three = MORE && __ballot(ng >= 3) != 0, two2 = MORE && has2 && __ballot(nh >= 2) != 0;
            const bool three2 = MORE && has2 && __ballot(nh >= 3) != 0;
            TermIds<G> i3, j2, j3;
            if (three) i3 = lidx[ng >= 3 ? g0 + 2 : kPadGroup];
            if (two2) j2 = lidx[nh >= 2 ? h0 + 1 : kPadGroup];
            if (three2) j3 = lidx[nh >= 3 ? h0 + 2 : kPadGroup];
            const int L = ch.l0 + q;
            if (L > L0) lds_wait_geq(&lds_done, L, L - 1);
            T s;
            if (three) {  // groups 0-2 in one round trip
                T ya[3][G];
#pragma unroll
                for (int j = 0; j < G; ++j) {
                    ya[0][j] = yb(i1.v[j]);
                    ya[1][j] = yb(i2.v[j]);
                    ya[2][j] = yb(i3.v[j]);
                }
                const TermGroup<T, G> v3 = lval[ng >= 3 ? g0 + 2 : kPadGroup];
                s = R.x;
#pragma unroll
                for (int j = 0; j < G; ++j) s = fma_t(-v1.v[j], ya[0][j], s);
#pragma unroll
                for (int j = 0; j < G; ++j) s = fma_t(-v2.v[j], ya[1][j], s);
#pragma unroll
                for (int j = 0; j < G; ++j) s = fma_t(-v3.v[j], ya[2][j], s);
                if (__ballot(ng >= 4))
                    for (int g = 3; g < ng; ++g) s = group_fma(s, lval[g0 + g], lidx[g0 + g]);
            } else {
                s = group_fma(R.x, v1, i1);
                if (two) {
                    s = group_fma(s, v2, i2);
                    if (!MORE && __ballot(ng >= 3))
                        for (int g = 2; g < ng; ++g) s = group_fma(s, lval[g0 + g], lidx[g0 + g]);
                }
            }
            if constexpr (KIND == 2) s = qdiv<T>(s, ldg[cr]);
            put(R.out, s);
            if (has2) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
                T t;
                if (two2) {  // groups 0-1 (or 0-2) in one round trip
                    T yb0[G], yb1[G], yb2[G];
#pragma unroll
                    for (int j = 0; j < G; ++j) {
                        yb0[j] = yb(j1.v[j]);
                        yb1[j] = yb(j2.v[j]);
                        if (three2) yb2[j] = yb(j3.v[j]);
                    }
                    const TermGroup<T, G> w0 = lval[h0], w1 = lval[nh >= 2 ? h0 + 1 : kPadGroup];
                    TermGroup<T, G> w2;
                    if (three2) w2 = lval[nh >= 3 ? h0 + 2 : kPadGroup];
                    t = R2.x;
#pragma unroll
                    for (int j = 0; j < G; ++j) t = fma_t(-w0.v[j], yb0[j], t);
#pragma unroll
                    for (int j = 0; j < G; ++j) t = fma_t(-w1.v[j], yb1[j], t);
                    if (three2) {
#pragma unroll
                        for (int j = 0; j < G; ++j) t = fma_t(-w2.v[j], yb2[j], t);
                    }
                    const int gn = three2 ? 3 : 2;
                    if (__ballot(nh > gn))
                        for (int g = gn; g < nh; ++g) t = group_fma(t, lval[h0 + g], lidx[h0 + g]);
                } else {
                    t = group_fma(R2.x, lval[h0], j1);
                    if (__ballot(nh >= 2))
                        for (int g = 1; g < nh; ++g) t = group_fma(t, lval[h0 + g], lidx[h0 + g]);
                }
                if constexpr (KIND == 2) t = qdiv<T>(t, ldg[cr2]);
                put(R2.out, t);
            }
            lds_publish(&lds_done, L + (has2 ? 2 : 1), lane == 0);  // after the y stores
            if (a.trace && lane == 0 && L + 1 < a.trace_cap / 2)  // diagnostics: pair end stamps
                a.trace[a.trace_cap / 2 + L + 1] = a.trace_clk ? clock64() : wall_clock64();
        }
    };
    // NAR: this thread may compute narrow runs (the loaders of LW > 0 never
    // do: their instance of levels() leaves that code, and its registers, out)
    auto levels = [&](const rsp::LevelChunk &ch, auto nar) {
        constexpr bool NAR = decltype(nar)::value;
        const int x0 = ch.x0, nl = ch.l1 - ch.l0;
#if RSP_THIN_LONG_READLANE
        auto vat = [&](int k) { return lval[k / G].v[k % G]; };
        auto yat = [&](int k) { return yb(lidx[k / G].v[k % G]); };
#endif
        for (int q = 0; q < nl;) {
            if (narrow(q)) {
                const int qe = run_end(q, nl);
                if constexpr (NAR) {
                const int K = min(a.narrow_waves, LW > 0 ? LW : (int)(blockDim.x >> 6));  // waves of this launch
                if (KIND != 2 && G == 2 && a.narrow_split) {  // (G = 4: the registers are not there)
                    if constexpr (KIND != 2 && G == 2)
                        if (tid < 64) narrow_run_split(ch, q, qe);
                } else if (PAIRS && K > 1) {  // (its own instantiation: the registers)
                    if constexpr (PAIRS)
                        if (tid < 64 * K) narrow_run_mw2(ch, q, qe, K);
                } else if (K > 1) {
                    if (tid < 64 * K) narrow_run_mw(ch, q, qe, K);
                } else if (tid < 64) {
                    if (a.trace)
                        narrow_run(ch, q, qe, std::true_type());
                    else
                        narrow_run(ch, q, qe, std::false_type());
                }
                }
                lds_barrier();
                q = qe;
                continue;
            }
            const int l = ch.l0 + q;
            const int lp = lptr[q], off = lp - x0, cnt = lptr[q + 1] - lp, ns = lns[q];
            if (tid < ns) {  // (ns <= kChunkRows <= NTH)
                const ThinRow<T> r = lrow[off + tid];
                T s = row_value(r);
                if constexpr (KIND == 2) s = qdiv<T>(s, ldg[off + tid]);
                put(r.out, s);
            }
            for (int r = ns + (tid >> 6); r < cnt; r += NTH / 64) {  // long rows: a wave each
                const ThinRow<T> t = lrow[off + r];
#if RSP_THIN_LONG_READLANE
                const int k0 = G * (t.g & 0xffff);
                T s = wave_chain<T>(t.x, k0, k0 + G * (t.g >> 16), tid & 63, vat, yat);
#else
                // every lane runs the row's chain on broadcast LDS operands,
                // group g+1's values, indices and y read under group g's fmas
                // (the same terms in the same order as wave_chain: same bits)
                const int g0 = t.g & 0xffff, ng = t.g >> 16;
                T s = ng > 0 ? groups_fma(t.x, g0, g0 + ng) : t.x;
#endif
                if constexpr (KIND == 2) s = qdiv<T>(s, ldg[off + r]);
                if ((tid & 63) == 0) put(t.out, s);
            }
            lds_barrier();
            if (a.trace && tid == 0 && l < a.trace_cap / 2)  // diagnostics: level end stamps
                a.trace[a.trace_cap / 2 + l] = a.trace_clk ? clock64() : wall_clock64();
            ++q;
        }
    };
    // chunk records through the constant address space: scalar loads, which
    // the y stores cannot alias and which leave vmcnt to the prefetch
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
        r.st0 = q[6];
        r.st1 = q[7];
        return r;
    };
    // Pipeline: while chunk c's levels run, the streams of chunk c+1 and the y
    // of its staged terms (their list loaded one chunk earlier) are loading,
    // and the staged-term list of chunk c+2. Streams have no dependent loads,
    // so one chunk of lead hides them.
    const int cl = c1 - 1;
    int px0 = 0, px1 = 0;  // the chunk to flush at the next switch
    if (LW == 0 || lt >= 0) {  // the loaders (every thread when LW == 0)
        rsp::LevelChunk rc = chunk(c0), rn = chunk(min(c0 + 1, cl));
        Pre p = load_pre(rc);
        StgY w = load_stgy(load_stg(rc));
        Stg sn = load_stg(rn);
        for (int c = c0; c < c1; ++c) {
            stage(c, px0, px1, rc, p, w);
            const rsp::LevelChunk cur = rc;
            if (c + 1 < c1) {
                const rsp::LevelChunk r2 = chunk(min(c + 2, cl));
                p = load_pre(rn);                           // chunk c+1's streams
                if (rn.st1 > rn.st0) w = load_stgy(sn);     // ... and its staged y
                if (r2.st1 > r2.st0) sn = load_stg(r2);     // chunk c+2's staged terms
                rc = rn;
                rn = r2;
            }
            mark_by(c, 4, 0);  // diagnostics: prefetch issued (wave 0 / last wave)
            mark_by(c, 5, NTH - 64);
            levels(cur, std::integral_constant<bool, LW == 0>());
            mark(c, 3);
            px0 = cur.x0;
            px1 = cur.x1;
        }
    } else {  // the first LW waves: the same barriers, no prefetch (so none of its registers)
        for (int c = c0; c < c1; ++c) {
            const rsp::LevelChunk cur = chunk(c);
            mark(c, 0);
            __syncthreads();  // stage(): the loaders restage the chunk between these two
            mark(c, 1);
            lds_barrier();
            mark(c, 2);
            mark_by(c, 4, 0);
            levels(cur, std::true_type());
            mark(c, 3);
            px0 = cur.x0;
            px1 = cur.x1;
        }
    }
    // the last chunk's rows (its levels ended with a barrier)
    for (int t = tid; t < px1 - px0; t += NTH) y[lrowi[t]] = ybuf[(px0 + t - base) & (rsp::kYWin - 1)];
}

// --------------------------------------------------------------- launchers

// Workgroups of a flow launch: with static items every one must be resident
// at once (rsp::FlowCtl): the occupancy query, less one workgroup per CU of
// margin (it can overstate by one, MI355X_MICROARCH.md residency notes),
// caps the requested grid.
template <auto KERNEL>
static int flow_grid(const rsp::FlowCtl &fc, int want, int cus, int items) {
    static int occ = 0;  // per kernel
    if (occ == 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, KERNEL, 256, 0) != hipSuccess) nb = 1;
        occ = max(nb - 1, 1);
    }
    // (start tickets need no residency: the same grid keeps the walk of the
    // static one; tests oversubscribe it, RSP_ILU_FLOW_GRID_X, so that
    // workgroups wait for others to end and steals carry the launch)
    const int g = min(want, cus * occ) * ((fc.mode & rsp::kFlowTickets) ? fc.grid_x : 1);
    return max(1, min(min(g, rsp::kFlowOwnMax), (items + 3) / 4));
}

// A flow launch of `items` items on `grid` 4-wave workgroups: its claim base,
// and the host mirror advanced by the claims it will make (rsp::FlowCtl).
static unsigned long long flow_claims(const rsp::FlowCtl &fc, int items, int grid) {
    const unsigned long long base = *fc.claim_host;
    if (fc.mode & rsp::kFlowTickets) return (*fc.tk_seq)++;  // the launch's counter slot (FlowClaims)
    if (!(fc.mode & rsp::kFlowClaims)) return base;  // static items: no claims
    *fc.claim_host = base + (unsigned long long)items + 2ull * 4ull * (unsigned long long)grid;
    return base;
}

template <typename T, int B>
static hipError_t launch_factor(const IluArgs &a, hipStream_t s) {
    if (a.fac_one) {
        if (a.n > 0) hipLaunchKernelGGL((ilu0_scale_lower<T>), dim3((a.n + 255) / 256), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    const LevelPlan &P = a.plan;
    int fr = 0;  // next flow run (sorted by level)
    int flow_launched = 0;
    if (a.flow && a.nfruns > 0) {  // the flow rows' upper values become kNotYet (ilu0_flow_prep)
        const int nitems = a.fruns[a.nfruns - 1].c1;
        hipLaunchKernelGGL((ilu0_flow_prep<T>), dim3((nitems + 3) / 4), dim3(256), 0, s, a, nitems);
    }
    for (int g = 0; g < P.nseg; ++g) {
        const rsp::LevelSeg sg = P.segs[g];
        if (sg.thin) {
            hipLaunchKernelGGL((ilu0_rounds<T>), dim3(1), dim3(kThinThreads), 0, s, a, sg.c0, sg.c1);
            continue;
        }
        for (int l = sg.lb; l < sg.le; ++l) {
            while (fr < a.nfruns && a.fruns[fr].lb < l) ++fr;
            if (a.flow && fr < a.nfruns && a.fruns[fr].lb == l) {  // flow run: one persistent launch
                const rsp::FacFlowRun r = a.fruns[fr];
                const bool tk = a.fc.mode & rsp::kFlowTickets;
                const int grid = tk ? flow_grid<ilu0_flow<T, true>>(a.fc, a.flow_grid, a.flow_cus, r.c1 - r.c0)
                                    : flow_grid<ilu0_flow<T, false>>(a.fc, a.flow_grid, a.flow_cus, r.c1 - r.c0);
                const unsigned long long base = flow_claims(a.fc, r.c1 - r.c0, grid);
                if (tk)
                    hipLaunchKernelGGL((ilu0_flow<T, true>), dim3(grid), dim3(256), 0, s, a, r.c0, r.c1, base);
                else
                    hipLaunchKernelGGL((ilu0_flow<T, false>), dim3(grid), dim3(256), 0, s, a, r.c0, r.c1, base);
                ++flow_launched;
                l = r.le - 1;
                continue;
            }
            const int off = P.ptr_host[l], cnt = P.ptr_host[l + 1] - off;
            if (cnt <= 0) continue;
            const rsp::FacSlotLevel *sl = a.fat_slots && a.fslev ? &a.fslev[l] : nullptr;
            if (sl && sl->stride > 0 && sl->rm > 0 && sl->qm > 0) {
                const int *lvl = a.fslots + sl->off;
                auto kern = sl->rm <= 64 ? (sl->qm <= 128 ? ilu0_level_slot<T, 1, 2>
                                                          : sl->qm <= 512 ? ilu0_level_slot<T, 1, 8>
                                                                          : ilu0_level_slot<T, 1, 16>)
                                         : (sl->qm <= 128 ? ilu0_level_slot<T, 4, 2>
                                                          : sl->qm <= 512 ? ilu0_level_slot<T, 4, 8>
                                                                          : ilu0_level_slot<T, 4, 16>);
                hipLaunchKernelGGL(kern, dim3(cnt), dim3(64), 0, s, a, lvl, sl->stride, sl->rm, sl->qm);
            } else if (a.fat_lds)
                hipLaunchKernelGGL((ilu0_level_lds<T, B>), dim3(cnt), dim3(64), 0, s, a, off);
            else
                hipLaunchKernelGGL((ilu0_level<T, B>), dim3((cnt + kIluWaves - 1) / kIluWaves),
                                   dim3(64 * kIluWaves), 0, s, a, off, cnt);
        }
    }
    // ilu0_flow_prep tagged the upper values of EVERY flow run's rows; only the
    // run's own launch restores them. A run the level walk skipped would leave
    // its rows tagged (a corrupt factor reported as success): fail the call.
    if (a.flow && flow_launched != a.nfruns) return hipErrorLaunchFailure;
    return hipGetLastError();
}

template <typename T, int KIND, int B>
static hipError_t launch_solve(const TrsvArgs &a, hipStream_t s) {
    const LevelPlan &P = a.plan;
    const T alpha = (T)a.alpha;
    {  // the streams every level reads (term values, alpha x_i, u_ii in level order)
        const int nk = max(P.nterms, a.n);
        if (nk > 0) hipLaunchKernelGGL((trsv_stream<T, KIND>), dim3((nk + 255) / 256), dim3(256), 0, s, a, alpha);
    }
    for (int g = 0; g < P.nseg; ++g) {
        const rsp::LevelSeg sg = P.segs[g];
        if (sg.thin) {
            // term groups of 2 for DAGs of short chains (the plan padded them so)
            // the two-levels-per-turn narrow runs (L / L^T): RSP_ILU_NARROW_PAIRS
            // 1 / 0 forces them; by default (-1) for DAGs of <= 32 rows per
            // level on average (the deep circuits: config 3, same box, dc1
            // 5.18 -> 4.94 ms, matrix-new_3 6.09 -> 5.81, G2_circuit 3.45 ->
            // 3.22; on wider DAGs' narrow runs they cost: parabolic_fem 3.55
            // -> 3.95, Dubcova3 2.59 -> 2.84, thermomech_TK 0.95 -> 1.00)
            const bool pr = KIND != 2 && (a.narrow_pairs > 0 || (a.narrow_pairs < 0 && a.n <= 32LL * P.nlev));
            // the pair loop's waves never load the next chunk (LW = 4;
            // RSP_ILU_LOADERS=0 turns that off)
            const bool ldr = pr && a.loaders != 0;
            auto kern = P.group == 2 ? (pr ? (ldr ? trsv_thin_pf<T, KIND, 2, KIND != 2, 4> : trsv_thin_pf<T, KIND, 2, KIND != 2>)
                                           : trsv_thin_pf<T, KIND, 2>)
                                     : (pr ? (ldr ? trsv_thin_pf<T, KIND, 4, KIND != 2, 4> : trsv_thin_pf<T, KIND, 4, KIND != 2>)
                                           : trsv_thin_pf<T, KIND, 4>);
            hipLaunchKernelGGL(kern, dim3(1), dim3(kThinThreads), 0, s, a, sg.c0, sg.c1, P.ptr_host[sg.lb]);
            continue;
        }
        if (a.flow && sg.c1 > sg.c0) {  // flow segment: one persistent launch
            const bool tk = a.fc.mode & rsp::kFlowTickets;
            const int grid = tk ? flow_grid<trsv_flow<T, KIND, true>>(a.fc, a.flow_grid, a.flow_cus, sg.c1 - sg.c0)
                                : flow_grid<trsv_flow<T, KIND, false>>(a.fc, a.flow_grid, a.flow_cus, sg.c1 - sg.c0);
            const unsigned long long base = flow_claims(a.fc, sg.c1 - sg.c0, grid);
            if (tk)
                hipLaunchKernelGGL((trsv_flow<T, KIND, true>), dim3(grid), dim3(256), 0, s, a, sg.c0, sg.c1, base);
            else
                hipLaunchKernelGGL((trsv_flow<T, KIND, false>), dim3(grid), dim3(256), 0, s, a, sg.c0, sg.c1, base);
            continue;
        }
        for (int l = sg.lb; l < sg.le; ++l) {
            const int off = P.ptr_host[l], cnt = P.ptr_host[l + 1] - off;
            if (cnt <= 0) continue;
            const int ns = P.nshort_host[l], nb = (ns + 255) / 256;
            const int nw = P.nwave_host ? P.nwave_host[l] : cnt, nwb = (nw - ns + 3) / 4;
            const int sb = P.sbase_host ? P.sbase_host[l] : -1;
            hipLaunchKernelGGL((trsv_level<T, KIND, B>), dim3(nb + nwb + (cnt - nw)), dim3(256), 0,
                               s, a, off, cnt, ns, nb, nw, nwb, sb);
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

void warm_ilu() {  // see rsp_kernels.h
    int o = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, trsv_stream<float, 0>, 256, 0);
}
#ifndef RSP_FTZ_BUILD
// Slot rows of the fat factor levels (analysis, once per pattern). Padding
// is written too: divisor positions -1 and pairs (0, 0), so every value
// index the factor kernel loads from a slot is a valid position.
__global__ __launch_bounds__(64) void ilu0_slot_build(IluArgs a, const int4 *__restrict__ desc,
                                                      const long long *__restrict__ offs,
                                                      int *__restrict__ slots) {
    const int lane = threadIdx.x;
    const int4 d = desc[blockIdx.x];
    int *q = slots + offs[blockIdx.x];
    const int x = d.x, rm = d.y, qm = d.z;
    const int i = a.plan.rows[x], rs = a.rowptr[i], re = a.rowptr[i + 1];
    const int nr = re - rs, nlo = a.dpos[i] - rs;
    const int q0 = a.upd_ptr[rs], nq = a.upd_ptr[re] - q0;
    const bool global = nr > rsp::kFacRow || nq > rsp::kFacPairs;
    if (lane < 8) {
        const int h[8] = {i, rs, nlo, nr, nq, a.hasdiag[i], global ? 1 : 0, 0};
        q[lane] = h[lane];
    }
    for (int y = lane; y < rm; y += 64) {
        const bool in = !global && y < nr, lower = in && y < nlo;
        q[8 + y] = lower ? a.udiv[rs + y] : -1;
        q[8 + rm + y] = in ? ((a.upd_ptr[rs + y] - q0) | ((lower ? a.lord[rs + y] - rs : 0) << 11) |
                              ((lower ? a.lend[rs + y] - rs : 0) << 20))
                           : 0;
    }
    const int pa = rsp::fac_pairs_at(rm);
    for (int u = lane; u < qm; u += 64) {
        const bool in = !global && u < nq;
        q[pa + 2 * u] = in ? a.upd_u[q0 + u] : 0;
        q[pa + 2 * u + 1] = in ? a.upd_l[q0 + u] - rs : 0;
    }
}

hipError_t ilu0_build_slots(const IluArgs &a, const int4 *desc, const long long *offs, int nrows, int *slots,
                            hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    hipLaunchKernelGGL(ilu0_slot_build, dim3(nrows), dim3(64), 0, s, a, desc, offs, slots);
    return hipGetLastError();
}

hipError_t ilu0_factor_f64(const IluArgs &a, hipStream_t s) { return factor_dispatch<double>(a, s); }
hipError_t trsv_lower_n_f64(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<double, 0>(a, s); }
hipError_t trsv_lower_t_f64(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<double, 1>(a, s); }
hipError_t trsv_upper_f64(const TrsvArgs &a, hipStream_t s) { return solve_dispatch<double, 2>(a, s); }
#endif

}  // namespace RSP_KNS
