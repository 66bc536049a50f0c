// ilu_analysis.hip — the data-parallel half of the ILU(0) analysis on the
// MI355X (rsp_ilu0_analysis; the reference's csrilu02_analysis,
// GPU/ilu0.cu:196-217): pattern validation, diagonal positions, the
// structural-zero min-reduce, and the symbolic factor (every position's
// update list, the intra-row stages, the stage order of each row's lower
// positions, the divisor positions). What stays on the host (ilu_analysis.cpp)
// is what is sequential along the dependency chains: the level sets (a row's
// level needs its producers' levels: longest paths of the DAG, one O(nnz)
// pass) and the greedy chunking of the launch plans.
//
// Update lists: position t = (i, j) receives the pair (p = (i, k), q = (k, j))
// for every lower position p of row i with k < j and j in row k's upper part,
// in ascending k — the same lists, in the same order, as the host's
// ilu_symbolic (count pass, exclusive scan, fill pass over the identical
// traversal; see an_pairs). Bitwise-equal plans are asserted through
// rsp_ilu0_plan_digest against rsp_ilu0_analysis_host.
//
// Integer work (HBM/latency-bound, no MFMA). Compiled once (no FTZ variant).

#include <hip/hip_runtime.h>
#include <limits.h>

#include <algorithm>

#include "rsp_kernels.h"

namespace rsp_k {

namespace {

constexpr int kAnThreads = 256;

// first position in [lo, hi) of ci with ci >= v (rows are sorted)
__device__ __forceinline__ int lower_bound_dev(const int *__restrict__ ci, int lo, int hi, int v) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ci[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Diagonal positions + structural zero, one thread per row (binary search:
// O(log len) even on a circuit's hub rows). The pattern was validated on the
// host before this launch (columns in range, rows strictly increasing:
// rsp_api.cpp ilu_symbolic_device returns INVALID_VALUE first), so flags[0]
// is never set here (round 6: the per-row validation loop held one thread
// for a hub row's whole length, ~1 ms on ASIC_320ks); flags[1] = min row
// without a diagonal (INT_MAX = none).
__global__ __launch_bounds__(kAnThreads) void an_rows(int n, const int *__restrict__ rp,
                                                       const int *__restrict__ ci, int *__restrict__ dpos,
                                                       int *__restrict__ hasdiag, int *__restrict__ flags) {
    const int i = blockIdx.x * kAnThreads + threadIdx.x;
    if (i >= n) return;
    const int rs = rp[i], re = rp[i + 1];
    const int d = lower_bound_dev(ci, rs, re, i);
    const int hd = (d < re && ci[d] == i) ? 1 : 0;
    dpos[i] = d;
    hasdiag[i] = hd;
    if (!hd) atomicMin(flags + 1, i);
}

// Update lists, push form, one wave (64-thread workgroup) per row i of a
// length class: for each lower position p = (i, k) in ascending order, the
// lanes take row k's upper entries q (columns > k, 64 at a time), find each
// column in row i after p (binary search: rows are sorted) and, on a hit at
// t, count (FILL = 0) or append (p, q) to t's list (FILL = 1). A row's
// per-position counters / cursors live in LDS (LDS_CAP entries; the wave's
// LDS accesses are in order, and the lanes of one step hit distinct columns),
// so every list comes out in ascending k, exactly as the host's ilu_symbolic.
// Rows longer than any LDS class (LDS_CAP = 0) use global cursors advanced by
// atomics, each step waited for before the next.
template <bool FILL, int LDS_CAP>
__global__ __launch_bounds__(64) void an_pairs(const int *__restrict__ rows, const int *__restrict__ rp,
                                               const int *__restrict__ ci, const int *__restrict__ dpos,
                                               const int *__restrict__ hasdiag, int *__restrict__ cnt_or_ptr,
                                               int *__restrict__ gcur, int *__restrict__ upd_l,
                                               int *__restrict__ upd_u) {
    __shared__ int c[LDS_CAP > 0 ? LDS_CAP : 1];
    const int lane = threadIdx.x;
    const int i = rows[blockIdx.x];
    const int rs = rp[i], re = rp[i + 1], di = dpos[i];
    int *cur = LDS_CAP > 0 ? c - rs : gcur;  // indexed by position
    for (int t = rs + lane; t < re; t += 64) cur[t] = FILL ? cnt_or_ptr[t] : 0;
    __syncthreads();
    for (int p = rs; p < di; p++) {
        const int k = ci[p];
        const int q1 = rp[k + 1];
        for (int qb = dpos[k] + hasdiag[k]; qb < q1; qb += 64) {
            const int q = qb + lane;
            if (q < q1) {
                const int col = ci[q];
                const int t = lower_bound_dev(ci, p + 1, re, col);
                if (t < re && ci[t] == col) {
                    if (LDS_CAP > 0) {
                        const int m = cur[t];
                        cur[t] = m + 1;
                        if (FILL) {
                            upd_l[m] = p;
                            upd_u[m] = q;
                        }
                    } else {
                        const int m = atomicAdd(cur + t, 1);
                        if (FILL) {
                            upd_l[m] = p;
                            upd_u[m] = q;
                        }
                    }
                }
            }
            if (LDS_CAP == 0) __builtin_amdgcn_s_waitcnt(0);  // this step's atomics before the next's
        }
    }
    __syncthreads();
    if (!FILL)
        for (int t = rs + lane; t < re; t += 64) cnt_or_ptr[t] = cur[t];
}

// The same lists for the rows of <= `cap` entries, with row i's columns
// staged in LDS beside its counters (dynamic LDS: 3 cap ints): the search for
// each column of row k in row i is an LDS binary search instead of a chain of
// global loads, and the (p, q) steps are FLATTENED: for 64 lower positions p
// at a time, the upper parts of their rows k are concatenated (an exclusive
// scan of their lengths) and the wave takes 64 consecutive (p, q) of that
// sequence per step, the next step's column loads issued before this step's
// searches (round 6: one step per p left a circuit row of hundreds of lower
// positions, most with rows k of a few upper entries, at one dependent load
// per p, ~0.5-0.9 ms per pass). Order: a step's lanes are in (p, q) order, so
// two lanes of one step that hit the same target t are ranked by lane (the
// lower lane has the smaller p) — the lists come out in ascending k as in the
// one-p-per-step walk. Counting needs no order (LDS atomic adds).
template <bool FILL>
__global__ __launch_bounds__(64) void an_pairs_lds(const int *__restrict__ rows, int cap, const int *__restrict__ rp,
                                                   const int *__restrict__ ci, const int *__restrict__ dpos,
                                                   const int *__restrict__ hasdiag, int *__restrict__ cnt_or_ptr,
                                                   int *__restrict__ upd_l, int *__restrict__ upd_u) {
    extern __shared__ int an_lds[];
    int *cur = an_lds, *cols = an_lds + cap, *tag = an_lds + 2 * cap;  // indexed by position - rs
    __shared__ int offs[64], qsl[64];
    const int lane = threadIdx.x;
    const int i = rows[blockIdx.x];
    const int rs = rp[i], re = rp[i + 1], di = dpos[i], len = re - rs;
    for (int t = lane; t < len; t += 64) {
        cur[t] = FILL ? cnt_or_ptr[rs + t] : 0;
        cols[t] = ci[rs + t];
    }
    __syncthreads();
    for (int pb = rs; pb < di; pb += 64) {
        const int np = min(64, di - pb);
        int qs = 0, nq = 0;  // lane j: row k = ci[pb + j]'s upper range
        if (lane < np) {
            const int k = cols[pb + lane - rs];
            qs = dpos[k] + hasdiag[k];
            nq = max(0, rp[k + 1] - qs);
        }
        int incl = nq;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const int total = __builtin_amdgcn_readlane(incl, 63);
        offs[lane] = incl - nq;  // lanes >= np: total
        qsl[lane] = qs;
        __syncthreads();
        // flattened index f -> (j, q): the largest j with offs[j] <= f
        auto locate = [&](int f, int &jj) {
            int lo = 0, hi = 63;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (offs[mid] <= f)
                    lo = mid;
                else
                    hi = mid - 1;
            }
            jj = lo;
            return qsl[lo] + f - offs[lo];
        };
        int j = 0, q = 0, col = -1;
        if (lane < total) {
            q = locate(lane, j);
            col = ci[q];
        }
        for (int fb = 0; fb < total; fb += 64) {
            int jn = 0, qn = 0, coln = -1;
            if (fb + 64 + lane < total) {
                qn = locate(fb + 64 + lane, jn);
                coln = ci[qn];
            }
            const int p = pb + j;
            int t = -1;
            if (col >= 0) {
                int lo = p + 1 - rs, hi = len;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (cols[mid] < col)
                        lo = mid + 1;
                    else
                        hi = mid;
                }
                if (lo < len && cols[lo] == col) t = lo;
            }
            if (!FILL) {
                if (t >= 0) atomicAdd(&cur[t], 1);
            } else {
                // lanes of this step sharing a target: ranked by lane
                // (volatile: the read-backs must not be folded into this
                // lane's own stores). One lane of a clashing group wins the
                // tag; the others mark the target, so the whole group sees it;
                // then one ballot per clashing group ranks its lanes
                volatile int *vtag = tag;
                if (t >= 0) vtag[t] = lane;
                const bool lost = t >= 0 && vtag[t] != lane;
                int rank = 0, last = 1;
                if (__any(lost)) {
                    if (lost) vtag[t] = 64;
                    const bool grp = t >= 0 && vtag[t] == 64;
                    unsigned long long todo = __ballot(grp);
                    while (todo) {
                        const int tl = __builtin_amdgcn_readlane(t, __builtin_ctzll(todo));
                        const unsigned long long mask = __ballot(grp && t == tl);
                        if (grp && t == tl) {
                            rank = __popcll(mask & ((1ull << lane) - 1ull));
                            last = (mask >> lane) == 1ull ? 1 : 0;
                        }
                        todo &= ~mask;
                    }
                }
                if (t >= 0) {
                    const int m = cur[t] + rank;
                    upd_l[m] = p;
                    upd_u[m] = q;
                    __builtin_amdgcn_wave_barrier();
                    if (last) cur[t] = m + 1;
                }
            }
            j = jn;
            q = qn;
            col = coln;
        }
        __syncthreads();  // (offs / qsl rewritten by the next batch)
    }
    __syncthreads();
    if (!FILL)
        for (int t = lane; t < len; t += 64) cnt_or_ptr[rs + t] = cur[t];
}

// Per row (one thread): intra-row stages of the lower positions (stage(t) =
// 1 + max stage of the l_ik its pairs read, 0 without pairs; positions in
// ascending order, so every read stage is final), the stable order of the
// lower positions by stage (lord; counting sort through `scratch`, which
// holds one counter per lower position), and lend (end of each position's
// stage group in lord order). Divisor positions of the lower entries (udiv).
__global__ __launch_bounds__(kAnThreads) void an_stages(int n, int maxlen, const int *__restrict__ rp,
                                                         const int *__restrict__ ci,
                                                         const int *__restrict__ dpos,
                                                         const int *__restrict__ hasdiag,
                                                         const int *__restrict__ ptr,
                                                         const int *__restrict__ upd_l, int *__restrict__ stage,
                                                         int *__restrict__ lord, int *__restrict__ lend,
                                                         int *__restrict__ udiv, int *__restrict__ scratch) {
    const int i = blockIdx.x * kAnThreads + threadIdx.x;
    if (i >= n) return;
    const int rs = rp[i], di = dpos[i], re = rp[i + 1];
    if (re - rs > maxlen) return;  // done on the host
    int smax = -1;
    for (int t = rs; t < di; t++) {
        int s = 0;
        for (int u = ptr[t]; u < ptr[t + 1]; u++) s = max(s, stage[upd_l[u]] + 1);
        stage[t] = s;
        smax = max(smax, s);
        const int k = ci[t];
        udiv[t] = hasdiag[k] ? dpos[k] : -1;
        scratch[t] = 0;
    }
    for (int t = di; t < re; t++) {
        stage[t] = 0;
        udiv[t] = -1;
        lord[t] = 0;
        lend[t] = 0;
    }
    if (di == rs) return;
    // counting sort by stage (stage < di - rs): counters at scratch[rs + s]
    for (int t = rs; t < di; t++) scratch[rs + stage[t]]++;
    int run = 0;
    for (int s = 0; s <= smax; s++) {
        const int c = scratch[rs + s];
        scratch[rs + s] = run;
        run += c;
    }
    for (int t = rs; t < di; t++) lord[rs + scratch[rs + stage[t]]++] = t;
    for (int x = di - rs - 1; x >= 0; x--) {
        const bool last = x == di - rs - 1 || stage[lord[rs + x]] != stage[lord[rs + x + 1]];
        lend[rs + x] = last ? rs + x + 1 : lend[rs + x + 1];
    }
}

// an_stages for one row per wave (the rows of (thread-kernel maxlen, 1024]
// entries, listed in `rows`): the same stage, udiv, lord, lend. Stages in
// LDS; a lower position's pairs read by the lanes (the next position's pair
// loads issued before this one's max-reduce: upd_l does not depend on the
// stages); the stable counting sort by stage as a wave: LDS histogram, scan,
// then positions placed 64 at a time in position order, each lane counting
// the lanes before it of its own stage (round 6: one thread per such row
// walked its pairs and sort through dependent global loads, ~0.6-1 ms per
// pass on the circuits).
__global__ __launch_bounds__(64) void an_stages_wave(const int *__restrict__ rows, const int *__restrict__ rp,
                                                      const int *__restrict__ ci, const int *__restrict__ dpos,
                                                      const int *__restrict__ hasdiag,
                                                      const int *__restrict__ ptr,
                                                      const int *__restrict__ upd_l, int *__restrict__ stage,
                                                      int *__restrict__ lord, int *__restrict__ lend,
                                                      int *__restrict__ udiv) {
    __shared__ int st[1024], base[1024], pl[1024];
    const int lane = threadIdx.x;
    const int i = rows[blockIdx.x];
    const int rs = rp[i], di = dpos[i], re = rp[i + 1], nl = di - rs;
    for (int t = di + lane; t < re; t += 64) {
        stage[t] = 0;
        udiv[t] = -1;
        lord[t] = 0;
        lend[t] = 0;
    }
    for (int x = lane; x < nl; x += 64) {
        const int k = ci[rs + x];
        udiv[rs + x] = hasdiag[k] ? dpos[k] : -1;
        base[x] = 0;
    }
    if (nl == 0) return;
    // stages, position by position; u ranges read 63 positions at a time
    // (lane x: the start of position xb + x's pairs, lane nx: the last end)
    int smax = 0;
    for (int xb = 0; xb < nl; xb += 63) {
        const int nx = min(63, nl - xb);
        const int u0l = lane <= nx ? ptr[rs + xb + lane] : 0;
        if (__builtin_amdgcn_readlane(u0l, 0) == __builtin_amdgcn_readlane(u0l, nx)) {
            // no pairs in these positions: stage 0 each, in parallel
            if (lane < nx) {
                st[xb + lane] = 0;
                stage[rs + xb + lane] = 0;
            }
            __syncthreads();  // (later positions read these slots from other lanes)
            continue;
        }
        int u0 = __builtin_amdgcn_readlane(u0l, 0);
        int u1 = __builtin_amdgcn_readlane(u0l, 1);
        int v = u0 + lane < u1 ? upd_l[u0 + lane] : -1;
        for (int x = 0; x < nx; x++) {
            int s = 0;
            const bool any = u1 > u0;  // (uniform)
            for (int u = u0;;) {
                const int un = u + 64;
                // the next load: this position's next 64 pairs, else the next position's first
                int vn = -1, u0n = u0, u1n = u1;
                if (un < u1) {
                    vn = un + lane < u1 ? upd_l[un + lane] : -1;
                } else if (x + 1 < nx) {
                    u0n = u1;
                    u1n = __builtin_amdgcn_readlane(u0l, x + 2);
                    vn = u0n + lane < u1n ? upd_l[u0n + lane] : -1;
                }
                if (v >= 0) s = max(s, st[v - rs] + 1);
                v = vn;
                if (un >= u1) {
                    u0 = u0n;
                    u1 = u1n;
                    break;
                }
                u = un;
            }
            // wave max (every lane ends with the row's value)
            if (any)
                for (int o = 32; o > 0; o >>= 1) s = max(s, __shfl_xor(s, o));
            st[xb + x] = s;  // every lane writes the same value, and reads only its own writes
            stage[rs + xb + x] = s;
            smax = max(smax, s);
        }
    }
    // histogram of the stages (< nl), exclusive scan into base
    __syncthreads();
    for (int x = lane; x < nl; x += 64) atomicAdd(&base[st[x]], 1);
    __syncthreads();
    int carry = 0;
    for (int sb = 0; sb <= smax; sb += 64) {
        const int sx = sb + lane;
        const int c = sx <= smax ? base[sx] : 0;
        int incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (sx <= smax) base[sx] = carry + incl - c;
        carry += __builtin_amdgcn_readlane(incl, 63);
    }
    __syncthreads();
    // stable placement, 64 positions at a time in position order
    for (int xb = 0; xb < nl; xb += 64) {
        const int x = xb + lane;
        const int s = x < nl ? st[x] : -1;
        int before = 0;
        for (int l = 0; l < 64; l++) before += (l < lane && __builtin_amdgcn_readlane(s, l) == s) ? 1 : 0;
        if (s >= 0) {
            const int pos = base[s] + before;
            pl[x] = pos;
            lord[rs + pos] = rs + x;
        }
        __syncthreads();
        if (s >= 0) atomicAdd(&base[s], 1);
        __syncthreads();
    }
    // base[s] is now the end of stage s's group
    for (int x = lane; x < nl; x += 64) lend[rs + pl[x]] = rs + base[st[x]];
}

inline unsigned grid_of(long long count) { return (unsigned)((count + kAnThreads - 1) / kAnThreads); }

}  // namespace

void warm_analysis() {  // see rsp_kernels.h
    int o = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, an_rows, kAnThreads, 0);
}

hipError_t ilu_an_rows(int n, const int *rp, const int *ci, int *dpos, int *hasdiag, int *flags,
                       hipStream_t s) {
    if (n <= 0) return hipSuccess;
    an_rows<<<grid_of(n), kAnThreads, 0, s>>>(n, rp, ci, dpos, hasdiag, flags);
    return hipGetLastError();
}

// Row length classes of the pair kernels: <= 1024 entries (4 KB of LDS per
// wave), <= 16384 (64 KB), longer (global cursors). rows_c*: the rows of each
// class (device), counts n_c*.
template <bool FILL>
static hipError_t an_pairs_launch(const int *const rows_c[3], const int n_c[3], int cap0, const int *rp, const int *ci,
                                  const int *dpos, const int *hasdiag, int *cnt_or_ptr, int *gcur, int *upd_l,
                                  int *upd_u, hipStream_t s) {
    if (n_c[0] > 0)
        an_pairs_lds<FILL><<<n_c[0], 64, 3 * cap0 * sizeof(int), s>>>(rows_c[0], cap0, rp, ci, dpos, hasdiag,
                                                                    cnt_or_ptr, upd_l, upd_u);
    if (n_c[1] > 0)
        an_pairs<FILL, 16384><<<n_c[1], 64, 0, s>>>(rows_c[1], rp, ci, dpos, hasdiag, cnt_or_ptr, gcur, upd_l, upd_u);
    if (n_c[2] > 0)
        an_pairs<FILL, 0><<<n_c[2], 64, 0, s>>>(rows_c[2], rp, ci, dpos, hasdiag, cnt_or_ptr, gcur, upd_l, upd_u);
    return hipGetLastError();
}

hipError_t ilu_an_count(const int *const rows_c[3], const int n_c[3], int cap0, const int *rp, const int *ci,
                        const int *dpos, const int *hasdiag, int *cnt, int *gcur, hipStream_t s) {
    return an_pairs_launch<false>(rows_c, n_c, cap0, rp, ci, dpos, hasdiag, cnt, gcur, nullptr, nullptr, s);
}

// Exclusive prefix sum of `count` ints (cnt -> ptr) in three passes: block
// sums (1024 elements per 256-thread block), a one-block scan of those, then
// each block's local scan plus its offset. temp holds the block sums; with
// temp == nullptr only *temp_bytes is set.
namespace {
constexpr int kScanPer = 1024;  // elements per block (4 per thread)

__device__ __forceinline__ int block_excl_scan(int v, int *lds, int *total) {
    // inclusive scan over 256 threads in LDS (Hillis-Steele), returns exclusive
    const int t = threadIdx.x;
    lds[t] = v;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
        const int a = t >= d ? lds[t - d] : 0;
        __syncthreads();
        lds[t] += a;
        __syncthreads();
    }
    const int incl = lds[t];
    if (total) *total = lds[255];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(256) void scan_sums(const int *__restrict__ in, int count, int *__restrict__ sums) {
    __shared__ int lds[256];
    const int base = blockIdx.x * kScanPer + threadIdx.x * 4;
    int v = 0;
    for (int j = 0; j < 4; j++) v += base + j < count ? in[base + j] : 0;
    int tot;
    block_excl_scan(v, lds, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// one block scans the (<= 256 * 1024) block sums in place, exclusive
__global__ __launch_bounds__(256) void scan_top(int *__restrict__ sums, int nb) {
    __shared__ int lds[256];
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += 256 * 4) {
        const int base = b0 + threadIdx.x * 4;
        int v[4], loc = 0;
        for (int j = 0; j < 4; j++) {
            v[j] = base + j < nb ? sums[base + j] : 0;
            loc += v[j];
        }
        int tot;
        int ex = block_excl_scan(loc, lds, &tot) + carry;
        for (int j = 0; j < 4; j++) {
            if (base + j < nb) sums[base + j] = ex;
            ex += v[j];
        }
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void scan_apply(const int *__restrict__ in, int count,
                                                  const int *__restrict__ sums, int *__restrict__ out) {
    __shared__ int lds[256];
    const int base = blockIdx.x * kScanPer + threadIdx.x * 4;
    int v[4], loc = 0;
    for (int j = 0; j < 4; j++) {
        v[j] = base + j < count ? in[base + j] : 0;
        loc += v[j];
    }
    int ex = block_excl_scan(loc, lds, nullptr) + sums[blockIdx.x];
    for (int j = 0; j < 4; j++) {
        if (base + j < count) out[base + j] = ex;
        ex += v[j];
    }
}
}  // namespace

hipError_t ilu_an_scan(const int *cnt, int *ptr, int count, void *temp, size_t *temp_bytes, hipStream_t s) {
    const int nb = (count + kScanPer - 1) / kScanPer;
    if (!temp) {
        *temp_bytes = (size_t)std::max(nb, 1) * sizeof(int);
        return hipSuccess;
    }
    if (count <= 0) return hipSuccess;
    int *sums = (int *)temp;
    scan_sums<<<nb, 256, 0, s>>>(cnt, count, sums);
    scan_top<<<1, 256, 0, s>>>(sums, nb);
    scan_apply<<<nb, 256, 0, s>>>(cnt, count, sums, ptr);
    return hipGetLastError();
}

hipError_t ilu_an_fill(const int *const rows_c[3], const int n_c[3], int cap0, const int *rp, const int *ci,
                       const int *dpos, const int *hasdiag, const int *ptr, int *gcur, int *upd_l, int *upd_u,
                       hipStream_t s) {
    return an_pairs_launch<true>(rows_c, n_c, cap0, rp, ci, dpos, hasdiag, const_cast<int *>(ptr), gcur, upd_l, upd_u,
                                 s);
}

hipError_t ilu_an_stages(int n, int maxlen, const int *rp, const int *ci, const int *dpos, const int *hasdiag,
                         const int *ptr, const int *upd_l, int *stage, int *lord, int *lend, int *udiv,
                         int *scratch, const int *wrows, int nwrows, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    an_stages<<<grid_of(n), kAnThreads, 0, s>>>(n, maxlen, rp, ci, dpos, hasdiag, ptr, upd_l, stage, lord, lend,
                                                udiv, scratch);
    if (nwrows > 0)
        an_stages_wave<<<nwrows, 64, 0, s>>>(wrows, rp, ci, dpos, hasdiag, ptr, upd_l, stage, lord, lend, udiv);
    return hipGetLastError();
}

// The update pairs of the listed rows, packed back to back (row r's pairs at
// cbase[r]): the host factor plan reads only its thin rows' pairs.
__global__ __launch_bounds__(256) void an_gather_pairs(const int *__restrict__ rows, int nrows,
                                                       const int *__restrict__ rp, const int *__restrict__ ptr,
                                                       const int *__restrict__ cbase, const int *__restrict__ upd_l,
                                                       const int *__restrict__ upd_u, int *__restrict__ out_l,
                                                       int *__restrict__ out_u) {
    for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
        const int i = rows[r], q0 = ptr[rp[i]], q1 = ptr[rp[i + 1]], o = cbase[r] - q0;
        for (int q = q0 + (int)threadIdx.x; q < q1; q += 256) {
            out_l[o + q] = upd_l[q];
            out_u[o + q] = upd_u[q];
        }
    }
}

hipError_t ilu_an_gather_pairs(const int *rows, int nrows, const int *rp, const int *ptr, const int *cbase,
                               const int *upd_l, const int *upd_u, int *out_l, int *out_u, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    an_gather_pairs<<<std::min(nrows, 65536), 256, 0, s>>>(rows, nrows, rp, ptr, cbase, upd_l, upd_u, out_l, out_u);
    return hipGetLastError();
}

// ------------------------------------------------ solve plans: per-term half
// (ilu_analysis.cpp solve_plan_terms restated; see SolveTermsArgs)
namespace {

// a row's padded terms and the offset of its late terms (ilu_analysis.cpp
// split_padded / late_offset restated)
__device__ __forceinline__ int st_split_padded(int ne, int cnt, int g) {
    const int pe = (ne + g - 1) / g * g, pl = (cnt - ne + g - 1) / g * g;
    return max(g, pe + pl);
}
__device__ __forceinline__ int st_row_terms(const rsp_k::SolveTermsArgs &a, int i, int *j0) {
    if (a.kind == 0) {
        *j0 = a.rp[i];
        return a.dpos[i] - *j0;
    }
    *j0 = a.ltp[i];
    return a.ltp[i + 1] - *j0;
}

// one wave per level-order slot x: its flat terms [t0, next t0) — the row's
// terms in the split order (a thin row's late terms from the first group
// after its early ones), pads (position -1, source the zero slot) elsewhere —
// y index "zero slot" (thin runs overwrite theirs), slot_of, default row record
__global__ __launch_bounds__(256) void st_rows(rsp_k::SolveTermsArgs a) {
    const int x = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (x >= a.nx) return;
    const rsp::RowTask t = a.tasks[x];
    const int i = t.i;
    int j0;
    const int cnt = st_row_terms(a, i, &j0);
    const int ne = a.kind == 2 || !a.ne ? 0 : a.ne[i], g = a.group;  // no ne / lpos: the reference's order
    const int lo = t.t1 - t.t0 == st_split_padded(ne, cnt, g) ? (ne + g - 1) / g * g : ne;
    const int tend = x + 1 < a.nx ? a.tasks[x + 1].t0 : a.total;
    for (int q = lane; q < tend - t.t0; q += 64) {
        const int k = t.t0 + q;
        const int o = q < ne ? q : (q >= lo && q - lo < cnt - ne ? ne + q - lo : -1);  // term, or pad
        int tp = -1, c = rsp::kPadSrc;
        if (o >= 0) {
            const int j = j0 + o;
            tp = a.kind == 0 ? (a.lpos ? a.lpos[j] : j) : a.lts[j];
            c = a.kind == 0 ? a.ci[tp] : a.ltc[j];
        }
        a.tpos[k] = tp;
        a.src[k] = c;
        a.sid[k] = rsp::kYWin;
    }
    if (lane == 0) {
        a.slot_of[i] = x;
        a.trow[x] = rsp::ThinRowPlan{0, 0, 0, -1};
    }
}

__device__ __forceinline__ int block_sum(int v, int *lds) {
    int tot;
    block_excl_scan(v, lds, &tot);
    return tot;
}

// one workgroup per chunk: the window remap of its terms (a producer earlier
// in the run and at most kYWin slots before the end of the consumer's level
// is read from the LDS window) and the count of its staged terms
__global__ __launch_bounds__(256) void st_remap(rsp_k::SolveTermsArgs a) {
    __shared__ int lds[256];
    const int c = blockIdx.x;
    const rsp::LevelChunk ch = a.chunks[c];
    const int base = a.cbase[c];
    int m = 0;
    for (int k = ch.k0 + (int)threadIdx.x; k < ch.k1; k += 256) {
        int sc = a.src[k];
        if (sc >= 0) {
            int lo = ch.x0, hi = ch.x1;  // the slot whose terms hold k (thin rows: t0 strictly increasing)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (a.tasks[mid].t0 <= k)
                    lo = mid;
                else
                    hi = mid;
            }
            int l0 = ch.l0, l1 = ch.l1;  // ... and its level
            while (l1 - l0 > 1) {
                const int mid = (l0 + l1) >> 1;
                if (a.ptr[mid] <= lo)
                    l0 = mid;
                else
                    l1 = mid;
            }
            const int sj = a.slot_of[sc];
            if (sj >= base && sj < a.ptr[l0]) {
                const int rj = sj - base;
                if (a.ptr[l0 + 1] - base - rj <= rsp::kYWin) {
                    sc = -((rj & (rsp::kYWin - 1)) + 1);
                    a.src[k] = sc;
                }
            }
        }
        m += sc >= 0;
    }
    const int tot = block_sum(m, lds);
    if (threadIdx.x == 0) a.nst[c] = tot;
}

// one workgroup per chunk: its staged range, row records, y indices and
// staged terms (in term order: a block scan per 256 terms)
__global__ __launch_bounds__(256) void st_fill(rsp_k::SolveTermsArgs a) {
    __shared__ int lds[256];
    const int c = blockIdx.x;
    const rsp::LevelChunk ch = a.chunks[c];
    const int base = a.cbase[c], st0 = a.nst_ptr[c];
    if (threadIdx.x == 0) {
        a.chunks[c].st0 = st0;
        a.chunks[c].st1 = a.nst_ptr[c + 1];
        if (c == 0 && a.nst_ptr[a.nch] == 0) a.stg[0] = rsp::StagedTerm{0, 0};  // the empty list's entry
    }
    const int G = a.group;
    for (int x = ch.x0 + (int)threadIdx.x; x < ch.x1; x += 256) {
        const rsp::RowTask t = a.tasks[x];
        int j0;
        const int cnt = st_row_terms(a, t.i, &j0), ne = a.kind == 2 || !a.ne ? 0 : a.ne[t.i];
        const int eg = t.t1 - t.t0 == st_split_padded(ne, cnt, G) ? (ne + G - 1) / G : 0;  // early groups
        a.trow[x] = rsp::ThinRowPlan{(t.t0 - ch.k0) / G | ((t.t1 - t.t0) / G) << 16,
                                     ((x - base) & (rsp::kYWin - 1)) | eg << 16, t.i, t.d};
    }
    int run = st0;
    for (int kb = ch.k0; kb < ch.k1; kb += 256) {
        const int k = kb + (int)threadIdx.x;
        const int sc = k < ch.k1 ? a.src[k] : -1;
        int tot;
        const int pos = block_excl_scan(sc >= 0 ? 1 : 0, lds, &tot);
        if (k < ch.k1) {
            if (sc < 0) {
                a.sid[k] = -sc - 1;
            } else {
                a.sid[k] = rsp::kYWin + 1 + (k - ch.k0);
                a.stg[run + pos] = rsp::StagedTerm{k - ch.k0, sc};
            }
        }
        run += tot;
    }
}

}  // namespace

hipError_t ilu_an_solve_terms(const SolveTermsArgs &a, hipStream_t s) {
    if (a.total <= 0 || a.nx <= 0 || a.nch <= 0) return hipErrorInvalidValue;  // the caller writes the empty plan
    st_rows<<<(unsigned)((a.nx + 3) / 4), 256, 0, s>>>(a);
    st_remap<<<a.nch, 256, 0, s>>>(a);
    hipError_t e = hipMemsetAsync(a.nst + a.nch, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    size_t tb = 0;
    (void)ilu_an_scan(nullptr, nullptr, a.nch + 1, nullptr, &tb, s);
    e = ilu_an_scan(a.nst, a.nst_ptr, a.nch + 1, a.scan, &tb, s);
    if (e != hipSuccess) return e;
    st_fill<<<a.nch, 256, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace rsp_k
