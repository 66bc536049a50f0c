// ilu_blocks.cpp — plan of the block-inverse solve of a deep DAG (round 6;
// kernels: trsv_blocks.hip, layout: rsp::BlkDesc in rsp_kernels.h).
//
// The level-scheduled solve pays one dependent hand-off per level; on the
// circuits (~10^4 levels of ~10 rows) that is ~190 ns per level and the GPU
// loses to one CPU core. This plan cuts the rows, in level order, into
// blocks of <= kBlkRows rows and writes every row's unknown as a combination
// of its block's right-hand sides and of unknowns of EARLIER blocks (the
// block's partitioned inverse), so one block — several levels — is one
// dependent step of one wave.
//
// Every rule here is restated independently in oracle/rsp_oracle.c
// (oracle_trsv_blocks_*, steps 1-6), and the GPU result equals that
// restatement bit for bit:
//  * dependencies of row i: kind 0 (L) the strict lower part of row i,
//    column ascending; kind 1 (L^T) the rows j > i with l_ji != 0, j
//    descending (IluHostPlan::ltp / lts / ltc);
//  * positions: the DAG's level order, rows ascending inside a level;
//  * chunks of kBlkWin positions; no block crosses a chunk (a chunk is one
//    segment: one launch, its y in the LDS window);
//  * blocks, greedily inside a chunk: row p joins the current block (first
//    position s) while the block has < kBlkRows rows and p's pattern there
//    has <= kBlkYMax y terms, <= kBlkNear of them near (position >=
//    max(chunk start, s - kBlkNearWin)); else p starts a new block with its
//    own dependencies as pattern, and if that breaks the caps p is a long
//    block of its own;
//  * pattern: x sources (p and the x sources of its in-block dependencies),
//    then y sources (the in-block dependencies' y sources and the positions
//    of its dependencies before the block), each ascending.
// Chunks are independent (the near rule reads positions only), so they are
// planned in parallel; so are the blocks' coefficient recipes.
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <vector>

#include "ilu_analysis.h"

namespace rsp_an {

bool blocks_wanted(int n, int nlev) {
    const int m = env_int("RSP_ILU_BLOCKS", -1);
    if (m == 0 || n <= 0) return false;
    if (m > 0) return true;
    // deep DAGs: <= 32 rows per level on average (the circuits: ~10)
    return (long long)n <= 32LL * nlev;
}

namespace {

// One chunk's blocks and patterns (positions [c0, c1)), local numbering.
struct ChunkPlan {
    std::vector<int> pool;    // patterns, position by position
    std::vector<int> bstart;  // local blocks' first positions
    std::vector<char> islong;
};

}  // namespace

bool plan_blocks(int kind, const int *rp, const int *ci, const IluHostPlan &hp, BlkPlanHost &bp) {
    const int BS = rsp::kBlkRows, YMAX = env_int("RSP_BLK_YMAX", rsp::kBlkYMax), NMAX = env_int("RSP_BLK_NMAX", rsp::kBlkNear),
              NW = env_int("RSP_BLK_NW", rsp::kBlkNearWin), CH = env_int("RSP_BLK_CH", rsp::kBlkWin);
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    const int n = hp.n;
    const DagHost &dag = kind == 0 ? hp.L : hp.LT;
    bp = BlkPlanHost();
    bp.n = n;
    if (n <= 0 || (int)dag.rows.size() != n || dag.ptr.size() < 2) return false;
    auto dep_begin = [&](int i) { return kind == 0 ? rp[i] : hp.ltp[(size_t)i]; };
    auto dep_end = [&](int i) { return kind == 0 ? hp.dpos[(size_t)i] : hp.ltp[(size_t)i + 1]; };
    auto dep_src = [&](int o) { return kind == 0 ? ci[o] : hp.ltc[(size_t)o]; };
    auto dep_val = [&](int o) { return kind == 0 ? o : hp.lts[(size_t)o]; };
    // positions: level order, rows ascending inside a level
    hvec<int> &order = bp.order;
    order.assign(dag.rows.begin(), dag.rows.end());
    const int nlev = (int)dag.ptr.size() - 1;
    parallel_for(nlev, 256, [&](long long l0, long long l1) {
        for (long long l = l0; l < l1; l++)
            std::sort(order.begin() + dag.ptr[(size_t)l], order.begin() + dag.ptr[(size_t)l + 1]);
    });
    hvec<int> pos((size_t)n);
    parallel_for(n, 1 << 14, [&](long long p0, long long p1) {
        for (long long p = p0; p < p1; p++) pos[(size_t)order[(size_t)p]] = (int)p;
    });

    // ---- chunks: at most CH positions; a row with more than kBlkLongCap
    // dependencies at or after its chunk's start starts a new chunk (its
    // in-chunk terms then fit one record, trsv_blk_pro)
    std::vector<int> cs;  // chunk starts, then n
    {
        int c0 = 0;
        cs.push_back(0);
        for (int p = 1; p < n; p++) {
            bool cut = p - c0 == CH;
            if (!cut) {
                const int r = order[(size_t)p];
                int m = 0;
                for (int o = dep_begin(r); o < dep_end(r); o++) m += pos[(size_t)dep_src(o)] >= c0;
                cut = m > rsp::kBlkLongCap;
            }
            if (cut) {
                c0 = p;
                cs.push_back(p);
            }
        }
        cs.push_back(n);
    }
    // ---- blocks and patterns: chunk by chunk (in parallel), greedy inside
    const int nch = (int)cs.size() - 1;
    std::vector<ChunkPlan> cp((size_t)nch);
    hvec<int> nx((size_t)n), lblk((size_t)n);
    hvec<long long> lpo((size_t)n);  // chunk-local pattern offsets
    parallel_for(nch, 1, [&](long long g0, long long g1) {
        std::vector<int> stamp((size_t)n, -1), xs, ys;
        int tag = 0;
        for (long long g = g0; g < g1; g++) {
            const int c0 = cs[(size_t)g], c1 = cs[(size_t)g + 1];
            ChunkPlan &C = cp[(size_t)g];
            std::vector<int> &pool = C.pool;
            pool.reserve((size_t)(c1 - c0) * 12);
            int b = 0, bsize = 0, bst = c0, near = 0;
            // the candidate pattern of p in a block starting at s (s == p: alone)
            auto cand = [&](int p, int r, int s) {
                const int lo = std::max(c0, s - NW);
                xs.clear();
                ys.clear();
                near = 0;
                ++tag;
                xs.push_back(p);
                stamp[(size_t)p] = tag;
                for (int o = dep_begin(r); o < dep_end(r); o++) {
                    const int q = pos[(size_t)dep_src(o)];
                    if (q >= s) {
                        const long long k0 = lpo[(size_t)q], k1 = lpo[(size_t)q + 1];
                        for (long long k = k0; k < k1; k++) {
                            const int u = pool[(size_t)k];
                            if (stamp[(size_t)u] == tag) continue;
                            stamp[(size_t)u] = tag;
                            (k - k0 < nx[(size_t)q] ? xs : ys).push_back(u);
                        }
                    } else if (stamp[(size_t)q] != tag) {
                        stamp[(size_t)q] = tag;
                        ys.push_back(q);
                    }
                }
                for (int u : ys) near += u >= lo;
            };
            for (int p = c0; p < c1; p++) {
                const int r = order[(size_t)p];
                bool ok = false;
                lpo[(size_t)p] = (long long)pool.size();  // (the end of p - 1's pattern, read by cand)
                if (bsize > 0) {
                    cand(p, r, bst);
                    ok = bsize < BS && (int)ys.size() <= YMAX && near <= NMAX;
                    if (!ok) {
                        C.bstart.push_back(bst);
                        C.islong.push_back(0);
                        b++;
                        bsize = 0;
                    }
                }
                if (!ok) cand(p, r, p);
                std::sort(xs.begin(), xs.end());
                std::sort(ys.begin(), ys.end());
                nx[(size_t)p] = (int)xs.size();
                pool.insert(pool.end(), xs.begin(), xs.end());
                pool.insert(pool.end(), ys.begin(), ys.end());
                lblk[(size_t)p] = b;
                if (bsize == 0) bst = p;
                bsize++;
                if (!ok && ((int)ys.size() > YMAX || near > NMAX)) {  // a long row: a block of its own
                    C.bstart.push_back(bst);
                    C.islong.push_back(1);
                    b++;
                    bsize = 0;
                }
            }
            if (bsize > 0) {
                C.bstart.push_back(bst);
                C.islong.push_back(0);
            }
        }
    });
    // global numbering: block and entry offsets of each chunk
    std::vector<int> cb((size_t)nch + 1, 0);
    std::vector<long long> ce((size_t)nch + 1, 0);
    for (int g = 0; g < nch; g++) {
        cb[(size_t)g + 1] = cb[(size_t)g] + (int)cp[(size_t)g].bstart.size();
        ce[(size_t)g + 1] = ce[(size_t)g] + (long long)cp[(size_t)g].pool.size();
    }
    const int nb = cb[(size_t)nch];
    if (ce[(size_t)nch] >= INT_MAX - 1) return false;  // int entry offsets
    const int E = (int)ce[(size_t)nch];
    bp.nb = nb;
    hvec<int> pool((size_t)E), blk((size_t)n);
    hvec<long long> po((size_t)n + 1);
    std::vector<int> bstart((size_t)nb + 1);
    std::vector<char> islong((size_t)nb);
    bp.segs.resize((size_t)nch);
    parallel_for(nch, 1, [&](long long g0, long long g1) {
        for (long long g = g0; g < g1; g++) {
            const int c0 = cs[(size_t)g], c1 = cs[(size_t)g + 1];
            const ChunkPlan &C = cp[(size_t)g];
            std::copy(C.pool.begin(), C.pool.end(), pool.begin() + ce[(size_t)g]);
            for (int p = c0; p < c1; p++) {
                po[(size_t)p] = ce[(size_t)g] + lpo[(size_t)p];
                blk[(size_t)p] = cb[(size_t)g] + lblk[(size_t)p];
            }
            for (size_t k = 0; k < C.bstart.size(); k++) {
                bstart[(size_t)cb[(size_t)g] + k] = C.bstart[k];
                islong[(size_t)cb[(size_t)g] + k] = C.islong[k];
            }
            bp.segs[(size_t)g] = {cb[(size_t)g], cb[(size_t)g + 1], c0, c1};
        }
    });
    po[(size_t)n] = E;
    bstart[(size_t)nb] = n;
    cp.clear();
    const double t_greedy = ms();

    // ---- each row's far / near split; each block's far wait and near width
    bp.rows.resize((size_t)n);
    bp.ref.resize((size_t)E + 1);
    bp.ref[(size_t)E] = 0;  // (a pad: loaders read one entry past an empty list)
    bp.desc.assign((size_t)nb, rsp::BlkDesc{});
    parallel_for(nb, 256, [&](long long q0, long long q1) {
        for (long long q = q0; q < q1; q++) {
            const int p0 = bstart[(size_t)q], p1 = bstart[(size_t)q + 1];
            const int c0 = *(std::upper_bound(cs.begin(), cs.end(), p0) - 1), thr = std::max(c0, p0 - NW);
            int kn = 0;
            for (int p = p0; p < p1; p++) {
                const long long k0 = po[(size_t)p], kx = k0 + nx[(size_t)p], k1 = po[(size_t)p + 1];
                const long long kf = std::lower_bound(pool.begin() + kx, pool.begin() + k1, thr) - pool.begin();
                bp.rows[(size_t)p] = {(int)k0, nx[(size_t)p], (int)(k1 - kx), (int)(kf - kx)};
                kn = std::max(kn, (int)(k1 - kf));
                for (long long k = k0; k < kx; k++) bp.ref[(size_t)k] = order[(size_t)pool[(size_t)k]];
                for (long long k = kx; k < k1; k++) bp.ref[(size_t)k] = pool[(size_t)k];
            }
            rsp::BlkDesc &d = bp.desc[(size_t)q];
            d.p0 = p0;
            d.np = p1 - p0;
            d.kind = islong[(size_t)q] ? 1 : 0;
            d.eoff = (int)po[(size_t)p0];
            d.ne = (int)(po[(size_t)p1] - po[(size_t)p0]);
            // a long row: its in-chunk terms in rounds of 64 (trsv_blk_pro)
            d.kn = islong[(size_t)q] ? (kn + 63) / 64 : kn;
        }
    });
    const double t_rows = ms();

    // ---- coefficient recipes, in intra-block level order (two passes over
    // the blocks in parallel: counts, then the arrays at their offsets)
    hvec<int> ilev((size_t)n), nitem((size_t)nb), ndep((size_t)nb);
    parallel_for(nb, 64, [&](long long q0, long long q1) {
        for (long long q = q0; q < q1; q++) {
            rsp::BlkDesc &d = bp.desc[(size_t)q];
            int nd = 0, ni = 0, maxl = 0;
            for (int p = d.p0; p < d.p0 + d.np; p++) {
                const int r = order[(size_t)p];
                int lev = 0;
                for (int o = dep_begin(r); o < dep_end(r); o++) {
                    nd++;
                    const int s = pos[(size_t)dep_src(o)];
                    if (s >= d.p0) {
                        lev = std::max(lev, ilev[(size_t)s] + 1);
                        ni += (int)(po[(size_t)s + 1] - po[(size_t)s]);
                    } else {
                        ni++;
                    }
                }
                ilev[(size_t)p] = lev;
                maxl = std::max(maxl, lev);
            }
            d.nd = nd;
            d.nlev = maxl + 1;
            ndep[(size_t)q] = nd;
            nitem[(size_t)q] = ni;
        }
    });
    std::vector<long long> roff((size_t)nb + 1, 0);
    long long dsum = 0, lsum = 0, osum = 0;
    for (int q = 0; q < nb; q++) {
        rsp::BlkDesc &d = bp.desc[(size_t)q];
        d.doff = (int)dsum;
        d.loff = (int)lsum;
        d.ovf = 0;
        if (d.kind && d.kn > rsp::kBlkNear) {  // record overflow: rounds past kBlkNear
            d.ovf = (int)osum;
            osum += 64LL * (d.kn - rsp::kBlkNear);
        }
        dsum += ndep[(size_t)q];
        lsum += d.nlev + 1;
        roff[(size_t)q + 1] = roff[(size_t)q] + nitem[(size_t)q];
        if (!d.kind) {
            if (d.nd >= 65536 || d.ne >= 65535) return false;  // (the caps keep them far below)
            bp.lds_elems = std::max(bp.lds_elems, d.nd + 1 + d.ne);
            // eord + rptr (ne + 1) + recipe items + level bounds (nlev + 1)
            const long long w = 2LL * d.ne + 1 + nitem[(size_t)q] + d.nlev + 1;
            if (w > (1 << 20)) return false;
            bp.lds_words = std::max(bp.lds_words, (int)w);
        }
    }
    if (dsum >= INT_MAX || roff[(size_t)nb] >= INT_MAX || lsum >= INT_MAX || osum >= INT_MAX) return false;
    bp.novf = osum;
    bp.vpos.resize((size_t)std::max<long long>(dsum, 1));
    bp.eord.resize((size_t)E);
    bp.rptr.resize((size_t)E + 1);
    bp.rit.resize((size_t)std::max<long long>(roff[(size_t)nb], 1));
    bp.lptr.resize((size_t)lsum);
    bp.rptr[(size_t)E] = (int)roff[(size_t)nb];
    parallel_for(nb, 64, [&](long long q0, long long q1) {
        std::vector<int> where((size_t)n, -1), cnt, first;
        std::vector<std::pair<int, unsigned>> items;
        std::vector<unsigned> sorted;
        for (long long q = q0; q < q1; q++) {
            const rsp::BlkDesc &d = bp.desc[(size_t)q];
            const int p0 = d.p0, p1 = d.p0 + d.np;
            const bool lng = d.kind != 0;
            items.clear();
            int dd = 0;
            for (int p = p0; p < p1; p++) {
                const int r = order[(size_t)p];
                const long long k0 = po[(size_t)p], k1 = po[(size_t)p + 1];
                const int base = (int)(k0 - d.eoff);
                for (long long k = k0; k < k1; k++) where[(size_t)pool[(size_t)k]] = (int)(k - k0);
                for (int o = dep_begin(r); o < dep_end(r); o++, dd++) {
                    bp.vpos[(size_t)d.doff + dd] = dep_val(o);
                    const int s = pos[(size_t)dep_src(o)];
                    if (s >= p0) {  // in the block (never for a long row)
                        for (long long k = po[(size_t)s]; k < po[(size_t)s + 1]; k++)
                            items.push_back({base + where[(size_t)pool[(size_t)k]],
                                             ((unsigned)dd << 16) | (unsigned)(1 + (k - d.eoff))});
                    } else {
                        items.push_back({base + where[(size_t)s], lng ? (unsigned)dd : ((unsigned)dd << 16)});
                    }
                }
                for (long long k = k0; k < k1; k++) where[(size_t)pool[(size_t)k]] = -1;
            }
            // each entry's items in dependency order (stable by entry)
            cnt.assign((size_t)d.ne + 1, 0);
            for (const auto &it : items) cnt[(size_t)it.first + 1]++;
            for (int e = 0; e < d.ne; e++) cnt[(size_t)e + 1] += cnt[(size_t)e];
            first.assign(cnt.begin(), cnt.end());
            sorted.resize(items.size());
            for (const auto &it : items) sorted[(size_t)cnt[(size_t)it.first]++] = it.second;
            // slots by intra-block level, then position, then entry
            long long slot = d.eoff, ro = roff[(size_t)q];
            for (int l = 0; l < d.nlev; l++) {
                bp.lptr[(size_t)d.loff + l] = (int)slot;
                for (int p = p0; p < p1; p++) {
                    if (ilev[(size_t)p] != l) continue;
                    const int base = (int)(po[(size_t)p] - d.eoff), m = (int)(po[(size_t)p + 1] - po[(size_t)p]);
                    for (int t = 0; t < m; t++, slot++) {
                        const int e = base + t;
                        bp.eord[(size_t)slot] = (unsigned)e | (t == nx[(size_t)p] - 1 ? 0x80000000u : 0u);
                        bp.rptr[(size_t)slot] = (int)ro;
                        for (int k = first[(size_t)e]; k < first[(size_t)e + 1]; k++)
                            bp.rit[(size_t)ro++] = sorted[(size_t)k];
                    }
                }
            }
            bp.lptr[(size_t)d.loff + d.nlev] = (int)slot;
        }
    });
    int nlong = 0;
    for (char c : islong) nlong += c;
    bp.nlong = nlong;
    bp.entries = E;
    if (env_int("RSP_ILU_BLK_STATS", 0)) {  // diagnostics
        long long near = 0, far = 0, x = 0, kn = 0;
        for (const rsp::BlkRow &r : bp.rows) {
            x += r.nx;
            far += r.nfar;
            near += r.ny - r.nfar;
        }
        for (const rsp::BlkDesc &d : bp.desc) kn += d.kn;
        long long prev = 0, bprev = 0;  // y terms of earlier segments; blocks with any
        for (const rsp::BlkSeg &sg : bp.segs)
            for (int q = sg.b0; q < sg.b1; q++) {
                long long c = 0;
                for (int p = bp.desc[(size_t)q].p0; p < bp.desc[(size_t)q].p0 + bp.desc[(size_t)q].np; p++)
                    for (int k = bp.rows[(size_t)p].off + bp.rows[(size_t)p].nx;
                         k < bp.rows[(size_t)p].off + bp.rows[(size_t)p].nx + bp.rows[(size_t)p].ny; k++)
                        c += bp.ref[(size_t)k] < sg.p0;
                prev += c;
                bprev += c > 0;
            }
        fprintf(stderr, "plan_blocks kind=%d: y terms of earlier segments %lld (%.2f/row), blocks with any %lld of %d\n",
                kind, prev, (double)prev / n, bprev, nb);
        fprintf(stderr,
                "plan_blocks kind=%d n=%d levels=%d blocks=%d long=%d segments=%d entries=%d x/row=%.2f "
                "far/row=%.2f near/row=%.2f kn/block=%.2f lds_elems=%d deps=%zu recipes=%zu %.1f ms "
                "(greedy %.1f, rows %.1f)\n",
                kind, n, nlev, nb, nlong, (int)bp.segs.size(), E, (double)x / n, (double)far / n, (double)near / n,
                (double)kn / std::max(nb, 1), bp.lds_elems, bp.vpos.size(), bp.rit.size(), ms(), t_greedy, t_rows);
    }
    return true;
}

}  // namespace rsp_an
