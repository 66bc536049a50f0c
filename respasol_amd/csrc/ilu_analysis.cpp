// ilu_analysis.cpp — host half of the ILU(0) analysis (see ilu_analysis.h).
// Replaces the dependency analysis inside cusparse?csrilu02_analysis and
// cusparse?csrsv2_analysis (GPU/ilu0.cu:196-252). No HIP calls here.

#include "ilu_analysis.h"

#include <limits.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <thread>

namespace rsp_an {

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void Phases::start() {
    t_last = now_ms();
    next = 0;
}

void Phases::mark(const char *what) {
    const double t = now_ms();
    if (print) fprintf(stderr, "rsp_ilu0_analysis n=%d %-14s %8.2f ms\n", n, what, t - t_last);
    if (ms && next < kPhases) ms[next] = t - t_last;
    next++;
    t_last = t;
}

// rows grouped by level (stable: ascending row within a level)
static void group_levels(const std::vector<int> &lev, int nlev, std::vector<int> &ptr,
                         std::vector<int> &rows) {
    ptr.assign((size_t)nlev + 1, 0);
    for (int v : lev) ptr[(size_t)v + 1]++;
    for (int l = 0; l < nlev; l++) ptr[(size_t)l + 1] += ptr[(size_t)l];
    std::vector<int> fill(ptr.begin(), ptr.end() - 1);
    rows.assign(lev.size(), 0);
    for (size_t i = 0; i < lev.size(); i++) rows[(size_t)fill[(size_t)lev[i]]++] = (int)i;
}




// fma-chain batch for a mean chain length of total / count
static int chain_batch(long long total, long long count) {
    const double mean = count > 0 ? (double)total / (double)count : 0.0;
    return mean <= 2.5 ? 2 : (mean <= 5.0 ? 4 : 8);
}


// Solve plan of one DAG (see LevelPlan): tasks in level order over flat
// terms (term k of row i: matrix value at tpos[k], y of column col_of(k)),
// segments (a level is thin if it has <= thin_rows rows and its terms fit one
// chunk), the LDS-staged chunks of every thin run (<= kChunkRows rows and
// <= kChunkTerms terms each), and the y source of every term of a thin run:
// the LDS window slot (run index mod kYWin) if the column was produced earlier
// in the run and no later row of the run can have reused that slot by the end
// of the consumer's level, else the column (global y, or its value staged at
// the chunk start — the producer is then in an earlier chunk or before the
// run, so its store is visible after the chunk's full barrier).

// row_terms(i, emit) calls emit(tpos, col) for the terms of row i in order
template <typename RowTerms>
static void build_solve_plan(int n, const std::vector<int> &ptr, const std::vector<int> &rows,
                             int thin_rows, int group, const std::vector<int> &diag,
                             RowTerms row_terms, SolvePlan &sp) {
    const int nlev = (int)ptr.size() - 1;
    std::vector<int> order(rows);
    // segments: runs of thin levels / fat levels. A thin level's rows have
    // their terms padded to whole groups of `group` (at least one group):
    // pads are (position -1, source kPadSrc), i.e. a zero value times the zero
    // slot of the LDS y buffer — an exact no-op fma — so the thin kernel reads
    // a row as whole groups with vector loads and no length tests.
    // terms per row, counted once
    std::vector<int> nt_row((size_t)n, 0);
    for (int i = 0; i < n; i++) {
        int cnt = 0;
        row_terms(i, [&](int, int) { cnt++; });
        nt_row[(size_t)i] = cnt;
    }
    auto nterms = [&](int i) { return nt_row[(size_t)i]; };
    auto padded = [&](int cnt) { return std::max(1, (cnt + group - 1) / group) * group; };
    std::vector<int> lpad((size_t)std::max(nlev, 1), 0);
    for (int l = 0; l < nlev; l++)
        for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++) lpad[(size_t)l] += padded(nterms(order[(size_t)x]));
    sp.segs.clear();
    for (int l = 0; l < nlev; l++) {
        const int cnt = ptr[(size_t)l + 1] - ptr[(size_t)l];
        const int thin = (cnt <= thin_rows && cnt <= rsp::kThinThreads && cnt <= rsp::kChunkRows &&
                          lpad[(size_t)l] <= rsp::kChunkTerms) ? 1 : 0;
        if (!sp.segs.empty() && sp.segs.back().thin == thin && sp.segs.back().le == l)
            sp.segs.back().le = l + 1;
        else
            sp.segs.push_back({l, l + 1, thin, 0, 0, 0});
    }
    std::vector<char> thin_lev((size_t)std::max(nlev, 1), 0);
    for (const rsp::LevelSeg &sg : sp.segs)
        for (int l = sg.lb; l < sg.le; l++) thin_lev[(size_t)l] = (char)sg.thin;
    // within each level: short rows first (a thread each), longer rows after
    // them (a wave each). Short: <= kLongTerms terms in a thin run (LDS
    // operands); <= kFatLongTerms in a fat level, where a thread pays one
    // global round trip per batch of terms and a wave one per 64 terms.
    // A fat level's rows of > kHubTerms terms come last, a workgroup each.
    const int fat_long = env_int("RSP_ILU_FAT_LONG", rsp::kFatLongTerms);
    const int hub = env_int("RSP_ILU_HUB", rsp::kHubTerms);
    sp.nshort.assign((size_t)std::max(nlev, 1), 0);
    sp.nwave.assign((size_t)std::max(nlev, 1), 0);
    for (int l = 0; l < nlev; l++) {
        const int lim = thin_lev[(size_t)l] ? rsp::kLongTerms : fat_long;
        auto b = order.begin() + ptr[(size_t)l], e = order.begin() + ptr[(size_t)l + 1];
        auto mid = std::stable_partition(b, e, [&](int i) { return nterms(i) <= lim; });
        sp.nshort[(size_t)l] = (int)(mid - b);
        auto hb = thin_lev[(size_t)l] ? e : std::stable_partition(mid, e, [&](int i) { return nterms(i) <= hub; });
        sp.nwave[(size_t)l] = (int)(hb - b);
    }
    std::vector<int> col;
    sp.tasks.assign(std::max<size_t>(rows.size(), 1), rsp::RowTask{0, 0, 0, -1});
    sp.tpos.clear();
    {  // flat terms incl. pads: reserve once
        size_t total = 0;
        for (int l = 0; l < nlev; l++) total += (size_t)lpad[(size_t)l];
        total += (size_t)rows.size() * rsp::kFatLongTerms;
        sp.tpos.reserve(total);
        col.reserve(total);
    }
    // fat levels: each short row owns kFatLongTerms flat terms (its terms,
    // then pads), so trsv_level finds a row's terms at sbase + r * 8 without
    // reading its task first; t1 stays at the row's last real term
    const bool pad_fat = fat_long == rsp::kFatLongTerms && env_int("RSP_ILU_FAT_PAD", 1) != 0;
    sp.sbase.assign((size_t)std::max(nlev, 1), -1);
    for (int l = 0; l < nlev; l++) {
        const bool padl = pad_fat && !thin_lev[(size_t)l] && sp.nshort[(size_t)l] > 0;
        if (padl) sp.sbase[(size_t)l] = (int)sp.tpos.size();
        for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++) {
            const int i = order[(size_t)x];
            rsp::RowTask &t = sp.tasks[(size_t)x];
            t.i = i;
            t.t0 = (int)sp.tpos.size();
            row_terms(i, [&](int tp, int c) {
                sp.tpos.push_back(tp);
                col.push_back(c);
            });
            if (thin_lev[(size_t)l])
                while ((int)sp.tpos.size() - t.t0 < padded((int)sp.tpos.size() - t.t0)) {
                    sp.tpos.push_back(-1);
                    col.push_back(-1);
                }
            t.t1 = (int)sp.tpos.size();
            if (padl && x - ptr[(size_t)l] < sp.nshort[(size_t)l])
                while ((int)sp.tpos.size() - t.t0 < rsp::kFatLongTerms) {
                    sp.tpos.push_back(-1);
                    col.push_back(-1);
                }
            t.d = diag.empty() ? -1 : diag[(size_t)i];
        }
    }
    // flow segments: fat segments of two or more levels run as one persistent
    // launch (trsv_flow) over work items in level order — a level's short rows
    // in groups of 64 (a lane each), then its wave and hub rows (a wave each).
    // Short rows must fit one batch of kFatLongTerms terms (RSP_ILU_FAT_LONG).
    sp.fitems.clear();
    const int gate_d = env_int("RSP_ILU_FLOW_GATE", 3);  // levels between an item and its gate (0: none)
    if (fat_long <= rsp::kFatLongTerms && env_int("RSP_ILU_FLOW_PLAN", 1) != 0)
        for (rsp::LevelSeg &sg : sp.segs) {
            if (sg.thin || sg.le - sg.lb < 2) continue;
            sg.c0 = (int)sp.fitems.size();
            for (int l = sg.lb; l < sg.le; l++) {
                const int p0 = ptr[(size_t)l], cnt = ptr[(size_t)l + 1] - p0, ns = sp.nshort[(size_t)l];
                const int sb = sp.sbase[(size_t)l];
                // gate: the last row of level l - gate_d when it is in this segment
                const int lg = l - gate_d;
                const int gate = gate_d > 0 && lg >= sg.lb && ptr[(size_t)lg + 1] > ptr[(size_t)lg]
                                     ? order[(size_t)ptr[(size_t)lg + 1] - 1] : -1;
                for (int r = 0; r < ns; r += 64)
                    sp.fitems.push_back({p0 + r, std::min(64, ns - r), sb >= 0 ? sb + r * rsp::kFatLongTerms : -1, gate});
                for (int r = ns; r < cnt; r++) sp.fitems.push_back({p0 + r, 0, -1, gate});
            }
            sg.c1 = (int)sp.fitems.size();
        }
    if (env_int("RSP_ILU_PLANSTATS", 0)) {  // diagnostics: the segment structure of this DAG
        int nthin = 0, nfat = 0, nflow = 0, lthin = 0, lfat = 0, lflow = 0;
        for (const rsp::LevelSeg &sg : sp.segs) {
            const int nl = sg.le - sg.lb;
            if (sg.thin) nthin++, lthin += nl;
            else if (sg.c1 > sg.c0) nflow++, lflow += nl;
            else nfat++, lfat += nl;
        }
        fprintf(stderr, "rsp_ilu0 plan n=%d levels=%d group=%d thin %d segs / %d levels, fat %d / %d, flow %d / %d (%zu items)\n",
                n, nlev, group, nthin, lthin, nfat, lfat, nflow, lflow, sp.fitems.size());
    }
    if (sp.fitems.empty()) sp.fitems.push_back({0, 0, -1, -1});  // keep the device array non-empty
    std::vector<int> lterms((size_t)std::max(nlev, 1), 0);
    for (int l = 0; l < nlev; l++)
        if (ptr[(size_t)l + 1] > ptr[(size_t)l])
            lterms[(size_t)l] = sp.tasks[(size_t)ptr[(size_t)l + 1] - 1].t1 - sp.tasks[(size_t)ptr[(size_t)l]].t0;
    sp.src = col;
    for (size_t k = 0; k < col.size(); k++)
        if (col[k] < 0) sp.src[k] = rsp::kPadSrc;
    for (rsp::LevelSeg &sg : sp.segs)
        if (sg.thin) sg.nth = rsp::kThinThreads;
    // chunks of the thin runs + term sources
    std::vector<int> slot_of((size_t)n, -1);
    for (size_t x = 0; x < order.size(); x++) slot_of[(size_t)order[x]] = (int)x;
    sp.chunks.clear();
    for (rsp::LevelSeg &sg : sp.segs) {
        if (!sg.thin) continue;
        sg.c0 = (int)sp.chunks.size();
        int crow = 0, cterm = 0;
        for (int l = sg.lb; l < sg.le; l++) {
            const int cnt = ptr[(size_t)l + 1] - ptr[(size_t)l];
            if (sp.chunks.size() == (size_t)sg.c0 || crow + cnt > rsp::kChunkRows ||
                cterm + lterms[(size_t)l] > rsp::kChunkTerms) {
                sp.chunks.push_back({l, l + 1, 0, 0, 0, 0, 0, 0});
                crow = 0;
                cterm = 0;
            } else {
                sp.chunks.back().l1 = l + 1;
            }
            crow += cnt;
            cterm += lterms[(size_t)l];
        }
        sg.c1 = (int)sp.chunks.size();
        const int base = ptr[(size_t)sg.lb];
        for (int l = sg.lb; l < sg.le; l++) {
            const int r_end = ptr[(size_t)l + 1] - base;
            for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++)
                for (int k = sp.tasks[(size_t)x].t0; k < sp.tasks[(size_t)x].t1; k++) {
                    if (col[(size_t)k] < 0) continue;  // pad
                    const int sj = slot_of[(size_t)col[(size_t)k]];
                    if (sj < base || sj >= ptr[(size_t)l]) continue;  // before the run
                    const int rj = sj - base;
                    if (r_end - rj <= rsp::kYWin) sp.src[(size_t)k] = -((rj & (rsp::kYWin - 1)) + 1);
                }
        }
    }
    if (sp.tpos.empty()) {  // keep the device arrays non-empty
        sp.tpos.push_back(0);
        sp.src.push_back(0);
    }
    // per chunk: slot and term ranges, the static row records (first group,
    // y window slot), each term's y index in the LDS y buffer (window slot,
    // the zero slot for pads, or its staged slot) and the staged terms
    sp.trow.assign(std::max<size_t>(rows.size(), 1), rsp::ThinRowPlan{0, 0, 0, -1});
    sp.sid.assign(sp.tpos.size(), rsp::kYWin);
    sp.stg.clear();
    for (const rsp::LevelSeg &sg : sp.segs) {
        if (!sg.thin) continue;
        const int base = ptr[(size_t)sg.lb];
        for (int c = sg.c0; c < sg.c1; c++) {
            rsp::LevelChunk &ch = sp.chunks[(size_t)c];
            ch.x0 = ptr[(size_t)ch.l0];
            ch.x1 = ptr[(size_t)ch.l1];
            ch.k0 = ch.x1 > ch.x0 ? sp.tasks[(size_t)ch.x0].t0 : 0;
            ch.k1 = ch.x1 > ch.x0 ? sp.tasks[(size_t)ch.x1 - 1].t1 : 0;
            ch.st0 = (int)sp.stg.size();
            for (int x = ch.x0; x < ch.x1; x++) {
                const rsp::RowTask &t = sp.tasks[(size_t)x];
                sp.trow[(size_t)x] = {(t.t0 - ch.k0) / group | ((t.t1 - t.t0) / group) << 16,
                                      (x - base) & (rsp::kYWin - 1), t.i, t.d};
                for (int k = t.t0; k < t.t1; k++) {
                    const int sc = sp.src[(size_t)k];
                    if (sc < 0) {
                        sp.sid[(size_t)k] = -sc - 1;  // window slot, or the zero slot for a pad
                    } else {
                        sp.sid[(size_t)k] = rsp::kYWin + 1 + (k - ch.k0);
                        sp.stg.push_back({k - ch.k0, sc});
                    }
                }
            }
            ch.st1 = (int)sp.stg.size();
        }
    }
    if (sp.stg.empty()) sp.stg.push_back({0, 0});
    if (sp.chunks.empty()) sp.chunks.push_back({0, 0, 0, 0, 0, 0, 0, 0});
}



// Factor plan of the L DAG (see IluArgs): segments (a level is thin if it
// has <= thin_rows rows and its positions / update pairs fit one chunk), the
// LDS-staged chunks of every thin run, and per chunk its items (the positions
// of its rows: lower ones in intra-row stage order, then upper ones) and update
// pairs with their sources: a chunk-local item when the producing row is in
// the chunk, else the position (its final value is staged at the chunk start).
// Factor plan of the L DAG (see IluArgs): segments (fat levels: one launch
// each; thin levels: one single-workgroup launch per run) and, for the thin
// runs, ROUNDS: a level's positions ("items") grouped so that a round's items
// are independent — a lower item of intra-row stage s is in round s, a row's
// upper items (diagonal included) in the round after its last lower stage.
// Every item depends only on earlier rounds (its own row's l_ik) and earlier
// levels (u_kj, u_kk). The run's items, in round order, are cut into LDS
// chunks (<= kRndItems items, kRndPairs update pairs, kRndStaged staged
// values, kRndRounds rounds; a round may be split between chunks). An item's
// operands are indices into the kernel's LDS value buffer by class: its own
// chunk's slots, the previous chunk's slots (kept in the other LDS buffer),
// values staged from vals at the chunk start (producers two or more chunks
// back, or before the run), or the zero slot (a missing u_kk).

static void build_factor_plan(int n, const std::vector<int> &rp, const std::vector<int> &ci,
                              const std::vector<int> &dpos, const std::vector<int> &hasdiag,
                              const IluSymbolic &sym, const std::vector<int> &ptr,
                              const std::vector<int> &rows, int thin_rows, FacPlan &fp) {
    const int nlev = (int)ptr.size() - 1;
    const int K = rsp::kRndItems, S = rsp::kRndStaged, kZero = 2 * rsp::kRndItems + rsp::kRndStaged;
    const int thin_items = env_int("RSP_ILU_THIN_FACTOR_ITEMS", rsp::kRndLevelItems);
    auto npairs = [&](int p) { return sym.upd_ptr[(size_t)p + 1] - sym.upd_ptr[(size_t)p]; };
    fp.segs.clear();
    for (int l = 0; l < nlev; l++) {
        const int cnt = ptr[(size_t)l + 1] - ptr[(size_t)l];
        long long items = 0;
        int maxp = 0;
        for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++) {
            const int i = rows[(size_t)x];
            items += rp[(size_t)i + 1] - rp[(size_t)i];
            for (int p = rp[(size_t)i]; p < rp[(size_t)i + 1]; p++) maxp = std::max(maxp, npairs(p));
        }
        const int thin = (cnt <= thin_rows && items <= thin_items && maxp <= rsp::kRndItemPairs) ? 1 : 0;
        if (!fp.segs.empty() && fp.segs.back().thin == thin && fp.segs.back().le == l)
            fp.segs.back().le = l + 1;
        else
            fp.segs.push_back({l, l + 1, thin, 0, 0, rsp::kThinThreads});
    }
    fp.chunks.clear();
    fp.items.clear();
    fp.pairs.clear();
    fp.staged.clear();
    fp.rounds.clear();
    // where each position was placed: chunk and slot (-1: not in this run yet)
    std::vector<int> pchunk((size_t)rp[(size_t)n], -1), pslot((size_t)rp[(size_t)n], 0);
    std::vector<int> stg_of((size_t)rp[(size_t)n], -1);  // staged slot in the current chunk
    std::vector<int> stg_list;                            // positions staged in the current chunk
    struct RItem {
        int round, pos, row;
    };
    std::vector<RItem> ritems, rsorted;  // a level's items
    std::vector<int> rcount;
    for (rsp::LevelSeg &sg : fp.segs) {
        if (!sg.thin) continue;
        sg.c0 = (int)fp.chunks.size();
        rsp::RndChunk ch{};
        int c = -1;  // current chunk id
        auto open_chunk = [&]() {
            for (int q : stg_list) stg_of[(size_t)q] = -1;
            stg_list.clear();
            c = (int)fp.chunks.size();
            ch = rsp::RndChunk{(int)fp.items.size(), (int)fp.items.size(), (int)fp.pairs.size(),
                               (int)fp.pairs.size(), (int)fp.staged.size(), (int)fp.staged.size(),
                               (int)fp.rounds.size(), (int)fp.rounds.size()};
            fp.chunks.push_back(ch);
        };
        auto close_chunk = [&]() {
            ch.i1 = (int)fp.items.size();
            ch.p1 = (int)fp.pairs.size();
            ch.s1 = (int)fp.staged.size();
            ch.r1 = (int)fp.rounds.size();
            fp.chunks[(size_t)c] = ch;
        };
        // operand class index of position q for an item of chunk c (new staged
        // values are appended to `fresh`; the caller commits or rolls back)
        auto ref = [&](int q, std::vector<int> &fresh) {
            const int qc = pchunk[(size_t)q];
            if (qc == c) return pslot[(size_t)q];
            if (qc >= 0 && qc == c - 1) return K + pslot[(size_t)q];
            if (stg_of[(size_t)q] >= 0) return 2 * K + stg_of[(size_t)q];
            for (size_t f = 0; f < fresh.size(); f++)
                if (fresh[f] == q) return 2 * K + (int)(stg_list.size() + f);
            fresh.push_back(q);
            return 2 * K + (int)(stg_list.size() + fresh.size() - 1);
        };
        open_chunk();
        long long last_round_key = -1;  // (level, round) of the chunk's last round
        std::vector<int> fresh, ipairs;
        for (int l = sg.lb; l < sg.le; l++) {
            ritems.clear();
            for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++) {
                const int i = rows[(size_t)x], rs = rp[(size_t)i], di = dpos[(size_t)i];
                int nst = 0;
                for (int p = rs; p < di; p++) {
                    ritems.push_back({sym.stage[(size_t)p], p, i});
                    nst = std::max(nst, sym.stage[(size_t)p] + 1);
                }
                for (int p = di; p < rp[(size_t)i + 1]; p++) ritems.push_back({nst, p, i});
            }
            {  // stable counting sort by round
                int rmax = 0;
                for (const RItem &ri : ritems) rmax = std::max(rmax, ri.round);
                rcount.assign((size_t)rmax + 2, 0);
                for (const RItem &ri : ritems) rcount[(size_t)ri.round + 1]++;
                for (int r = 0; r <= rmax; r++) rcount[(size_t)r + 1] += rcount[(size_t)r];
                rsorted.resize(ritems.size());
                for (const RItem &ri : ritems) rsorted[(size_t)rcount[(size_t)ri.round]++] = ri;
                ritems.swap(rsorted);
            }
            for (const RItem &ri : ritems) {
                const int p = ri.pos, i = ri.row;
                const long long key = (long long)(l - sg.lb) * 1000000007LL + ri.round;
                const bool lower = p < dpos[(size_t)i];
                for (int attempt = 0; attempt < 2; attempt++) {
                    fresh.clear();
                    ipairs.clear();
                    for (int u = sym.upd_ptr[(size_t)p]; u < sym.upd_ptr[(size_t)p + 1]; u++) {
                        const int lc = ref(sym.upd_l[(size_t)u], fresh), uc = ref(sym.upd_u[(size_t)u], fresh);
                        ipairs.push_back(lc | uc << 16);
                    }
                    int d = -1;
                    if (lower) {
                        const int k = ci[(size_t)p];
                        d = hasdiag[(size_t)k] ? ref(dpos[(size_t)k], fresh) : kZero;
                    }
                    const int slot = (int)fp.items.size() - ch.i0;
                    const bool new_round = key != last_round_key;
                    const bool fits = slot < K && (int)(fp.pairs.size() - ch.p0 + ipairs.size()) <= rsp::kRndPairs &&
                                      (int)(stg_list.size() + fresh.size()) <= S &&
                                      (int)(fp.rounds.size() - ch.r0) + (new_round ? 1 : 0) <= rsp::kRndRounds;
                    if (!fits && attempt == 0 && slot > 0) {  // next chunk (references re-resolved there)
                        close_chunk();
                        open_chunk();
                        last_round_key = -1;
                        continue;
                    }
                    // commit the item
                    for (int q : fresh) {
                        stg_of[(size_t)q] = (int)stg_list.size();
                        stg_list.push_back(q);
                        fp.staged.push_back(q);
                    }
                    if (new_round) {
                        fp.rounds.push_back(slot);
                        last_round_key = key;
                    }
                    const int pstart = (int)fp.pairs.size() - ch.p0;
                    fp.pairs.insert(fp.pairs.end(), ipairs.begin(), ipairs.end());
                    const int zr = (!lower && p == dpos[(size_t)i] && hasdiag[(size_t)i]) ? i : -1;
                    fp.items.push_back({p, pstart | (int)ipairs.size() << 16, d, zr});
                    pchunk[(size_t)p] = c;
                    pslot[(size_t)p] = slot;
                    break;
                }
            }
        }
        close_chunk();
        sg.c1 = (int)fp.chunks.size();
        for (int x = ptr[(size_t)sg.lb]; x < ptr[(size_t)sg.le]; x++) {  // positions leave the run
            const int i = rows[(size_t)x];
            for (int p = rp[(size_t)i]; p < rp[(size_t)i + 1]; p++) pchunk[(size_t)p] = -1;
        }
        for (int q : stg_list) stg_of[(size_t)q] = -1;
        stg_list.clear();
    }
    if (fp.items.empty()) fp.items.push_back({0, 0, -1, -1});
    for (std::vector<int> *v : {&fp.pairs, &fp.staged, &fp.rounds})
        if (v->empty()) v->push_back(0);
    if (fp.chunks.empty()) fp.chunks.push_back(rsp::RndChunk{});
}


// Symbolic ILU(0): the update list of every position (see IluArgs) and the
// intra-row stages of the lower positions. Row i is scattered into a dense
// column -> position map, then each lower k (ascending) walks row k's upper
// part; a hit at column j appends (pos l_ik, pos u_kj) to position (i, j).

// Host worker threads for the analysis: OMP_NUM_THREADS (the box's share of
// its cores; the machine may have many more) or the hardware count, <= 64.
static int host_threads() {
    int t = env_int("OMP_NUM_THREADS", 0);
    if (t <= 0) t = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 64));
}

// f(r0, r1) over contiguous row blocks of [0, n) on host_threads() threads.
template <typename F>
static void parallel_rows(int n, F f) {
    const int nt = n < 8192 ? 1 : host_threads();
    if (nt == 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
        th.emplace_back(f, (int)((long long)n * t / nt), (int)((long long)n * (t + 1) / nt));
    for (std::thread &x : th) x.join();
}

static bool ilu_symbolic(int n, const std::vector<int> &rp, const std::vector<int> &ci,
                         const std::vector<int> &dpos, const std::vector<int> &hasdiag,
                         IluSymbolic &s) {
    const int nnz = rp[(size_t)n];
    std::vector<int> cnt((size_t)nnz, 0);
    // pass 1: counts (rows are independent: a row writes only its own
    // positions' counts; each worker scatters its rows into its own map)
    std::mutex mu;
    long long total = 0;
    parallel_rows(n, [&](int r0, int r1) {
        std::vector<int> map((size_t)n, -1);
        long long part = 0;
        for (int i = r0; i < r1; i++) {
            for (int p = rp[(size_t)i]; p < rp[(size_t)i + 1]; p++) map[(size_t)ci[(size_t)p]] = p;
            for (int p = rp[(size_t)i]; p < dpos[(size_t)i]; p++) {
                const int k = ci[(size_t)p];
                for (int q = dpos[(size_t)k] + hasdiag[(size_t)k]; q < rp[(size_t)k + 1]; q++) {
                    const int t = map[(size_t)ci[(size_t)q]];
                    if (t > p) {
                        cnt[(size_t)t]++;
                        part++;
                    }
                }
            }
            for (int p = rp[(size_t)i]; p < rp[(size_t)i + 1]; p++) map[(size_t)ci[(size_t)p]] = -1;
        }
        std::lock_guard<std::mutex> g(mu);
        total += part;
    });
    if (total > INT_MAX) return false;
    s.upd_ptr.assign((size_t)nnz + 1, 0);
    for (int p = 0; p < nnz; p++) s.upd_ptr[(size_t)p + 1] = s.upd_ptr[(size_t)p] + cnt[(size_t)p];
    s.upd_l.resize((size_t)total);
    s.upd_u.resize((size_t)total);
    // pass 2: fill (k ascending per target, since p ascends) + stages
    std::vector<int> &stage = s.stage;
    stage.assign((size_t)nnz, 0);
    s.lord.assign((size_t)nnz, 0);
    s.lend.assign((size_t)nnz, 0);
    parallel_rows(n, [&](int r0, int r1) {
        std::vector<int> map((size_t)n, -1), order;
        for (int i = r0; i < r1; i++) {
            const int rs = rp[(size_t)i], di = dpos[(size_t)i];
            for (int p = rs; p < rp[(size_t)i + 1]; p++) map[(size_t)ci[(size_t)p]] = p;
            for (int p = rs; p < rp[(size_t)i + 1]; p++) cnt[(size_t)p] = s.upd_ptr[(size_t)p];  // fill
            for (int p = rs; p < di; p++) {
                const int k = ci[(size_t)p];
                for (int q = dpos[(size_t)k] + hasdiag[(size_t)k]; q < rp[(size_t)k + 1]; q++) {
                    const int t = map[(size_t)ci[(size_t)q]];
                    if (t > p) {
                        const int u = cnt[(size_t)t]++;
                        s.upd_l[(size_t)u] = p;
                        s.upd_u[(size_t)u] = q;
                        if (t < di) stage[(size_t)t] = std::max(stage[(size_t)t], stage[(size_t)p] + 1);
                    }
                }
            }
            for (int p = rs; p < rp[(size_t)i + 1]; p++) map[(size_t)ci[(size_t)p]] = -1;
            // lower positions by (stage, column)
            order.assign((size_t)(di - rs), 0);
            for (int p = rs; p < di; p++) order[(size_t)(p - rs)] = p;
            std::stable_sort(order.begin(), order.end(),
                             [&](int a, int b) { return stage[(size_t)a] < stage[(size_t)b]; });
            for (int x = 0; x < di - rs; x++) s.lord[(size_t)(rs + x)] = order[(size_t)x];
            for (int x = di - rs - 1; x >= 0; x--) {
                const bool last = x == di - rs - 1 ||
                                  stage[(size_t)order[(size_t)x]] != stage[(size_t)order[(size_t)x + 1]];
                s.lend[(size_t)(rs + x)] = last ? rs + x + 1 : s.lend[(size_t)(rs + x + 1)];
            }
        }
    });
    return true;
}

// The symbolic factor of a few given rows on the host (the device analysis
// leaves its long rows here: a hub row's lower positions form a long serial
// chain that one GPU lane walks at global-memory latency, where the host
// walks it in cache). cnt != nullptr: update-list counts of the rows'
// positions; else the pairs at ptr, the stages, the stage order and the
// divisor positions — every value exactly as ilu_symbolic / plan_symbolic.
void symbolic_rows(const std::vector<int> &rows, int n, const int *rp, const int *ci, const int *dpos,
                   const int *hasdiag, int *cnt, const int *ptr, int *upd_l, int *upd_u, int *stage, int *lord,
                   int *lend, int *udiv) {
    if (rows.empty()) return;
    std::vector<int> map((size_t)n, -1), cur, order;
    for (int i : rows) {
        const int rs = rp[i], re = rp[i + 1], di = dpos[i];
        for (int p = rs; p < re; p++) map[(size_t)ci[p]] = p;
        if (cnt) {
            for (int p = rs; p < re; p++) cnt[p] = 0;
        } else {
            cur.assign(ptr + rs, ptr + re);
            for (int p = rs; p < re; p++) stage[p] = 0;
        }
        for (int p = rs; p < di; p++) {
            const int k = ci[p];
            for (int q = dpos[k] + hasdiag[k]; q < rp[k + 1]; q++) {
                const int t = map[(size_t)ci[q]];
                if (t > p) {
                    if (cnt) {
                        cnt[t]++;
                    } else {
                        const int u = cur[(size_t)(t - rs)]++;
                        upd_l[u] = p;
                        upd_u[u] = q;
                        if (t < di) stage[t] = std::max(stage[t], stage[p] + 1);
                    }
                }
            }
        }
        for (int p = rs; p < re; p++) map[(size_t)ci[p]] = -1;
        if (cnt) continue;
        order.resize((size_t)(di - rs));
        for (int p = rs; p < di; p++) order[(size_t)(p - rs)] = p;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return stage[a] < stage[b]; });
        for (int x = 0; x < di - rs; x++) lord[rs + x] = order[(size_t)x];
        for (int x = di - rs - 1; x >= 0; x--) {
            const bool last = x == di - rs - 1 || stage[order[(size_t)x]] != stage[order[(size_t)x + 1]];
            lend[rs + x] = last ? rs + x + 1 : lend[rs + x + 1];
        }
        for (int p = di; p < re; p++) lord[p] = lend[p] = 0;
        for (int p = rs; p < re; p++) {
            const int k = ci[p];
            udiv[p] = (p < di && hasdiag[k]) ? dpos[k] : -1;
        }
    }
}

// The U DAG (extension: the true L.U apply, rsp_trsv_upper): row i waits
// for every j > i with u_ij != 0.
void plan_u(const int *rp, const int *ci, IluHostPlan &hp) {
    const int n = hp.n;
    const std::vector<int> &dpos = hp.dpos, &hasdiag = hp.hasdiag;
    std::vector<int> lvu((size_t)n, 0);
    int nlu = n > 0 ? 1 : 0;
    for (int i = n - 1; i >= 0; i--) {
        int l = 0;
        for (int p = dpos[(size_t)i] + hasdiag[(size_t)i]; p < rp[(size_t)i + 1]; p++)
            l = std::max(l, lvu[(size_t)ci[(size_t)p]] + 1);
        lvu[(size_t)i] = l;
        nlu = std::max(nlu, l + 1);
    }
    group_levels(lvu, nlu, hp.U.ptr, hp.U.rows);
    long long nu = 0;
    for (int i = 0; i < n; i++) nu += rp[(size_t)i + 1] - dpos[(size_t)i] - hasdiag[(size_t)i];
    hp.U.batch = chain_batch(nu, n);
    hp.U.group = env_int("RSP_ILU_GROUP", hp.U.batch == 2 ? 2 : 4) == 2 ? 2 : 4;
    std::vector<int> udiag((size_t)n);
    for (int i = 0; i < n; i++) udiag[(size_t)i] = hasdiag[(size_t)i] ? dpos[(size_t)i] : -1;
    const int thin_solve = std::min(env_int("RSP_ILU_THIN_SOLVE", rsp::kThinSolveRows), rsp::kThinThreads);
    build_solve_plan(n, hp.U.ptr, hp.U.rows, thin_solve, hp.U.group, udiag, [&](int i, auto emit) {
        for (int p = dpos[(size_t)i] + hasdiag[(size_t)i]; p < rp[(size_t)i + 1]; p++) emit(p, ci[(size_t)p]);
    }, hp.U.sp);
    hp.U.planned = true;
}

rsp_status_t plan_validate(int n, const int *rpp, const int *cip, IluHostPlan &hp) {
    hp = IluHostPlan();
    hp.n = n;
    if (n < 0 || (n > 0 && !rpp)) return RSP_STATUS_INVALID_VALUE;
    if (n > 0 && rpp[0] != 0) return RSP_STATUS_INVALID_VALUE;
    for (int i = 0; i < n; i++)
        if (rpp[i + 1] < rpp[i]) return RSP_STATUS_INVALID_VALUE;
    const int nnz_s = n > 0 ? rpp[n] : 0;
    if (nnz_s > 0 && !cip) return RSP_STATUS_INVALID_VALUE;
    hp.nnz_s = nnz_s;
    const int *rp = rpp, *ci = cip;
    // columns in range, and each row strictly increasing (the reference loader
    // sorts rows, loadMatrixMarket.cpp:237-242; csrilu02 requires sorted,
    // duplicate-free rows): otherwise INVALID_VALUE, never a wrong factor
    bool bad = false;
    {
        std::mutex mu;
        parallel_rows(n, [&](int r0, int r1) {
            bool b = false;
            for (int i = r0; i < r1 && !b; i++)
                for (int p = rp[i]; p < rp[i + 1]; p++) {
                    const int c = ci[p];
                    if (c < 0 || c >= n || (p > rp[i] && c <= ci[p - 1])) {
                        b = true;
                        break;
                    }
                }
            if (b) {
                std::lock_guard<std::mutex> g(mu);
                bad = true;
            }
        });
    }
    if (bad) return RSP_STATUS_INVALID_VALUE;
    std::vector<int> &dpos = hp.dpos, &hasdiag = hp.hasdiag;
    dpos.assign((size_t)n, 0);
    hasdiag.assign((size_t)n, 0);
    parallel_rows(n, [&](int r0, int r1) {
        for (int i = r0; i < r1; i++) {
            const int *b = ci + rp[i], *e = ci + rp[i + 1];
            const int *p = std::lower_bound(b, e, i);
            dpos[(size_t)i] = (int)(p - ci);
            hasdiag[(size_t)i] = (p != e && *p == i) ? 1 : 0;
        }
    });
    for (int i = 0; i < n; i++)  // the first missing diagonal (cusparseXcsrilu02_zeroPivot)
        if (!hasdiag[(size_t)i]) {
            hp.structural_zero = i;
            break;
        }
    return RSP_STATUS_SUCCESS;
}

void plan_levels(const int *rp, const int *ci, IluHostPlan &hp) {
    const int n = hp.n;
    const std::vector<int> &dpos = hp.dpos;
    // levels of the lower DAG (factor + L solve): the longest path ending at
    // each row — a sequential O(nnz) pass (each row needs its producers')
    std::vector<int> lv((size_t)n, 0);
    int nl = n > 0 ? 1 : 0;
    for (int i = 0; i < n; i++) {
        int l = 0;
        for (int p = rp[i]; p < dpos[(size_t)i]; p++) l = std::max(l, lv[(size_t)ci[p]] + 1);
        lv[(size_t)i] = l;
        nl = std::max(nl, l + 1);
    }
    // transposed strict lower: row k lists (j, pos) for l_jk, j descending
    std::vector<int> &ltp = hp.ltp, &lts = hp.lts, &ltc = hp.ltc;
    ltp.assign((size_t)n + 1, 0);
    for (int j = 0; j < n; j++)
        for (int p = rp[j]; p < dpos[(size_t)j]; p++) ltp[(size_t)ci[p] + 1]++;
    for (int k = 0; k < n; k++) ltp[(size_t)k + 1] += ltp[(size_t)k];
    lts.assign((size_t)ltp[(size_t)n], 0);
    ltc.assign((size_t)ltp[(size_t)n], 0);
    {
        std::vector<int> fill(ltp.begin(), ltp.end() - 1);
        for (int j = n - 1; j >= 0; j--)
            for (int p = rp[j]; p < dpos[(size_t)j]; p++) {
                const int k = ci[p];
                const int slot = fill[(size_t)k]++;
                lts[(size_t)slot] = p;
                ltc[(size_t)slot] = j;
            }
    }
    // levels of the L^T DAG: row i waits for every j > i with l_ji != 0
    std::vector<int> lvt((size_t)n, 0);
    int nlt = n > 0 ? 1 : 0;
    for (int j = n - 1; j >= 0; j--) {
        nlt = std::max(nlt, lvt[(size_t)j] + 1);
        for (int p = rp[j]; p < dpos[(size_t)j]; p++) {
            const int k = ci[p];
            lvt[(size_t)k] = std::max(lvt[(size_t)k], lvt[(size_t)j] + 1);
        }
    }
    group_levels(lv, nl, hp.L.ptr, hp.L.rows);
    group_levels(lvt, nlt, hp.LT.ptr, hp.LT.rows);
}

rsp_status_t plan_symbolic(const int *rpp, const int *cip, IluHostPlan &hp) {
    const int n = hp.n;
    const std::vector<int> rp(rpp, rpp + (size_t)n + 1), ci(cip, cip + (size_t)hp.nnz_s);
    if (!ilu_symbolic(n, rp, ci, hp.dpos, hp.hasdiag, hp.sym)) return RSP_STATUS_ALLOC_FAILED;
    // per lower position (i, k): the position of its divisor u_kk (-1: none)
    hp.udiv.assign((size_t)hp.nnz_s, -1);
    parallel_rows(n, [&](int r0, int r1) {
        for (int i = r0; i < r1; i++)
            for (int p = rp[(size_t)i]; p < hp.dpos[(size_t)i]; p++) {
                const int k = ci[(size_t)p];
                if (hp.hasdiag[(size_t)k]) hp.udiv[(size_t)p] = hp.dpos[(size_t)k];
            }
    });
    return RSP_STATUS_SUCCESS;
}

void plan_rest(const int *rpp, const int *cip, long long slot_cap, bool want_u, IluHostPlan &hp) {
    const int n = hp.n, nnz_s = hp.nnz_s;
    const std::vector<int> rp(rpp, rpp + (size_t)n + 1), ci(cip, cip + (size_t)nnz_s);
    const std::vector<int> &dpos = hp.dpos, &hasdiag = hp.hasdiag;
    const std::vector<int> &ltp = hp.ltp, &lts = hp.lts, &ltc = hp.ltc;
    // RSP_ILU_THIN_SOLVE / RSP_ILU_THIN_FACTOR: tuning knobs (0 = no thin runs)
    const int thin_solve = std::min(env_int("RSP_ILU_THIN_SOLVE", rsp::kThinSolveRows), rsp::kThinThreads);
    const int thin_factor = env_int("RSP_ILU_THIN_FACTOR", rsp::kThinFactorRows);
    IluSymbolic &sym = hp.sym;
    {
        long long nlo = 0;
        for (int i = 0; i < n; i++) nlo += dpos[(size_t)i] - rp[(size_t)i];
        hp.L.batch = hp.LT.batch = chain_batch(nlo, n);
        for (DagHost *d : {&hp.L, &hp.LT})  // thin-run term groups
            d->group = env_int("RSP_ILU_GROUP", d->batch == 2 ? 2 : 4) == 2 ? 2 : 4;
        hp.fac_batch = chain_batch((long long)sym.upd_l.size(), nnz_s);
    }
    // the factor plan and the solve plans (flat terms in level order, thin-run
    // chunks, y sources) are independent: built concurrently
    {
        std::vector<std::thread> th;
        const bool tm = env_int("RSP_ILU_TIMING", 0) >= 2;  // diagnostics: per-plan wall time
        auto timed = [tm, n](const char *what, auto fn) {
            const double t0 = now_ms();
            fn();
            if (tm) fprintf(stderr, "rsp_ilu0_analysis n=%d   plan %-10s %8.2f ms\n", n, what, now_ms() - t0);
        };
        th.emplace_back([&] {
            timed("factor", [&] {
                build_factor_plan(n, rp, ci, dpos, hasdiag, sym, hp.L.ptr, hp.L.rows, thin_factor, hp.fplan);
            });
        });
        th.emplace_back([&] {
            timed("L", [&] {
                build_solve_plan(n, hp.L.ptr, hp.L.rows, thin_solve, hp.L.group, std::vector<int>(),
                                 [&](int i, auto emit) {
                                     for (int p = rp[(size_t)i]; p < dpos[(size_t)i]; p++) emit(p, ci[(size_t)p]);
                                 }, hp.L.sp);
            });
        });
        th.emplace_back([&] {
            timed("LT", [&] {
                build_solve_plan(n, hp.LT.ptr, hp.LT.rows, thin_solve, hp.LT.group, std::vector<int>(),
                                 [&](int i, auto emit) {
                                     for (int q = ltp[(size_t)i]; q < ltp[(size_t)i + 1]; q++)
                                         emit(lts[(size_t)q], ltc[(size_t)q]);
                                 }, hp.LT.sp);
            });
        });
        if (want_u) th.emplace_back([&] { plan_u(rp.data(), ci.data(), hp); });
        for (std::thread &x : th) x.join();
    }
    hp.L.planned = hp.LT.planned = true;
    const std::vector<int> &rows_l = hp.L.rows;
    hp.frow.assign(std::max<size_t>(rows_l.size(), 1), rsp::FacRow{});
    for (size_t x = 0; x < rows_l.size(); x++) {
        const int i = rows_l[x], rs = rp[(size_t)i], re = rp[(size_t)i + 1];
        hp.frow[x] = rsp::FacRow{i, rs, dpos[(size_t)i], re, sym.upd_ptr[(size_t)rs], sym.upd_ptr[(size_t)re],
                                 hasdiag[(size_t)i], 0};
    }
    // fat factor levels in the slot layout (rsp::FacSlotLevel): each row's
    // structure at a fixed stride, so ilu0_level_slot reads it in one round
    // trip. A level whose padded slots would take more than twice its rows'
    // own structure (one large row among many small ones), or past the
    // budget, keeps the FacRow path.
    const std::vector<int> &lp = hp.L.ptr;
    const int nlev = (int)lp.size() - 1;
    hp.fslev.assign((size_t)std::max(nlev, 0), rsp::FacSlotLevel{0, 0, 0, 0, 0});
    long long total = 0;
    std::vector<int> slot_levels;
    for (const rsp::LevelSeg &sg : hp.fplan.segs) {
        if (sg.thin) continue;
        for (int l = sg.lb; l < sg.le; l++) {
            int rm = 0, qm = 0;
            long long own = 0;
            for (int x = lp[(size_t)l]; x < lp[(size_t)l + 1]; x++) {
                const int i = rows_l[(size_t)x], rs = rp[(size_t)i], re = rp[(size_t)i + 1];
                const int nq = sym.upd_ptr[(size_t)re] - sym.upd_ptr[(size_t)rs];
                if (re - rs <= rsp::kFacRow && nq <= rsp::kFacPairs) {
                    rm = std::max(rm, re - rs);
                    qm = std::max(qm, nq);
                }
                own += (rsp::fac_pairs_at(std::min(re - rs, rsp::kFacRow)) + 2 * std::min(nq, rsp::kFacPairs) + 3) & ~3;
            }
            if (rm == 0 || qm == 0) continue;
            const int stride = (rsp::fac_pairs_at(rm) + 2 * qm + 3) & ~3;
            const long long cnt = lp[(size_t)l + 1] - lp[(size_t)l];
            if (cnt * stride > 2 * own) continue;  // padding would dominate
            if (total + cnt * stride > slot_cap) continue;
            hp.fslev[(size_t)l] = rsp::FacSlotLevel{total, stride, rm, qm, 0};
            total += cnt * stride;
            slot_levels.push_back(l);
        }
    }
    hp.slot_total = total;
    // flow runs: maximal runs of >= 2 slot-layout fat levels without
    // global-path rows; items in level order, gated like the solve's
    hp.fruns.clear();
    hp.ffitems.clear();
    if (env_int("RSP_ILU_FLOW_PLAN", 1) != 0) {
        const int gate_d = env_int("RSP_ILU_FLOW_GATE", 3);
        auto flowable = [&](int l) {
            const rsp::FacSlotLevel &sl = hp.fslev[(size_t)l];
            if (sl.stride <= 0) return false;
            for (int x = lp[(size_t)l]; x < lp[(size_t)l + 1]; x++) {
                const int i = rows_l[(size_t)x], rs = rp[(size_t)i], re = rp[(size_t)i + 1];
                if (re - rs > rsp::kFacRow || sym.upd_ptr[(size_t)re] - sym.upd_ptr[(size_t)rs] > rsp::kFacPairs)
                    return false;
            }
            return true;
        };
        for (const rsp::LevelSeg &sg : hp.fplan.segs) {
            if (sg.thin) continue;
            for (int l = sg.lb; l < sg.le;) {
                if (!flowable(l)) {
                    l++;
                    continue;
                }
                int e = l + 1;
                while (e < sg.le && flowable(e)) e++;
                if (e - l >= 2) {
                    rsp::FacFlowRun r{l, e, (int)hp.ffitems.size(), 0};
                    for (int v = l; v < e; v++) {
                        const rsp::FacSlotLevel &sl = hp.fslev[(size_t)v];
                        const int lg = v - gate_d;
                        const int gate = gate_d > 0 && lg >= l && lp[(size_t)lg + 1] > lp[(size_t)lg]
                                             ? rows_l[(size_t)lp[(size_t)lg + 1] - 1] : -1;
                        for (int x = lp[(size_t)v]; x < lp[(size_t)v + 1]; x++)
                            hp.ffitems.push_back({sl.off + (long long)(x - lp[(size_t)v]) * sl.stride,
                                                  sl.rm | sl.qm << 16, gate});
                    }
                    r.c1 = (int)hp.ffitems.size();
                    hp.fruns.push_back(r);
                }
                l = e;
            }
        }
    }
    if (hp.ffitems.empty()) hp.ffitems.push_back({0, 0, -1});  // keep the device array non-empty
    for (int l : slot_levels) {
        const rsp::FacSlotLevel &sl = hp.fslev[(size_t)l];
        for (int x = lp[(size_t)l]; x < lp[(size_t)l + 1]; x++) {
            hp.slot_desc.push_back(int4{x, sl.rm, sl.qm, 0});
            hp.slot_offs.push_back(sl.off + (long long)(x - lp[(size_t)l]) * sl.stride);
        }
    }
}


rsp_status_t plan_host(int n, const int *rp, const int *ci, long long slot_cap, bool want_u, IluHostPlan &hp,
                       Phases &ph) {
    rsp_status_t st = plan_validate(n, rp, ci, hp);
    if (st != RSP_STATUS_SUCCESS) return st;
    ph.mark("validate");
    plan_levels(rp, ci, hp);
    ph.mark("levels");
    st = plan_symbolic(rp, ci, hp);
    if (st != RSP_STATUS_SUCCESS) return st;
    ph.mark("symbolic");
    plan_rest(rp, ci, slot_cap, want_u, hp);
    ph.mark("plans");
    return RSP_STATUS_SUCCESS;
}

namespace {
struct Fnv {  // FNV-1a over 8-byte words (bytes for the tail)
    uint64_t h = 1469598103934665603ULL;
    void bytes(const void *p, size_t n) {
        const unsigned char *c = (const unsigned char *)p;
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            uint64_t w;
            memcpy(&w, c + i, 8);
            h = (h ^ w) * 1099511628211ULL;
        }
        for (; i < n; i++) h = (h ^ c[i]) * 1099511628211ULL;
    }
    template <typename V>
    void vec(const std::vector<V> &v) {
        const uint64_t n = v.size();
        bytes(&n, sizeof(n));
        if (!v.empty()) bytes(v.data(), v.size() * sizeof(V));
    }
};
}  // namespace

uint64_t digest(const IluHostPlan &hp) {
    Fnv f;
    f.bytes(&hp.n, sizeof(hp.n));
    f.bytes(&hp.structural_zero, sizeof(hp.structural_zero));
    f.vec(hp.dpos);
    f.vec(hp.hasdiag);
    f.vec(hp.udiv);
    f.vec(hp.sym.upd_ptr);
    f.vec(hp.sym.upd_l);
    f.vec(hp.sym.upd_u);
    f.vec(hp.sym.lord);
    f.vec(hp.sym.lend);
    for (const DagHost *d : {&hp.L, &hp.LT}) {
        f.vec(d->ptr);
        f.vec(d->rows);
        f.vec(d->sp.tasks);
        f.vec(d->sp.tpos);
        f.vec(d->sp.src);
        f.vec(d->sp.segs);
        f.vec(d->sp.chunks);
        f.vec(d->sp.trow);
        f.vec(d->sp.sid);
        f.vec(d->sp.stg);
        f.vec(d->sp.nshort);
        f.vec(d->sp.nwave);
        f.vec(d->sp.sbase);
        f.vec(d->sp.fitems);
    }
    f.vec(hp.fplan.segs);
    f.vec(hp.fplan.chunks);
    f.vec(hp.fplan.items);
    f.vec(hp.fplan.pairs);
    f.vec(hp.fplan.staged);
    f.vec(hp.fplan.rounds);
    f.vec(hp.frow);
    f.vec(hp.fslev);
    f.vec(hp.slot_desc);
    f.vec(hp.slot_offs);
    f.vec(hp.fruns);
    f.vec(hp.ffitems);
    return f.h;
}

}  // namespace rsp_an
