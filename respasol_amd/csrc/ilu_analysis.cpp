// ilu_analysis.cpp — host half of the ILU(0) analysis (see ilu_analysis.h).
// Replaces the dependency analysis inside cusparse?csrilu02_analysis and
// cusparse?csrsv2_analysis (GPU/ilu0.cu:196-252). No HIP calls here.

#include "ilu_analysis.h"

#include <limits.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <unordered_map>
#include <mutex>
#include <thread>

namespace rsp_an {

// Block cache behind PoolAlloc (host_pool.h).
namespace {
constexpr size_t kHugePage = 2u << 20;
struct BlockCache {
    std::mutex m;
    std::multimap<size_t, void *> free_blocks;    // size -> block
    std::unordered_map<void *, size_t> live;      // block -> size
    size_t cached = 0;
    size_t cap = (size_t)std::max(0, env_int("RSP_HOST_POOL_MB", 1024)) << 20;
};
BlockCache &block_cache() {
    static BlockCache *c = new BlockCache();  // never destroyed: blocks may be freed during exit
    return *c;
}
}  // namespace

void *pool_get(size_t bytes) {
    const size_t r = (bytes + kHugePage - 1) & ~(kHugePage - 1);
    BlockCache &c = block_cache();
    {
        std::lock_guard<std::mutex> g(c.m);
        auto it = c.free_blocks.lower_bound(r);
        if (it != c.free_blocks.end() && it->first <= r + r / 4 + kHugePage) {  // best fit, little slack
            void *p = it->second;
            const size_t s = it->first;
            c.free_blocks.erase(it);
            c.cached -= s;
            c.live[p] = s;
            return p;
        }
    }
    void *p = nullptr;
    if (posix_memalign(&p, kHugePage, r) != 0 || !p) throw std::bad_alloc();
    (void)madvise(p, r, MADV_HUGEPAGE);  // a hint: without THP the block is just a block
    std::lock_guard<std::mutex> g(c.m);
    c.live[p] = r;
    return p;
}

void pool_put(void *p, size_t) {
    if (!p) return;
    BlockCache &c = block_cache();
    {
        std::lock_guard<std::mutex> g(c.m);
        auto it = c.live.find(p);
        if (it == c.live.end()) return;  // not ours (cannot happen through PoolAlloc)
        const size_t s = it->second;
        c.live.erase(it);
        if (c.cached + s <= c.cap) {
            c.free_blocks.emplace(s, p);
            c.cached += s;
            return;
        }
    }
    free(p);
}

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

// Host worker threads for the analysis: OMP_NUM_THREADS (the box's share of
// its cores; the machine may have many more) or the hardware count, <= 64.
static int host_threads() {
    int t = env_int("OMP_NUM_THREADS", 0);
    if (t <= 0) t = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 64));
}

// Persistent worker threads for the parallel loops below. A loop used to
// spawn and join its team each time (~0.2-0.5 ms per loop at 16 threads, and
// an analysis runs ~35 loops: tens of ms on a small matrix). A loop is a job
// of `nb` blocks claimed through an atomic counter; the calling thread works
// on its own job too, so a job always finishes even when every worker is busy
// (nested or concurrent loops: the plans of L, L^T and the factor run at the
// same time). Block boundaries are the same as before, so are the plans.
// Workers are created on first use (as many as host_threads() - 1 asks for,
// growing if a later call asks for more), detached, and live as long as the
// process.
class Pool {
    struct Job {
        std::function<void(int)> body;
        int nb = 0;
        std::atomic<int> next{0}, done{0};
        std::mutex m;
        std::condition_variable cv;
        std::exception_ptr err;  // the first exception of a block (rethrown by run)
        void work() {
            for (int b; (b = next.fetch_add(1, std::memory_order_relaxed)) < nb;) {
                try {
                    body(b);
                } catch (...) {
                    std::lock_guard<std::mutex> g(m);
                    if (!err) err = std::current_exception();
                }
                if (done.fetch_add(1, std::memory_order_acq_rel) + 1 == nb) {
                    std::lock_guard<std::mutex> g(m);
                    cv.notify_all();
                }
            }
        }
    };
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Job>> q_;
    int workers_ = 0;

    void worker() {
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return !q_.empty(); });
                j = std::move(q_.front());
                q_.pop_front();
            }
            j->work();
        }
    }

  public:
    static Pool &get() {
        static Pool *p = new Pool();  // never destroyed: its threads outlive static destructors
        return *p;
    }
    // body(b) for b in [0, nb) on up to `team` threads (the caller included)
    void run(int nb, int team, const std::function<void(int)> &body) {
        if (nb <= 0) return;
        team = std::max(1, std::min(team, nb));
        if (team == 1) {
            for (int b = 0; b < nb; b++) body(b);
            return;
        }
        auto j = std::make_shared<Job>();
        j->body = body;
        j->nb = nb;
        {
            std::lock_guard<std::mutex> g(m_);
            for (; workers_ < team - 1; workers_++) std::thread([this] { worker(); }).detach();
            for (int t = 1; t < team; t++) q_.push_back(j);
        }
        if (team == 2)
            cv_.notify_one();
        else
            cv_.notify_all();
        j->work();
        std::unique_lock<std::mutex> g(j->m);
        j->cv.wait(g, [&] { return j->done.load(std::memory_order_acquire) == nb; });
        // every block has finished (no worker still runs body over the
        // caller's locals): a block's exception is the caller's now
        if (j->err) std::rethrow_exception(j->err);
    }
};

// f(r0, r1) over contiguous row blocks of [0, n) on host_threads() threads.
template <typename F>
static void parallel_rows(int n, F f) {
    const int nt = n < 8192 ? 1 : host_threads();
    if (nt == 1) {
        f(0, n);
        return;
    }
    Pool::get().run(nt, nt, [&](int t) { f((int)((long long)n * t / nt), (int)((long long)n * (t + 1) / nt)); });
}

// f(lo, hi) over [0, n) in at most host_threads() contiguous blocks of at
// least `grain`.
template <typename F>
static void pfor(long long n, long long grain, F f) {
    const int nt = (int)std::max<long long>(1, std::min<long long>(host_threads(), n / std::max(grain, 1LL)));
    if (nt <= 1) {
        if (n > 0) f(0LL, n);
        return;
    }
    Pool::get().run(nt, nt, [&](int t) { f(n * t / nt, n * (t + 1) / nt); });
}

void parallel_for(long long n, long long grain, const std::function<void(long long, long long)> &f) {
    pfor(n, grain, [&](long long a, long long b) { f(a, b); });
}

// f(j) for j in [0, n), items handed out dynamically (uneven item costs:
// levels, segments, chunks); `work` estimates the total cost to size the team.
// Items are claimed in runs of about n / (64 team) (one claim per item made
// the many tiny levels of a deep DAG — 13 k on matrix-new_3 — cost ~1 ms
// per loop in claims alone; round 5).
template <typename F>
static void pfor_dyn(int n, long long work, long long grain, F f) {
    const int nt = (int)std::max<long long>(1, std::min<long long>({(long long)host_threads(), (long long)n,
                                                                     work / std::max(grain, 1LL)}));
    if (nt <= 1) {
        for (int j = 0; j < n; j++) f(j);
        return;
    }
    const int run = std::max(1, n / (64 * nt));
    Pool::get().run((n + run - 1) / run, nt, [&](int b) {
        for (int j = b * run, e = std::min(n, j + run); j < e; j++) f(j);
    });
}

// rows grouped by level (stable: ascending row within a level). A counting
// sort; on large level sets with few levels per row block, in parallel: each
// of T contiguous row blocks counts its levels, block t's rows of level v go
// after those of blocks < t (the same order as the sequential pass).
static void group_levels(const hvec<int> &lev, int nlev, hvec<int> &ptr,
                         hvec<int> &rows) {
    const int n = (int)lev.size();
    const int T = host_threads();
    ptr.assign((size_t)nlev + 1, 0);
    rows.resize(lev.size());
    if (n < (1 << 16) || T < 2 || (long long)nlev * T > n) {
        for (int v : lev) ptr[(size_t)v + 1]++;
        for (int l = 0; l < nlev; l++) ptr[(size_t)l + 1] += ptr[(size_t)l];
        hvec<int> fill(ptr.begin(), ptr.end() - 1);
        for (size_t i = 0; i < lev.size(); i++) rows[(size_t)fill[(size_t)lev[i]]++] = (int)i;
        return;
    }
    std::vector<int> cnt((size_t)T * nlev, 0);  // cnt[t * nlev + v]
    auto block = [&](int t, int &a, int &b) {
        a = (int)((long long)n * t / T);
        b = (int)((long long)n * (t + 1) / T);
    };
    pfor_dyn(T, n, 1, [&](int t) {
        int a, b;
        block(t, a, b);
        int *c = cnt.data() + (size_t)t * nlev;
        for (int i = a; i < b; i++) c[lev[(size_t)i]]++;
    });
    // per level: its start, then each block's offset within it (level-major)
    int run = 0;
    for (int v = 0; v < nlev; v++) {
        ptr[(size_t)v] = run;
        for (int t = 0; t < T; t++) {
            const int k = cnt[(size_t)t * nlev + v];
            cnt[(size_t)t * nlev + v] = run;
            run += k;
        }
    }
    ptr[(size_t)nlev] = run;
    pfor_dyn(T, n, 1, [&](int t) {
        int a, b;
        block(t, a, b);
        int *c = cnt.data() + (size_t)t * nlev;
        for (int i = a; i < b; i++) rows[(size_t)c[lev[(size_t)i]]++] = i;
    });
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

// Built in two parts, each in parallel phases (rows, levels and chunks as
// work items, prefix sums over level order in between):
//   solve_plan_rows  (host): segments, row classes and order, tasks, flow
//                    items, the thin runs' chunks (levels, slots, terms) —
//                    per-row and per-level decisions; row_count(i) = the
//                    number of terms of row i;
//   solve_plan_terms (host; the device analysis runs ilu_an_solve_terms
//                    instead, the same arrays bit for bit): per flat term
//                    its position and y source, the window remap, the thin
//                    runs' row records, y indices and staged terms.
// A thin-run row's padded terms: its early and its late terms (split order,
// IluHostPlan::lpos) each padded to whole groups, at least one group.
static inline int split_padded(int ne, int cnt, int group) {
    const int pe = (ne + group - 1) / group * group, pl = (cnt - ne + group - 1) / group * group;
    return std::max(group, pe + pl);
}

template <typename RowCount, typename RowEarly>
static void solve_plan_rows(int n, const hvec<int> &ptr, const hvec<int> &rows,
                            int thin_rows, int group, const hvec<int> &diag,
                            RowCount row_count, RowEarly row_early, SolvePlan &sp) {
    const int nlev = (int)ptr.size() - 1;
    const long long nx = (long long)rows.size();
    constexpr long long kGrain = 1 << 14;
    const bool tm = env_int("RSP_ILU_TIMING", 0) >= 4;  // diagnostics: sub-steps
    double tq = now_ms();
    auto step = [&](const char *what) {
        if (!tm) return;
        const double t = now_ms();
        fprintf(stderr, "rsp_ilu0_analysis n=%d       solve rows %-10s %6.2f ms\n", n, what, t - tq);
        tq = t;
    };
    hvec<int> order(rows);
    // (row_count / row_early are O(1) lookups: called where needed, not
    // copied into per-row arrays first)
    auto padded_row = [&](int i) { return split_padded(row_early(i), row_count(i), group); };
    hvec<int> lpad((size_t)std::max(nlev, 1), 0);
    pfor_dyn(nlev, nx, kGrain, [&](int l) {
        int t = 0;
        for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++) t += padded_row(order[(size_t)x]);
        lpad[(size_t)l] = t;
    });
    step("counts");
    // RSP_ILU_THIN_TERMS: tuning knob (a thin level's padded terms, <= kChunkTerms)
    const int thin_terms = std::min(env_int("RSP_ILU_THIN_TERMS", rsp::kThinSolveTerms), rsp::kChunkTerms);
    sp.segs.clear();
    for (int l = 0; l < nlev; l++) {
        const int cnt = ptr[(size_t)l + 1] - ptr[(size_t)l];
        const int thin = (cnt <= thin_rows && cnt <= rsp::kThinThreads && cnt <= rsp::kChunkRows &&
                          lpad[(size_t)l] <= thin_terms) ? 1 : 0;
        if (!sp.segs.empty() && sp.segs.back().thin == thin && sp.segs.back().le == l)
            sp.segs.back().le = l + 1;
        else
            sp.segs.push_back({l, l + 1, thin, 0, 0, 0});
    }
    hvec<char> thin_lev((size_t)std::max(nlev, 1), 0);
    for (const rsp::LevelSeg &sg : sp.segs)
        for (int l = sg.lb; l < sg.le; l++) thin_lev[(size_t)l] = (char)sg.thin;
    step("segs");
    // within each level (stable): short rows, then wave rows, then (fat
    // levels) hub rows
    const int fat_long = env_int("RSP_ILU_FAT_LONG", rsp::kFatLongDefault);
    const int hub = env_int("RSP_ILU_HUB", rsp::kHubTerms);
    sp.nshort.assign((size_t)std::max(nlev, 1), 0);
    sp.nwave.assign((size_t)std::max(nlev, 1), 0);
    pfor_dyn(nlev, nx, kGrain, [&](int l) {
        const int lim = thin_lev[(size_t)l] ? rsp::kLongTerms : fat_long;
        const int b = ptr[(size_t)l], e = ptr[(size_t)l + 1];
        int c[3] = {0, 0, 0};
        auto cls = [&](int i) {
            const int t = row_count(i);
            return t <= lim ? 0 : (thin_lev[(size_t)l] || t <= hub ? 1 : 2);
        };
        for (int x = b; x < e; x++) c[cls(order[(size_t)x])]++;
        sp.nshort[(size_t)l] = c[0];
        sp.nwave[(size_t)l] = c[0] + c[1];
        if (c[0] == e - b || c[1] == e - b || c[2] == e - b) return;  // one class: order unchanged
        hvec<int> tmp(order.begin() + b, order.begin() + e);
        int w[3] = {b, b + c[0], b + c[0] + c[1]};
        for (int i : tmp) order[(size_t)w[cls(i)]++] = i;
    });
    step("classes");
    // flat term ranges in level order: a thin row's terms padded to whole
    // groups; a padded fat level's short rows own kFatLongTerms terms each
    const bool pad_fat = fat_long == rsp::kFatLongTerms && env_int("RSP_ILU_FAT_PAD", 1) != 0;
    sp.sbase.assign((size_t)std::max(nlev, 1), -1);
    sp.tasks.assign(std::max<size_t>(rows.size(), 1), rsp::RowTask{0, 0, 0, -1});
    hvec<int> len((size_t)std::max(nx, 1LL), 0);
    pfor_dyn(nlev, nx, kGrain, [&](int l) {
        const bool padl = pad_fat && !thin_lev[(size_t)l] && sp.nshort[(size_t)l] > 0;
        for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++) {
            const int i = order[(size_t)x], t = row_count(i);
            const int t1 = thin_lev[(size_t)l] ? padded_row(i) : t;
            len[(size_t)x] = padl && x - ptr[(size_t)l] < sp.nshort[(size_t)l] ? std::max(t1, rsp::kFatLongTerms) : t1;
            sp.tasks[(size_t)x].t1 = t1;  // length for now
        }
    });
    step("lengths");
    long long total = 0;
    for (long long x = 0; x < nx; x++) {
        sp.tasks[(size_t)x].t0 = (int)total;
        total += len[(size_t)x];
    }
    for (int l = 0; l < nlev; l++)
        if (pad_fat && !thin_lev[(size_t)l] && sp.nshort[(size_t)l] > 0) sp.sbase[(size_t)l] = sp.tasks[(size_t)ptr[(size_t)l]].t0;
    sp.nterm = total;
    step("prefix");
    pfor(nx, kGrain, [&](long long a, long long b) {
        for (long long x = a; x < b; x++) {
            rsp::RowTask &t = sp.tasks[(size_t)x];
            t.i = order[(size_t)x];
            t.t1 += t.t0;
            t.d = diag.empty() ? -1 : diag[(size_t)t.i];
        }
    });
    step("tasks");
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
    if (sp.fitems.empty()) sp.fitems.push_back({0, 0, -1, -1});
    step("flow");
    hvec<int> lterms((size_t)std::max(nlev, 1), 0);
    for (int l = 0; l < nlev; l++)
        if (ptr[(size_t)l + 1] > ptr[(size_t)l])
            lterms[(size_t)l] = sp.tasks[(size_t)ptr[(size_t)l + 1] - 1].t1 - sp.tasks[(size_t)ptr[(size_t)l]].t0;
    for (rsp::LevelSeg &sg : sp.segs)
        if (sg.thin) sg.nth = rsp::kThinThreads;
    // chunks of the thin runs (greedy over levels): levels, slots, terms, and
    // each chunk's run base (the run's first slot)
    sp.chunks.clear();
    sp.cbase.clear();
    for (rsp::LevelSeg &sg : sp.segs) {
        if (!sg.thin) continue;
        sg.c0 = (int)sp.chunks.size();
        int crow = 0, cterm = 0;
        for (int l = sg.lb; l < sg.le; l++) {
            const int cnt = ptr[(size_t)l + 1] - ptr[(size_t)l];
            if (sp.chunks.size() == (size_t)sg.c0 || crow + cnt > rsp::kChunkRows ||
                cterm + lterms[(size_t)l] > rsp::kChunkTerms) {
                sp.chunks.push_back({l, l + 1, 0, 0, 0, 0, 0, 0});
                sp.cbase.push_back(ptr[(size_t)sg.lb]);
                crow = 0;
                cterm = 0;
            } else {
                sp.chunks.back().l1 = l + 1;
            }
            crow += cnt;
            cterm += lterms[(size_t)l];
        }
        sg.c1 = (int)sp.chunks.size();
    }
    for (rsp::LevelChunk &ch : sp.chunks) {
        ch.x0 = ptr[(size_t)ch.l0];
        ch.x1 = ptr[(size_t)ch.l1];
        ch.k0 = ch.x1 > ch.x0 ? sp.tasks[(size_t)ch.x0].t0 : 0;
        ch.k1 = ch.x1 > ch.x0 ? sp.tasks[(size_t)ch.x1 - 1].t1 : 0;
    }
    if (sp.chunks.empty()) {
        sp.chunks.push_back({0, 0, 0, 0, 0, 0, 0, 0});
        sp.cbase.push_back(0);
    }
    step("chunks");
}

// row_terms(i, emit) calls emit(tpos, col) for the terms of row i in order
// (row_count(i) of them, as given to solve_plan_rows; the first row_early(i)
// of them early). A thin row (its task spans split_padded terms) places its
// late terms at the first group after its early ones; other rows keep their
// terms contiguous (when split_padded equals the count the two coincide).
static inline int late_offset(int ne, int cnt, int len, int group) {
    return len == split_padded(ne, cnt, group) ? (ne + group - 1) / group * group : ne;
}
template <typename RowTerms, typename RowEarly>
static void solve_plan_terms(int n, const hvec<int> &ptr, int group, RowTerms row_terms, RowEarly row_early,
                             SolvePlan &sp) {
    constexpr long long kGrain = 1 << 14;
    const int nlev = (int)ptr.size() - 1;
    const long long nx = (long long)ptr[(size_t)nlev], total = sp.nterm;
    sp.tpos.assign((size_t)total, -1);
    hvec<int> col((size_t)total, -1);
    hvec<int> egroups((size_t)std::max(nx, 1LL), 0);  // thin rows: whole groups of early terms
    pfor(nx, kGrain, [&](long long a, long long b) {
        for (long long x = a; x < b; x++) {
            const rsp::RowTask &t = sp.tasks[(size_t)x];
            const int ne = row_early(t.i);
            int cnt = 0;
            row_terms(t.i, [&](int, int) { cnt++; });
            const int lo = late_offset(ne, cnt, t.t1 - t.t0, group);
            if (t.t1 - t.t0 == split_padded(ne, cnt, group)) egroups[(size_t)x] = lo / group;
            int o = 0;
            row_terms(t.i, [&](int tp, int c) {
                const int k = t.t0 + (o < ne ? o : lo + (o - ne));
                sp.tpos[(size_t)k] = tp;
                col[(size_t)k] = c;
                o++;
            });
        }
    });
    sp.src.resize((size_t)total);
    pfor(total, kGrain, [&](long long a, long long b) {
        for (long long k = a; k < b; k++) sp.src[(size_t)k] = col[(size_t)k] < 0 ? rsp::kPadSrc : col[(size_t)k];
    });
    hvec<int> slot_of((size_t)n, -1);
    pfor(nx, kGrain, [&](long long a, long long b) {
        for (long long x = a; x < b; x++) slot_of[(size_t)sp.tasks[(size_t)x].i] = (int)x;
    });
    hvec<int> thin_base((size_t)std::max(nlev, 1), -1);  // per thin level: its run's first slot
    for (const rsp::LevelSeg &sg : sp.segs)
        if (sg.thin)
            for (int l = sg.lb; l < sg.le; l++) thin_base[(size_t)l] = ptr[(size_t)sg.lb];
    // y sources of the thin runs' terms: the LDS window slot when the
    // producer is earlier in the run and still in the window
    pfor_dyn(nlev, nx, kGrain, [&](int l) {
        const int base = thin_base[(size_t)l];
        if (base < 0) return;
        const int r_end = ptr[(size_t)l + 1] - base;
        for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++)
            for (int k = sp.tasks[(size_t)x].t0; k < sp.tasks[(size_t)x].t1; k++) {
                if (col[(size_t)k] < 0) continue;  // pad
                const int sj = slot_of[(size_t)col[(size_t)k]];
                if (sj < base || sj >= ptr[(size_t)l]) continue;  // before the run
                const int rj = sj - base;
                if (r_end - rj <= rsp::kYWin) sp.src[(size_t)k] = -((rj & (rsp::kYWin - 1)) + 1);
            }
    });
    if (sp.tpos.empty()) {
        sp.tpos.push_back(0);
        sp.src.push_back(0);
    }
    // per chunk: static row records, term y indices, staged terms (counted
    // per chunk, then filled at their prefix offsets)
    sp.trow.assign(std::max<size_t>((size_t)nx, 1), rsp::ThinRowPlan{0, 0, 0, -1});
    sp.sid.assign(sp.tpos.size(), rsp::kYWin);
    const int nch = (int)sp.chunks.size();
    hvec<int> nst((size_t)std::max(nch, 1), 0);
    pfor_dyn(nch, nx, kGrain, [&](int c) {
        const rsp::LevelChunk &ch = sp.chunks[(size_t)c];
        int m = 0;
        for (int x = ch.x0; x < ch.x1; x++)
            for (int k = sp.tasks[(size_t)x].t0; k < sp.tasks[(size_t)x].t1; k++) m += sp.src[(size_t)k] >= 0;
        nst[(size_t)c] = m;
    });
    long long nstg = 0;
    for (int c = 0; c < nch; c++) {
        sp.chunks[(size_t)c].st0 = (int)nstg;
        nstg += nst[(size_t)c];
        sp.chunks[(size_t)c].st1 = (int)nstg;
    }
    sp.stg.assign((size_t)nstg, rsp::StagedTerm{0, 0});
    pfor_dyn(nch, nx, kGrain, [&](int c) {
        const rsp::LevelChunk &ch = sp.chunks[(size_t)c];
        const int base = sp.cbase[(size_t)c];
        int st = ch.st0;
        for (int x = ch.x0; x < ch.x1; x++) {
            const rsp::RowTask &t = sp.tasks[(size_t)x];
            sp.trow[(size_t)x] = {(t.t0 - ch.k0) / group | ((t.t1 - t.t0) / group) << 16,
                                  ((x - base) & (rsp::kYWin - 1)) | egroups[(size_t)x] << 16, t.i, t.d};
            for (int k = t.t0; k < t.t1; k++) {
                const int sc = sp.src[(size_t)k];
                if (sc < 0) {
                    sp.sid[(size_t)k] = -sc - 1;
                } else {
                    sp.sid[(size_t)k] = rsp::kYWin + 1 + (k - ch.k0);
                    sp.stg[(size_t)st++] = {k - ch.k0, sc};
                }
            }
        }
    });
    if (sp.stg.empty()) sp.stg.push_back({0, 0});
}

// Both parts on the host.
template <typename RowCount, typename RowTerms, typename RowEarly>
static void build_solve_plan(int n, const hvec<int> &ptr, const hvec<int> &rows,
                             int thin_rows, int group, const hvec<int> &diag,
                             RowCount row_count, RowTerms row_terms, RowEarly row_early, SolvePlan &sp) {
    solve_plan_rows(n, ptr, rows, thin_rows, group, diag, row_count, row_early, sp);
    solve_plan_terms(n, ptr, group, row_terms, row_early, sp);
}

// Which levels of the L DAG the factor runs thin. A level runs thin up to
// kRndFlowItems positions; up to kRndLevelItems when it could not run in a
// flow launch anyway (a row past the slot layout's kFacRow entries /
// kFacPairs pairs: circuit hubs); and never with a position of more than
// kRndItemPairs update pairs. Wider levels are fat: in a flow run they
// spread over all CUs, where a thin run stages every position through one
// (A/B knobs RSP_ILU_THIN_FACTOR_ITEMS / RSP_ILU_THIN_FACTOR_FLOW).
static hvec<char> factor_thin_levels(const int *rp, const hvec<int> &upd_ptr,
                                            const hvec<int> &ptr, const hvec<int> &rows,
                                            int thin_rows, hvec<long long> *items_out) {
    const int nlev = (int)ptr.size() - 1;
    const int thin_items = env_int("RSP_ILU_THIN_FACTOR_ITEMS", rsp::kRndLevelItems);
    const int thin_flow = env_int("RSP_ILU_THIN_FACTOR_FLOW", rsp::kRndFlowItems);
    hvec<long long> litems((size_t)std::max(nlev, 1), 0);
    hvec<char> thin((size_t)std::max(nlev, 1), 0);
    pfor_dyn(nlev, (long long)rows.size(), 1 << 14, [&](int l) {
        long long items = 0;
        int maxp = 0;
        bool hub = false;
        for (int x = ptr[(size_t)l]; x < ptr[(size_t)l + 1]; x++) {
            const int i = rows[(size_t)x], rs = rp[(size_t)i], re = rp[(size_t)i + 1];
            items += re - rs;
            for (int p = rs; p < re; p++) maxp = std::max(maxp, upd_ptr[(size_t)p + 1] - upd_ptr[(size_t)p]);
            hub |= re - rs > rsp::kFacRow || upd_ptr[(size_t)re] - upd_ptr[(size_t)rs] > rsp::kFacPairs;
        }
        litems[(size_t)l] = items;
        const int cnt = ptr[(size_t)l + 1] - ptr[(size_t)l];
        const long long lim = hub ? thin_items : std::min(thin_items, thin_flow);
        thin[(size_t)l] = (cnt <= thin_rows && items <= lim && maxp <= rsp::kRndItemPairs) ? 1 : 0;
    });
    if (items_out) items_out->swap(litems);
    return thin;
}

static int thin_factor_rows() { return env_int("RSP_ILU_THIN_FACTOR", rsp::kThinFactorRows); }

hvec<int> factor_thin_rows(const int *rp, const IluHostPlan &hp) {
    const hvec<char> thin = factor_thin_levels(rp, hp.sym.upd_ptr, hp.L.ptr, hp.L.rows, thin_factor_rows(),
                                                      nullptr);
    hvec<int> out;
    for (size_t l = 0; l + 1 < hp.L.ptr.size(); l++)
        if (thin[l])
            for (int x = hp.L.ptr[l]; x < hp.L.ptr[l + 1]; x++) out.push_back(hp.L.rows[(size_t)x]);
    return out;
}

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
//
// Built in parallel. A thin segment is cut at level boundaries into pieces
// of about RSP_ILU_PIECE_ITEMS positions (default kRndPieceItems); each
// piece is planned on its own (greedily, as above) and the pieces are joined
// in order with an EMPTY chunk between two pieces of a segment: ilu0_rounds issues a chunk's gathers at
// the previous chunk's switch, so the empty chunk's switch is where the
// earlier piece's last stores are complete before the next piece stages them
// (a piece sees every value before it as staged). Per position, where[] holds
// the chunk key (piece + 1, chunk within the piece) and slot it was placed at:
// keys are unique over the whole plan, so a piece reading a position another
// piece is writing concurrently (never its own chunk or the one before) only
// ever gets "not here" — the relaxed atomics make those reads well defined.
// The staged positions of the current chunk sit in a piece-private hash.
static constexpr int kRndPieceItems = 1 << 16;  // the largest piece (round 4 A/B: 2^17 / 2^16 / 2^15 gave factor 58.58 / 58.58 / 58.73 ms); see build_factor_plan

static void build_factor_plan(int n, const int *rp, const int *ci,
                              const hvec<int> &dpos, const hvec<int> &hasdiag,
                              const IluSymbolic &sym, const hvec<int> &ptr,
                              const hvec<int> &rows, int thin_rows, FacPlan &fp) {
    const int nlev = (int)ptr.size() - 1;
    const int K = rsp::kRndItems, S = rsp::kRndStaged, kZero = 2 * rsp::kRndItems + rsp::kRndStaged;
    const int nnz = rp[(size_t)n];
    const double t0 = now_ms();
    hvec<long long> litems;
    const hvec<char> lthin = factor_thin_levels(rp, sym.upd_ptr, ptr, rows, thin_rows, &litems);
    const double t_thin = now_ms() - t0;
    // piece size: about 1/32 of the thin positions, within [2^15, 2^16] — a
    // function of the pattern only, so the plan is the same on every host
    // (round 5: a fixed 2^16 left the circuits' 7-13 pieces, ~120 ns per
    // position each, as the analysis' longest step; each extra piece adds an
    // empty chunk to the factor, ~1.5 us: a 2^14 floor gave config-3 analysis
    // -15 ms for +0.6 % on the circuits' factor, profiles/r05_piece_ab.txt)
    long long thin_total = 0;
    for (int l = 0; l < nlev; l++)
        if (lthin[(size_t)l]) thin_total += litems[(size_t)l];
    const long long piece_items = std::max(
        1LL, (long long)env_int("RSP_ILU_PIECE_ITEMS",
                                (int)std::min<long long>(kRndPieceItems, std::max<long long>(1 << 15, thin_total / 32))));
    // pairs of position p of thin row i (packed, see IluSymbolic::pair_base)
    auto pair_off = [&](int i) {
        return sym.pair_base.empty() ? 0 : sym.pair_base[(size_t)i] - sym.upd_ptr[(size_t)rp[(size_t)i]];
    };
    fp.segs.clear();
    for (int l = 0; l < nlev; l++) {
        const int thin = lthin[(size_t)l];
        if (!fp.segs.empty() && fp.segs.back().thin == thin && fp.segs.back().le == l)
            fp.segs.back().le = l + 1;
        else
            fp.segs.push_back({l, l + 1, thin, 0, 0, rsp::kThinThreads});
    }
    struct Piece {
        int seg, lb, le;
        FacPlan out;  // chunk records relative to the piece's own arrays
    };
    hvec<Piece> pieces;
    for (int s = 0; s < (int)fp.segs.size(); s++) {
        const rsp::LevelSeg &sg = fp.segs[(size_t)s];
        if (!sg.thin) continue;
        long long acc = 0;
        int lb = sg.lb;
        for (int l = sg.lb; l < sg.le; l++) {
            acc += litems[(size_t)l];
            if (acc >= piece_items && l + 1 < sg.le) {
                pieces.push_back({s, lb, l + 1, FacPlan()});
                lb = l + 1;
                acc = 0;
            }
        }
        pieces.push_back({s, lb, sg.le, FacPlan()});
    }
    hvec<unsigned long long> where((size_t)std::max(nnz, 1), 0ull);
    const double t_where = now_ms() - t0;
    auto wload = [&](int q) { return __atomic_load_n(&where[(size_t)q], __ATOMIC_RELAXED); };
    pfor_dyn((int)pieces.size(), nnz, 1 << 15, [&](int pi) {
        Piece &pc = pieces[(size_t)pi];
        FacPlan &o = pc.out;
        // staged positions of the current chunk: open addressing, epoch-stamped
        constexpr int kH = 4 * rsp::kRndStaged;
        hvec<int> hkey(kH), hval(kH), hep(kH, 0);
        int epoch = 0, nstg = 0;
        auto hslot = [&](int q) { return (int)(((unsigned)q * 2654435761u) >> 18) & (kH - 1); };
        auto hfind = [&](int q) {
            for (int h = hslot(q);; h = (h + 1) & (kH - 1)) {
                if (hep[(size_t)h] != epoch) return -1;
                if (hkey[(size_t)h] == q) return hval[(size_t)h];
            }
        };
        auto hput = [&](int q, int v) {
            int h = hslot(q);
            while (hep[(size_t)h] == epoch) h = (h + 1) & (kH - 1);
            hep[(size_t)h] = epoch;
            hkey[(size_t)h] = q;
            hval[(size_t)h] = v;
        };
        const unsigned long long pkey = (unsigned long long)(pi + 1) << 28;
        int c = -1;  // chunk within the piece
        unsigned long long ckey = 0;
        rsp::RndChunk ch{};
        auto open_chunk = [&]() {
            epoch++;
            nstg = 0;
            c = (int)o.chunks.size();
            ckey = pkey | (unsigned long long)c;
            ch = rsp::RndChunk{(int)o.items.size(), (int)o.items.size(), (int)o.pairs.size(), (int)o.pairs.size(),
                               (int)o.staged.size(), (int)o.staged.size(), (int)o.rounds.size(), (int)o.rounds.size()};
            o.chunks.push_back(ch);
        };
        auto close_chunk = [&]() {
            ch.i1 = (int)o.items.size();
            ch.p1 = (int)o.pairs.size();
            ch.s1 = (int)o.staged.size();
            ch.r1 = (int)o.rounds.size();
            o.chunks[(size_t)c] = ch;
        };
        // this item's not-yet-staged operands (fresh), looked up by a second
        // epoch-stamped hash: an item of a hub row has up to kRndItemPairs
        // pairs, and a linear search of its fresh list was quadratic in them
        constexpr int kF = 4 * rsp::kRndItemPairs;  // >= 2 x the 2 kRndItemPairs operands
        hvec<int> fkey(kF), fval(kF), fep(kF, 0);
        int fepoch = 0;
        // first slot of the item's round in its chunk: a position placed at
        // or after it is computed in the same round, so it is no operand
        // slot. Only a one-level factor (IluHostPlan::fac_one) reads such a
        // position — a u_kk of a row without lower entries, final from the
        // start — and stages its input instead; in an L-level plan every
        // operand lies in an earlier round, so this never triggers there.
        int rstart = 0;
        auto ref = [&](int q, hvec<int> &fresh) {
            const unsigned long long w = wload(q), wk = w >> 12;
            if (wk == ckey && (int)(w & 0xfff) < rstart) return (int)(w & 0xfff);
            if (c > 0 && wk == ckey - 1) return K + (int)(w & 0xfff);
            const int st = hfind(q);
            if (st >= 0) return 2 * K + st;
            int h = (int)(((unsigned)q * 2654435761u) >> 20) & (kF - 1);
            for (; fep[(size_t)h] == fepoch; h = (h + 1) & (kF - 1))
                if (fkey[(size_t)h] == q) return 2 * K + (int)(nstg + fval[(size_t)h]);
            fep[(size_t)h] = fepoch;
            fkey[(size_t)h] = q;
            fval[(size_t)h] = (int)fresh.size();
            fresh.push_back(q);
            return 2 * K + (int)(nstg + fresh.size() - 1);
        };
        struct RItem {
            int round, pos, row;
        };
        hvec<RItem> ritems, rsorted;
        hvec<int> rcount, fresh, ipairs;
        open_chunk();
        long long last_round_key = -1;
        int last_round_level = -1;  // level of the chunk's last round (-1: none yet)
        for (int l = pc.lb; l < pc.le; l++) {
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
                const long long key = (long long)(l - pc.lb) * 1000000007LL + ri.round;
                const bool lower = p < dpos[(size_t)i];
                for (int attempt = 0; attempt < 2; attempt++) {
                    fresh.clear();
                    fepoch++;
                    ipairs.clear();
                    rstart = key != last_round_key ? (int)o.items.size() - ch.i0
                                                   : (o.rounds.back() & ~rsp::kRndLevelStart);
                    const int po = pair_off(i);
                    for (int u = sym.upd_ptr[(size_t)p]; u < sym.upd_ptr[(size_t)p + 1]; u++) {
                        const int lc = ref(sym.upd_l[(size_t)(u + po)], fresh), uc = ref(sym.upd_u[(size_t)(u + po)], fresh);
                        ipairs.push_back(lc | uc << 16);
                    }
                    int d = -1;
                    if (lower) {
                        const int k = ci[(size_t)p];
                        d = hasdiag[(size_t)k] ? ref(dpos[(size_t)k], fresh) : kZero;
                    }
                    const int slot = (int)o.items.size() - ch.i0;
                    const bool new_round = key != last_round_key;
                    const bool fits = slot < K && (int)(o.pairs.size() - ch.p0 + ipairs.size()) <= rsp::kRndPairs &&
                                      nstg + (int)fresh.size() <= S &&
                                      (int)(o.rounds.size() - ch.r0) + (new_round ? 1 : 0) <= rsp::kRndRounds;
                    if (!fits && attempt == 0 && slot > 0) {
                        close_chunk();
                        open_chunk();
                        last_round_key = -1;
                        last_round_level = -1;
                        continue;
                    }
                    for (int q : fresh) {
                        hput(q, nstg++);
                        o.staged.push_back(q);
                    }
                    if (new_round) {  // flagged where it opens a level in this chunk
                        o.rounds.push_back(slot | (l != last_round_level ? rsp::kRndLevelStart : 0));
                        last_round_key = key;
                        last_round_level = l;
                    }
                    const int pstart = (int)o.pairs.size() - ch.p0;
                    o.pairs.insert(o.pairs.end(), ipairs.begin(), ipairs.end());
                    const int zr = (!lower && p == dpos[(size_t)i] && hasdiag[(size_t)i]) ? i : -1;
                    o.items.push_back({p, pstart | (int)ipairs.size() << 16, d, zr});
                    __atomic_store_n(&where[(size_t)p], ckey << 12 | (unsigned long long)slot, __ATOMIC_RELAXED);
                    break;
                }
            }
        }
        close_chunk();
    });
    const double t_pieces = now_ms() - t0;
    // join: pieces in order, an empty chunk between two pieces of a segment
    fp.chunks.clear();
    fp.items.clear();
    fp.pairs.clear();
    fp.staged.clear();
    fp.rounds.clear();
    size_t ni = 0, np = 0, ns = 0, nr = 0, nc = 0;
    for (const Piece &pc : pieces) {
        ni += pc.out.items.size();
        np += pc.out.pairs.size();
        ns += pc.out.staged.size();
        nr += pc.out.rounds.size();
        nc += pc.out.chunks.size() + 1;
    }
    fp.items.reserve(ni);
    fp.pairs.reserve(np);
    fp.staged.reserve(ns);
    fp.rounds.reserve(nr);
    fp.chunks.reserve(nc);
    for (size_t q = 0; q < pieces.size(); q++) {
        const Piece &pc = pieces[q];
        rsp::LevelSeg &sg = fp.segs[(size_t)pc.seg];
        const int bi = (int)fp.items.size(), bp = (int)fp.pairs.size(), bs = (int)fp.staged.size(),
                  br = (int)fp.rounds.size();
        if (q == 0 || pieces[q - 1].seg != pc.seg)
            sg.c0 = (int)fp.chunks.size();
        else
            fp.chunks.push_back(rsp::RndChunk{bi, bi, bp, bp, bs, bs, br, br});  // the separator
        for (rsp::RndChunk r : pc.out.chunks) {
            r.i0 += bi, r.i1 += bi, r.p0 += bp, r.p1 += bp, r.s0 += bs, r.s1 += bs, r.r0 += br, r.r1 += br;
            fp.chunks.push_back(r);
        }
        fp.items.insert(fp.items.end(), pc.out.items.begin(), pc.out.items.end());
        fp.pairs.insert(fp.pairs.end(), pc.out.pairs.begin(), pc.out.pairs.end());
        fp.staged.insert(fp.staged.end(), pc.out.staged.begin(), pc.out.staged.end());
        fp.rounds.insert(fp.rounds.end(), pc.out.rounds.begin(), pc.out.rounds.end());
        sg.c1 = (int)fp.chunks.size();
    }
    if (fp.items.empty()) fp.items.push_back({0, 0, -1, -1});
    for (hvec<int> *v : {&fp.pairs, &fp.staged, &fp.rounds})
        if (v->empty()) v->push_back(0);
    if (fp.chunks.empty()) fp.chunks.push_back(rsp::RndChunk{});
    if (env_int("RSP_ILU_TIMING", 0) >= 3)
        fprintf(stderr, "rsp_ilu0_analysis n=%d     factor plan: thin levels %.2f where %.2f pieces (%zu) %.2f join %.2f ms\n",
                n, t_thin, t_where, pieces.size(), t_pieces, now_ms() - t0);
}

// Symbolic ILU(0): the update list of every position (see IluArgs) and the
// intra-row stages of the lower positions. Row i is scattered into a dense
// column -> position map, then each lower k (ascending) walks row k's upper
// part; a hit at column j appends (pos l_ik, pos u_kj) to position (i, j).

static bool ilu_symbolic(int n, const hvec<int> &rp, const hvec<int> &ci,
                         const hvec<int> &dpos, const hvec<int> &hasdiag,
                         IluSymbolic &s) {
    const int nnz = rp[(size_t)n];
    hvec<int> cnt((size_t)nnz, 0);
    // pass 1: counts (rows are independent: a row writes only its own
    // positions' counts; each worker scatters its rows into its own map)
    std::mutex mu;
    long long total = 0;
    parallel_rows(n, [&](int r0, int r1) {
        hvec<int> map((size_t)n, -1);
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
    hvec<int> &stage = s.stage;
    stage.assign((size_t)nnz, 0);
    s.lord.assign((size_t)nnz, 0);
    s.lend.assign((size_t)nnz, 0);
    parallel_rows(n, [&](int r0, int r1) {
        hvec<int> map((size_t)n, -1), order;
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

static void symbolic_row(int i, std::vector<int> &map, std::vector<int> &cur, std::vector<int> &order,
                         const int *rp, const int *ci, const int *dpos, const int *hasdiag, int *cnt,
                         const int *ptr, int *upd_l, int *upd_u, int *stage, int *lord, int *lend, int *udiv);

// The symbolic factor of a few given rows on the host (the device analysis
// leaves its long rows here: a hub row's lower positions form a long serial
// chain that one GPU lane walks at global-memory latency, where the host
// walks it in cache). cnt != nullptr: update-list counts of the rows'
// positions; else the pairs at ptr, the stages, the stage order and the
// divisor positions — every value exactly as ilu_symbolic / plan_symbolic.
void symbolic_rows(const hvec<int> &rows, int n, const int *rp, const int *ci, const int *dpos,
                   const int *hasdiag, int *cnt, const int *ptr, int *upd_l, int *upd_u, int *stage, int *lord,
                   int *lend, int *udiv) {
    if (rows.empty()) return;
    // rows in parallel (each writes only its own positions and update-list
    // slots; round 5: the hub rows were one sequential pass, ~1-1.7 ms per
    // circuit, twice), in blocks of rows: a block has ONE column map of n
    // entries, reset after each row at the row's own columns only, so the
    // pass stays O(nnz of the rows' DAG) plus O(n) per block (a map per row
    // cost O(n) per long row: quadratic on patterns with many long rows)
    const int nr = (int)rows.size();
    const int nblk = std::max(1, std::min(nr, 2 * host_threads()));
    pfor_dyn(nblk, (long long)nr << 14, 1 << 14, [&](int b) {
        std::vector<int> map((size_t)n, -1), cur, order;
        for (int ri = (int)((long long)nr * b / nblk); ri < (int)((long long)nr * (b + 1) / nblk); ri++)
            symbolic_row(rows[(size_t)ri], map, cur, order, rp, ci, dpos, hasdiag, cnt, ptr, upd_l, upd_u, stage,
                         lord, lend, udiv);
    });
}

// One row of symbolic_rows; `map` is all -1 on entry and on return.
static void symbolic_row(int i, std::vector<int> &map, std::vector<int> &cur, std::vector<int> &order,
                         const int *rp, const int *ci, const int *dpos, const int *hasdiag, int *cnt,
                         const int *ptr, int *upd_l, int *upd_u, int *stage, int *lord, int *lend, int *udiv) {
    {
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
        if (cnt) return;
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
    const hvec<int> &dpos = hp.dpos, &hasdiag = hp.hasdiag;
    hvec<int> lvu((size_t)n, 0);
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
    hvec<int> udiag((size_t)n);
    for (int i = 0; i < n; i++) udiag[(size_t)i] = hasdiag[(size_t)i] ? dpos[(size_t)i] : -1;
    const int thin_solve = std::min(env_int("RSP_ILU_THIN_SOLVE", rsp::kThinSolveRows), rsp::kThinThreads);
    build_solve_plan(n, hp.U.ptr, hp.U.rows, thin_solve, hp.U.group, udiag,
                     [&](int i) { return rp[(size_t)i + 1] - dpos[(size_t)i] - hasdiag[(size_t)i]; },
                     [&](int i, auto emit) {
        for (int p = dpos[(size_t)i] + hasdiag[(size_t)i]; p < rp[(size_t)i + 1]; p++) emit(p, ci[(size_t)p]);
    }, [](int) { return 0; }, hp.U.sp);  // (the U solve keeps the reference order: no split)
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
    hvec<int> &dpos = hp.dpos, &hasdiag = hp.hasdiag;
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

// The split term order of both solve DAGs (IluHostPlan::lpos): per row, its
// early terms, then its late ones (producer one level below the row's), each
// part in the reference's order; a stable partition per row, rows in
// parallel. (The oracle restates it: rsp_oracle.c ORACLE_TRSV_SPLIT.)
static void split_terms(const int *rp, const int *ci, IluHostPlan &hp) {
    const int n = hp.n;
    const hvec<int> &dpos = hp.dpos, &lv = hp.lev_l, &lvt = hp.lev_lt;
    if (!hp.split) {  // the reference's order: every term "late", none moved. Left
        // empty (identity order, no early terms: the consumers treat an empty
        // lpos / ne as that) instead of materialised: the fill was 1-4 ms of
        // the level phase on the 1 M-row patterns (round 5)
        hp.lpos.clear();
        hp.ne_l.clear();
        hp.ne_lt.clear();
        return;
    }
    hp.lpos.assign((size_t)std::max(hp.nnz_s, 1), 0);
    hp.ne_l.assign((size_t)std::max(n, 1), 0);
    hp.ne_lt.assign((size_t)std::max(n, 1), 0);
    parallel_rows(n, [&](int r0, int r1) {
        hvec<int> late, late_c;
        for (int i = r0; i < r1; i++) {
            // L: row i reads y_j, j = ci[p] < i
            int k = rp[i];
            late.clear();
            for (int p = rp[i]; p < dpos[(size_t)i]; p++) {
                if (lv[(size_t)ci[p]] == lv[(size_t)i] - 1)
                    late.push_back(p);
                else
                    hp.lpos[(size_t)k++] = p;
            }
            hp.ne_l[(size_t)i] = k - rp[i];
            for (int p : late) hp.lpos[(size_t)k++] = p;
            // L^T: row i reads y_j, j = ltc[q] > i, q in [ltp[i], ltp[i+1])
            const int q0 = hp.ltp[(size_t)i], q1 = hp.ltp[(size_t)i + 1];
            late.clear();
            late_c.clear();
            int w = q0;
            for (int q = q0; q < q1; q++) {
                const int j = hp.ltc[(size_t)q], tp = hp.lts[(size_t)q];
                if (lvt[(size_t)j] == lvt[(size_t)i] - 1) {
                    late.push_back(tp);
                    late_c.push_back(j);
                } else {
                    hp.lts[(size_t)w] = tp;
                    hp.ltc[(size_t)w++] = j;
                }
            }
            hp.ne_lt[(size_t)i] = w - q0;
            for (size_t u = 0; u < late.size(); u++) {
                hp.lts[(size_t)w] = late[u];
                hp.ltc[(size_t)w++] = late_c[u];
            }
        }
    });
}

// The lower DAG's levels (factor + L solve): the longest path ending at each
// row (each row needs its producers'). rsp_ilu0_analysis waits for these only.
void plan_levels_lower(const int *rp, const int *ci, IluHostPlan &hp) {
    const int n = hp.n;
    const hvec<int> &dpos = hp.dpos;
    const double t0 = now_ms();
    hvec<int> &lv = hp.lev_l;
    lv.assign((size_t)n, 0);
    int nl = n > 0 ? 1 : 0;
    for (int i = 0; i < n; i++) {
        int l = 0;
        for (int p = rp[i]; p < dpos[(size_t)i]; p++) l = std::max(l, lv[(size_t)ci[p]] + 1);
        lv[(size_t)i] = l;
        nl = std::max(nl, l + 1);
    }
    group_levels(lv, nl, hp.L.ptr, hp.L.rows);
    if (env_int("RSP_ILU_TIMING", 0) >= 3)
        fprintf(stderr, "rsp_ilu0_analysis n=%d     levels: L %.2f ms\n", n, now_ms() - t0);
}

// The solves-only half of the level analysis: the L^T DAG's levels and the
// transposed strict lower part (two independent passes, run concurrently:
// each is memory-latency bound), then the split term order. Round 6: started
// by the solve plans' thread, so the analysis proper (the reference's
// csrilu02_analysis) no longer waits for it. The split order reads the L
// levels too: with split = false it is left to the caller (plan_levels).
void plan_levels_upper(const int *rp, const int *ci, IluHostPlan &hp, bool split) {
    const int n = hp.n;
    hp.split = env_int("RSP_ILU_SPLIT", 0) != 0;
    const hvec<int> &dpos = hp.dpos;
    const double t0 = now_ms();
    double t_lt = 0, t_tr = 0;  // diagnostics (RSP_ILU_TIMING >= 3): each pass's wall time
    // levels of the L^T DAG: row i waits for every j > i with l_ji != 0
    Task tt([&] {
        hvec<int> &lvt = hp.lev_lt;
        lvt.assign((size_t)n, 0);
        int nlt = n > 0 ? 1 : 0;
        for (int j = n - 1; j >= 0; j--) {
            nlt = std::max(nlt, lvt[(size_t)j] + 1);
            for (int p = rp[j]; p < dpos[(size_t)j]; p++) {
                const int k = ci[p];
                lvt[(size_t)k] = std::max(lvt[(size_t)k], lvt[(size_t)j] + 1);
            }
        }
        group_levels(lvt, nlt, hp.LT.ptr, hp.LT.rows);
        t_lt = now_ms() - t0;
    });
    // transposed strict lower: row k lists (j, pos) for l_jk, j descending.
    // Rows in parallel: counts and slots by relaxed atomics, then each
    // column's slots sorted by j (descending; one entry per j, so the order
    // is unique whatever the interleaving). Round 5: the sequential form was
    // the level phase's longest pass (tmt_unsym 9.4 ms against 4.4 / 4.6 ms
    // for the two level passes).
    hvec<int> &ltp = hp.ltp, &lts = hp.lts, &ltc = hp.ltc;
    ltp.assign((size_t)n + 1, 0);
    parallel_rows(n, [&](int r0, int r1) {
        for (int j = r0; j < r1; j++)
            for (int p = rp[j]; p < dpos[(size_t)j]; p++) __atomic_fetch_add(&ltp[(size_t)ci[p] + 1], 1, __ATOMIC_RELAXED);
    });
    for (int k = 0; k < n; k++) ltp[(size_t)k + 1] += ltp[(size_t)k];
    lts.resize((size_t)ltp[(size_t)n]);
    ltc.resize((size_t)ltp[(size_t)n]);
    {
        hvec<int> fill(ltp.begin(), ltp.end() - 1);
        parallel_rows(n, [&](int r0, int r1) {
            for (int j = r0; j < r1; j++)
                for (int p = rp[j]; p < dpos[(size_t)j]; p++) {
                    const int slot = __atomic_fetch_add(&fill[(size_t)ci[p]], 1, __ATOMIC_RELAXED);
                    lts[(size_t)slot] = p;
                    ltc[(size_t)slot] = j;
                }
        });
    }
    parallel_rows(n, [&](int k0, int k1) {
        std::vector<std::pair<int, int>> tmp;
        for (int k = k0; k < k1; k++) {
            const int a = ltp[(size_t)k], b = ltp[(size_t)k + 1];
            if (b - a <= 32) {  // insertion sort, j descending
                for (int x = a + 1; x < b; x++) {
                    const int cj = ltc[(size_t)x], cp = lts[(size_t)x];
                    int y = x - 1;
                    for (; y >= a && ltc[(size_t)y] < cj; y--) {
                        ltc[(size_t)y + 1] = ltc[(size_t)y];
                        lts[(size_t)y + 1] = lts[(size_t)y];
                    }
                    ltc[(size_t)y + 1] = cj;
                    lts[(size_t)y + 1] = cp;
                }
            } else {
                tmp.resize((size_t)(b - a));
                for (int x = a; x < b; x++) tmp[(size_t)(x - a)] = {ltc[(size_t)x], lts[(size_t)x]};
                std::sort(tmp.begin(), tmp.end(), [](const std::pair<int, int> &u, const std::pair<int, int> &v) {
                    return u.first > v.first;
                });
                for (int x = a; x < b; x++) {
                    ltc[(size_t)x] = tmp[(size_t)(x - a)].first;
                    lts[(size_t)x] = tmp[(size_t)(x - a)].second;
                }
            }
        }
    });
    t_tr = now_ms() - t0;
    tt.join();
    const double t_j = now_ms() - t0;
    if (split) split_terms(rp, ci, hp);
    if (env_int("RSP_ILU_TIMING", 0) >= 3)
        fprintf(stderr, "rsp_ilu0_analysis n=%d     levels: LT %.2f transpose %.2f joined %.2f split %.2f ms\n",
                n, t_lt, t_tr, t_j, now_ms() - t0 - t_j);
}

void plan_levels(const int *rp, const int *ci, IluHostPlan &hp) {
    hp.split = env_int("RSP_ILU_SPLIT", 0) != 0;
    Task tl([&] { plan_levels_lower(rp, ci, hp); });
    plan_levels_upper(rp, ci, hp, false);
    tl.join();
    split_terms(rp, ci, hp);
}

rsp_status_t plan_symbolic(const int *rpp, const int *cip, IluHostPlan &hp) {
    const int n = hp.n;
    const hvec<int> rp(rpp, rpp + (size_t)n + 1), ci(cip, cip + (size_t)hp.nnz_s);
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

static void timed_plan(int n, const char *what, const std::function<void()> &fn) {
    const double t0 = now_ms();
    fn();
    if (env_int("RSP_ILU_TIMING", 0) >= 2)  // diagnostics: per-plan wall time
        fprintf(stderr, "rsp_ilu0_analysis n=%d   plan %-10s %8.2f ms\n", n, what, now_ms() - t0);
}

// RSP_ILU_THIN_SOLVE / RSP_ILU_THIN_FACTOR: tuning knobs (0 = no thin runs)
static int thin_solve_rows() {
    return std::min(env_int("RSP_ILU_THIN_SOLVE", rsp::kThinSolveRows), rsp::kThinThreads);
}

// The L and L^T solve plans; terms_on_host = false builds only the per-row
// half (the device analysis builds the per-term half on the MI355X:
// rsp_k::ilu_an_solve_terms).
static void plan_solves_impl(const int *rp, const int *ci, IluHostPlan &hp, bool terms_on_host) {
    const int n = hp.n;
    const hvec<int> &dpos = hp.dpos;
    const hvec<int> &ltp = hp.ltp, &lts = hp.lts, &ltc = hp.ltc;
    const int thin_solve = thin_solve_rows();
    long long nlo = 0;
    for (int i = 0; i < n; i++) nlo += dpos[(size_t)i] - rp[(size_t)i];
    hp.L.batch = hp.LT.batch = chain_batch(nlo, n);
    auto cnt_l = [&](int i) { return dpos[(size_t)i] - rp[(size_t)i]; };
    auto cnt_lt = [&](int i) { return ltp[(size_t)i + 1] - ltp[(size_t)i]; };
    // thin-run term groups, per DAG. Reference order (default): 2 only where
    // groups of 4 would save almost no groups (sum ceil(c/2) <= 1.15 sum
    // ceil(c/4): chains of <= 2 terms, the 2-D grids), else 4 — a circuit's
    // short mean chain hides hub rows of thousands of terms (config 3, same
    // box: G2_circuit solve 3.21 -> 2.66 ms, ASIC_320ks 1.52 -> 1.31, ss1
    // 1.34 -> 1.16 against the round-3 rule of 2 for every DAG of mean chain
    // <= 2.5; ecology2 / tmt_unsym keep 2: 4.26 / 4.22 against 4.49 / 4.45 ms
    // with 4; profiles/r04_ilu_group_ab.txt). Split order (RSP_ILU_SPLIT=1):
    // 2 where a row's two parts are short on average (mean chain <= 5 terms).
    auto group_of = [&](auto cnt) {
        if (hp.split) return n > 0 && (double)nlo / n <= 5.0 ? 2 : 4;
        long long s2 = 0, s4 = 0;
        for (int i = 0; i < n; i++) {
            const int c = cnt(i);
            s2 += (c + 1) / 2;
            s4 += (c + 3) / 4;
        }
        return 100 * s2 <= 115 * s4 ? 2 : 4;
    };
    const int g_env = env_int("RSP_ILU_GROUP", 0);
    hp.L.group = g_env ? (g_env == 2 ? 2 : 4) : group_of(cnt_l);
    hp.LT.group = g_env ? (g_env == 2 ? 2 : 4) : group_of(cnt_lt);
    // split term order (IluHostPlan::lpos): early terms first
    // (empty: the reference's order, split_terms)
    auto ne_l = [&](int i) { return hp.ne_l.empty() ? 0 : hp.ne_l[(size_t)i]; };
    auto ne_lt = [&](int i) { return hp.ne_lt.empty() ? 0 : hp.ne_lt[(size_t)i]; };
    // the two DAGs' plans (flat terms in level order, thin-run chunks, y
    // sources) are independent: built concurrently
    Task tl([&] {
        timed_plan(n, "L", [&] {
            solve_plan_rows(n, hp.L.ptr, hp.L.rows, thin_solve, hp.L.group, hvec<int>(), cnt_l, ne_l, hp.L.sp);
            if (terms_on_host)
                solve_plan_terms(n, hp.L.ptr, hp.L.group, [&](int i, auto emit) {
                    for (int o = rp[(size_t)i]; o < dpos[(size_t)i]; o++) {
                        const int p = hp.lpos.empty() ? o : hp.lpos[(size_t)o];
                        emit(p, ci[(size_t)p]);
                    }
                }, ne_l, hp.L.sp);
        });
    });
    timed_plan(n, "LT", [&] {
        solve_plan_rows(n, hp.LT.ptr, hp.LT.rows, thin_solve, hp.LT.group, hvec<int>(), cnt_lt, ne_lt, hp.LT.sp);
        if (terms_on_host)
            solve_plan_terms(n, hp.LT.ptr, hp.LT.group, [&](int i, auto emit) {
                for (int q = ltp[(size_t)i]; q < ltp[(size_t)i + 1]; q++) emit(lts[(size_t)q], ltc[(size_t)q]);
            }, ne_lt, hp.LT.sp);
    });
    tl.join();
    hp.L.planned = hp.LT.planned = true;
}

void plan_solves(const int *rp, const int *ci, IluHostPlan &hp) { plan_solves_impl(rp, ci, hp, true); }
void plan_solves_rows(const int *rp, const int *ci, IluHostPlan &hp) { plan_solves_impl(rp, ci, hp, false); }

void plan_factor(const int *rp, const int *ci, long long slot_cap, IluHostPlan &hp) {
    const int n = hp.n, nnz_s = hp.nnz_s;
    const hvec<int> &dpos = hp.dpos, &hasdiag = hp.hasdiag;
    const int thin_factor = thin_factor_rows();
    IluSymbolic &sym = hp.sym;
    hp.fac_batch = chain_batch((long long)sym.upd_ptr[(size_t)nnz_s], nnz_s);
    // No update pairs at all (a stored lower triangle): the factor is
    // l_ik = a_ik / a_kk for every lower position and nothing else, and the
    // a_kk are never written with other bits, so every row goes in ONE level
    // (IluHostPlan::F) instead of the L DAG's — for G2_circuit 5 799 levels.
    // The positions' arithmetic is unchanged (same division, same operands):
    // same bits. In that level a row may read a u_kk that the row k's own
    // work item rewrites concurrently with identical bits (fat kernels) or
    // that a thin run has not placed yet (its rounds are in order: lower
    // items in round 0, a row's diagonal in round 1, so a round-0 item finds
    // the divisor "not here" and stages the input). No flow run (one level).
    // RSP_ILU_FAC_ONE=0 keeps L's levels (A/B).
    hp.fac_one = n > 0 && sym.upd_ptr[(size_t)nnz_s] == 0 && env_int("RSP_ILU_FAC_ONE", 1) != 0;
    if (hp.fac_one) {
        hp.F.ptr = hvec<int>{0, n};
        hp.F.rows.resize((size_t)n);
        pfor(n, 1 << 16, [&](long long a, long long b) {
            for (long long x = a; x < b; x++) hp.F.rows[(size_t)x] = (int)x;
        });
    } else {
        hp.F = DagHost();
    }
    hp.fac_scale = hp.fac_one && env_int("RSP_ILU_FAC_SCALE", 1) != 0;
    if (hp.fac_scale) {  // ilu0_scale_lower needs no plan
        hp.fplan = FacPlan();
        hp.frow.assign(1, rsp::FacRow{});
        hp.fslev.clear();
        hp.slot_desc.clear();
        hp.slot_offs.clear();
        hp.slot_total = 0;
        hp.fruns.clear();
        hp.ffitems.assign(1, rsp::FacFlowItem{0, 0, -1});
        return;
    }
    const hvec<int> &lp = hp.fac_one ? hp.F.ptr : hp.L.ptr;
    const hvec<int> &rows_l = hp.fac_one ? hp.F.rows : hp.L.rows;
    timed_plan(n, "factor", [&] {
        build_factor_plan(n, rp, ci, dpos, hasdiag, sym, lp, rows_l, thin_factor, hp.fplan);
    });
    const long long nx = (long long)rows_l.size();
    hp.frow.assign(std::max<size_t>(rows_l.size(), 1), rsp::FacRow{});
    pfor(nx, 1 << 14, [&](long long a, long long b) {
        for (long long x = a; x < b; x++) {
            const int i = rows_l[(size_t)x], rs = rp[(size_t)i], re = rp[(size_t)i + 1];
            hp.frow[(size_t)x] = rsp::FacRow{i, rs, dpos[(size_t)i], re, sym.upd_ptr[(size_t)rs],
                                             sym.upd_ptr[(size_t)re], hasdiag[(size_t)i], 0};
        }
    });
    // fat factor levels in the slot layout (rsp::FacSlotLevel): each row's
    // structure at a fixed stride, so ilu0_level_slot reads it in one round
    // trip. A level whose padded slots would take more than twice its rows'
    // own structure (one large row among many small ones), or past the
    // budget, keeps the FacRow path. Per level (parallel): the largest
    // LDS-path row and pair count, the rows' own structure size, whether
    // every row fits the LDS path (flow runs); then the offsets in order.
    const int nlev = (int)lp.size() - 1;
    hp.fslev.assign((size_t)std::max(nlev, 0), rsp::FacSlotLevel{0, 0, 0, 0, 0});
    struct LevStat {
        int rm, qm, all_lds, fat;
        long long own;
    };
    hvec<LevStat> ls((size_t)std::max(nlev, 1), LevStat{0, 0, 0, 0, 0});
    for (const rsp::LevelSeg &sg : hp.fplan.segs)
        if (!sg.thin)
            for (int l = sg.lb; l < sg.le; l++) ls[(size_t)l].fat = 1;
    pfor_dyn(nlev, nx, 1 << 14, [&](int l) {
        LevStat &st = ls[(size_t)l];
        if (!st.fat) return;
        st.all_lds = 1;
        for (int x = lp[(size_t)l]; x < lp[(size_t)l + 1]; x++) {
            const rsp::FacRow &fr = hp.frow[(size_t)x];
            const int nr = fr.re - fr.rs, nq = fr.q1 - fr.q0;
            if (nr <= rsp::kFacRow && nq <= rsp::kFacPairs) {
                st.rm = std::max(st.rm, nr);
                st.qm = std::max(st.qm, nq);
            } else {
                st.all_lds = 0;
            }
            st.own += (rsp::fac_pairs_at(std::min(nr, rsp::kFacRow)) + 2 * std::min(nq, rsp::kFacPairs) + 3) & ~3;
        }
    });
    long long total = 0;
    hvec<int> slot_levels;
    // RSP_ILU_SLOT_PAD: A/B knob, the padded size a level may take over its
    // rows' own structure (2 / 4 / 16: config-3 fp64 factor 58.6 / 58.7 /
    // 58.6 ms; the ~280 single fat levels per run left on the FacRow path
    // are hub-row levels, not padding-dominated ones)
    const long long pad_ratio = std::max(1, env_int("RSP_ILU_SLOT_PAD", 2));
    for (int l = 0; l < nlev; l++) {
        const LevStat &st = ls[(size_t)l];
        if (!st.fat || st.rm == 0) continue;
        // a level without update pairs keeps one (padding) pair slot per row:
        // the kernels' pair loads are clamped to the level's qm - 1
        const int qm = std::max(st.qm, 1);
        const int stride = (rsp::fac_pairs_at(st.rm) + 2 * qm + 3) & ~3;
        const long long cnt = lp[(size_t)l + 1] - lp[(size_t)l];
        if (cnt * stride > pad_ratio * st.own) continue;  // padding would dominate
        if (total + cnt * stride > slot_cap) continue;
        hp.fslev[(size_t)l] = rsp::FacSlotLevel{total, stride, st.rm, qm, 0};
        total += cnt * stride;
        slot_levels.push_back(l);
    }
    hp.slot_total = total;
    // flow runs: maximal runs of >= 2 slot-layout fat levels without
    // global-path rows; items in level order, gated like the solve's
    hp.fruns.clear();
    hp.ffitems.clear();
    if (env_int("RSP_ILU_FLOW_PLAN", 1) != 0) {
        const int gate_d = env_int("RSP_ILU_FLOW_GATE", 3);
        auto flowable = [&](int l) { return hp.fslev[(size_t)l].stride > 0 && ls[(size_t)l].all_lds; };
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
                    const int c0 = hp.fruns.empty() ? 0 : hp.fruns.back().c1;
                    hp.fruns.push_back(rsp::FacFlowRun{l, e, c0, c0 + lp[(size_t)e] - lp[(size_t)l]});
                }
                l = e;
            }
        }
        hp.ffitems.resize(hp.fruns.empty() ? 0 : (size_t)hp.fruns.back().c1);
        for (const rsp::FacFlowRun &r : hp.fruns)
            pfor_dyn(r.le - r.lb, lp[(size_t)r.le] - lp[(size_t)r.lb], 1 << 14, [&](int j) {
                const int v = r.lb + j;
                const rsp::FacSlotLevel &sl = hp.fslev[(size_t)v];
                const int lg = v - gate_d;
                const int gate = gate_d > 0 && lg >= r.lb && lp[(size_t)lg + 1] > lp[(size_t)lg]
                                     ? rows_l[(size_t)lp[(size_t)lg + 1] - 1] : -1;
                for (int x = lp[(size_t)v]; x < lp[(size_t)v + 1]; x++)
                    hp.ffitems[(size_t)(r.c0 + x - lp[(size_t)r.lb])] =
                        rsp::FacFlowItem{sl.off + (long long)(x - lp[(size_t)v]) * sl.stride, sl.rm | sl.qm << 16, gate};
            });
    }
    if (hp.ffitems.empty()) hp.ffitems.push_back({0, 0, -1});  // keep the device array non-empty
    hvec<long long> sd0(slot_levels.size() + 1, 0);
    for (size_t j = 0; j < slot_levels.size(); j++)
        sd0[j + 1] = sd0[j] + lp[(size_t)slot_levels[j] + 1] - lp[(size_t)slot_levels[j]];
    hp.slot_desc.resize((size_t)sd0.back());
    hp.slot_offs.resize((size_t)sd0.back());
    pfor_dyn((int)slot_levels.size(), sd0.back(), 1 << 14, [&](int j) {
        const int l = slot_levels[(size_t)j];
        const rsp::FacSlotLevel &sl = hp.fslev[(size_t)l];
        for (int x = lp[(size_t)l]; x < lp[(size_t)l + 1]; x++) {
            const size_t o = (size_t)(sd0[(size_t)j] + x - lp[(size_t)l]);
            hp.slot_desc[o] = int4{x, sl.rm, sl.qm, 0};
            hp.slot_offs[o] = sl.off + (long long)(x - lp[(size_t)l]) * sl.stride;
        }
    });
}


void plan_rest(const int *rp, const int *ci, long long slot_cap, bool want_u, IluHostPlan &hp) {
    Task ts([&] {
        plan_solves(rp, ci, hp);
        if (want_u) plan_u(rp, ci, hp);
    });
    plan_factor(rp, ci, slot_cap, hp);
    ts.join();
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
    // the plans see what they see after the device analysis: no host copy of
    // the stage order, stage ends or divisor positions (kept for the digest)
    hvec<int> lord, lend, udiv;
    lord.swap(hp.sym.lord);
    lend.swap(hp.sym.lend);
    udiv.swap(hp.udiv);
    // ... and, like it, only the thin rows' update pairs, packed (the full
    // lists are kept for the digest)
    hvec<int> upd_l, upd_u;
    if (env_int("RSP_ILU_PACK_PAIRS", 1)) {
        const hvec<int> trows = factor_thin_rows(rp, hp);
        hvec<int> pl, pu;
        hp.sym.pair_base.assign((size_t)std::max(n, 1), 0);
        for (int i : trows) {
            hp.sym.pair_base[(size_t)i] = (int)pl.size();
            for (int q = hp.sym.upd_ptr[(size_t)rp[i]]; q < hp.sym.upd_ptr[(size_t)rp[i + 1]]; q++) {
                pl.push_back(hp.sym.upd_l[(size_t)q]);
                pu.push_back(hp.sym.upd_u[(size_t)q]);
            }
        }
        upd_l.swap(hp.sym.upd_l);
        upd_u.swap(hp.sym.upd_u);
        hp.sym.upd_l.swap(pl);
        hp.sym.upd_u.swap(pu);
    }
    plan_rest(rp, ci, slot_cap, want_u, hp);
    // block-inverse plans of the deep DAGs (as rsp_ilu0_analysis)
    if (blocks_wanted(n, (int)hp.L.ptr.size() - 1)) hp.has_lb = plan_blocks(0, rp, ci, hp, hp.Lb);
    if (blocks_wanted(n, (int)hp.LT.ptr.size() - 1)) hp.has_ltb = plan_blocks(1, rp, ci, hp, hp.LTb);
    lord.swap(hp.sym.lord);
    lend.swap(hp.sym.lend);
    udiv.swap(hp.udiv);
    if (!hp.sym.pair_base.empty()) {
        hp.sym.pair_base.clear();
        hp.sym.upd_l.swap(upd_l);
        hp.sym.upd_u.swap(upd_u);
    }
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
    void vec(const hvec<V> &v) {
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
    for (const BlkPlanHost *b : {&hp.Lb, &hp.LTb}) {
        f.bytes(&b->nb, sizeof(b->nb));
        f.bytes(&b->lds_elems, sizeof(b->lds_elems));
        f.bytes(&b->lds_words, sizeof(b->lds_words));
        f.vec(b->order);
        f.vec(b->desc);
        f.vec(b->rows);
        f.vec(b->ref);
        f.vec(b->vpos);
        f.vec(b->eord);
        f.vec(b->lptr);
        f.vec(b->rptr);
        f.vec(b->rit);
        f.vec(b->segs);
    }
    f.bytes(&hp.fac_one, sizeof(hp.fac_one));
    f.bytes(&hp.fac_scale, sizeof(hp.fac_scale));
    f.vec(hp.F.ptr);
    f.vec(hp.F.rows);
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
