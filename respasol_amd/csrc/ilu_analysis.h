// ilu_analysis.h — host half of the ILU(0) analysis (rsp_ilu0_analysis, the
// reference's csrilu02_analysis + 2x csrsv2_analysis, GPU/ilu0.cu:196-252):
// validation, diagonal positions, level sets of the L / L^T / U DAGs, the
// symbolic factor (update lists, intra-row stages) and the launch plans of
// the factor and the solves. Pure host C++ (no HIP calls): rsp_api.cpp
// downloads the pattern, calls plan_host and uploads the result in one
// arena; rsp_ilu0_analysis_host runs it on host arrays (tests, profiling).
#ifndef RSP_ILU_ANALYSIS_H
#define RSP_ILU_ANALYSIS_H

#include <stdint.h>
#include <stdlib.h>

#include <exception>
#include <functional>
#include <thread>
#include <utility>
#include <vector>

#include "rsp.h"
#include "host_pool.h"
#include "rsp_kernels.h"

namespace rsp_an {

// A helper thread of the analysis whose exception (std::bad_alloc from the
// pool, say) is carried to join(), which rethrows it in the caller; the
// destructor joins too, so a caller that unwinds first never leaves it
// running over the caller's locals (nor calls std::terminate).
class Task {
    std::exception_ptr err_;
    std::thread t_;

  public:
    template <typename F>
    explicit Task(F f) : t_([this, f] {
          try {
              f();
          } catch (...) {
              err_ = std::current_exception();
          }
      }) {}
    Task(const Task &) = delete;
    Task &operator=(const Task &) = delete;
    void join() {
        if (t_.joinable()) t_.join();
        if (err_) std::rethrow_exception(std::exchange(err_, nullptr));
    }
    ~Task() {
        if (t_.joinable()) t_.join();
    }
};

inline int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

struct SolvePlan {
    hvec<int> sbase;   // per level: first flat term of its padded short rows, -1 = none
    hvec<int> nshort;  // per level
    hvec<int> nwave;   // per level: short + wave rows (the rest: hub rows)
    hvec<rsp::RowTask> tasks;
    hvec<int> tpos, src;
    hvec<rsp::LevelSeg> segs;
    hvec<rsp::LevelChunk> chunks;
    hvec<rsp::ThinRowPlan> trow;
    hvec<int> sid;
    hvec<rsp::StagedTerm> stg;
    hvec<rsp::FlowItem> fitems;  // flow segments' work items (LevelSeg c0 / c1 of a fat segment)
    hvec<int> cbase;  // per chunk: its thin run's first slot (not in the digest: derived)
    int nterm = 0;           // flat terms (tpos.size() once the terms are built; >= 1 then)
};

// Symbolic ILU(0) data (built by ilu_symbolic below).
struct IluSymbolic {
    hvec<int> upd_ptr, upd_l, upd_u, lord, lend;
    hvec<int> stage;  // per lower position: its intra-row stage
    // empty: upd_l / upd_u hold every pair (indexed as upd_ptr). Else only
    // the pairs of the rows of the factor's thin levels, packed: row i's pair
    // u at pair_base[i] + u - upd_ptr[rowptr[i]] (the device analysis
    // downloads no more; the factor plan reads no other row's pairs).
    hvec<int> pair_base;
};

struct FacPlan {
    hvec<rsp::LevelSeg> segs;
    hvec<rsp::RndChunk> chunks;
    hvec<rsp::RndItem> items;
    hvec<int> pairs, staged, rounds;
};

// One DAG's levels and solve plan.
struct DagHost {
    hvec<int> ptr, rows;  // level pointers, rows in level order
    SolvePlan sp;
    int batch = 8, group = 4;
    bool planned = false;
};

// The block-inverse solve plan of a deep DAG (ilu_blocks.cpp; rsp::BlkDesc).
struct BlkPlanHost {
    int n = 0, nb = 0, nlong = 0, entries = 0;
    int lds_elems = 0;  // coefficient build: LDS values (T) of the largest normal block
    int lds_words = 0;  // ... and 32-bit words of its slot data (eord, rptr, recipe items, levels)
    long long novf = 0; // long blocks' record overflow entries
    hvec<int> order;    // position -> row
    hvec<rsp::BlkDesc> desc;
    hvec<rsp::BlkRow> rows;
    hvec<int> ref, vpos, lptr, rptr;
    hvec<unsigned> eord, rit;
    hvec<rsp::BlkSeg> segs;
};

// Everything the analysis computes on the host.
struct IluHostPlan {
    int n = 0, nnz_s = 0, structural_zero = -1;
    hvec<int> dpos, hasdiag, udiv;
    IluSymbolic sym;
    DagHost L, LT, U;
    // block-inverse solve plans of L / L^T where the DAG is deep (blocks_wanted)
    BlkPlanHost Lb, LTb;
    bool has_lb = false, has_ltb = false;
    // The factor's level sets: L's, or ONE level holding every row (F, with
    // fac_one set) for a pattern without update pairs — a stored lower
    // triangle (the symmetric matrices' storage), where no position of any
    // row's upper part is ever updated, so every u_kk a division reads is
    // final from the start and the L DAG's order constrains nothing.
    DagHost F;
    bool fac_one = false;
    // fac_one and the factor is ilu0_scale_lower (one launch, no plan: the
    // factor plan, FacRow records and slots stay empty); RSP_ILU_FAC_SCALE=0
    // at analysis time plans the one level instead (A/B, tests)
    bool fac_scale = false;
    // transposed strict lower part (row k: (position of l_jk, j), j descending)
    hvec<int> ltp, lts, ltc;
    // the solves' term order. Default: the reference's (L column ascending,
    // L^T the column sweep: lpos is the identity, ne_* = 0). RSP_ILU_SPLIT=1
    // (split = 1; round 4, measured slower): a row's terms from
    // the level just below its own in the DAG ("late") after its other
    // ("early") terms, each part in the reference's order. L: lpos[rp[i] + o]
    // = position of the o-th term of row i; L^T: lts / ltc above, permuted
    // per row the same way; ne_l / ne_lt = early terms per row. lev_l /
    // lev_lt: the levels.
    int split = 0;
    hvec<int> lpos, ne_l, ne_lt, lev_l, lev_lt;
    FacPlan fplan;
    int fac_batch = 8;
    hvec<rsp::FacRow> frow;
    // fat factor levels in the slot layout: per factor level (stride 0: FacRow
    // path), the rows to write (desc) and their offsets, total ints
    hvec<rsp::FacSlotLevel> fslev;
    hvec<int4> slot_desc;
    hvec<long long> slot_offs;
    long long slot_total = 0;
    // flow runs of the factor (rsp::FacFlowRun / FacFlowItem)
    hvec<rsp::FacFlowRun> fruns;
    hvec<rsp::FacFlowItem> ffitems;
};

// Phase timer (RSP_ILU_TIMING=1 prints; phase_ms collects when given).
struct Phases {
    bool print = false;
    int n = 0;
    double *ms = nullptr;  // [kPhases]
    int next = 0;
    void mark(const char *what);
    void start();
    double t_last = 0.0;
};
constexpr int kPhases = 6;  // phase slots of Phases::ms (marks in call order)

// The host analysis in phases (rsp_ilu0_analysis runs validate and symbolic
// on the GPU instead, and fills hp.dpos / hasdiag / structural_zero / sym
// from there):
//   plan_validate: pattern checks, diagonal positions, structural zero;
//   plan_levels:   level sets of L and L^T, the transposed L (sequential);
//   plan_symbolic: update lists, stages, stage order, divisor positions;
//   plan_solves:   the L and L^T solve plans (needs the levels only);
//   plan_factor:   the factor plan, FacRow records, slot layout, flow runs
//                  (needs sym.upd_ptr / upd_l / upd_u / stage);
//   plan_rest:     both (the solves on a second thread).
rsp_status_t plan_validate(int n, const int *rp, const int *ci, IluHostPlan &hp);
// The rows of the L DAG's levels the factor runs thin (needs the levels and
// sym.upd_ptr): the only rows whose update pairs the factor plan reads.
hvec<int> factor_thin_rows(const int *rp, const IluHostPlan &hp);
void plan_levels(const int *rp, const int *ci, IluHostPlan &hp);        // both halves below
void plan_levels_lower(const int *rp, const int *ci, IluHostPlan &hp);  // L levels (the factor's)
void plan_levels_upper(const int *rp, const int *ci, IluHostPlan &hp,  // L^T levels, transposed lower,
                       bool split = true);                             // split order (needs L levels)
rsp_status_t plan_symbolic(const int *rp, const int *ci, IluHostPlan &hp);
void plan_solves(const int *rp, const int *ci, IluHostPlan &hp);
// ... their per-row half only (SolvePlan without tpos / src / trow / sid /
// stg and the chunks' staged ranges: rsp_k::ilu_an_solve_terms builds those)
void plan_solves_rows(const int *rp, const int *ci, IluHostPlan &hp);
void plan_factor(const int *rp, const int *ci, long long slot_cap, IluHostPlan &hp);
void plan_rest(const int *rp, const int *ci, long long slot_cap, bool want_u, IluHostPlan &hp);
// The symbolic factor of the given rows on the host (the device analysis'
// long rows): counts when cnt != nullptr, else pairs at ptr + stages, stage
// order, divisor positions (arrays indexed by position).
void symbolic_rows(const hvec<int> &rows, int n, const int *rp, const int *ci, const int *dpos,
                   const int *hasdiag, int *cnt, const int *ptr, int *upd_l, int *upd_u, int *stage, int *lord,
                   int *lend, int *udiv);
// All of it. rp / ci: base 0, rp[n] stored entries. slot_cap_ints:
// budget of the fat-level slot layout. The U DAG plan (the --true-lu
// extension) is built only when want_u. Returns INVALID_VALUE for a malformed
// or unsorted pattern, ALLOC_FAILED if the update lists overflow int.
rsp_status_t plan_host(int n, const int *rp, const int *ci, long long slot_cap_ints, bool want_u,
                       IluHostPlan &hp, Phases &ph);
// Block-inverse solves (ilu_blocks.cpp): whether a DAG of n rows and nlev
// levels gets one (RSP_ILU_BLOCKS: -1 auto = deep DAGs, <= 32 rows per level
// on average; 0 never; 1 always), and its plan (kind 0: L, 1: L^T; needs the
// DAG's levels, dpos and for L^T ltp / lts / ltc). false: no plan (the
// level-scheduled solve runs).
bool blocks_wanted(int n, int nlev);
bool plan_blocks(int kind, const int *rp, const int *ci, const IluHostPlan &hp, BlkPlanHost &bp);
// Build the U DAG's levels and solve plan (lazily, on first use).
void plan_u(const int *rp, const int *ci, IluHostPlan &hp);
// 64-bit digest (FNV-1a) of every array of the plan (tests: identical plans).
uint64_t digest(const IluHostPlan &hp);

// f(lo, hi) over [0, n) in contiguous blocks of >= grain on the analysis'
// worker pool (also used by the SpMV planner, rsp_api.cpp make_tile_plan)
void parallel_for(long long n, long long grain, const std::function<void(long long, long long)> &f);

}  // namespace rsp_an

#endif
