// rsp_api.cpp — implementation of include/rsp.h (the C-ABI operator library
// librsp.so). Host-side planning (SpMV row-block schedule, ILU(0) level sets)
// plus launches of the kernels in spmv.hip / ilu0.hip. Mirrors the cuSPARSE
// lifecycle the reference drivers use (GPU/spmv.cu:122-186,
// GPU/ilu0.cu:82-310); see include/rsp.h for the per-call mapping.

#include "rsp.h"

#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <unordered_map>
#include <memory>
#include <new>
#include <chrono>
#include <mutex>
#include <functional>
#include <thread>
#include <vector>

#include "rsp_kernels.h"
#include "ilu_analysis.h"

using rsp_an::env_int;

using rsp::SpmvBlock;
using rsp::SpmvLongRow;
using rsp::SpmvTile;

struct rsp_context {
    int device;
    hipStream_t stream;
    int ftz;
    int spmv_variant;  // RSP_SPMV_VARIANT (tuning knob, default 0)
    int num_cus;
    // diagnostic trace buffers (RSP_ILU_FTRACE / RSP_ILU_TRACE), allocated
    // on the handle's device on first use, freed by rsp_destroy
    unsigned long long *d_ftrace;
    unsigned long long *d_strace;
};

// The SpMV schedule lives in device memory owned by the matrix descriptor
// (d_plan), not in the caller's workspace: it is built once, at
// rsp_spmv_buffer_size time (where the reference calls
// cusparseSpMV_bufferSize, GPU/spmv.cu:159-164, outside its timed loop), so
// the reference's exact call sequence create_csr -> bufferSize -> malloc ->
// 50x SpMV pays no planning inside a timed call, and any number of matrices
// may share one workspace without re-planning.
struct rsp_spmat {
    int64_t rows, cols, nnz;
    int *rowptr;
    int *colidx;
    void *vals;
    rsp_datatype_t type;
    // schedule state
    int planned;                // d_plan holds a schedule for plan_type / local_cols
    int plan_device;            // device d_plan was allocated on
    void *d_plan;               // [tiles | long rows | partials | col bases | 16-bit offsets]
    size_t plan_cap;            // bytes allocated at d_plan
    rsp_datatype_t plan_type;
    int nblocks, nlong, nslots;
    int nnz_s;                  // rowptr[rows] seen by the planner
    size_t off_long, off_part;  // byte offsets inside d_plan
    size_t off_cbase, off_cidx, off_runs;
    int64_t nnz_c16;            // entries read through 16-bit column offsets or slot indices
    int64_t nnz_staged;         // ... of which in staged tiles (x staged in LDS)
    int64_t local_cols;         // rsp_spmat_set_local_cols (-1: not split)
    int nint;                   // interior tiles at the front of the schedule
    unsigned long long plan_gen;  // unique per plan / value rebind (batch staleness key)
};

namespace {
std::atomic<unsigned long long> g_plan_next{1};
unsigned long long plan_new_gen() { return g_plan_next.fetch_add(1); }
}  // namespace

struct rsp_ilu0_info {
    int analysed;
    int n, nnz_s;
    const int *rowptr, *colidx;  // device pattern captured at analysis
    int structural_zero;         // -1 = none
    int factored;
    int *d_dpos, *d_hasdiag;
    int *d_upd_ptr, *d_upd_l, *d_upd_u, *d_lord, *d_lend, *d_udiv;
    // d_zero: [0] numerical zero pivot (atomicMin), [1] generation of the
    // last factor call whose flow wait gave up, [2..4] the same for the L,
    // L^T and U solves (rsp::FlowCtl), [6..7] the flow claim counter
    int *d_zero;
    unsigned long long claim_host = 0;  // flow claims issued (rsp::FlowCtl)
    int *d_fdone = nullptr;             // ticket flow launches: per item, the epoch that finished it (rsp::FlowCtl)
    unsigned *d_tk = nullptr;           // ticket flow launches: two slots of counters (rsp::FlowCtl::tickets)
    unsigned long long tk_seq = 0;      // ticket flow launches enqueued (rsp::FlowCtl::tk_seq)
    unsigned flow_epoch = 0;            // epochs handed out (rsp::FlowCtl)
    int solve_gen[3] = {0, 0, 0};       // per solve kind: generation of the last call
    long long n_updates;
    // one level set per DAG: L (factor + L solve), L^T, U
    struct Dag {
        rsp_an::hvec<int> ptr;                  // host level pointers
        int *d_rows = nullptr, *d_ptr = nullptr;
        rsp::RowTask *d_tasks = nullptr;       // solve: task per level-order slot
        int *d_tpos = nullptr, *d_src = nullptr;  // solve: flat terms
        rsp::LevelChunk *d_chunks = nullptr;   // solve: LDS-staged chunks of thin runs
        rsp::ThinRowPlan *d_trow = nullptr;    // solve: thin-run row records
        int *d_sid = nullptr;                  // solve: thin-run y indices per term
        rsp::StagedTerm *d_stg = nullptr;      // solve: thin-run staged terms
        rsp::FlowItem *d_fitems = nullptr;     // solve: flow segments' work items
        int nterms = 0;                        // solve: flat terms
        int *d_nshort = nullptr;               // solve: short rows per level (device)
        rsp_an::hvec<int> nshort;               // (host)
        rsp_an::hvec<int> nwave;                // solve: short + wave rows per level (host)
        rsp_an::hvec<int> sbase;                // solve: padded short rows' first term per level (host)
        rsp_an::hvec<rsp::LevelSeg> segs;       // thread-per-row solve plan
        int batch = 8;                         // solve fma-chain batch
        int group = 4;                         // thin-run term groups (2 or 4)
    } L, LT, U, F;  // F: the factor's one level when fac_one (ptr, d_rows, d_ptr; rsp_an::IluHostPlan::F)
    // block-inverse solve plans of deep L / L^T DAGs (rsp_an::plan_blocks,
    // trsv_blocks.hip); on = false: the level-scheduled solve runs
    struct BlkDag {
        bool on = false;
        int nb = 0, lds_elems = 0, lds_words = 0, entries = 0, nlong = 0;
        rsp_an::hvec<rsp::BlkSeg> segs;  // host
        int *d_order = nullptr, *d_ref = nullptr, *d_vpos = nullptr, *d_lptr = nullptr, *d_rptr = nullptr;
        rsp::BlkDesc *d_desc = nullptr;
        rsp::BlkRow *d_rows = nullptr;
        unsigned *d_eord = nullptr, *d_rit = nullptr;
        void *d_ev = nullptr, *d_yp = nullptr;  // scratch, fp64-sized
        void *d_rc = nullptr;  // block records (fp64-sized: 64 x 144 B per block)
    } Lb, LTb;
    bool fac_one = false, fac_scale = false;  // fac_scale: the factor is ilu0_scale_lower (IluHostPlan::fac_scale)
    const Dag &fdag() const { return fac_one ? F : L; }  // the factor's level sets
    rsp_an::hvec<rsp::LevelSeg> fac_segs;       // wave-per-row factor plan over fdag()
    void *d_sval = nullptr, *d_sx = nullptr, *d_sdg = nullptr;  // solve streams (trsv_stream)
    rsp::RndChunk *d_rchunks = nullptr;        // round-based factor chunks (thin runs)
    rsp::RndItem *d_ritems = nullptr;
    rsp::FacRow *d_frow = nullptr;
    int *d_fslots = nullptr;                   // fat factor levels, slot layout (ilu0_level_slot)
    rsp_an::hvec<rsp::FacFlowRun> fruns;        // factor flow runs (ilu0_flow)
    rsp::FacFlowItem *d_ffitems = nullptr;
    void *d_forig = nullptr;                   // flow rows' upper input values (ilu0_flow_prep), fp64-sized
    int fac_gen = 0;
    rsp_an::hvec<rsp::FacSlotLevel> fslev;      // per factor level (stride 0: FacRow path)
    int *d_rpairs = nullptr, *d_rstaged = nullptr, *d_rrounds = nullptr;
    int fac_batch;
    void *d_arena = nullptr;    // one allocation holding the analysis' arrays (Arena)
    void *d_arena_u = nullptr;  // the U plan's (built on first use)
    void *d_arena_sym = nullptr;    // device analysis: dpos, hasdiag, upd_ptr, lord, lend, udiv, scratch
    void *d_arena_pairs = nullptr;  // device analysis: upd_l, upd_u
    void *d_usval = nullptr;    // U solve term values (trsv_stream), in d_arena_u
    unsigned long long digest = 0;  // rsp_an::digest of the host plan
    std::unique_ptr<rsp_an::IluHostPlan> host;  // kept for the solve plans and the U plan
    rsp_an::hvec<int> host_rp, host_ci;
    // The L and L^T solve plans (the reference's two csrsv2_analysis calls,
    // GPU/ilu0.cu:228-252): built on a worker thread that rsp_ilu0_analysis
    // starts once the levels exist and leaves running; ilu_solves_ready
    // (rsp_trsv_analysis, or the first solve) joins it and uploads them.
    // (Declared after host / host_rp / host_ci, which it reads: destroyed,
    // i.e. joined, before them.)
    std::unique_ptr<rsp_an::Task> solves_task;
    bool solves_ready = false;
    bool dev_terms = true;      // the per-term half of the solve plans is built on the device
    void *d_arena_s = nullptr;  // the solve plans' allocation
    rsp_handle_t han = nullptr; // the handle of the analysis (its stream uploads the solve plans)
    // Recovery of a call whose flow wait gave up (a co-running kernel kept
    // some of the flow launch's workgroups from being scheduled past the
    // give-up bound): rsp_ilu0_zero_pivot / rsp_trsv_zero_pivot re-run it
    // without flow launches (every level its own launch: no co-residency
    // needed), from the factor's input values — copied before every factor
    // that has flow runs — or the solve's unchanged x. RSP_ILU_FLOW_RECOVER=0
    // reports EXECUTION_FAILED instead (the round-4 behaviour).
    // A recovered call's output feeds the calls made after it (the L^T solve
    // reads the L solve's y; a solve reads the factor's values), so those are
    // re-run too, in call order (seq).
    void *d_fbackup = nullptr;
    size_t fbackup_bytes = 0;
    long long call_seq = 0;
    struct FacCall {
        long long seq = 0;
        int valid = 0;
        int ftz = 0;  // the handle's FTZ mode at the call
        rsp_datatype_t type = RSP_R_64F;
        void *vals = nullptr;
    } last_fac;
    struct SolveCall {
        long long seq = 0;
        int valid = 0;
        int ftz = 0;
        rsp_operation_t op = RSP_OPERATION_NON_TRANSPOSE;
        double alpha = 1.0;
        rsp_datatype_t type = RSP_R_64F;
        const void *vals = nullptr, *x = nullptr;
        void *y = nullptr;
    } last_solve[3];
};

#define RSP_CHECK_HIP(call)                                                     \
    do {                                                                        \
        hipError_t e_ = (call);                                                 \
        if (e_ != hipSuccess)                                                   \
            return e_ == hipErrorOutOfMemory ? RSP_STATUS_ALLOC_FAILED          \
                                             : RSP_STATUS_EXECUTION_FAILED;     \
    } while (0)

extern "C" {

int rsp_get_version(void) { return RSP_VERSION_MAJOR * 1000 + RSP_VERSION_MINOR; }

const char *rsp_get_error_string(rsp_status_t s) {
    switch (s) {
        case RSP_STATUS_SUCCESS: return "RSP_STATUS_SUCCESS";
        case RSP_STATUS_NOT_INITIALIZED: return "RSP_STATUS_NOT_INITIALIZED";
        case RSP_STATUS_ALLOC_FAILED: return "RSP_STATUS_ALLOC_FAILED";
        case RSP_STATUS_INVALID_VALUE: return "RSP_STATUS_INVALID_VALUE";
        case RSP_STATUS_ARCH_MISMATCH: return "RSP_STATUS_ARCH_MISMATCH";
        case RSP_STATUS_EXECUTION_FAILED: return "RSP_STATUS_EXECUTION_FAILED";
        case RSP_STATUS_INTERNAL_ERROR: return "RSP_STATUS_INTERNAL_ERROR";
        case RSP_STATUS_MATRIX_TYPE_NOT_SUPPORTED: return "RSP_STATUS_MATRIX_TYPE_NOT_SUPPORTED";
        case RSP_STATUS_ZERO_PIVOT: return "RSP_STATUS_ZERO_PIVOT";
        case RSP_STATUS_NOT_SUPPORTED: return "RSP_STATUS_NOT_SUPPORTED";
    }
    return "RSP_STATUS_UNKNOWN";
}

rsp_status_t rsp_create(rsp_handle_t *handle) {
    if (!handle) return RSP_STATUS_INVALID_VALUE;
    *handle = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return RSP_STATUS_NOT_INITIALIZED;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return RSP_STATUS_NOT_INITIALIZED;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RSP_STATUS_ARCH_MISMATCH;
    rsp_context *c = new (std::nothrow) rsp_context;
    if (!c) return RSP_STATUS_ALLOC_FAILED;
    c->device = dev;
    c->stream = nullptr;
    c->ftz = 0;
    const char *v = getenv("RSP_SPMV_VARIANT");
    c->spmv_variant = v ? atoi(v) : 0;
    c->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    // every kernel code object loaded now, as cusparseCreate sets itself up
    // outside the reference's timed calls (a lazily loaded one cost the
    // first timed SpMV of a --ref-sequence run 1.2-1.5 ms, measured)
    rsp_k::warm_spmv();
    rsp_k_ftz::warm_spmv();
    rsp_k::warm_ilu();
    rsp_k_ftz::warm_ilu();
    rsp_k::warm_analysis();
    c->d_ftrace = nullptr;
    c->d_strace = nullptr;
    *handle = c;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_destroy(rsp_handle_t h) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (h->d_ftrace || h->d_strace) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(h->device);
        if (h->d_ftrace) (void)hipFree(h->d_ftrace);
        if (h->d_strace) (void)hipFree(h->d_strace);
        (void)hipSetDevice(cur);
    }
    delete h;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_set_stream(rsp_handle_t h, void *stream) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    h->stream = (hipStream_t)stream;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_get_stream(rsp_handle_t h, void **stream) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!stream) return RSP_STATUS_INVALID_VALUE;
    *stream = (void *)h->stream;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_set_ftz(rsp_handle_t h, int enable) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    h->ftz = enable ? 1 : 0;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_get_ftz(rsp_handle_t h, int *enable) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!enable) return RSP_STATUS_INVALID_VALUE;
    *enable = h->ftz;
    return RSP_STATUS_SUCCESS;
}

/* ------------------------------------------------------------------ CSR */

rsp_status_t rsp_create_csr(rsp_spmat_t *mat, int64_t rows, int64_t cols, int64_t nnz,
                            void *d_row_offsets, void *d_col_ind, void *d_values,
                            rsp_datatype_t value_type) {
    if (!mat) return RSP_STATUS_INVALID_VALUE;
    *mat = nullptr;
    if (rows < 0 || cols < 0 || nnz < 0 || rows > INT_MAX - 1 || cols > INT_MAX || nnz > INT_MAX)
        return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    if (!d_row_offsets && rows > 0) return RSP_STATUS_INVALID_VALUE;
    if ((!d_col_ind || !d_values) && nnz > 0) return RSP_STATUS_INVALID_VALUE;
    rsp_spmat *a = new (std::nothrow) rsp_spmat;
    if (!a) return RSP_STATUS_ALLOC_FAILED;
    memset(a, 0, sizeof(*a));
    a->rows = rows;
    a->cols = cols;
    a->nnz = nnz;
    a->rowptr = (int *)d_row_offsets;
    a->colidx = (int *)d_col_ind;
    a->vals = d_values;
    a->type = value_type;
    a->planned = 0;
    a->d_plan = nullptr;
    a->local_cols = -1;
    *mat = a;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_spmat_set_local_cols(rsp_spmat_t mat, int64_t ncols_local) {
    if (!mat || ncols_local < 0 || ncols_local > mat->cols) return RSP_STATUS_INVALID_VALUE;
    mat->local_cols = ncols_local;
    mat->planned = 0;  // re-plan on the next call
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_csr_set_values(rsp_spmat_t mat, void *d_values, rsp_datatype_t value_type) {
    if (!mat) return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    if (d_values != mat->vals) mat->plan_gen = plan_new_gen();  // batches hold the old pointer
    mat->vals = d_values;
    if (value_type != mat->type) mat->planned = 0;  // tile size depends on type
    mat->type = value_type;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_destroy_spmat(rsp_spmat_t mat) {
    if (!mat) return RSP_STATUS_INVALID_VALUE;
    if (mat->d_plan) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(mat->plan_device);
        (void)hipFree(mat->d_plan);
        (void)hipSetDevice(cur);
    }
    delete mat;
    return RSP_STATUS_SUCCESS;
}

/* ----------------------------------------------------------------- SpMV */

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct SpmvBounds {
    size_t nblocks, nlong, nslots;
};

static SpmvBounds spmv_bounds(int64_t rows, int64_t nnz, int cap) {
    // greedy packing: two consecutive size-closed tiles exceed `cap`, long
    // rows contribute <= nnz/cap + 1 chunks each side.
    // + every row longer than kSpmvLongRow may sit in a tile of its own and
    // close the tile before it: <= 2 * nnz / kSpmvLongRow extra tiles.
    SpmvBounds b;
    size_t q = (size_t)(nnz / cap) + 1;
    size_t l = (size_t)(nnz / rsp::kSpmvLongRow) + 1;
    b.nlong = q;
    b.nslots = 2 * q + 1;
    b.nblocks = 6 * q + 2 * l + (size_t)(rows / rsp::kSpmvMaxRows) + 8;
    b.nblocks += std::min<size_t>(b.nblocks, 8192);  // headroom for spread-out small plans
    return b;
}

// Workspace: [tiles | long rows | chunk partials | per-tile column base |
// 16-bit column offsets (2 B per stored entry) | staged tiles' runs].
struct SpmvLayout {
    size_t off_long, off_part, off_cbase, off_cidx, off_runs, bytes;
};
static SpmvLayout spmv_layout(const SpmvBounds &b, size_t elem, int64_t nnz, size_t run_ints = 0) {
    SpmvLayout l;
    l.off_long = align256(b.nblocks * sizeof(SpmvBlock));
    l.off_part = l.off_long + align256(b.nlong * sizeof(SpmvLongRow));
    l.off_cbase = l.off_part + align256(b.nslots * 2 * elem);  // value + ticket per slot
    l.off_cidx = l.off_cbase + align256(b.nblocks * sizeof(int));
    l.off_runs = l.off_cidx + align256((size_t)std::max<int64_t>(nnz, 0) * sizeof(uint16_t));
    l.bytes = l.off_runs + align256(run_ints * sizeof(int));
    return l;
}

static int tile_cap(rsp_datatype_t t) {
    return t == RSP_R_64F ? SpmvTile<double>::kMaxNnz : SpmvTile<float>::kMaxNnz;
}
static int chunk_cap(rsp_datatype_t t) {
    return t == RSP_R_64F ? SpmvTile<double>::kChunk : SpmvTile<float>::kChunk;
}
static size_t elem_size(rsp_datatype_t t) { return t == RSP_R_64F ? 8 : 4; }
// Tile row cuts: RSP_SPMV_VARIANT bit 6 aligns them to 128-B y lines, bit 7
// to 64 B (tuning knob; default unaligned).
static int spmv_row_align(rsp_handle_t h, rsp_datatype_t t) {
    const int e = (int)elem_size(t);
    return (h->spmv_variant & 64) ? 128 / e : (h->spmv_variant & 128) ? 64 / e : 1;
}

static rsp_status_t spmv_plan(rsp_handle_t h, rsp_spmat_t mat, rsp_datatype_t compute_type);

static rsp_status_t rsp_spmv_buffer_size_impl(rsp_handle_t h, rsp_operation_t op, const void *alpha,
                                  rsp_spmat_t mat, const void *beta, rsp_datatype_t compute_type,
                                  size_t *buffer_size) {
    (void)alpha;
    (void)beta;
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!mat || !buffer_size) return RSP_STATUS_INVALID_VALUE;
    if (op != RSP_OPERATION_NON_TRANSPOSE) return RSP_STATUS_NOT_SUPPORTED;
    if (compute_type != mat->type) return RSP_STATUS_NOT_SUPPORTED;
    // the schedule is built here, into the matrix's own device memory (the
    // reference calls bufferSize once, before its timed loop); the caller's
    // workspace is not needed
    if (!mat->planned || mat->plan_type != compute_type) {
        rsp_status_t st = spmv_plan(h, mat, compute_type);
        if (st != RSP_STATUS_SUCCESS) return st;
    }
    *buffer_size = 0;
    return RSP_STATUS_SUCCESS;
}

// Greedy row-block schedule over host row offsets (see spmv.hip header).
// Rows longer than kSpmvLongRow get tiles of their own (one per `chunk`
// entries); the others are packed into tiles of <= cap entries / maxrows rows.
static int build_spmv_plan(const int *rp, int m, int cap, int chunk, rsp_an::hvec<SpmvBlock> &blocks,
                           rsp_an::hvec<SpmvLongRow> &longrows, int *nslots,
                           int maxrows = rsp::kSpmvMaxRows, int row_align = 1) {
    blocks.clear();
    longrows.clear();
    int slots = 0;
    int r = 0;
    while (r < m) {
        int len = rp[r + 1] - rp[r];
        if (len > rsp::kSpmvLongRow) {
            if (len <= chunk) {  // one chunk: reduced and written in place
                SpmvBlock b;
                b.r0 = r;
                b.r1 = rsp::kSpmvWholeRow;
                b.k0 = rp[r];
                b.k1 = rp[r + 1];
                blocks.push_back(b);
                r++;
                continue;
            }
            SpmvLongRow lr;
            lr.row = r;
            lr.first = slots;
            lr.nchunks = 0;
            lr.pad = 0;
            for (int k = rp[r]; k < rp[r + 1]; k += chunk) {
                SpmvBlock b;
                b.r0 = r;
                b.r1 = -(slots + 1);
                b.k0 = k;
                b.k1 = std::min(k + chunk, rp[r + 1]);
                blocks.push_back(b);
                slots++;
                lr.nchunks++;
            }
            longrows.push_back(lr);
            r++;
            continue;
        }
        int start = r, nnz = 0;
        while (r < m && r - start < maxrows) {
            int l = rp[r + 1] - rp[r];
            // a tile always takes its first row (<= kSpmvLongRow <= kMaxNnz)
            if (l > rsp::kSpmvLongRow || (r > start && nnz + l > cap)) break;
            nnz += l;
            r++;
        }
        // row_align > 1: end a packed tile on a multiple of row_align rows,
        // so its y stores cover whole lines, where the tile keeps >= 3/4 of
        // its entries
        if (row_align > 1 && r < m && r % row_align != 0) {
            const int ra = r - r % row_align;
            if (ra > start && (int64_t)(rp[ra] - rp[start]) * 4 >= (int64_t)(rp[r] - rp[start]) * 3) r = ra;
        }
        SpmvBlock b;
        b.r0 = start;
        b.r1 = r;
        b.k0 = rp[start];
        b.k1 = rp[r];
        blocks.push_back(b);
    }
    *nslots = slots;
    return 0;
}

// A complete SpMV schedule over host row offsets `rp` and column indices `ci`:
// tiles (interior tiles first when local_cols >= 0), long rows, per-tile
// column base and the 16-bit column offsets.
struct TilePlan {
    rsp_an::hvec<SpmvBlock> blocks;
    rsp_an::hvec<SpmvLongRow> longrows;
    int nslots = 0, nint = 0;
    rsp_an::hvec<int> cbase;
    rsp_an::hvec<uint16_t> c16;
    rsp_an::hvec<int> runs;  // staged tiles' run descriptors (int pairs), SpmvArgs::runs
    int64_t nnz_c16 = 0;     // entries read through 16-bit offsets or slot indices
    int64_t nnz_staged = 0;  // ... of which in staged tiles
};

// spread > 0: a plan of fewer tiles than `spread` (the resident workgroup
// slots it may use) is re-packed into up to `spread` smaller tiles, so a lone
// launch does not leave slots idle. Long rows do not depend on the packing
// cap (they are cut at the fixed chunk), so every spread of one matrix has
// the same long rows and partial slots.
static void make_tile_plan(const int *rp, const int *ci, int m, int64_t nnz_bound,
                           rsp_datatype_t type, int64_t spread, int64_t local_cols, bool use_c16,
                           TilePlan &p, int row_align = 1, bool use_stage = true) {
    const int chunk = chunk_cap(type);
    const int cap = tile_cap(type);
    const int align = row_align;
    const int maxrows = type == RSP_R_64F ? SpmvTile<double>::kMaxRows : SpmvTile<float>::kMaxRows;
    build_spmv_plan(rp, m, cap, chunk, p.blocks, p.longrows, &p.nslots, maxrows, align);
    const int64_t nb = (int64_t)p.blocks.size();
    if (spread > 0 && nb > 0 && nb < spread) {
        const SpmvBounds bb = spmv_bounds(m, std::max<int64_t>(nnz_bound, 0), chunk);
        const int64_t nnz_s = rp[(size_t)m];
        int c = (int)std::max<int64_t>(64, std::min<int64_t>(cap, (nnz_s + spread - 1) / spread));
        for (int tries = 0; tries < 32 && c < cap; tries++) {
            rsp_an::hvec<SpmvBlock> b2;
            rsp_an::hvec<SpmvLongRow> l2;
            int s2 = 0;
            build_spmv_plan(rp, m, c, chunk, b2, l2, &s2, maxrows, align);
            if ((int64_t)b2.size() <= spread && b2.size() <= bb.nblocks) {
                p.blocks.swap(b2);
                p.longrows.swap(l2);
                p.nslots = s2;
                break;
            }
            c += std::max(8, c / 16);
        }
    }
    // Random-band matrices (round 4): tiles whose columns lie in a band
    // narrower than 65536 but scattered over it (more runs than a staged
    // tile's run table holds) are staged by an explicit column LIST instead
    // (below); that needs at most kStageSlots distinct columns per tile, so
    // such a matrix is re-packed with tiles of at most kStageSlots entries
    // (the canonical summation order does not depend on the packing). Judged
    // on a sample of 64 tiles; not for spread plans (already small tiles).
    const int ucap = type == RSP_R_64F ? SpmvTile<double>::kStageSlots : SpmvTile<float>::kStageSlots;
    const bool list_ok = use_stage && use_c16 && type == RSP_R_64F && SpmvTile<double>::kStageList &&
                         env_int("RSP_SPMV_STAGE_LIST", 1) != 0;
    if (list_ok && (int64_t)p.blocks.size() == nb && nb > 0) {
        int64_t band = 0, all = 0;
        std::vector<int> cols;
        const size_t step = std::max<size_t>(1, p.blocks.size() / 64);
        for (size_t t = 0; t < p.blocks.size(); t += step) {
            const SpmvBlock &bk = p.blocks[t];
            if (bk.r1 < 0 || bk.k1 <= bk.k0) continue;
            cols.assign(ci + bk.k0, ci + bk.k1);
            std::sort(cols.begin(), cols.end());
            cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
            int R = 1;
            for (size_t u = 1; u < cols.size(); u++) R += cols[u] != cols[u - 1] + 1;
            all += bk.k1 - bk.k0;
            if (cols.back() - cols.front() <= 65535 && R > rsp::kStageRuns && (int)cols.size() > ucap)
                band += bk.k1 - bk.k0;
        }
        if (2 * band > all) {
            rsp_an::hvec<SpmvBlock> b2;
            rsp_an::hvec<SpmvLongRow> l2;
            int s2 = 0;
            // RSP_SPMV_LIST_CAP (A/B knob): a smaller tile for the re-packed plan
            const int lcap = std::min(std::max(env_int("RSP_SPMV_LIST_CAP", ucap), 64), ucap);
            build_spmv_plan(rp, m, std::min(cap, lcap), chunk, b2, l2, &s2, maxrows, align);
            p.blocks.swap(b2);
            p.longrows.swap(l2);
            p.nslots = s2;
        }
    }
    // split schedule (rsp_spmat_set_local_cols): tiles reading own columns
    // only first; long-row tiles always in the second part (with the fixup)
    p.nint = 0;
    if (local_cols >= 0) {
        auto interior = [&](const SpmvBlock &b) {
            if (b.r1 < 0) return false;
            for (int k = b.k0; k < b.k1; k++)
                if (ci[(size_t)k] >= local_cols) return false;
            return true;
        };
        auto mid = std::stable_partition(p.blocks.begin(), p.blocks.end(), interior);
        p.nint = (int)(mid - p.blocks.begin());
    }
    // 16-bit column offsets: a tile whose columns span < 65536 reads
    // col = cbase + off (2 B per entry instead of 4; the int32 colidx is not
    // read for it). Staged tiles (round 4, spmv.hip stream_products_staged):
    // where the tile's distinct columns are few (at most kStageSlots, at most
    // RSP_SPMV_STAGE_PCT % of its entries, default 80) in at most kStageRuns
    // contiguous runs, its 16-bit values are instead the entries' slots in the
    // sorted list of those columns, and the runs ({first column, first slot},
    // then {0, slots}) go to `runs`. Tiles are planned in parallel.
    const int64_t nnz_s = m > 0 ? rp[(size_t)m] : 0;
    p.cbase.assign(p.blocks.size(), -1);
    p.c16.clear();
    p.runs.clear();
    p.nnz_c16 = 0;
    p.nnz_staged = 0;
    if (use_c16 && nnz_s > 0 && nnz_s <= nnz_bound) {
        p.c16.assign((size_t)nnz_s, 0);
        const long long nt = (long long)p.blocks.size();
        const long long pct = std::min(std::max(env_int("RSP_SPMV_STAGE_PCT", 80), 0), 100);
        const int64_t xelem = type == RSP_R_64F ? 8 : 4;
        std::vector<std::vector<int>> truns(use_stage ? (size_t)nt : 0);
        std::vector<char> tmode(use_stage ? (size_t)nt : 0, 0);  // 1 runs, 2 list
        std::atomic<int64_t> n16{0}, nst{0};
        rsp_an::parallel_for(nt, 64, [&](long long t0, long long t1) {
            std::vector<int> cols;
            int64_t c16n = 0, stn = 0;
            for (long long t = t0; t < t1; t++) {
                const SpmvBlock &bk = p.blocks[(size_t)t];
                if (bk.k1 <= bk.k0) continue;
                int lo = ci[(size_t)bk.k0], hi = lo;
                for (int k = bk.k0 + 1; k < bk.k1; k++) {
                    lo = std::min(lo, ci[(size_t)k]);
                    hi = std::max(hi, ci[(size_t)k]);
                }
                if (hi - lo > 65535) continue;
                const int len = bk.k1 - bk.k0;
                c16n += len;
                // staged x loads use 32-bit byte offsets into a buffer resource of
                // 0x7ffffffc bytes (spmv.hip stream_products_staged): a tile whose
                // columns reach past that keeps the plain 16-bit offsets
                const bool x_in_rsrc = ((int64_t)hi + 1) * xelem <= (int64_t)0x7ffffffc;
                if (use_stage && bk.r1 >= 0 && x_in_rsrc) {  // (long-row chunks keep the offsets)
                    cols.assign(ci + bk.k0, ci + bk.k1);
                    std::sort(cols.begin(), cols.end());
                    cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
                    const int U = (int)cols.size();
                    int R = 1;
                    for (int u = 1; u < U; u++) R += cols[(size_t)u] != cols[(size_t)u - 1] + 1;
                    const bool runs_mode = U <= ucap && R <= rsp::kStageRuns && 100LL * U <= pct * len;
                    const bool list_mode = !runs_mode && list_ok && U <= ucap && R > rsp::kStageRuns;
                    if (runs_mode || list_mode) {
                        std::vector<int> &r = truns[(size_t)t];
                        tmode[(size_t)t] = runs_mode ? 1 : 2;
                        if (runs_mode) {
                            r.reserve(2 * (size_t)(R + 1));
                            for (int u = 0; u < U; u++)
                                if (u == 0 || cols[(size_t)u] != cols[(size_t)u - 1] + 1) {
                                    r.push_back(cols[(size_t)u]);
                                    r.push_back(u);
                                }
                            r.push_back(0);
                            r.push_back(U);
                        } else {  // {base column, U}, then the U column offsets as uint16, padded to 8 B
                            r.assign(2 + 2 * (size_t)((U + 3) / 4), 0);
                            r[0] = cols[0];
                            r[1] = U;
                            uint16_t *o = reinterpret_cast<uint16_t *>(r.data() + 2);
                            for (int u = 0; u < U; u++) o[u] = (uint16_t)(cols[(size_t)u] - cols[0]);
                        }
                        for (int k = bk.k0; k < bk.k1; k++)
                            p.c16[(size_t)k] = (uint16_t)(std::lower_bound(cols.begin(), cols.end(), ci[(size_t)k]) -
                                                          cols.begin());
                        stn += len;
                        continue;
                    }
                }
                p.cbase[(size_t)t] = lo;
                for (int k = bk.k0; k < bk.k1; k++) p.c16[(size_t)k] = (uint16_t)(ci[(size_t)k] - lo);
            }
            n16 += c16n;
            nst += stn;
        });
        p.nnz_c16 = n16;
        p.nnz_staged = nst;
        if (use_stage) {  // descriptors concatenated in tile order; cbase = -2 - (pair offset << 8 | runs)
            for (size_t t = 0; t < truns.size(); t++) {
                const std::vector<int> &r = truns[t];
                if (r.empty()) continue;
                const int64_t off = (int64_t)p.runs.size() / 2;
                // runs mode: descriptors + sentinel; list mode: 255 (header {base, U} + offsets)
                const int nr = tmode[t] == 2 ? 255 : (int)r.size() / 2 - 1;
                if (off >= (1LL << 22)) {  // (encoding range; never reached on real matrices)
                    p.nnz_c16 -= p.blocks[t].k1 - p.blocks[t].k0;
                    p.nnz_staged -= p.blocks[t].k1 - p.blocks[t].k0;
                    continue;  // cbase stays -1: the int32 path
                }
                p.cbase[t] = -2 - (int)((off << 8) | nr);
                p.runs.insert(p.runs.end(), r.begin(), r.end());
            }
        }
    }
}

// Row offsets and column indices of `mat` on the host, validated (base 0,
// non-decreasing offsets, columns inside [0, cols)).
static rsp_status_t download_pattern(rsp_handle_t h, rsp_spmat_t mat, rsp_an::hvec<int> &rp,
                                     rsp_an::hvec<int> &ci) {
    const int m = (int)mat->rows;
    rp.assign((size_t)m + 1, 0);
    ci.clear();
    if (m > 0) {
        RSP_CHECK_HIP(hipMemcpyAsync(rp.data(), mat->rowptr, ((size_t)m + 1) * sizeof(int),
                                     hipMemcpyDeviceToHost, h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
    }
    if (m > 0 && rp[0] != 0) return RSP_STATUS_INVALID_VALUE;  // base 0 only
    for (int i = 0; i < m; i++)
        if (rp[i + 1] < rp[i]) return RSP_STATUS_INVALID_VALUE;
    // the stored entries must lie inside the colidx / vals arrays (nnz long)
    if (m > 0 && (int64_t)rp[(size_t)m] > mat->nnz) return RSP_STATUS_INVALID_VALUE;
    // Column indices are gathered unchecked by the kernel: validate them once
    // here (outside the timed loop) so a malformed matrix is an INVALID_VALUE
    // status, never an out-of-bounds read of x on the GPU.
    if (m > 0 && rp[(size_t)m] > 0) {
        if (!mat->colidx) return RSP_STATUS_INVALID_VALUE;
        ci.resize((size_t)rp[(size_t)m]);
        RSP_CHECK_HIP(hipMemcpyAsync(ci.data(), mat->colidx, ci.size() * sizeof(int),
                                     hipMemcpyDeviceToHost, h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
        const int ncols = (int)mat->cols;
        for (int c : ci)
            if ((unsigned)c >= (unsigned)ncols) return RSP_STATUS_INVALID_VALUE;
    }
    return RSP_STATUS_SUCCESS;
}

static int64_t spmv_resident_tiles(rsp_handle_t h, rsp_datatype_t t) {
    return (int64_t)rsp_k::spmv_tiles_per_cu((int)elem_size(t)) * h->num_cus;
}

// Build the schedule of `mat` for `compute_type` into the matrix's own device
// memory (host-blocking; see struct rsp_spmat).
static rsp_status_t spmv_plan(rsp_handle_t h, rsp_spmat_t mat, rsp_datatype_t compute_type) {
    const int m = (int)mat->rows;
    rsp_an::hvec<int> rp, ci;
    rsp_status_t st = download_pattern(h, mat, rp, ci);
    if (st != RSP_STATUS_SUCCESS) return st;
    // Full tiles for every matrix. Rounds 3-4 spread a scattered (circuit)
    // matrix with fewer tiles than resident slots over up to that many small
    // tiles; once the row reduce stopped stalling on 33-256-entry rows (round
    // 5: branch-free steps, heavy rows eight lanes each) the full tiles are
    // faster per call: dc1 8.75 -> 7.02 us, G2_circuit 8.13 -> 6.10, ASIC_320ks
    // 11.77 -> 9.22, ss1 8.49 -> 6.61, matrix-new_3 9.10 -> 6.71
    // (profiles/r05_heavy_rows_ab.txt). RSP_SPMV_VARIANT bit 9 still spreads
    // every small matrix (A/B), bit 5 keeps every tile on the int32 indices.
    // A batch re-plans its members itself (rsp_spmv_batch_create). Tiling
    // never changes the result (canonical summation order).
    const bool spread = (h->spmv_variant & 512) != 0;
    TilePlan p;
    make_tile_plan(rp.data(), ci.data(), m, mat->nnz, compute_type,
                   spread ? spmv_resident_tiles(h, compute_type) : 0,
                   mat->local_cols, !(h->spmv_variant & 32), p, spmv_row_align(h, compute_type),
                   !(h->spmv_variant & rsp::kSpmvVariantNoStage));
    const rsp_an::hvec<SpmvBlock> &blocks = p.blocks;
    const rsp_an::hvec<SpmvLongRow> &longrows = p.longrows;
    const int nslots = p.nslots, nint = p.nint;
    const rsp_an::hvec<int> &cbase = p.cbase;
    const rsp_an::hvec<uint16_t> &c16 = p.c16;
    const int64_t nnz_c16 = p.nnz_c16;
    // exact layout of this schedule in the matrix's device memory (grown,
    // never shrunk, on a re-plan)
    SpmvBounds b{blocks.size(), longrows.size(), (size_t)nslots};
    const SpmvLayout lay = spmv_layout(b, elem_size(compute_type), (int64_t)c16.size(), p.runs.size());
    mat->planned = 0;
    if (lay.bytes > mat->plan_cap || !mat->d_plan) {
        if (mat->d_plan) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(mat->plan_device);
            (void)hipFree(mat->d_plan);
            (void)hipSetDevice(cur);
            mat->d_plan = nullptr;
            mat->plan_cap = 0;
        }
        RSP_CHECK_HIP(hipMalloc(&mat->d_plan, std::max<size_t>(lay.bytes, 256)));
        mat->plan_cap = std::max<size_t>(lay.bytes, 256);
        RSP_CHECK_HIP(hipGetDevice(&mat->plan_device));
    }
    char *buf = (char *)mat->d_plan;
    if (!blocks.empty()) {
        RSP_CHECK_HIP(hipMemcpyAsync(buf, blocks.data(), blocks.size() * sizeof(SpmvBlock),
                                     hipMemcpyHostToDevice, h->stream));
        RSP_CHECK_HIP(hipMemcpyAsync(buf + lay.off_cbase, cbase.data(), cbase.size() * sizeof(int),
                                     hipMemcpyHostToDevice, h->stream));
    }
    if (!c16.empty())
        RSP_CHECK_HIP(hipMemcpyAsync(buf + lay.off_cidx, c16.data(), c16.size() * sizeof(uint16_t),
                                     hipMemcpyHostToDevice, h->stream));
    if (!p.runs.empty())
        RSP_CHECK_HIP(hipMemcpyAsync(buf + lay.off_runs, p.runs.data(), p.runs.size() * sizeof(int),
                                     hipMemcpyHostToDevice, h->stream));
    const size_t off_long = lay.off_long, off_part = lay.off_part;
    if (!longrows.empty())
        RSP_CHECK_HIP(hipMemcpyAsync(buf + off_long, longrows.data(),
                                     longrows.size() * sizeof(SpmvLongRow), hipMemcpyHostToDevice,
                                     h->stream));
    // partial slots: the long rows' arrival tickets start (and stay) at 0
    if (nslots > 0)
        RSP_CHECK_HIP(hipMemsetAsync(buf + off_part, 0, (size_t)nslots * 2 * elem_size(compute_type),
                                     h->stream));
    RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
    mat->planned = 1;
    mat->plan_type = compute_type;
    mat->nblocks = (int)blocks.size();
    mat->nint = nint;
    mat->plan_gen = plan_new_gen();
    mat->nlong = (int)longrows.size();
    mat->nslots = nslots;
    mat->nnz_s = m > 0 ? rp[(size_t)m] : 0;
    mat->off_long = off_long;
    mat->off_part = off_part;
    mat->off_cbase = lay.off_cbase;
    mat->off_cidx = lay.off_cidx;
    mat->off_runs = lay.off_runs;
    mat->nnz_c16 = nnz_c16;
    mat->nnz_staged = p.nnz_staged;
    return RSP_STATUS_SUCCESS;
}

static rsp_status_t rsp_spmv_preprocess_impl(rsp_handle_t h, rsp_operation_t op, const void *alpha,
                                 rsp_spmat_t mat, const void *d_x, const void *beta, void *d_y,
                                 rsp_datatype_t compute_type, void *d_buffer) {
    (void)alpha;
    (void)beta;
    (void)d_x;
    (void)d_y;
    (void)d_buffer;
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!mat) return RSP_STATUS_INVALID_VALUE;
    if (op != RSP_OPERATION_NON_TRANSPOSE) return RSP_STATUS_NOT_SUPPORTED;
    if (compute_type != mat->type) return RSP_STATUS_NOT_SUPPORTED;
    return spmv_plan(h, mat, compute_type);  // explicit request: always re-plan
}

rsp_status_t rsp_spmv_plan_info(rsp_spmat_t mat, int64_t *tiles, int64_t *entries_16bit) {
    if (!mat || !tiles || !entries_16bit) return RSP_STATUS_INVALID_VALUE;
    if (!mat->planned) return RSP_STATUS_NOT_INITIALIZED;
    *tiles = mat->nblocks;
    *entries_16bit = mat->nnz_c16;
    return RSP_STATUS_SUCCESS;
}

static rsp_status_t spmv_run(rsp_handle_t h, rsp_operation_t op, const void *alpha, rsp_spmat_t mat,
                             const void *d_x, const void *beta, void *d_y,
                             rsp_datatype_t compute_type, void *d_buffer, int part) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!mat || !alpha || !beta) return RSP_STATUS_INVALID_VALUE;
    if (op != RSP_OPERATION_NON_TRANSPOSE) return RSP_STATUS_NOT_SUPPORTED;
    if (compute_type != mat->type) return RSP_STATUS_NOT_SUPPORTED;
    if (mat->rows > 0 && (!d_y || (mat->cols > 0 && !d_x))) return RSP_STATUS_INVALID_VALUE;
    (void)d_buffer;  // the schedule lives in the matrix (struct rsp_spmat)
    if (!mat->planned || mat->plan_type != compute_type) {  // lazily, if bufferSize was skipped
        rsp_status_t st = spmv_plan(h, mat, compute_type);
        if (st != RSP_STATUS_SUCCESS) return st;
    }
    char *plan = (char *)mat->d_plan;
    rsp::SpmvArgs a;
    a.m = (int)mat->rows;
    a.rowptr = mat->rowptr;
    a.colidx = mat->colidx;
    a.vals = mat->vals;
    a.x = d_x;
    a.y = d_y;
    a.blocks = (const SpmvBlock *)plan;
    a.nblocks = mat->nblocks;
    a.cbases = (const int *)(plan + mat->off_cbase);
    a.cidx = (const unsigned short *)(plan + mat->off_cidx);
    a.runs = (const int *)(plan + mat->off_runs);
    a.cmax = mat->cols > 0 ? (int)(mat->cols - 1) : 0;
    a.longrows = (const SpmvLongRow *)(plan + mat->off_long);
    a.nlong = mat->nlong;
    a.partials = plan + mat->off_part;
    if (compute_type == RSP_R_64F) {
        a.alpha = *(const double *)alpha;
        a.beta = *(const double *)beta;
    } else {
        a.alpha = *(const float *)alpha;
        a.beta = *(const float *)beta;
    }
    if (part != 0) {  // split schedule: part 1 = interior tiles, part 2 = the rest + fixup
        if (a.beta != 0.0) return RSP_STATUS_INVALID_VALUE;
        if (part == 1) {
            a.nblocks = mat->nint;
            a.nlong = 0;
        } else {
            a.blocks += mat->nint;
            a.cbases += mat->nint;
            a.nblocks = mat->nblocks - mat->nint;
        }
    }
    a.vector_ok = ((((uintptr_t)mat->colidx) | ((uintptr_t)mat->vals)) & 15) == 0;
    a.nnz = mat->nnz_s;
    a.variant = h->spmv_variant;
    hipError_t e;
    if (compute_type == RSP_R_64F)
        e = rsp_k::spmv_f64(a, h->stream);
    else
        e = h->ftz ? rsp_k_ftz::spmv_f32(a, h->stream) : rsp_k::spmv_f32(a, h->stream);
    return e == hipSuccess ? RSP_STATUS_SUCCESS : RSP_STATUS_EXECUTION_FAILED;
}

static rsp_status_t rsp_spmv_impl(rsp_handle_t h, rsp_operation_t op, const void *alpha, rsp_spmat_t mat,
                      const void *d_x, const void *beta, void *d_y, rsp_datatype_t compute_type,
                      void *d_buffer) {
    return spmv_run(h, op, alpha, mat, d_x, beta, d_y, compute_type, d_buffer, 0);
}

static rsp_status_t rsp_spmv_part_impl(rsp_handle_t h, const void *alpha, rsp_spmat_t mat, const void *d_x,
                           const void *beta, void *d_y, rsp_datatype_t compute_type,
                           void *d_buffer, int part) {
    if (part < 0 || part > 2) return RSP_STATUS_INVALID_VALUE;
    return spmv_run(h, RSP_OPERATION_NON_TRANSPOSE, alpha, mat, d_x, beta, d_y, compute_type,
                    d_buffer, part);
}

/* ------------------------------------------------------- batched SpMV */

struct rsp_spmv_batch {
    rsp_datatype_t type;
    int part;
    rsp_an::hvec<rsp_spmat_t> mats;
    rsp_an::hvec<unsigned long long> plan_gen;  // schedules as copied (stale check)
    rsp_an::hvec<rsp::SpmvBatchArgs> launches;  // one per kSpmvBatchMax matrices
    void *d_mem = nullptr;                      // entries, tiles, long rows of every launch
    int64_t tiles = 0, entries_16bit = 0;       // rsp_spmv_batch_info
    ~rsp_spmv_batch() {
        if (d_mem) (void)hipFree(d_mem);
    }
};

static rsp_status_t rsp_spmv_batch_create_impl(rsp_handle_t h, int count, const rsp_spmat_t *mats,
                                   const void *const *d_x, void *const *d_y,
                                   void *const *d_buffers, rsp_datatype_t compute_type,
                                   int part, rsp_spmv_batch_t *batch) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    (void)d_buffers;  // workspaces are not needed: schedules live in the matrices
    if (!batch || count < 0 || (count > 0 && (!mats || !d_x || !d_y)))
        return RSP_STATUS_INVALID_VALUE;
    if (part < 0 || part > 2) return RSP_STATUS_INVALID_VALUE;
    if (compute_type != RSP_R_64F && compute_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    *batch = nullptr;
    for (int j = 0; j < count; j++) {
        rsp_spmat_t A = mats[j];
        if (!A) return RSP_STATUS_INVALID_VALUE;
        if (A->type != compute_type) return RSP_STATUS_NOT_SUPPORTED;
        if (A->rows > 0 && (!d_y[j] || (A->cols > 0 && !d_x[j]))) return RSP_STATUS_INVALID_VALUE;
        if (!A->planned || A->plan_type != compute_type) {
            rsp_status_t st = spmv_plan(h, A, compute_type);
            if (st != RSP_STATUS_SUCCESS) return st;
        }
    }
    std::unique_ptr<rsp_spmv_batch> b(new rsp_spmv_batch());
    b->type = compute_type;
    b->part = part;
    // The batch carries its own schedules. Each matrix's own plan is spread
    // over the whole chip for a lone launch (rsp_spmv_preprocess); in a
    // batch that only shrinks the tiles, which cost the moderate set 35 %
    // (0.145 vs 0.108 ms per step). So members are planned with
    // full tiles, and spread only when the launch's tiles together do not
    // fill the resident slots (each matrix over its nnz share of them).
    // Long rows and their partial slots are the same in every spread of a
    // matrix; the batch keeps its own partials and tickets per member, so a
    // matrix may appear in several batches and several times in one (the
    // same A with several right-hand sides), and a batch never shares
    // tickets with single calls of its matrices.
    const int64_t R = spmv_resident_tiles(h, compute_type);
    const bool spread_ok = !(h->spmv_variant & 16), c16_ok = !(h->spmv_variant & 32);
    const bool stage_ok = !(h->spmv_variant & rsp::kSpmvVariantNoStage);
    rsp_an::hvec<TilePlan> plans((size_t)count);
    // layout: per launch [entries | tiles | tile column bases | long rows |
    // 16-bit column offsets of each matrix | long-row partials and tickets of
    // each matrix (zero)], each 16-B aligned
    struct Span { int first, count; size_t off_e, off_t, off_c, off_l; rsp_an::hvec<size_t> off_16, off_p, off_r; };
    rsp_an::hvec<Span> spans;
    size_t bytes = 0;
    auto tile_range = [part](const TilePlan &p, int *t0, int *t1) {
        *t0 = part == 2 ? p.nint : 0;
        *t1 = part == 1 ? p.nint : (int)p.blocks.size();
    };
    for (int first = 0; first < count; first += rsp::kSpmvBatchMax) {
        Span sp{first, std::min(rsp::kSpmvBatchMax, count - first), 0, 0, 0, 0, {}, {}, {}};
        rsp_an::hvec<rsp_an::hvec<int>> rps((size_t)sp.count), cis((size_t)sp.count);
        int64_t nt_full = 0, nnz_all = 0;
        for (int q = 0; q < sp.count; q++) {
            rsp_spmat_t A = mats[first + q];
            rsp_status_t st = download_pattern(h, A, rps[q], cis[q]);
            if (st != RSP_STATUS_SUCCESS) return st;
            make_tile_plan(rps[q].data(), cis[q].data(), (int)A->rows, A->nnz, compute_type, 0,
                           A->local_cols, c16_ok, plans[first + q], spmv_row_align(h, compute_type), stage_ok);
            int t0, t1;
            tile_range(plans[first + q], &t0, &t1);
            nt_full += t1 - t0;
            nnz_all += A->rows > 0 ? rps[q][(size_t)A->rows] : 0;
        }
        if (spread_ok && nt_full < R)
            for (int q = 0; q < sp.count; q++) {
                rsp_spmat_t A = mats[first + q];
                const int64_t nnz_q = A->rows > 0 ? rps[q][(size_t)A->rows] : 0;
                const int64_t share = std::max<int64_t>(1, R * nnz_q / std::max<int64_t>(1, nnz_all));
                make_tile_plan(rps[q].data(), cis[q].data(), (int)A->rows, A->nnz, compute_type,
                               share, A->local_cols, c16_ok, plans[first + q],
                               spmv_row_align(h, compute_type), stage_ok);
            }
        int nt = 0, nl = 0;
        for (int q = 0; q < sp.count; q++) {
            const TilePlan &p = plans[first + q];
            rsp_spmat_t A = mats[first + q];
            // the long rows index partial slots of the matrix's own workspace
            if ((int)p.longrows.size() != A->nlong || p.nslots != A->nslots)
                return RSP_STATUS_INTERNAL_ERROR;
            int t0, t1;
            tile_range(p, &t0, &t1);
            nt += t1 - t0;
            nl += part == 1 ? 0 : (int)p.longrows.size();
        }
        sp.off_e = bytes;
        bytes += (size_t)sp.count * sizeof(rsp::SpmvBatchEntry);
        sp.off_t = bytes;
        bytes += (size_t)nt * sizeof(SpmvBlock);
        sp.off_c = bytes;
        bytes += ((size_t)nt * sizeof(int) + 15) & ~(size_t)15;
        sp.off_l = bytes;
        bytes += ((size_t)nl * sizeof(SpmvLongRow) + 15) & ~(size_t)15;
        for (int q = 0; q < sp.count; q++) {
            sp.off_16.push_back(bytes);
            bytes += (plans[first + q].c16.size() * sizeof(uint16_t) + 15) & ~(size_t)15;
        }
        for (int q = 0; q < sp.count; q++) {
            sp.off_r.push_back(bytes);
            bytes += (plans[first + q].runs.size() * sizeof(int) + 15) & ~(size_t)15;
        }
        for (int q = 0; q < sp.count; q++) {
            sp.off_p.push_back(bytes);
            const size_t pb = (size_t)plans[first + q].nslots * 2 * elem_size(compute_type);
            bytes += (pb + 15) & ~(size_t)15;
        }
        spans.push_back(sp);
    }
    // Layout invariant (the round-4 fault was a zero-fill that reached the
    // entries and tiles of a later launch): every region of every launch lies
    // inside the allocation, after the previous one, and overlaps no other;
    // in particular each member's partials and tickets (zeros of the image,
    // written by nothing else here) are its own.
    {
        size_t end = 0;
        auto region = [&](size_t off, size_t len) {
            const bool ok = off >= end && off + len <= bytes;
            end = off + len;
            return ok;
        };
        for (const Span &sp : spans) {
            int nt = 0, nl = 0;
            for (int q = 0; q < sp.count; q++) {
                int t0, t1;
                tile_range(plans[sp.first + q], &t0, &t1);
                nt += t1 - t0;
                nl += part == 1 ? 0 : (int)plans[sp.first + q].longrows.size();
            }
            bool ok = region(sp.off_e, (size_t)sp.count * sizeof(rsp::SpmvBatchEntry)) &&
                      region(sp.off_t, (size_t)nt * sizeof(SpmvBlock)) && region(sp.off_c, (size_t)nt * sizeof(int)) &&
                      region(sp.off_l, (size_t)nl * sizeof(SpmvLongRow));
            for (int q = 0; ok && q < sp.count; q++) ok = region(sp.off_16[q], plans[sp.first + q].c16.size() * 2);
            for (int q = 0; ok && q < sp.count; q++) ok = region(sp.off_r[q], plans[sp.first + q].runs.size() * 4);
            for (int q = 0; ok && q < sp.count; q++)
                ok = region(sp.off_p[q], (size_t)plans[sp.first + q].nslots * 2 * elem_size(compute_type));
            if (!ok) return RSP_STATUS_INTERNAL_ERROR;
        }
    }
    if (bytes > 0) RSP_CHECK_HIP(hipMalloc(&b->d_mem, bytes));
    rsp_an::hvec<unsigned char> host(bytes);
    for (const Span &sp : spans) {
        rsp::SpmvBatchArgs a{};
        a.entries = (const rsp::SpmvBatchEntry *)((char *)b->d_mem + sp.off_e);
        a.tiles = (const SpmvBlock *)((char *)b->d_mem + sp.off_t);
        a.cbases = (const int *)((char *)b->d_mem + sp.off_c);
        a.longrows = (const SpmvLongRow *)((char *)b->d_mem + sp.off_l);
        a.count = sp.count;
        for (int q = 0; q <= rsp::kSpmvBatchMax; q++)
            a.tiles_at.begin[q] = a.longs_at.begin[q] = INT_MAX;
        int nt = 0, nl = 0;
        for (int q = 0; q < sp.count; q++) {
            rsp_spmat_t A = mats[sp.first + q];
            const TilePlan &p = plans[sp.first + q];
            int t0, t1;
            tile_range(p, &t0, &t1);
            const int nlq = part == 1 ? 0 : (int)p.longrows.size();
            rsp::SpmvBatchEntry e{};
            e.rowptr = A->rowptr;
            e.colidx = A->colidx;
            e.vals = A->vals;
            e.x = d_x[sp.first + q];
            e.y = d_y[sp.first + q];
            e.partials = (void *)((char *)b->d_mem + sp.off_p[q]);  // this member's own
            e.cidx = (const unsigned short *)((char *)b->d_mem + sp.off_16[q]);
            e.runs = (const int *)((char *)b->d_mem + sp.off_r[q]);
            e.cmax = A->cols > 0 ? (int)(A->cols - 1) : 0;
            e.nnz = A->nnz_s;
            e.vector_ok = ((((uintptr_t)A->colidx) | ((uintptr_t)A->vals)) & 15) == 0;
            memcpy(host.data() + sp.off_e + (size_t)q * sizeof(e), &e, sizeof(e));
            a.tiles_at.begin[q] = nt;
            a.longs_at.begin[q] = nl;
            for (int t = t0; t < t1; t++)
                if (p.cbase[(size_t)t] != -1) b->entries_16bit += p.blocks[(size_t)t].k1 - p.blocks[(size_t)t].k0;
            b->tiles += t1 - t0;
            if (t1 > t0) {
                memcpy(host.data() + sp.off_t + (size_t)nt * sizeof(SpmvBlock), p.blocks.data() + t0,
                       (size_t)(t1 - t0) * sizeof(SpmvBlock));
                memcpy(host.data() + sp.off_c + (size_t)nt * sizeof(int), p.cbase.data() + t0,
                       (size_t)(t1 - t0) * sizeof(int));
            }
            if (nlq > 0)
                memcpy(host.data() + sp.off_l + (size_t)nl * sizeof(SpmvLongRow), p.longrows.data(),
                       (size_t)nlq * sizeof(SpmvLongRow));
            if (!p.c16.empty())
                memcpy(host.data() + sp.off_16[q], p.c16.data(), p.c16.size() * sizeof(uint16_t));
            if (!p.runs.empty())
                memcpy(host.data() + sp.off_r[q], p.runs.data(), p.runs.size() * sizeof(int));
            nt += t1 - t0;
            nl += nlq;
        }
        a.tiles_at.begin[sp.count] = nt;
        a.longs_at.begin[sp.count] = nl;
        b->launches.push_back(a);
    }
    // the image is value-initialised, so every member's long-row partials and
    // tickets go up as 0 (tickets start, and stay, at 0 between launches)
    if (bytes > 0) RSP_CHECK_HIP(hipMemcpy(b->d_mem, host.data(), bytes, hipMemcpyHostToDevice));
    for (int j = 0; j < count; j++) {
        b->mats.push_back(mats[j]);
        b->plan_gen.push_back(mats[j]->plan_gen);
    }
    *batch = b.release();
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_spmv_batch_run(rsp_handle_t h, rsp_spmv_batch_t b, const void *alpha,
                                const void *beta) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!b || !alpha || !beta) return RSP_STATUS_INVALID_VALUE;
    for (size_t j = 0; j < b->mats.size(); j++) {  // re-planned since create: stale copy
        const rsp_spmat_t A = b->mats[j];
        if (!A->planned || A->plan_gen != b->plan_gen[j]) return RSP_STATUS_INVALID_VALUE;
    }
    const double av = b->type == RSP_R_64F ? *(const double *)alpha : *(const float *)alpha;
    const double bv = b->type == RSP_R_64F ? *(const double *)beta : *(const float *)beta;
    if (b->part != 0 && bv != 0.0) return RSP_STATUS_INVALID_VALUE;
    for (rsp::SpmvBatchArgs a : b->launches) {
        a.alpha = av;
        a.beta = bv;
        a.variant = h->spmv_variant;
        hipError_t e;
        if (b->type == RSP_R_64F)
            e = rsp_k::spmv_batch_f64(a, h->stream);
        else
            e = h->ftz ? rsp_k_ftz::spmv_batch_f32(a, h->stream) : rsp_k::spmv_batch_f32(a, h->stream);
        if (e != hipSuccess) return RSP_STATUS_EXECUTION_FAILED;
    }
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_spmv_batch_info(rsp_spmv_batch_t b, int64_t *tiles, int64_t *entries_16bit) {
    if (!b || !tiles || !entries_16bit) return RSP_STATUS_INVALID_VALUE;
    *tiles = b->tiles;
    *entries_16bit = b->entries_16bit;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_spmv_batch_destroy(rsp_spmv_batch_t b) {
    if (!b) return RSP_STATUS_INVALID_VALUE;
    delete b;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_gather(rsp_handle_t h, rsp_datatype_t value_type, int64_t n, const int64_t *d_idx,
                        const void *d_src, void *d_dst) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    if (n < 0 || (n > 0 && (!d_idx || !d_src || !d_dst))) return RSP_STATUS_INVALID_VALUE;
    hipError_t e = rsp_k::gather(value_type == RSP_R_64F ? 8 : 4, n, d_idx, d_src, d_dst, h->stream);
    return e == hipSuccess ? RSP_STATUS_SUCCESS : RSP_STATUS_EXECUTION_FAILED;
}

rsp_status_t rsp_scatter(rsp_handle_t h, rsp_datatype_t value_type, int64_t n, const int64_t *d_idx,
                         const void *d_src, void *d_dst) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    if (n < 0 || (n > 0 && (!d_idx || !d_src || !d_dst))) return RSP_STATUS_INVALID_VALUE;
    hipError_t e = rsp_k::scatter(value_type == RSP_R_64F ? 8 : 4, n, d_idx, d_src, d_dst, h->stream);
    return e == hipSuccess ? RSP_STATUS_SUCCESS : RSP_STATUS_EXECUTION_FAILED;
}

/* --------------------------------------------------------------- ILU(0) */

static void ilu_free_device(rsp_ilu0_info *f) {
    f->solves_task.reset();  // (joins a solve planning still running)
    f->solves_ready = false;
    if (f->d_arena_s) (void)hipFree(f->d_arena_s);
    f->d_arena_s = nullptr;
    // every array except the slot layout lives in the arenas
    if (f->d_arena) (void)hipFree(f->d_arena);
    if (f->d_arena_u) (void)hipFree(f->d_arena_u);
    if (f->d_arena_sym) (void)hipFree(f->d_arena_sym);
    if (f->d_arena_pairs) (void)hipFree(f->d_arena_pairs);
    f->d_arena_sym = f->d_arena_pairs = nullptr;
    if (f->d_fslots) (void)hipFree(f->d_fslots);
    if (f->d_fbackup) (void)hipFree(f->d_fbackup);
    f->d_fbackup = nullptr;
    f->fbackup_bytes = 0;
    f->last_fac = rsp_ilu0_info::FacCall();
    for (rsp_ilu0_info::SolveCall &c : f->last_solve) c = rsp_ilu0_info::SolveCall();
    f->d_arena = f->d_arena_u = nullptr;
    f->d_usval = nullptr;
    f->d_fslots = nullptr;
    f->d_dpos = f->d_hasdiag = f->d_zero = f->d_fdone = nullptr;
    f->d_tk = nullptr;
    f->d_upd_ptr = f->d_upd_l = f->d_upd_u = f->d_lord = f->d_lend = f->d_udiv = nullptr;
    f->d_sval = f->d_sx = f->d_sdg = nullptr;
    f->fslev.clear();
    f->fruns.clear();
    f->d_ffitems = nullptr;
    f->d_forig = nullptr;
    f->d_frow = nullptr;
    f->d_rchunks = nullptr;
    f->d_ritems = nullptr;
    f->d_rpairs = f->d_rstaged = f->d_rrounds = nullptr;
    for (rsp_ilu0_info::Dag *d : {&f->L, &f->LT, &f->U, &f->F}) *d = rsp_ilu0_info::Dag();
    f->Lb = rsp_ilu0_info::BlkDag();
    f->LTb = rsp_ilu0_info::BlkDag();
    f->fac_one = f->fac_scale = false;
}

rsp_status_t rsp_create_ilu0_info(rsp_ilu0_info_t *info) {
    if (!info) return RSP_STATUS_INVALID_VALUE;
    rsp_ilu0_info *f = new (std::nothrow) rsp_ilu0_info();
    if (!f) return RSP_STATUS_ALLOC_FAILED;
    f->analysed = 0;
    f->structural_zero = -1;
    f->factored = 0;
    f->d_dpos = f->d_hasdiag = nullptr;
    f->d_zero = nullptr;
    f->d_upd_ptr = f->d_upd_l = f->d_upd_u = f->d_lord = f->d_lend = f->d_udiv = nullptr;
    f->n_updates = 0;
    *info = f;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_destroy_ilu0_info(rsp_ilu0_info_t info) {
    if (!info) return RSP_STATUS_INVALID_VALUE;
    ilu_free_device(info);
    delete info;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_ilu0_buffer_size(rsp_handle_t h, int n, int nnz, rsp_datatype_t value_type,
                                  rsp_ilu0_info_t info, size_t *buffer_size) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!info || !buffer_size || n < 0 || nnz < 0) return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    *buffer_size = 0;
    return RSP_STATUS_SUCCESS;
}

}  // extern "C"

// Device helpers of the ILU analysis upload.
template <typename V>
static hipError_t upload_vec(V **dst, const rsp_an::hvec<V> &v) {
    size_t bytes = std::max<size_t>(v.size(), 1) * sizeof(V);
    hipError_t e = hipMalloc((void **)dst, bytes);
    if (e != hipSuccess) return e;
    if (!v.empty()) e = hipMemcpy(*dst, v.data(), v.size() * sizeof(V), hipMemcpyHostToDevice);
    return e;
}

// Many arrays in ONE device allocation: add() records each array (host data
// to copy, or space only), commit() makes one hipMalloc and one copy per
// array. (One allocation per array — ~40 per analysis — had cost more than
// the copies themselves.)
struct Arena {
    struct Item {
        void **dst;
        const void *src;
        size_t bytes, copy, off;
    };
    rsp_an::hvec<Item> items;
    size_t total = 0;
    void add(void **dst, const void *src, size_t bytes, size_t copy) {
        items.push_back({dst, src, bytes, copy, total});
        total += (bytes + 255) & ~(size_t)255;
    }
    template <typename V>
    void up(V **dst, const rsp_an::hvec<V> &v) {
        add((void **)dst, v.empty() ? nullptr : v.data(), std::max<size_t>(v.size(), 1) * sizeof(V),
            v.size() * sizeof(V));
    }
    void space(void **dst, size_t bytes) { add(dst, nullptr, bytes, 0); }
    hipError_t commit(void **base, hipStream_t s) {
        *base = nullptr;
        if (total == 0) return hipSuccess;
        hipError_t e = hipMalloc(base, total);
        if (e != hipSuccess) return e;
        for (const Item &it : items) {
            *it.dst = (char *)*base + it.off;
            if (it.copy && e == hipSuccess)
                e = hipMemcpyAsync(*it.dst, it.src, it.copy, hipMemcpyHostToDevice, s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e;
    }
};

// Upload one DAG's solve plan (into the arena `ar`) and keep its host parts.
static void dag_upload(Arena &ar, rsp_ilu0_info::Dag &d, const rsp_an::DagHost &h) {
    d.ptr = h.ptr;
    d.batch = h.batch;
    d.group = h.group;
    d.segs = h.sp.segs;
    d.nshort = h.sp.nshort;
    d.nwave = h.sp.nwave;
    d.sbase = h.sp.sbase;
    d.nterms = (int)h.sp.tpos.size();
    if (!d.d_rows) {  // (L's levels may be in the factor's arena already)
        ar.up(&d.d_rows, h.rows);
        ar.up(&d.d_ptr, h.ptr);
    }
    ar.up(&d.d_tasks, h.sp.tasks);
    ar.up(&d.d_nshort, h.sp.nshort);
    ar.up(&d.d_tpos, h.sp.tpos);
    ar.up(&d.d_src, h.sp.src);
    ar.up(&d.d_chunks, h.sp.chunks);
    ar.up(&d.d_trow, h.sp.trow);
    ar.up(&d.d_sid, h.sp.sid);
    ar.up(&d.d_stg, h.sp.stg);
    ar.up(&d.d_fitems, h.sp.fitems);
}

// Upload a block-inverse solve plan (into the arena) with its scratch.
static void blk_upload(Arena &ar, rsp_ilu0_info::BlkDag &d, const rsp_an::BlkPlanHost &h) {
    d.on = true;
    d.nb = h.nb;
    d.lds_elems = h.lds_elems;
    d.lds_words = h.lds_words;
    d.entries = h.entries;
    d.nlong = h.nlong;
    d.segs = h.segs;
    ar.up(&d.d_order, h.order);
    ar.up(&d.d_desc, h.desc);
    ar.up(&d.d_rows, h.rows);
    ar.up(&d.d_ref, h.ref);
    ar.up(&d.d_vpos, h.vpos);
    ar.up(&d.d_eord, h.eord);
    ar.up(&d.d_lptr, h.lptr);
    ar.up(&d.d_rptr, h.rptr);
    ar.up(&d.d_rit, h.rit);
    ar.space(&d.d_ev, ((size_t)h.entries + 1) * sizeof(double));
    ar.space(&d.d_yp, ((size_t)h.n + 1) * sizeof(double));  // (+ a spare cell, trsv_blk_seg)
    ar.space(&d.d_rc, (size_t)h.nb * 64 * 144);
}

// Upload one DAG's per-row solve plan (L or L^T) into the arena and reserve
// the per-term arrays, which rsp_k::ilu_an_solve_terms then builds on the
// device (t: its arguments; pointers set at commit, the rest by the caller).
static void dag_upload_rows(Arena &ar, rsp_ilu0_info::Dag &d, const rsp_an::DagHost &h, int n,
                            rsp_k::SolveTermsArgs &t) {
    d.ptr = h.ptr;
    d.batch = h.batch;
    d.group = h.group;
    d.segs = h.sp.segs;
    d.nshort = h.sp.nshort;
    d.nwave = h.sp.nwave;
    d.sbase = h.sp.sbase;
    d.nterms = std::max(h.sp.nterm, 1);
    const size_t nx = h.rows.size(), nch = h.sp.chunks.size();
    long long thin_terms = 0;
    for (const rsp::LevelChunk &ch : h.sp.chunks) thin_terms += ch.k1 - ch.k0;
    if (!d.d_rows) {  // (L's levels may be in the factor's arena already)
        ar.up(&d.d_rows, h.rows);
        ar.up(&d.d_ptr, h.ptr);
    }
    ar.up(&d.d_tasks, h.sp.tasks);
    ar.up(&d.d_nshort, h.sp.nshort);
    ar.space((void **)&d.d_tpos, (size_t)d.nterms * 4);
    ar.space((void **)&d.d_src, (size_t)d.nterms * 4);
    ar.space((void **)&d.d_sid, (size_t)d.nterms * 4);
    ar.up(&d.d_chunks, h.sp.chunks);  // staged ranges written on the device
    ar.space((void **)&d.d_trow, std::max<size_t>(nx, 1) * sizeof(rsp::ThinRowPlan));
    ar.space((void **)&d.d_stg, (size_t)std::max(thin_terms, 1LL) * sizeof(rsp::StagedTerm));
    ar.up(&d.d_fitems, h.sp.fitems);
    ar.up((int **)&t.cbase, h.sp.cbase);
    ar.space((void **)&t.slot_of, (size_t)std::max(n, 1) * 4);
    ar.space((void **)&t.nst, (nch + 1) * 4);
    ar.space((void **)&t.nst_ptr, (nch + 1) * 4);
    size_t tb = 0;
    (void)rsp_k::ilu_an_scan(nullptr, nullptr, (int)nch + 1, nullptr, &tb, nullptr);
    ar.space(&t.scan, std::max<size_t>(tb, 16));
    t.n = n;
    t.nx = (int)nx;
    t.total = h.sp.nterm;
    t.nch = (int)nch;
    t.group = h.group;
}

// After the commit: the per-term arrays of a DAG uploaded by dag_upload_rows.
static hipError_t dag_build_terms(rsp_ilu0_info::Dag &d, rsp_k::SolveTermsArgs &t, hipStream_t s) {
    t.tasks = d.d_tasks;
    t.ptr = d.d_ptr;
    t.chunks = d.d_chunks;
    t.tpos = d.d_tpos;
    t.src = d.d_src;
    t.sid = d.d_sid;
    t.trow = d.d_trow;
    t.stg = d.d_stg;
    return rsp_k::ilu_an_solve_terms(t, s);
}

// Tests only (RSP_ILU_DIGEST): the device-built per-term arrays back into the
// host plan, so the digest covers them.
static hipError_t dag_download_terms(const rsp_ilu0_info::Dag &d, const rsp_k::SolveTermsArgs &t,
                                     rsp_an::DagHost &h, hipStream_t s) {
    rsp_an::SolvePlan &sp = h.sp;
    int nstg = 0;
    hipError_t e = hipMemcpyAsync(&nstg, t.nst_ptr + t.nch, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    sp.tpos.resize((size_t)d.nterms);
    sp.src.resize((size_t)d.nterms);
    sp.sid.resize((size_t)d.nterms);
    sp.trow.resize(std::max<size_t>((size_t)t.nx, 1));
    sp.stg.resize((size_t)std::max(nstg, 1));
    e = hipMemcpyAsync(sp.tpos.data(), d.d_tpos, sp.tpos.size() * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(sp.src.data(), d.d_src, sp.src.size() * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(sp.sid.data(), d.d_sid, sp.sid.size() * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(sp.trow.data(), d.d_trow, sp.trow.size() * sizeof(rsp::ThinRowPlan), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(sp.stg.data(), d.d_stg, sp.stg.size() * sizeof(rsp::StagedTerm), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(sp.chunks.data(), d.d_chunks, sp.chunks.size() * sizeof(rsp::LevelChunk),
                           hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e;
}

extern "C" {


// Budget of the fat factor slot layout (ints): RSP_ILU_SLOT_CAP_MB if set,
// else the smaller of 2 GB and 1/8 of the device memory free now.
static long long slot_cap_ints() {
    long long cap_mb = env_int("RSP_ILU_SLOT_CAP_MB", -1);
    if (cap_mb < 0) {
        size_t fr = 0, tot = 0;
        cap_mb = 2048;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) cap_mb = std::min<long long>(cap_mb, (long long)(fr >> 23));
    }
    return cap_mb * (1LL << 20) / 4;
}

// The data-parallel analysis on the device (ilu_analysis.hip), overlapped
// with the host level sets: validation, diagonal positions and structural
// zero, then the symbolic factor (update lists, stages, stage order, divisor
// positions), which stays on the device for the factor kernels; the host gets
// back the pattern, dpos / hasdiag, the update lists and stages its plans
// read. Rows longer than kAnDevRow entries (circuit hubs: a long serial chain
// of lower positions, slow at one GPU lane's memory latency) are done on the
// host (rsp_an::symbolic_rows) and their ranges uploaded. Fills hp (levels
// included).
static constexpr int kAnDevRow = 1024;
// device rows longer than this get one wave each for their stages (the
// thread-per-row kernel takes the rest; RSP_AN_WAVE_ROW overrides, A/B)
static constexpr int kAnWaveRow = 128;
static rsp_status_t ilu_symbolic_device(rsp_handle_t h, rsp_ilu0_info *f, const int *d_rp, const int *d_ci,
                                        const rsp_an::hvec<int> &rp, rsp_an::hvec<int> &ci, rsp_an::IluHostPlan &hp,
                                        rsp_an::Phases &ph, const std::function<void()> &after_levels) {
    const int n = hp.n, nnz_s = hp.nnz_s;
    hipStream_t s = h->stream;
    const bool tm3 = env_int("RSP_ILU_TIMING", 0) >= 3;  // diagnostics: sub-phase wall times
    auto t_last = std::chrono::steady_clock::now();
    auto sub = [&](const char *what) {
        if (!tm3) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "rsp_ilu0_analysis n=%d     %-22s %8.2f ms\n", n, what,
                std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    rsp_an::hvec<int> dev_rows, long_rows, wave_rows;
    const int wave_row = (int)env_int("RSP_AN_WAVE_ROW", kAnWaveRow);
    int cap0 = 1;  // the longest device row: the pair kernel's LDS per row
    for (int i = 0; i < n; i++) {
        const int len = rp[(size_t)i + 1] - rp[(size_t)i];
        if (len > kAnDevRow) {
            long_rows.push_back(i);
        } else {
            cap0 = std::max(cap0, len);
            if (len > wave_row) wave_rows.push_back(i);
        }
    }
    rsp_an::resize_uninit(dev_rows, (size_t)(n - (int)long_rows.size()));
    if (long_rows.empty()) {  // every row (FEM / stencil patterns): 0 .. n-1 in parallel
        rsp_an::parallel_for(n, 1 << 16, [&](long long a, long long b) {
            for (long long i = a; i < b; i++) dev_rows[(size_t)i] = (int)i;
        });
    } else {
        size_t w = 0;
        for (int i = 0; i < n; i++)
            if (rp[(size_t)i + 1] - rp[(size_t)i] <= kAnDevRow) dev_rows[w++] = i;
    }
    // The host level pass needs only the pattern: download it first, check it
    // (columns in range, rows strictly increasing: the device check below
    // returns the same verdict), take the diagonal positions from it and run
    // the level pass on a thread of its own while the device validates,
    // counts, scans and fills (round 4: the level pass used to wait for all
    // of that).
    if (nnz_s > 0) {
        RSP_CHECK_HIP(hipMemcpyAsync(ci.data(), d_ci, (size_t)nnz_s * 4, hipMemcpyDeviceToHost, s));
        RSP_CHECK_HIP(hipStreamSynchronize(s));
    }
    sub("D2H pattern");
    {
        // (and the diagonal flags and the structural zero: the device rows
        // kernel below computes the same arrays for the device, so nothing of
        // it is read back — round 5: two synchronisations fewer per analysis)
        std::atomic<int> bad{0}, szero{INT_MAX};
        rsp_an::resize_uninit(hp.dpos, (size_t)n);
        rsp_an::resize_uninit(hp.hasdiag, (size_t)n);
        rsp_an::parallel_for(n, 1 << 14, [&](long long r0, long long r1) {
            int sz = INT_MAX;
            for (long long i = r0; i < r1; i++) {
                const int a = rp[(size_t)i], b = rp[(size_t)i + 1];
                int d = b, prev = -1;
                for (int p = a; p < b; p++) {
                    const int c = ci[(size_t)p];
                    if (c < 0 || c >= n || c <= prev) bad.store(1, std::memory_order_relaxed);
                    if (d == b && c >= (int)i) d = p;
                    prev = c;
                }
                hp.dpos[(size_t)i] = d;
                const int hd = d < b && ci[(size_t)d] == (int)i ? 1 : 0;
                hp.hasdiag[(size_t)i] = hd;
                if (!hd && sz == INT_MAX) sz = (int)i;
            }
            for (int cur = szero.load(); sz < cur && !szero.compare_exchange_weak(cur, sz);) {
            }
        });
        if (bad.load()) return RSP_STATUS_INVALID_VALUE;  // a column out of range or a row not increasing
        hp.structural_zero = szero.load() == INT_MAX ? -1 : szero.load();
    }
    sub("host check + dpos");
    // (the L levels: the factor's; L^T's are the solve plans' thread's first step)
    rsp_an::Task levels([&] { rsp_an::plan_levels_lower(rp.data(), ci.data(), hp); });
    size_t scan_bytes = 0;
    RSP_CHECK_HIP(rsp_k::ilu_an_scan(nullptr, nullptr, nnz_s + 1, nullptr, &scan_bytes, s));
    Arena ar;
    int *d_flags = nullptr, *d_cnt = nullptr, *d_stage = nullptr, *d_scratch = nullptr, *d_rows = nullptr;
    void *d_scan = nullptr;
    ar.space((void **)&f->d_dpos, (size_t)std::max(n, 1) * 4);
    ar.space((void **)&f->d_hasdiag, (size_t)std::max(n, 1) * 4);
    ar.space((void **)&d_flags, 2 * 4);
    ar.space((void **)&d_cnt, ((size_t)nnz_s + 1) * 4);
    ar.space((void **)&f->d_upd_ptr, ((size_t)nnz_s + 1) * 4);
    ar.space((void **)&d_stage, (size_t)std::max(nnz_s, 1) * 4);
    ar.space((void **)&f->d_lord, (size_t)std::max(nnz_s, 1) * 4);
    ar.space((void **)&f->d_lend, (size_t)std::max(nnz_s, 1) * 4);
    ar.space((void **)&f->d_udiv, (size_t)std::max(nnz_s, 1) * 4);
    ar.space((void **)&d_scratch, (size_t)std::max(nnz_s, 1) * 4);
    ar.space(&d_scan, std::max<size_t>(scan_bytes, 16));
    ar.up(&d_rows, dev_rows);
    int *d_wrows = nullptr;
    ar.up(&d_wrows, wave_rows);
    sub("arena");
    RSP_CHECK_HIP(ar.commit(&f->d_arena_sym, s));
    // the device's diagonal positions and flags (its validation flags are not
    // read: the host check above gave the same verdict)
    RSP_CHECK_HIP(rsp_k::ilu_an_rows(n, d_rp, d_ci, f->d_dpos, f->d_hasdiag, d_flags, s));
    const int n_c[3] = {(int)dev_rows.size(), 0, 0};
    const int *rows_c[3] = {d_rows, nullptr, nullptr};
    RSP_CHECK_HIP(rsp_k::ilu_an_count(rows_c, n_c, cap0, d_rp, d_ci, f->d_dpos, f->d_hasdiag, d_cnt, d_scratch, s));
    sub("rows + count kernels");
    // the long rows' counts on the host
    rsp_an::hvec<int> hcnt(long_rows.empty() ? 0 : (size_t)nnz_s);
    rsp_an::symbolic_rows(long_rows, n, rp.data(), ci.data(), hp.dpos.data(), hp.hasdiag.data(), hcnt.data(),
                          nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
    for (int i : long_rows)
        RSP_CHECK_HIP(hipMemcpyAsync(d_cnt + rp[(size_t)i], hcnt.data() + rp[(size_t)i],
                                     (size_t)(rp[(size_t)i + 1] - rp[(size_t)i]) * 4, hipMemcpyHostToDevice, s));
    sub("long-row counts");
    RSP_CHECK_HIP(hipMemsetAsync(d_cnt + nnz_s, 0, 4, s));
    RSP_CHECK_HIP(rsp_k::ilu_an_scan(d_cnt, f->d_upd_ptr, nnz_s + 1, d_scan, &scan_bytes, s));
    rsp_an::resize_uninit(hp.sym.upd_ptr, (size_t)nnz_s + 1);
    RSP_CHECK_HIP(hipMemcpyAsync(hp.sym.upd_ptr.data(), f->d_upd_ptr, ((size_t)nnz_s + 1) * 4,
                                 hipMemcpyDeviceToHost, s));
    RSP_CHECK_HIP(hipStreamSynchronize(s));
    sub("scan + D2H upd_ptr");
    ph.mark("device rows");
    // a pair count past int would overflow the plans' indices
    const int total = hp.sym.upd_ptr[(size_t)nnz_s];
    if (total < 0) return RSP_STATUS_ALLOC_FAILED;
    Arena ap;
    ap.space((void **)&f->d_upd_l, (size_t)std::max(total, 1) * 4);
    ap.space((void **)&f->d_upd_u, (size_t)std::max(total, 1) * 4);
    RSP_CHECK_HIP(ap.commit(&f->d_arena_pairs, s));
    sub("pairs arena");
    RSP_CHECK_HIP(rsp_k::ilu_an_fill(rows_c, n_c, cap0, d_rp, d_ci, f->d_dpos, f->d_hasdiag, f->d_upd_ptr, d_scratch,
                                     f->d_upd_l, f->d_upd_u, s));
    RSP_CHECK_HIP(rsp_k::ilu_an_stages(n, std::min(wave_row, kAnDevRow), d_rp, d_ci, f->d_dpos, f->d_hasdiag, f->d_upd_ptr, f->d_upd_l,
                                       d_stage, f->d_lord, f->d_lend, f->d_udiv, d_scratch, d_wrows,
                                       (int)wave_rows.size(), s));
    // the level sets (host thread, started above) while the device fills the update lists
    levels.join();
    ph.mark("levels");
    after_levels();  // the solve plans need nothing more: started here
    // the host factor plan reads the update pairs of its thin rows only: those
    // are packed on the device and downloaded (FEM matrices have tens of
    // millions of pairs, nearly all in fat levels). Not with host-built hub
    // rows (their lists are uploaded from full host arrays) or for the tests'
    // plan digest (which covers the full arrays).
    const bool pack = long_rows.empty() && !env_int("RSP_ILU_DIGEST", 0) && env_int("RSP_ILU_PACK_PAIRS", 1);
    bool want_stage = true;  // the factor plan reads the stages of its thin rows only
    if (pack) {
        const rsp_an::hvec<int> trows = rsp_an::factor_thin_rows(rp.data(), hp);
        want_stage = !trows.empty();
        rsp_an::hvec<int> cbase(trows.size() + 1, 0);
        for (size_t r = 0; r < trows.size(); r++) {
            const int i = trows[r];
            cbase[r + 1] = cbase[r] + hp.sym.upd_ptr[(size_t)rp[(size_t)i + 1]] - hp.sym.upd_ptr[(size_t)rp[(size_t)i]];
        }
        const int packed = cbase.back();
        hp.sym.pair_base.assign((size_t)std::max(n, 1), 0);
        for (size_t r = 0; r < trows.size(); r++) hp.sym.pair_base[(size_t)trows[r]] = cbase[r];
        rsp_an::resize_uninit(hp.sym.upd_l, (size_t)packed);
        rsp_an::resize_uninit(hp.sym.upd_u, (size_t)packed);
        if (packed > 0) {
            Arena ag;
            int *d_trows = nullptr, *d_cbase = nullptr, *d_pl = nullptr, *d_pu = nullptr;
            void *d_gather = nullptr;
            ag.up(&d_trows, trows);
            ag.up(&d_cbase, cbase);
            ag.space((void **)&d_pl, (size_t)packed * 4);
            ag.space((void **)&d_pu, (size_t)packed * 4);
            RSP_CHECK_HIP(ag.commit(&d_gather, s));
            hipError_t e = rsp_k::ilu_an_gather_pairs(d_trows, (int)trows.size(), d_rp, f->d_upd_ptr, d_cbase,
                                                      f->d_upd_l, f->d_upd_u, d_pl, d_pu, s);
            if (e == hipSuccess) e = hipMemcpyAsync(hp.sym.upd_l.data(), d_pl, (size_t)packed * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipMemcpyAsync(hp.sym.upd_u.data(), d_pu, (size_t)packed * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            (void)hipFree(d_gather);
            RSP_CHECK_HIP(e);
        }
    } else {
        rsp_an::resize_uninit(hp.sym.upd_l, (size_t)total);
        rsp_an::resize_uninit(hp.sym.upd_u, (size_t)total);
        if (total > 0) {
            RSP_CHECK_HIP(hipMemcpyAsync(hp.sym.upd_l.data(), f->d_upd_l, (size_t)total * 4, hipMemcpyDeviceToHost, s));
            RSP_CHECK_HIP(hipMemcpyAsync(hp.sym.upd_u.data(), f->d_upd_u, (size_t)total * 4, hipMemcpyDeviceToHost, s));
        }
    }
    rsp_an::resize_uninit(hp.sym.stage, want_stage ? (size_t)nnz_s : 0);
    if (nnz_s > 0 && want_stage)
        RSP_CHECK_HIP(hipMemcpyAsync(hp.sym.stage.data(), d_stage, (size_t)nnz_s * 4, hipMemcpyDeviceToHost, s));
    RSP_CHECK_HIP(hipStreamSynchronize(s));
    sub("D2H pairs + stages");
    if (!long_rows.empty()) {  // the long rows' lists, stages, stage order, divisors on the host
        rsp_an::hvec<int> lord((size_t)nnz_s), lend((size_t)nnz_s), udiv((size_t)nnz_s);
        rsp_an::symbolic_rows(long_rows, n, rp.data(), ci.data(), hp.dpos.data(), hp.hasdiag.data(), nullptr,
                              hp.sym.upd_ptr.data(), hp.sym.upd_l.data(), hp.sym.upd_u.data(), hp.sym.stage.data(),
                              lord.data(), lend.data(), udiv.data());
        for (int i : long_rows) {
            const size_t rs = (size_t)rp[(size_t)i], len = (size_t)(rp[(size_t)i + 1] - rp[(size_t)i]);
            const size_t q0 = (size_t)hp.sym.upd_ptr[rs], nq = (size_t)hp.sym.upd_ptr[rs + len] - q0;
            if (nq > 0) {
                RSP_CHECK_HIP(hipMemcpyAsync(f->d_upd_l + q0, hp.sym.upd_l.data() + q0, nq * 4, hipMemcpyHostToDevice, s));
                RSP_CHECK_HIP(hipMemcpyAsync(f->d_upd_u + q0, hp.sym.upd_u.data() + q0, nq * 4, hipMemcpyHostToDevice, s));
            }
            RSP_CHECK_HIP(hipMemcpyAsync(f->d_lord + rs, lord.data() + rs, len * 4, hipMemcpyHostToDevice, s));
            RSP_CHECK_HIP(hipMemcpyAsync(f->d_lend + rs, lend.data() + rs, len * 4, hipMemcpyHostToDevice, s));
            RSP_CHECK_HIP(hipMemcpyAsync(f->d_udiv + rs, udiv.data() + rs, len * 4, hipMemcpyHostToDevice, s));
        }
        RSP_CHECK_HIP(hipStreamSynchronize(s));
    }
    sub("long rows");
    ph.mark("device symbolic");
    return RSP_STATUS_SUCCESS;
}

static rsp_status_t rsp_ilu0_analysis_impl(rsp_handle_t h, int n, int nnz, const int *d_row_offsets,
                               const int *d_col_ind, rsp_ilu0_info_t f) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    // diagnostics: RSP_ILU_TIMING=1 prints the wall time of each analysis phase
    rsp_an::Phases ph;
    ph.print = env_int("RSP_ILU_TIMING", 0) != 0;
    ph.n = n;
    ph.start();
    if (!f || n < 0 || nnz < 0 || (n > 0 && !d_row_offsets)) return RSP_STATUS_INVALID_VALUE;
    const bool tm3 = env_int("RSP_ILU_TIMING", 0) >= 3;  // diagnostics: preamble sub-phases
    auto t_pre = std::chrono::steady_clock::now();
    auto pre = [&](const char *what) {
        if (!tm3) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "rsp_ilu0_analysis n=%d     %-22s %8.2f ms\n", n, what,
                std::chrono::duration<double, std::milli>(t - t_pre).count());
        t_pre = t;
    };
    ilu_free_device(f);
    pre("free");
    f->analysed = 0;
    f->factored = 0;
    f->structural_zero = -1;
    f->host.reset();
    // the pattern to the host (row offsets first: the stored entries must lie
    // inside the declared arrays before colidx is read)
    rsp_an::hvec<int> rp((size_t)n + 1, 0);
    if (n > 0) {
        RSP_CHECK_HIP(hipMemcpyAsync(rp.data(), d_row_offsets, ((size_t)n + 1) * sizeof(int),
                                     hipMemcpyDeviceToHost, h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
    }
    if (rp[0] != 0) return RSP_STATUS_INVALID_VALUE;
    for (int i = 0; i < n; i++)
        if (rp[(size_t)i + 1] < rp[(size_t)i]) return RSP_STATUS_INVALID_VALUE;
    const int nnz_s = rp[(size_t)n];
    if (nnz_s > 0 && !d_col_ind) return RSP_STATUS_INVALID_VALUE;
    if (nnz_s > nnz) return RSP_STATUS_INVALID_VALUE;  // entries past the declared arrays
    pre("D2H rowptr + checks");
    rsp_an::hvec<int> ci;
    rsp_an::resize_uninit(ci, (size_t)nnz_s);  // (downloaded whole below)
    std::unique_ptr<rsp_an::IluHostPlan> hp(new (std::nothrow) rsp_an::IluHostPlan());
    if (!hp) return RSP_STATUS_ALLOC_FAILED;
    hp->n = n;
    hp->nnz_s = nnz_s;
    // the solve plans are built on a second thread from the moment the levels
    // exist, under the symbolic factor's transfers and the factor plan
    // their per-term half is built on the device after the upload
    // (RSP_ILU_HOST_TERMS=1: on the host, as rsp_ilu0_analysis_host does; A/B)
    const bool dev_terms = n > 0 && !env_int("RSP_ILU_HOST_TERMS", 0);
    // (declared after rp, ci, hp: destroyed - joined - before them if the
    // factor plan throws)
    // the solve plans' thread outlives this call (rsp_ilu0_info::solves_task):
    // it holds the buffers, which move into the info below, not the locals
    std::unique_ptr<rsp_an::Task> solves;
    const int *rpd = rp.data(), *cid = ci.data();
    rsp_an::IluHostPlan *H = hp.get();
    rsp_status_t st = ilu_symbolic_device(h, f, d_row_offsets, d_col_ind, rp, ci, *hp, ph, [&] {
        solves.reset(new rsp_an::Task([rpd, cid, H, n, dev_terms] {
            rsp_an::plan_levels_upper(rpd, cid, *H);  // L^T levels, the transposed lower part
            // block-inverse plans of the deep DAGs, beside the row plans
            auto blk = [&](int kind) {
                const rsp_an::DagHost &dg = kind == 0 ? H->L : H->LT;
                if (!rsp_an::blocks_wanted(n, (int)dg.ptr.size() - 1)) return;
                bool &has = kind == 0 ? H->has_lb : H->has_ltb;
                has = rsp_an::plan_blocks(kind, rpd, cid, *H, kind == 0 ? H->Lb : H->LTb);
            };
            rsp_an::Task bl([&] { blk(0); }), bt([&] { blk(1); });
            if (dev_terms)
                rsp_an::plan_solves_rows(rpd, cid, *H);
            else
                rsp_an::plan_solves(rpd, cid, *H);
            bl.join();
            bt.join();
        }));
    });
    if (st == RSP_STATUS_SUCCESS) rsp_an::plan_factor(rp.data(), ci.data(), slot_cap_ints(), *hp);
    if (st != RSP_STATUS_SUCCESS) {
        solves.reset();  // (joined before the buffers it reads go)
        ilu_free_device(f);
        return st;
    }
    // the U DAG (--true-lu extension) is planned on its first use
    ph.mark("plans");
    f->structural_zero = hp->structural_zero;
    f->n_updates = nnz_s > 0 ? (long long)hp->sym.upd_ptr[(size_t)nnz_s] : 0;
    f->fac_batch = hp->fac_batch;
    f->fac_segs = hp->fplan.segs;
    f->fslev = hp->fslev;
    if (env_int("RSP_ILU_DIGEST", 0)) {  // tests only: the device-only symbolic arrays too
        hp->sym.lord.resize((size_t)nnz_s);
        hp->sym.lend.resize((size_t)nnz_s);
        hp->udiv.resize((size_t)nnz_s);
        hipError_t e = hipSuccess;
        if (nnz_s > 0) {
            e = hipMemcpyAsync(hp->sym.lord.data(), f->d_lord, (size_t)nnz_s * 4, hipMemcpyDeviceToHost, h->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(hp->sym.lend.data(), f->d_lend, (size_t)nnz_s * 4, hipMemcpyDeviceToHost, h->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(hp->udiv.data(), f->d_udiv, (size_t)nnz_s * 4, hipMemcpyDeviceToHost, h->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        }
        f->digest = e == hipSuccess ? 1 : 0;  // computed once the solve terms exist (below)
    }
    // (diagnostics, RSP_ILU_TIMING >= 3: the upload's steps)
    auto t_up = std::chrono::steady_clock::now();
    auto up_step = [&](const char *what) {
        if (!tm3) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "rsp_ilu0_analysis n=%d     upload: %-16s %8.2f ms\n", n, what,
                std::chrono::duration<double, std::milli>(t - t_up).count());
        t_up = t;
    };
    // everything in one device allocation
    Arena ar;
    ar.up(&f->d_rchunks, hp->fplan.chunks);
    ar.up(&f->d_ritems, hp->fplan.items);
    ar.up(&f->d_rpairs, hp->fplan.pairs);
    ar.up(&f->d_rstaged, hp->fplan.staged);
    ar.up(&f->d_rrounds, hp->fplan.rounds);
    ar.up(&f->d_frow, hp->frow);
    ar.up(&f->d_ffitems, hp->ffitems);
    f->fruns = hp->fruns;
    f->fac_one = hp->fac_one;  // the factor's one level (rsp_an::IluHostPlan::F), else L's
    f->fac_scale = hp->fac_scale;
    if (hp->fac_one) {
        f->F.ptr = hp->F.ptr;
        ar.up(&f->F.d_rows, hp->F.rows);
        ar.up(&f->F.d_ptr, hp->F.ptr);
    } else {  // the factor walks L's levels (the solve plans add the rest of L at ilu_solves_ready)
        f->L.ptr = hp->L.ptr;
        ar.up(&f->L.d_rows, hp->L.rows);
        ar.up(&f->L.d_ptr, hp->L.ptr);
    }
    // flow runs: the saved upper input values of their rows (ilu0_flow_prep)
    if (!hp->fruns.empty()) ar.space(&f->d_forig, (size_t)std::max(hp->nnz_s, 1) * sizeof(double));
    ar.space((void **)&f->d_zero, 8 * sizeof(int));  // zero pivot, flow give-ups, claim counter
    // flow items (factor rows; solve items hold >= 1 row each, U's included) <= n
    ar.space((void **)&f->d_fdone, (size_t)std::max(n, 1) * sizeof(int));
    ar.space((void **)&f->d_tk, 2 * rsp::kFlowTicketCtrs * sizeof(unsigned));
    int4 *d_desc = nullptr;
    long long *d_offs = nullptr;
    if (!hp->slot_desc.empty()) {
        ar.up(&d_desc, hp->slot_desc);
        ar.up(&d_offs, hp->slot_offs);
    }
    up_step("arena build");
    hipError_t e = ar.commit(&f->d_arena, h->stream);
    up_step("commit (H2D)");
    if (e == hipSuccess) e = hipMemsetD32(f->d_zero, INT_MAX, 1);
    if (e == hipSuccess) e = hipMemsetD32(f->d_zero + 1, 0, 7);
    if (e == hipSuccess) e = hipMemsetD32(f->d_fdone, 0, (size_t)std::max(n, 1));
    if (e == hipSuccess) e = hipMemsetD32(f->d_tk, 0, 2 * rsp::kFlowTicketCtrs);
    f->tk_seq = 0;
    f->fac_gen = 0;
    f->claim_host = 0;
    f->flow_epoch = 0;
    f->solve_gen[0] = f->solve_gen[1] = f->solve_gen[2] = 0;
    // fat factor slots, written on the device from the uploaded symbolic
    // arrays; the layout is an optimisation: without its memory, or if the
    // build fails, the FacRow path factors every fat level (same bits)
    if (e == hipSuccess && hp->slot_total > 0) {
        hipError_t es = hipMalloc((void **)&f->d_fslots, (size_t)hp->slot_total * sizeof(int));
        if (es == hipSuccess) {
            rsp::IluArgs a{};
            a.n = n;
            a.rowptr = d_row_offsets;
            a.dpos = f->d_dpos;
            a.hasdiag = f->d_hasdiag;
            a.upd_ptr = f->d_upd_ptr;
            a.upd_l = f->d_upd_l;
            a.upd_u = f->d_upd_u;
            a.lord = f->d_lord;
            a.lend = f->d_lend;
            a.udiv = f->d_udiv;
            a.plan.rows = f->fdag().d_rows;
            es = rsp_k::ilu0_build_slots(a, d_desc, d_offs, (int)hp->slot_desc.size(), f->d_fslots, h->stream);
            if (es == hipSuccess) es = hipStreamSynchronize(h->stream);
        }
        up_step("factor slots");
        if (es != hipSuccess) {
            (void)hipGetLastError();
            if (f->d_fslots) (void)hipFree(f->d_fslots);
            f->d_fslots = nullptr;
            f->fslev.assign(f->fslev.size(), rsp::FacSlotLevel{0, 0, 0, 0, 0});
            f->fruns.clear();  // the flow runs read the slots too
        }
    }
    ph.mark("upload");
    if (e != hipSuccess) {
        ilu_free_device(f);
        return e == hipErrorOutOfMemory ? RSP_STATUS_ALLOC_FAILED : RSP_STATUS_EXECUTION_FAILED;
    }
    // (the buffers keep their addresses: the solve plans' thread reads them on)
    f->host_rp.swap(rp);
    f->host_ci.swap(ci);
    f->host = std::move(hp);
    f->solves_task = std::move(solves);
    f->dev_terms = dev_terms;
    f->han = h;
    f->n = n;
    f->nnz_s = nnz_s;
    f->rowptr = d_row_offsets;
    f->colidx = d_col_ind;
    f->analysed = 1;
    return RSP_STATUS_SUCCESS;
}

// The L and L^T solve plans (rsp_trsv_analysis, or the first solve): wait
// for their thread (started by rsp_ilu0_analysis) and upload them — the row
// plans, the block-inverse plans of deep DAGs, the solve streams — and build
// their per-term half on the device. Once per analysis.
static rsp_status_t ilu_solves_ready(rsp_handle_t h, rsp_ilu0_info *f) {
    if (f->solves_ready) return RSP_STATUS_SUCCESS;
    if (!f->analysed || !f->host || !h) return RSP_STATUS_INVALID_VALUE;
    if (f->solves_task) {
        std::unique_ptr<rsp_an::Task> t = std::move(f->solves_task);
        try {
            t->join();
        } catch (...) {  // the plans are incomplete: the info needs a new analysis
            f->analysed = 0;
            throw;  // (guarded: an error status)
        }
    }
    rsp_an::IluHostPlan *hp = f->host.get();
    const int n = f->n;
    const bool dev_terms = f->dev_terms;
    const int *d_row_offsets = f->rowptr, *d_col_ind = f->colidx;
    const bool tm3 = env_int("RSP_ILU_TIMING", 0) >= 3;  // diagnostics
    auto t_up = std::chrono::steady_clock::now();
    auto up_step = [&](const char *what) {
        if (!tm3) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "rsp_trsv_analysis n=%d     upload: %-16s %8.2f ms\n", n, what,
                std::chrono::duration<double, std::milli>(t - t_up).count());
        t_up = t;
    };
    Arena ar;
    rsp_k::SolveTermsArgs tl{}, tt{};
    if (dev_terms) {
        dag_upload_rows(ar, f->L, hp->L, n, tl);
        dag_upload_rows(ar, f->LT, hp->LT, n, tt);
        tl.kind = 0;
        tl.rp = d_row_offsets;
        tl.ci = d_col_ind;
        // the split term order (rsp_an::split_terms); none (nullptr) for the
        // reference's order
        if (!hp->lpos.empty()) {
            ar.up((int **)&tl.lpos, hp->lpos);
            ar.up((int **)&tl.ne, hp->ne_l);
            ar.up((int **)&tt.ne, hp->ne_lt);
        }
        tt.kind = 1;
        ar.up((int **)&tt.ltp, hp->ltp);
        ar.up((int **)&tt.lts, hp->lts);
        ar.up((int **)&tt.ltc, hp->ltc);
    } else {
        dag_upload(ar, f->L, hp->L);
        dag_upload(ar, f->LT, hp->LT);
    }
    if (hp->has_lb) blk_upload(ar, f->Lb, hp->Lb);
    if (hp->has_ltb) blk_upload(ar, f->LTb, hp->LTb);
    // solve streams: values per flat term, alpha x and u_ii per level-order slot (fp64 size)
    const size_t nt = (size_t)std::max({f->L.nterms, f->LT.nterms, 1});
    ar.space(&f->d_sval, nt * sizeof(double));
    ar.space(&f->d_sx, (size_t)std::max(n, 1) * sizeof(double));
    ar.space(&f->d_sdg, (size_t)std::max(n, 1) * sizeof(double));
    up_step("arena build");
    hipError_t e = ar.commit(&f->d_arena_s, h->stream);
    up_step("commit (H2D)");
    if (e == hipSuccess && dev_terms) {
        tl.dpos = f->d_dpos;
        e = dag_build_terms(f->L, tl, h->stream);
        if (e == hipSuccess) e = dag_build_terms(f->LT, tt, h->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    up_step("solve terms");
    if (e == hipSuccess && env_int("RSP_ILU_DIGEST", 0)) {  // tests only
        if (dev_terms) {
            e = dag_download_terms(f->L, tl, hp->L, h->stream);
            if (e == hipSuccess) e = dag_download_terms(f->LT, tt, hp->LT, h->stream);
        }
        f->digest = e == hipSuccess && f->digest ? rsp_an::digest(*hp) : 0;
    }
    if (e != hipSuccess) {
        if (f->d_arena_s) (void)hipFree(f->d_arena_s);
        f->d_arena_s = nullptr;
        f->L = f->LT = rsp_ilu0_info::Dag();
        f->Lb = f->LTb = rsp_ilu0_info::BlkDag();
        f->analysed = 0;  // (the factor's L levels went with L: analyse again)
        return e == hipErrorOutOfMemory ? RSP_STATUS_ALLOC_FAILED : RSP_STATUS_EXECUTION_FAILED;
    }
    // host copies kept for the U plan, built on first use (rsp_trsv_upper)
    hp->sym = rsp_an::IluSymbolic();
    hp->fplan = rsp_an::FacPlan();
    hp->L = rsp_an::DagHost();
    hp->LT = rsp_an::DagHost();
    hp->F = rsp_an::DagHost();
    hp->Lb = rsp_an::BlkPlanHost();
    hp->LTb = rsp_an::BlkPlanHost();
    hp->ltp.clear();
    hp->lts.clear();
    hp->ltc.clear();
    hp->udiv.clear();
    hp->frow.clear();
    hp->slot_desc.clear();
    hp->slot_offs.clear();
    f->solves_ready = true;
    return RSP_STATUS_SUCCESS;
}

// The U DAG's plan (rsp_trsv_upper, the --true-lu extension), on first use.
static rsp_status_t ilu_plan_u(rsp_handle_t h, rsp_ilu0_info *f) {
    if (f->U.d_ptr) return RSP_STATUS_SUCCESS;
    if (!f->host) return RSP_STATUS_INTERNAL_ERROR;
    rsp_an::plan_u(f->host_rp.data(), f->host_ci.data(), *f->host);
    Arena ar;
    dag_upload(ar, f->U, f->host->U);
    // its streams (the L / L^T ones are sized for those DAGs' terms)
    ar.space(&f->d_usval, (size_t)std::max(f->U.nterms, 1) * sizeof(double));
    hipError_t e = ar.commit(&f->d_arena_u, h->stream);
    f->host->U = rsp_an::DagHost();
    if (e != hipSuccess) {
        if (f->d_arena_u) (void)hipFree(f->d_arena_u);
        f->d_arena_u = nullptr;
        f->U = rsp_ilu0_info::Dag();
        return e == hipErrorOutOfMemory ? RSP_STATUS_ALLOC_FAILED : RSP_STATUS_EXECUTION_FAILED;
    }
    return RSP_STATUS_SUCCESS;
}

static rsp_status_t rsp_ilu0_analysis_host_impl(int n, const int *row_offsets, const int *col_ind,
                                    int *levels_lower, int *levels_upper, uint64_t *digest,
                                    double *phase_ms) {
    rsp_an::Phases ph;
    ph.n = n;
    ph.ms = phase_ms;
    if (phase_ms)
        for (int i = 0; i < rsp_an::kPhases; i++) phase_ms[i] = 0.0;
    ph.start();
    rsp_an::IluHostPlan hp;
    rsp_status_t st = rsp_an::plan_host(n, row_offsets, col_ind, 1LL << 29, false, hp, ph);
    if (st != RSP_STATUS_SUCCESS) return st;
    if (levels_lower) *levels_lower = (int)hp.L.ptr.size() - 1;
    if (levels_upper) *levels_upper = (int)hp.LT.ptr.size() - 1;
    if (digest) *digest = rsp_an::digest(hp);
    return RSP_STATUS_SUCCESS;
}

static rsp_status_t rsp_spmv_plan_host_impl(int m, const int *rp, const int *ci, int64_t nnz,
                                            rsp_datatype_t type, int64_t *tiles, int64_t *e16,
                                            int64_t *est) {
    if (m < 0 || (m > 0 && (!rp || !ci)) || !tiles || !e16 || !est) return RSP_STATUS_INVALID_VALUE;
    if (type != RSP_R_64F && type != RSP_R_32F) return RSP_STATUS_NOT_SUPPORTED;
    TilePlan p;
    make_tile_plan(rp, ci, m, nnz, type, 0, -1, true, p);
    const int ucap = type == RSP_R_64F ? SpmvTile<double>::kStageSlots : SpmvTile<float>::kStageSlots;
    for (size_t t = 0; t < p.blocks.size(); t++) {
        const SpmvBlock &b = p.blocks[t];
        const int cb = p.cbase[t];
        if (cb == -1) continue;
        for (int k = b.k0; k < b.k1; k++) {
            int col;
            if (cb >= 0) {
                col = cb + p.c16[(size_t)k];
            } else {
                const int code = -2 - cb, nr = code & 255, off = code >> 8;
                if (nr == 255) {  // list mode (fp64): {base, U}, then U uint16 offsets
                    if (type != RSP_R_64F) return RSP_STATUS_INTERNAL_ERROR;
                    if ((size_t)2 * off + 2 > p.runs.size()) return RSP_STATUS_INTERNAL_ERROR;
                    const int *r = p.runs.data() + 2 * (size_t)off;
                    const int U = r[1];
                    if (U < 1 || U > ucap || (size_t)2 * off + 2 + 2 * (size_t)((U + 3) / 4) > p.runs.size())
                        return RSP_STATUS_INTERNAL_ERROR;
                    const uint16_t *o = reinterpret_cast<const uint16_t *>(r + 2);
                    for (int u = 1; u < U; u++)
                        if (o[u] <= o[u - 1]) return RSP_STATUS_INTERNAL_ERROR;
                    const int u = p.c16[(size_t)k];
                    if (u >= U) return RSP_STATUS_INTERNAL_ERROR;
                    if (r[0] + o[u] != ci[k]) return RSP_STATUS_INTERNAL_ERROR;
                    continue;
                }
                if (nr < 1 || nr > rsp::kStageRuns || (size_t)2 * (off + nr + 1) > p.runs.size())
                    return RSP_STATUS_INTERNAL_ERROR;
                const int *r = p.runs.data() + 2 * (size_t)off;
                const int U = r[2 * nr + 1];
                if (r[1] != 0 || U > ucap) return RSP_STATUS_INTERNAL_ERROR;
                for (int j = 1; j <= nr; j++)
                    if (r[2 * j + 1] <= r[2 * j - 1] || (j < nr && r[2 * j] <= r[2 * j - 2] + (r[2 * j + 1] - r[2 * j - 1]) - 1))
                        return RSP_STATUS_INTERNAL_ERROR;
                const int u = p.c16[(size_t)k];
                if (u >= U) return RSP_STATUS_INTERNAL_ERROR;
                int j = 0;
                while (j + 1 < nr && r[2 * (j + 1) + 1] <= u) j++;
                col = r[2 * j] + (u - r[2 * j + 1]);
            }
            if (col != ci[k]) return RSP_STATUS_INTERNAL_ERROR;
        }
    }
    *tiles = (int64_t)p.blocks.size();
    *e16 = p.nnz_c16;
    *est = p.nnz_staged;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_ilu0_plan_digest(rsp_ilu0_info_t f, uint64_t *digest) {
    if (!f || !digest || !f->analysed) return RSP_STATUS_INVALID_VALUE;
    const rsp_status_t st = ilu_solves_ready(f->han, f);  // (the digest covers the solve plans)
    if (st != RSP_STATUS_SUCCESS) return st;
    if (!f->digest) return RSP_STATUS_INVALID_VALUE;
    *digest = f->digest;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_ilu0_solve_blocks(rsp_ilu0_info_t f, int *blocks_lower, int *blocks_upper) {
    if (!f || !blocks_lower || !blocks_upper || !f->analysed) return RSP_STATUS_INVALID_VALUE;
    const rsp_status_t st = ilu_solves_ready(f->han, f);
    if (st != RSP_STATUS_SUCCESS) return st;
    *blocks_lower = f->Lb.on ? f->Lb.nb : 0;
    *blocks_upper = f->LTb.on ? f->LTb.nb : 0;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_ilu0_levels(rsp_ilu0_info_t f, int *levels_lower, int *levels_upper) {
    if (!f || !f->analysed) return RSP_STATUS_INVALID_VALUE;
    if (levels_upper) {  // (the L^T levels come with the solve plans)
        const rsp_status_t st = ilu_solves_ready(f->han, f);
        if (st != RSP_STATUS_SUCCESS) return st;
    }
    if (levels_lower) *levels_lower = (int)f->L.ptr.size() - 1;
    if (levels_upper) *levels_upper = (int)f->LT.ptr.size() - 1;
    return RSP_STATUS_SUCCESS;
}

// the recovery runs (rsp_ilu0_info::d_fbackup / last_solve), defined below
static bool flow_recover();
static rsp_status_t ilu_factor_run(rsp_handle_t h, rsp_ilu0_info_t f, rsp_datatype_t value_type, void *d_values,
                                   bool flow_ok);
static rsp_status_t rsp_trsv_lower_unit_impl(rsp_handle_t h, rsp_operation_t op, const void *alpha,
                                             rsp_ilu0_info_t f, rsp_datatype_t value_type, const void *d_values,
                                             const void *d_x, void *d_y, bool flow_ok);
static rsp_status_t rsp_trsv_upper_impl(rsp_handle_t h, const void *alpha, rsp_ilu0_info_t f,
                                        rsp_datatype_t value_type, const void *d_values, const void *d_x, void *d_y,
                                        bool flow_ok);

// Re-run one recorded solve without flow launches (rsp_ilu0_info::last_solve).
static rsp_status_t rerun_solve(rsp_handle_t h, rsp_ilu0_info *f, int which) {
    const rsp_ilu0_info::SolveCall c = f->last_solve[which];
    const double a64 = c.alpha;
    const float a32 = (float)c.alpha;
    const void *al = c.type == RSP_R_64F ? (const void *)&a64 : (const void *)&a32;
    const int ftz = h->ftz;
    h->ftz = c.ftz;  // the mode of the call being re-run
    const rsp_status_t st = which == RSP_TRSV_U
                                ? rsp_trsv_upper_impl(h, al, f, c.type, c.vals, c.x, c.y, false)
                                : rsp_trsv_lower_unit_impl(h, c.op, al, f, c.type, c.vals, c.x, c.y, false);
    h->ftz = ftz;
    return st;
}

// The recorded solves made after call `seq`, in call order (their inputs
// came from the call being recovered).
struct LaterSolves {
    int w[3];
    int k = 0;
};
static LaterSolves later_solves(const rsp_ilu0_info *f, long long seq) {
    LaterSolves l;
    for (int w = 0; w < 3; w++)
        if (f->last_solve[w].valid && f->last_solve[w].seq > seq) l.w[l.k++] = w;
    std::sort(l.w, l.w + l.k, [&](int a, int b) { return f->last_solve[a].seq < f->last_solve[b].seq; });
    return l;
}
// Whether a re-run of `first` (a solve kind, or -1 for the factor) and then
// of the solves `l` reads the inputs the original calls read: no recorded
// call after a re-run call may have written (its y) over that call's x or
// values. The ping-pong pattern (L solve r -> z, then L^T z -> r) overwrites
// the L solve's x, so its re-run would read the L^T result: not recoverable.
static bool overlaps(const void *a, size_t na, const void *b, size_t nb) {
    const char *p = (const char *)a, *q = (const char *)b;
    return p && q && p < q + nb && q < p + na;
}
static bool rerun_inputs_intact(const rsp_ilu0_info *f, int first, const LaterSolves &l) {
    int seq[4], k = 0;
    if (first >= 0) seq[k++] = first;
    for (int j = 0; j < l.k; j++) seq[k++] = l.w[j];
    for (int a = 0; a < k; a++) {
        const rsp_ilu0_info::SolveCall &c = f->last_solve[seq[a]];
        const size_t ny = (size_t)f->n * elem_size(c.type), nv = (size_t)f->nnz_s * elem_size(c.type);
        for (int b = a + 1; b < k; b++) {
            const rsp_ilu0_info::SolveCall &d = f->last_solve[seq[b]];
            if (overlaps(d.y, (size_t)f->n * elem_size(d.type), c.x, ny) ||
                overlaps(d.y, (size_t)f->n * elem_size(d.type), c.vals, nv))
                return false;
        }
    }
    if (first < 0 && f->last_fac.valid)  // the factor's values are restored from the copy, but a
        for (int a = 0; a < k; a++) {    // later solve must not have written into them
            const rsp_ilu0_info::SolveCall &d = f->last_solve[seq[a]];
            if (overlaps(d.y, (size_t)f->n * elem_size(d.type), f->last_fac.vals,
                         (size_t)f->nnz_s * elem_size(f->last_fac.type)))
                return false;
        }
    return true;
}

static rsp_status_t rerun_solves(rsp_handle_t h, rsp_ilu0_info *f, const LaterSolves &l) {
    for (int j = 0; j < l.k; j++) {
        const rsp_status_t st = rerun_solve(h, f, l.w[j]);
        if (st != RSP_STATUS_SUCCESS) return st;
    }
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_ilu0_zero_pivot(rsp_handle_t h, rsp_ilu0_info_t f, int *position) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !position) return RSP_STATUS_INVALID_VALUE;
    *position = -1;
    if (!f->analysed) return RSP_STATUS_INVALID_VALUE;
    int pos = f->structural_zero;
    int z[2] = {INT_MAX, 0};  // zero pivot, give-up generation of the factor calls
    RSP_CHECK_HIP(hipMemcpyAsync(z, f->d_zero, sizeof(z), hipMemcpyDeviceToHost, h->stream));
    RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
    // the last factor's flow wait gave up: its values are wrong. Recovered
    // (rsp_ilu0_info::d_fbackup): the input values restored, the factor run
    // again without flow launches; else reported.
    if (f->factored && f->fac_gen > 0 && z[1] == f->fac_gen) {
        if (!f->last_fac.valid || !flow_recover()) return RSP_STATUS_EXECUTION_FAILED;
        const LaterSolves later = later_solves(f, f->last_fac.seq);
        if (!rerun_inputs_intact(f, -1, later)) return RSP_STATUS_EXECUTION_FAILED;
        f->last_fac.valid = 0;
        RSP_CHECK_HIP(hipMemcpyAsync(f->last_fac.vals, f->d_fbackup, (size_t)f->nnz_s * elem_size(f->last_fac.type),
                                     hipMemcpyDeviceToDevice, h->stream));
        const int ftz = h->ftz;
        h->ftz = f->last_fac.ftz;  // the mode of the call being re-run
        rsp_status_t st = ilu_factor_run(h, f, f->last_fac.type, f->last_fac.vals, false);
        h->ftz = ftz;
        if (st == RSP_STATUS_SUCCESS) st = rerun_solves(h, f, later);
        if (st != RSP_STATUS_SUCCESS) return st;
        RSP_CHECK_HIP(hipMemcpyAsync(z, f->d_zero, sizeof(z), hipMemcpyDeviceToHost, h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
        if (z[1] == f->fac_gen) return RSP_STATUS_EXECUTION_FAILED;
    }
    if (f->factored && z[0] != INT_MAX && (pos < 0 || z[0] < pos)) pos = z[0];
    if (pos >= 0) {
        *position = pos;
        return RSP_STATUS_ZERO_PIVOT;
    }
    return RSP_STATUS_SUCCESS;
}

// cusparseXcsrsv2_zeroPivot for the solves (reference: the csrsv2 info
// objects of GPU/ilu0.cu:143-150). Host-blocking. EXECUTION_FAILED: the last
// solve of that kind gave up a flow wait (its y is wrong; never expected, a
// bound instead of a GPU hang). The unit-lower solves have no pivots; the U
// solve (extension) reports the factor's zero pivot, which it divides by.
rsp_status_t rsp_trsv_zero_pivot(rsp_handle_t h, rsp_ilu0_info_t f, int which, int *position) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !position || which < RSP_TRSV_L || which > RSP_TRSV_U) return RSP_STATUS_INVALID_VALUE;
    *position = -1;
    if (!f->analysed) return RSP_STATUS_INVALID_VALUE;
    int z[5];
    RSP_CHECK_HIP(hipMemcpyAsync(z, f->d_zero, sizeof(z), hipMemcpyDeviceToHost, h->stream));
    RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
    const int g = f->solve_gen[which];
    if (g > 0 && z[2 + which] == g) {  // recovered: the solve (and the solves after it) run again
        if (!f->last_solve[which].valid || !flow_recover()) return RSP_STATUS_EXECUTION_FAILED;
        const LaterSolves later = later_solves(f, f->last_solve[which].seq);
        if (!rerun_inputs_intact(f, which, later)) return RSP_STATUS_EXECUTION_FAILED;
        rsp_status_t st = rerun_solve(h, f, which);
        if (st == RSP_STATUS_SUCCESS) st = rerun_solves(h, f, later);
        if (st != RSP_STATUS_SUCCESS) return st;
        RSP_CHECK_HIP(hipMemcpyAsync(z, f->d_zero, sizeof(z), hipMemcpyDeviceToHost, h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
        if (z[2 + which] == f->solve_gen[which]) return RSP_STATUS_EXECUTION_FAILED;
    }
    if (which == RSP_TRSV_U) {
        int pos = f->structural_zero;
        if (f->factored && z[0] != INT_MAX && (pos < 0 || z[0] < pos)) pos = z[0];
        if (pos >= 0) {
            *position = pos;
            return RSP_STATUS_ZERO_PIVOT;
        }
    }
    return RSP_STATUS_SUCCESS;
}

// Flow launch control of one call (rsp::FlowCtl): status word and generation,
// give-up bound, the info's claim counter.
static rsp::FlowCtl flow_ctl(rsp_ilu0_info *f, int word, int gen) {
    rsp::FlowCtl c;
    c.status = f->d_zero + word;
    c.gen = gen;
    const long long us = std::max(env_int("RSP_ILU_FLOW_TIMEOUT_US", 200000), 0);
    c.ticks = (unsigned long long)us * 100ull;  // 100 MHz wall clock
    c.claim = reinterpret_cast<unsigned long long *>(f->d_zero + 6);
    c.claim_host = &f->claim_host;
    c.mode = env_int("RSP_ILU_FLOW_MODE", rsp::kFlowTickets);
    c.done = f->d_fdone;
    c.tickets = f->d_tk;
    c.grid_x = std::max(env_int("RSP_ILU_FLOW_GRID_X", 1), 1);
    c.tk_seq = &f->tk_seq;
    // (2^32 calls of one info before an epoch repeats; 0 is the array's initial value)
    if (++f->flow_epoch == 0) f->flow_epoch = 1;
    c.epoch = f->flow_epoch;
    return c;
}

static rsp::LevelPlan level_plan(const rsp_ilu0_info::Dag &d, const rsp_an::hvec<rsp::LevelSeg> &segs,
                                 int batch) {
    rsp::LevelPlan p;
    p.rows = d.d_rows;
    p.ptr_dev = d.d_ptr;
    p.ptr_host = d.ptr.data();
    p.nlev = (int)d.ptr.size() - 1;
    p.segs = segs.data();
    p.nseg = (int)segs.size();
    p.batch = batch;
    p.group = d.group;
    p.tasks = d.d_tasks;
    p.sbase_host = d.sbase.empty() ? nullptr : d.sbase.data();
    p.tpos = d.d_tpos;
    p.src = d.d_src;
    p.chunks = d.d_chunks;
    p.trow = d.d_trow;
    p.sid = d.d_sid;
    p.stg = d.d_stg;
    p.fitems = d.d_fitems;
    p.has_flow = 0;
    for (const rsp::LevelSeg &sg : segs) p.has_flow |= !sg.thin && sg.c1 > sg.c0;
    p.nterms = d.nterms;
    p.nshort = d.d_nshort;
    p.nshort_host = d.nshort.data();
    p.nwave_host = d.nwave.empty() ? nullptr : d.nwave.data();
    return p;
}

static bool flow_recover() { return env_int("RSP_ILU_FLOW_RECOVER", 1) != 0; }

// One factor call (flow_ok = false: no flow launch, every fat level its own
// launch — the recovery run of rsp_ilu0_zero_pivot).
static rsp_status_t ilu_factor_run(rsp_handle_t h, rsp_ilu0_info_t f, rsp_datatype_t value_type,
                                   void *d_values, bool flow_ok) {
    RSP_CHECK_HIP(hipMemsetD32Async(f->d_zero, INT_MAX, 1, h->stream));
    rsp::IluArgs a;
    a.n = f->n;
    a.rowptr = f->rowptr;
    a.colidx = f->colidx;
    a.dpos = f->d_dpos;
    a.hasdiag = f->d_hasdiag;
    a.vals = d_values;
    a.zero_pivot = f->d_zero;
    a.upd_ptr = f->d_upd_ptr;
    a.upd_l = f->d_upd_l;
    a.upd_u = f->d_upd_u;
    a.lord = f->d_lord;
    a.lend = f->d_lend;
    a.udiv = f->d_udiv;
    a.frow = f->d_frow;
    a.fslots = f->d_fslots;
    a.fslev = f->fslev.empty() ? nullptr : f->fslev.data();
    a.fat_slots = f->d_fslots && env_int("RSP_ILU_FAT_SLOT", 1) != 0;
    a.fat_lds = env_int("RSP_ILU_FAT_LDS", 1) != 0;
    a.defer_rounds = env_int("RSP_ILU_DEFER", 8);  // A/B knob (thin factor runs)
    a.narrow_waves = std::min(std::max(env_int("RSP_ILU_FNARROW_WAVES", 4), 1), rsp::kThinThreads / 64);
    a.rchunks = f->d_rchunks;
    a.ritems = f->d_ritems;
    a.rpairs = f->d_rpairs;
    a.rstaged = f->d_rstaged;
    a.rrounds = f->d_rrounds;
    a.plan = level_plan(f->fdag(), f->fac_segs, f->fac_batch);
    a.fac_one = f->fac_scale;
    a.fitems = f->d_ffitems;
    a.fruns = f->fruns.empty() ? nullptr : f->fruns.data();
    a.nfruns = a.fat_slots ? (int)f->fruns.size() : 0;
    a.lev = nullptr;
    a.forig = f->d_forig;
    if (f->fac_gen >= (1 << 30)) {  // generations wrap
        RSP_CHECK_HIP(hipMemsetD32Async(f->d_zero + 1, 0, 1, h->stream));  // no stale give-up
        f->fac_gen = 0;
    }
    a.gen = ++f->fac_gen;
    a.flow = flow_ok && env_int("RSP_ILU_FLOW", 1) != 0;
    a.flow_grid = h->num_cus * std::min(std::max(env_int("RSP_ILU_FLOW_WPC", 4), 4), 16) / 4;
    a.flow_cus = h->num_cus;
    a.flow_sleep = std::min(std::max(env_int("RSP_ILU_FLOW_SLEEP", 1), 1), 64);
    a.fc = flow_ctl(f, 1, a.gen);
    // diagnostics: RSP_ILU_FTRACE=<file> appends per-chunk shader-clock stamps
    // of the thin factor runs (host-blocking; never set in timed runs)
    const char *trace_file = getenv("RSP_ILU_FTRACE");
    unsigned long long *&d_trace = h->d_ftrace;
    const int trace_cap = 1 << 22;
    a.trace = nullptr;
    a.trace_cap = 0;
    if (trace_file) {
        if (!d_trace) RSP_CHECK_HIP(hipMalloc((void **)&d_trace, trace_cap * sizeof(unsigned long long)));
        RSP_CHECK_HIP(hipMemsetAsync(d_trace, 0, trace_cap * sizeof(unsigned long long), h->stream));
        a.trace = d_trace;
        a.trace_cap = trace_cap;
    }
    hipError_t e;
    if (value_type == RSP_R_64F)
        e = rsp_k::ilu0_factor_f64(a, h->stream);
    else
        e = h->ftz ? rsp_k_ftz::ilu0_factor_f32(a, h->stream) : rsp_k::ilu0_factor_f32(a, h->stream);
    if (trace_file && e == hipSuccess) {
        rsp_an::hvec<unsigned long long> t(trace_cap);
        RSP_CHECK_HIP(hipMemcpyAsync(t.data(), d_trace, t.size() * sizeof(t[0]), hipMemcpyDeviceToHost,
                                     h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
        if (FILE *fp = fopen(trace_file, "a")) {
            fprintf(fp, "# factor n=%d\n", f->n);
            for (int c = 0; c < trace_cap / 4; c++)
                if (t[4 * (size_t)c])
                    fprintf(fp, "%d %llu %llu %llu %llu %llu\n", c, t[4 * (size_t)c], t[4 * (size_t)c + 1],
                            t[4 * (size_t)c + 2], t[4 * (size_t)c + 3] & 0xffffffffull, t[4 * (size_t)c + 3] >> 32);
            fclose(fp);
        }
    }
    f->factored = 1;
    return e == hipSuccess ? RSP_STATUS_SUCCESS : RSP_STATUS_EXECUTION_FAILED;
}

static rsp_status_t rsp_ilu0_factor_impl(rsp_handle_t h, rsp_ilu0_info_t f, rsp_datatype_t value_type,
                             void *d_values) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !f->analysed || (f->nnz_s > 0 && !d_values)) return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    // a factor with flow runs keeps its input values for a recovery run
    // (rsp_ilu0_info::d_fbackup): one device copy of the values per call
    f->last_fac.valid = 0;
    const bool flows = !f->fruns.empty() && f->d_fslots && env_int("RSP_ILU_FLOW", 1) != 0 &&
                       env_int("RSP_ILU_FAT_SLOT", 1) != 0;
    if (flows && f->nnz_s > 0 && flow_recover()) {
        const size_t bytes = (size_t)f->nnz_s * elem_size(value_type);
        if (f->fbackup_bytes < bytes) {
            if (f->d_fbackup) (void)hipFree(f->d_fbackup);
            f->d_fbackup = nullptr;
            f->fbackup_bytes = 0;
            RSP_CHECK_HIP(hipMalloc(&f->d_fbackup, bytes));
            f->fbackup_bytes = bytes;
        }
        RSP_CHECK_HIP(hipMemcpyAsync(f->d_fbackup, d_values, bytes, hipMemcpyDeviceToDevice, h->stream));
        f->last_fac.valid = 1;
        f->last_fac.seq = ++f->call_seq;
        f->last_fac.ftz = h->ftz;
        f->last_fac.type = value_type;
        f->last_fac.vals = d_values;
    }
    return ilu_factor_run(h, f, value_type, d_values, true);
}

static rsp::TrsvArgs trsv_args(rsp_handle_t h, rsp_ilu0_info *f, const void *alpha, rsp_datatype_t t,
                               const void *vals, const void *x, void *y) {
    rsp::TrsvArgs a;
    a.n = f->n;
    a.rowptr = f->rowptr;
    a.colidx = f->colidx;
    a.dpos = f->d_dpos;
    a.hasdiag = f->d_hasdiag;
    a.vals = vals;
    a.x = x;
    a.y = y;
    a.alpha = (t == RSP_R_64F) ? *(const double *)alpha : (double)*(const float *)alpha;
    a.plan = level_plan(f->L, f->L.segs, f->L.batch);
    a.sval = f->d_sval;
    a.sx = f->d_sx;
    a.sdg = f->d_sdg;
    a.trace = nullptr;
    a.trace_cap = 0;
    a.trace_clk = 0;
    a.wave_lds = env_int("RSP_ILU_WAVE_LDS", 1);
    a.narrow_waves = std::min(std::max(env_int("RSP_ILU_NARROW_WAVES", 4), 1), rsp::kThinThreads / 64);
    a.narrow_split = env_int("RSP_ILU_NARROW_SPLIT", 0) != 0;  // (default off: slower)
    a.narrow_pairs = env_int("RSP_ILU_NARROW_PAIRS", -1);  // -1: by the DAG's level width (launcher)
    a.loaders = env_int("RSP_ILU_LOADERS", 1);
    a.flow = env_int("RSP_ILU_FLOW", 1) != 0;
    // 256-thread workgroups, RSP_ILU_FLOW_WPC waves per CU: 8 for the solves
    // (config 3, start tickets: solve 34.34 -> 33.95 ms against 4; the
    // factor's flow stays at 4: 40.11 vs 40.15 ms); no residency is needed
    // with start tickets, the static walk (RSP_ILU_FLOW_MODE=0) needs the
    // whole grid resident (flow_grid caps it by the occupancy query)
    a.flow_grid = h->num_cus * std::min(std::max(env_int("RSP_ILU_FLOW_WPC", 8), 4), 16) / 4;
    a.flow_cus = h->num_cus;
    a.flow_sleep = std::min(std::max(env_int("RSP_ILU_FLOW_SLEEP", 1), 1), 64);
    return a;
}

// A solve call of kind `which` (RSP_TRSV_*): its generation (status word
// 2 + which; generations restart with the factor's wrap-around below 2^30).
static hipError_t trsv_begin(rsp_handle_t h, rsp_ilu0_info *f, int which, rsp::TrsvArgs &a) {
    int &g = f->solve_gen[which];
    if (g >= (1 << 30)) {  // wrap: no stale give-up may match a new generation
        const hipError_t e = hipMemsetD32Async(f->d_zero + 2 + which, 0, 1, h->stream);
        if (e != hipSuccess) return e;
        g = 0;
    }
    a.fc = flow_ctl(f, 2 + which, ++g);
    return hipSuccess;
}

// A solve call's arguments, kept for its recovery run (rsp_ilu0_info::last_solve).
static void remember_solve(rsp_handle_t h, rsp_ilu0_info *f, int which, rsp_operation_t op, const void *alpha,
                           rsp_datatype_t t, const void *vals, const void *x, void *y) {
    rsp_ilu0_info::SolveCall &c = f->last_solve[which];
    c.seq = ++f->call_seq;
    c.valid = 1;
    c.ftz = h->ftz;
    c.op = op;
    c.alpha = t == RSP_R_64F ? *(const double *)alpha : (double)*(const float *)alpha;
    c.type = t;
    c.vals = vals;
    c.x = x;
    c.y = y;
}

// flow_ok = false: the recovery run of rsp_trsv_zero_pivot (no flow launch)
static rsp_status_t rsp_trsv_lower_unit_impl(rsp_handle_t h, rsp_operation_t op, const void *alpha,
                                 rsp_ilu0_info_t f, rsp_datatype_t value_type,
                                 const void *d_values, const void *d_x, void *d_y, bool flow_ok) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !f->analysed || !alpha) return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    if (f->n > 0 && (!d_x || !d_y || d_x == d_y)) return RSP_STATUS_INVALID_VALUE;
    if (op != RSP_OPERATION_NON_TRANSPOSE && op != RSP_OPERATION_TRANSPOSE) return RSP_STATUS_INVALID_VALUE;
    {
        const rsp_status_t st = ilu_solves_ready(h, f);  // (rsp_trsv_analysis not called: done here)
        if (st != RSP_STATUS_SUCCESS) return st;
    }
    remember_solve(h, f, op == RSP_OPERATION_NON_TRANSPOSE ? RSP_TRSV_L : RSP_TRSV_LT, op, alpha, value_type,
                   d_values, d_x, d_y);
    rsp::TrsvArgs a = trsv_args(h, f, alpha, value_type, d_values, d_x, d_y);
    a.flow = a.flow && flow_ok;
    // diagnostics: RSP_ILU_TRACE=<file> appends per-chunk timestamps of the
    // prefetching thin kernel (host-blocking; never set in timed runs)
    const char *trace_file = getenv("RSP_ILU_TRACE");
    unsigned long long *&d_trace = h->d_strace;
    const int trace_cap = 4 << 20;
    if (trace_file) {
        if (!d_trace) RSP_CHECK_HIP(hipMalloc((void **)&d_trace, trace_cap * sizeof(unsigned long long)));
        RSP_CHECK_HIP(hipMemsetAsync(d_trace, 0, trace_cap * sizeof(unsigned long long), h->stream));
        a.trace = d_trace;
        a.trace_cap = trace_cap;
        a.trace_clk = env_int("RSP_ILU_TRACE_CLK", 0);
    }
    hipError_t e;
    const bool f64 = value_type == RSP_R_64F, ftz = h->ftz != 0;
    if (op != RSP_OPERATION_NON_TRANSPOSE && op != RSP_OPERATION_TRANSPOSE) return RSP_STATUS_INVALID_VALUE;
    RSP_CHECK_HIP(trsv_begin(h, f, op == RSP_OPERATION_NON_TRANSPOSE ? RSP_TRSV_L : RSP_TRSV_LT, a));
    // a deep DAG: the block-inverse solve (trsv_blocks.hip; RSP_ILU_BLOCKS=0
    // at solve time runs the level-scheduled solve of the same analysis)
    const rsp_ilu0_info::BlkDag &bd = op == RSP_OPERATION_NON_TRANSPOSE ? f->Lb : f->LTb;
    if (bd.on && env_int("RSP_ILU_BLOCKS", -1) != 0) {
        rsp::BlkArgs b{};
        b.n = f->n;
        b.nb = bd.nb;
        b.order = bd.d_order;
        b.desc = bd.d_desc;
        b.rows = bd.d_rows;
        b.ref = bd.d_ref;
        b.vpos = bd.d_vpos;
        b.eord = bd.d_eord;
        b.lptr = bd.d_lptr;
        b.rptr = bd.d_rptr;
        b.rit = bd.d_rit;
        b.segs = bd.segs.data();
        b.nseg = (int)bd.segs.size();
        b.lds_elems = bd.lds_elems;
        b.lds_words = bd.lds_words;
        b.rc = bd.d_rc;
        b.vals = d_values;
        b.x = d_x;
        b.y = d_y;
        b.alpha = a.alpha;
        b.ev = bd.d_ev;
        b.yp = bd.d_yp;
        e = f64 ? rsp_k::trsv_blocks_f64(b, h->stream)
                : (ftz ? rsp_k_ftz::trsv_blocks_f32(b, h->stream) : rsp_k::trsv_blocks_f32(b, h->stream));
        return e == hipSuccess ? RSP_STATUS_SUCCESS : RSP_STATUS_EXECUTION_FAILED;
    }
    if (op == RSP_OPERATION_NON_TRANSPOSE) {
        e = f64 ? rsp_k::trsv_lower_n_f64(a, h->stream)
                : (ftz ? rsp_k_ftz::trsv_lower_n_f32(a, h->stream) : rsp_k::trsv_lower_n_f32(a, h->stream));
    } else if (op == RSP_OPERATION_TRANSPOSE) {
        a.plan = level_plan(f->LT, f->LT.segs, f->LT.batch);
        e = f64 ? rsp_k::trsv_lower_t_f64(a, h->stream)
                : (ftz ? rsp_k_ftz::trsv_lower_t_f32(a, h->stream) : rsp_k::trsv_lower_t_f32(a, h->stream));
    } else {
        return RSP_STATUS_INVALID_VALUE;
    }
    if (trace_file && e == hipSuccess) {
        rsp_an::hvec<unsigned long long> t(trace_cap);
        RSP_CHECK_HIP(hipMemcpyAsync(t.data(), d_trace, t.size() * sizeof(t[0]), hipMemcpyDeviceToHost,
                                     h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
        if (FILE *fp = fopen(trace_file, "a")) {
            fprintf(fp, "# solve op=%d n=%d\n", (int)op, f->n);
            for (int l = 0; l < trace_cap / 2; l++)
                if (t[(size_t)trace_cap / 2 + l])
                    fprintf(fp, "L %d %llu\n", l, t[(size_t)trace_cap / 2 + l]);
            for (int c = 0; c < trace_cap / 16; c++)
                if (t[8 * (size_t)c] || t[8 * (size_t)c + 3])
                    fprintf(fp, "%d %llu %llu %llu %llu %llu %llu\n", c, t[8 * (size_t)c],
                            t[8 * (size_t)c + 1], t[8 * (size_t)c + 2], t[8 * (size_t)c + 3],
                            t[8 * (size_t)c + 4], t[8 * (size_t)c + 5]);
            fclose(fp);
        }
    }
    return e == hipSuccess ? RSP_STATUS_SUCCESS : RSP_STATUS_EXECUTION_FAILED;
}

static rsp_status_t rsp_trsv_upper_impl(rsp_handle_t h, const void *alpha, rsp_ilu0_info_t f,
                            rsp_datatype_t value_type, const void *d_values, const void *d_x,
                            void *d_y, bool flow_ok) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !f->analysed || !alpha) return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    if (f->n > 0 && (!d_x || !d_y || d_x == d_y)) return RSP_STATUS_INVALID_VALUE;
    rsp_status_t st = ilu_solves_ready(h, f);  // (the solve streams)
    if (st != RSP_STATUS_SUCCESS) return st;
    st = ilu_plan_u(h, f);  // planned on first use
    if (st != RSP_STATUS_SUCCESS) return st;
    remember_solve(h, f, RSP_TRSV_U, RSP_OPERATION_NON_TRANSPOSE, alpha, value_type, d_values, d_x, d_y);
    rsp::TrsvArgs a = trsv_args(h, f, alpha, value_type, d_values, d_x, d_y);
    a.flow = a.flow && flow_ok;
    a.plan = level_plan(f->U, f->U.segs, f->U.batch);
    a.sval = f->d_usval;
    RSP_CHECK_HIP(trsv_begin(h, f, RSP_TRSV_U, a));
    hipError_t e;
    if (value_type == RSP_R_64F)
        e = rsp_k::trsv_upper_f64(a, h->stream);
    else
        e = h->ftz ? rsp_k_ftz::trsv_upper_f32(a, h->stream) : rsp_k::trsv_upper_f32(a, h->stream);
    return e == hipSuccess ? RSP_STATUS_SUCCESS : RSP_STATUS_EXECUTION_FAILED;
}


}  // extern "C"

// C-ABI entry points never let a C++ exception out (std::bad_alloc from the
// host plans' pools, say): it becomes a status, after `cleanup`.
template <typename F, typename C>
static rsp_status_t guarded(F body, C cleanup) {
    try {
        return body();
    } catch (const std::bad_alloc &) {
        cleanup();
        return RSP_STATUS_ALLOC_FAILED;
    } catch (...) {
        cleanup();
        return RSP_STATUS_INTERNAL_ERROR;
    }
}

extern "C" {


rsp_status_t rsp_spmv_buffer_size(rsp_handle_t h, rsp_operation_t op, const void *alpha,
                                  rsp_spmat_t mat, const void *beta, rsp_datatype_t compute_type,
                                  size_t *buffer_size) {
    return guarded([&] { return rsp_spmv_buffer_size_impl(h, op, alpha, mat, beta, compute_type, buffer_size); }, [] {});
}

rsp_status_t rsp_spmv_preprocess(rsp_handle_t h, rsp_operation_t op, const void *alpha,
                                 rsp_spmat_t mat, const void *d_x, const void *beta, void *d_y,
                                 rsp_datatype_t compute_type, void *d_buffer) {
    return guarded([&] { return rsp_spmv_preprocess_impl(h, op, alpha, mat, d_x, beta, d_y, compute_type, d_buffer); }, [] {});
}

rsp_status_t rsp_spmv(rsp_handle_t h, rsp_operation_t op, const void *alpha, rsp_spmat_t mat,
                      const void *d_x, const void *beta, void *d_y, rsp_datatype_t compute_type,
                      void *d_buffer) {
    return guarded([&] { return rsp_spmv_impl(h, op, alpha, mat, d_x, beta, d_y, compute_type, d_buffer); }, [] {});
}

rsp_status_t rsp_spmv_part(rsp_handle_t h, const void *alpha, rsp_spmat_t mat, const void *d_x,
                           const void *beta, void *d_y, rsp_datatype_t compute_type,
                           void *d_buffer, int part) {
    return guarded([&] { return rsp_spmv_part_impl(h, alpha, mat, d_x, beta, d_y, compute_type, d_buffer, part); }, [] {});
}

rsp_status_t rsp_spmv_batch_create(rsp_handle_t h, int count, const rsp_spmat_t *mats,
                                   const void *const *d_x, void *const *d_y,
                                   void *const *d_buffers, rsp_datatype_t compute_type,
                                   int part, rsp_spmv_batch_t *batch) {
    return guarded([&] { return rsp_spmv_batch_create_impl(h, count, mats, d_x, d_y, d_buffers, compute_type, part, batch); }, [] {});
}

rsp_status_t rsp_ilu0_analysis(rsp_handle_t h, int n, int nnz, const int *d_row_offsets,
                               const int *d_col_ind, rsp_ilu0_info_t f) {
    return guarded([&] { return rsp_ilu0_analysis_impl(h, n, nnz, d_row_offsets, d_col_ind, f); }, [&] { if (f) { ilu_free_device(f); f->analysed = 0; } });
}

rsp_status_t rsp_ilu0_analysis_host(int n, const int *row_offsets, const int *col_ind,
                                    int *levels_lower, int *levels_upper, uint64_t *digest,
                                    double *phase_ms) {
    return guarded([&] { return rsp_ilu0_analysis_host_impl(n, row_offsets, col_ind, levels_lower, levels_upper, digest, phase_ms); }, [] {});
}

rsp_status_t rsp_ilu0_factor(rsp_handle_t h, rsp_ilu0_info_t f, rsp_datatype_t value_type,
                             void *d_values) {
    return guarded([&] { return rsp_ilu0_factor_impl(h, f, value_type, d_values); }, [] {});
}

rsp_status_t rsp_trsv_analysis(rsp_handle_t h, rsp_operation_t op, rsp_ilu0_info_t f) {
    return guarded([&] {
        if (!h) return RSP_STATUS_NOT_INITIALIZED;
        if (!f || !f->analysed) return RSP_STATUS_INVALID_VALUE;
        if (op != RSP_OPERATION_NON_TRANSPOSE && op != RSP_OPERATION_TRANSPOSE) return RSP_STATUS_INVALID_VALUE;
        return ilu_solves_ready(h, f);
    }, [] {});
}

rsp_status_t rsp_trsv_lower_unit(rsp_handle_t h, rsp_operation_t op, const void *alpha,
                                 rsp_ilu0_info_t f, rsp_datatype_t value_type,
                                 const void *d_values, const void *d_x, void *d_y) {
    return guarded([&] { return rsp_trsv_lower_unit_impl(h, op, alpha, f, value_type, d_values, d_x, d_y, true); }, [] {});
}

rsp_status_t rsp_trsv_upper(rsp_handle_t h, const void *alpha, rsp_ilu0_info_t f,
                            rsp_datatype_t value_type, const void *d_values, const void *d_x,
                            void *d_y) {
    return guarded([&] { return rsp_trsv_upper_impl(h, alpha, f, value_type, d_values, d_x, d_y, true); }, [] {});
}

rsp_status_t rsp_spmv_plan_host(int m, const int *row_offsets, const int *col_ind, int64_t nnz,
                                rsp_datatype_t compute_type, int64_t *tiles, int64_t *entries_16bit,
                                int64_t *entries_staged) {
    return guarded([&] { return rsp_spmv_plan_host_impl(m, row_offsets, col_ind, nnz, compute_type, tiles,
                                                        entries_16bit, entries_staged); }, [] {});
}

}  // extern "C"
