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
#include <thread>
#include <vector>

#include "rsp_kernels.h"

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
    size_t off_cbase, off_cidx;
    int64_t nnz_c16;            // entries read through 16-bit column offsets
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
    int *d_zero;
    long long n_updates;
    // one level set per DAG: L (factor + L solve), L^T, U
    struct Dag {
        std::vector<int> ptr;                  // host level pointers
        int *d_rows = nullptr, *d_ptr = nullptr;
        rsp::RowTask *d_tasks = nullptr;       // solve: task per level-order slot
        int *d_tpos = nullptr, *d_src = nullptr;  // solve: flat terms
        rsp::LevelChunk *d_chunks = nullptr;   // solve: LDS-staged chunks of thin runs
        rsp::ThinRowPlan *d_trow = nullptr;    // solve: thin-run row records
        int *d_sid = nullptr;                  // solve: thin-run y indices per term
        rsp::StagedTerm *d_stg = nullptr;      // solve: thin-run staged terms
        int nterms = 0;                        // solve: flat terms
        int *d_nshort = nullptr;               // solve: short rows per level (device)
        std::vector<int> nshort;               // (host)
        std::vector<int> nwave;                // solve: short + wave rows per level (host)
        std::vector<int> sbase;                // solve: padded short rows' first term per level (host)
        std::vector<rsp::LevelSeg> segs;       // thread-per-row solve plan
        int batch = 8;                         // solve fma-chain batch
        int group = 4;                         // thin-run term groups (2 or 4)
    } L, LT, U;
    std::vector<rsp::LevelSeg> fac_segs;       // wave-per-row factor plan over L
    void *d_sval = nullptr, *d_sx = nullptr, *d_sdg = nullptr;  // solve streams (trsv_stream)
    rsp::RndChunk *d_rchunks = nullptr;        // round-based factor chunks (thin runs)
    rsp::RndItem *d_ritems = nullptr;
    rsp::FacRow *d_frow = nullptr;
    int *d_fslots = nullptr;                   // fat factor levels, slot layout (ilu0_level_slot)
    std::vector<rsp::FacSlotLevel> fslev;      // per L level (stride 0: FacRow path)
    int *d_rpairs = nullptr, *d_rstaged = nullptr, *d_rrounds = nullptr;
    int fac_batch;
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
// 16-bit column offsets (2 B per stored entry)].
struct SpmvLayout {
    size_t off_long, off_part, off_cbase, off_cidx, bytes;
};
static SpmvLayout spmv_layout(const SpmvBounds &b, size_t elem, int64_t nnz) {
    SpmvLayout l;
    l.off_long = align256(b.nblocks * sizeof(SpmvBlock));
    l.off_part = l.off_long + align256(b.nlong * sizeof(SpmvLongRow));
    l.off_cbase = l.off_part + align256(b.nslots * 2 * elem);  // value + ticket per slot
    l.off_cidx = l.off_cbase + align256(b.nblocks * sizeof(int));
    l.bytes = l.off_cidx + align256((size_t)std::max<int64_t>(nnz, 0) * sizeof(uint16_t));
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

rsp_status_t rsp_spmv_buffer_size(rsp_handle_t h, rsp_operation_t op, const void *alpha,
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
static int build_spmv_plan(const int *rp, int m, int cap, int chunk, std::vector<SpmvBlock> &blocks,
                           std::vector<SpmvLongRow> &longrows, int *nslots,
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
    std::vector<SpmvBlock> blocks;
    std::vector<SpmvLongRow> longrows;
    int nslots = 0, nint = 0;
    std::vector<int> cbase;
    std::vector<uint16_t> c16;
    int64_t nnz_c16 = 0;
};

// spread > 0: a plan of fewer tiles than `spread` (the resident workgroup
// slots it may use) is re-packed into up to `spread` smaller tiles, so a lone
// launch does not leave slots idle. Long rows do not depend on the packing
// cap (they are cut at the fixed chunk), so every spread of one matrix has
// the same long rows and partial slots.
static void make_tile_plan(const int *rp, const int *ci, int m, int64_t nnz_bound,
                           rsp_datatype_t type, int64_t spread, int64_t local_cols, bool use_c16,
                           TilePlan &p, int row_align = 1) {
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
            std::vector<SpmvBlock> b2;
            std::vector<SpmvLongRow> l2;
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
    // read for it).
    const int64_t nnz_s = m > 0 ? rp[(size_t)m] : 0;
    p.cbase.assign(p.blocks.size(), -1);
    p.c16.clear();
    p.nnz_c16 = 0;
    if (use_c16 && nnz_s > 0 && nnz_s <= nnz_bound) {
        p.c16.assign((size_t)nnz_s, 0);
        for (size_t t = 0; t < p.blocks.size(); t++) {
            const SpmvBlock &bk = p.blocks[t];
            if (bk.k1 <= bk.k0) continue;
            int lo = ci[(size_t)bk.k0], hi = lo;
            for (int k = bk.k0 + 1; k < bk.k1; k++) {
                lo = std::min(lo, ci[(size_t)k]);
                hi = std::max(hi, ci[(size_t)k]);
            }
            if (hi - lo > 65535) continue;
            p.cbase[t] = lo;
            p.nnz_c16 += bk.k1 - bk.k0;
            for (int k = bk.k0; k < bk.k1; k++) p.c16[(size_t)k] = (uint16_t)(ci[(size_t)k] - lo);
        }
    }
}

// Row offsets and column indices of `mat` on the host, validated (base 0,
// non-decreasing offsets, columns inside [0, cols)).
static rsp_status_t download_pattern(rsp_handle_t h, rsp_spmat_t mat, std::vector<int> &rp,
                                     std::vector<int> &ci) {
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
    std::vector<int> rp, ci;
    rsp_status_t st = download_pattern(h, mat, rp, ci);
    if (st != RSP_STATUS_SUCCESS) return st;
    const int chunk = chunk_cap(compute_type);
    // A matrix with fewer tiles than the chip holds resident workgroups (R)
    // leaves slots idle and runs each tile latency-bound: spread it over up
    // to R smaller tiles (measured +2.7 % on the moderate set per matrix;
    // plans of >= 2 waves are left alone, they lost 1 % this way). A batch
    // re-plans its members itself (rsp_spmv_batch_create). Tiling never
    // changes the result (canonical summation order). RSP_SPMV_VARIANT bit 4
    // turns spreading off, bit 5 keeps every tile on the int32 indices.
    TilePlan p;
    make_tile_plan(rp.data(), ci.data(), m, mat->nnz, compute_type,
                   (h->spmv_variant & 16) ? 0 : spmv_resident_tiles(h, compute_type),
                   mat->local_cols, !(h->spmv_variant & 32), p, spmv_row_align(h, compute_type));
    const std::vector<SpmvBlock> &blocks = p.blocks;
    const std::vector<SpmvLongRow> &longrows = p.longrows;
    const int nslots = p.nslots, nint = p.nint;
    const std::vector<int> &cbase = p.cbase;
    const std::vector<uint16_t> &c16 = p.c16;
    const int64_t nnz_c16 = p.nnz_c16;
    (void)chunk;
    // exact layout of this schedule in the matrix's device memory (grown,
    // never shrunk, on a re-plan)
    SpmvBounds b{blocks.size(), longrows.size(), (size_t)nslots};
    const SpmvLayout lay = spmv_layout(b, elem_size(compute_type), (int64_t)c16.size());
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
    mat->nnz_c16 = nnz_c16;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_spmv_preprocess(rsp_handle_t h, rsp_operation_t op, const void *alpha,
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

rsp_status_t rsp_spmv(rsp_handle_t h, rsp_operation_t op, const void *alpha, rsp_spmat_t mat,
                      const void *d_x, const void *beta, void *d_y, rsp_datatype_t compute_type,
                      void *d_buffer) {
    return spmv_run(h, op, alpha, mat, d_x, beta, d_y, compute_type, d_buffer, 0);
}

rsp_status_t rsp_spmv_part(rsp_handle_t h, const void *alpha, rsp_spmat_t mat, const void *d_x,
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
    std::vector<rsp_spmat_t> mats;
    std::vector<unsigned long long> plan_gen;  // schedules as copied (stale check)
    std::vector<rsp::SpmvBatchArgs> launches;  // one per kSpmvBatchMax matrices
    void *d_mem = nullptr;                      // entries, tiles, long rows of every launch
    int64_t tiles = 0, entries_16bit = 0;       // rsp_spmv_batch_info
    ~rsp_spmv_batch() {
        if (d_mem) (void)hipFree(d_mem);
    }
};

rsp_status_t rsp_spmv_batch_create(rsp_handle_t h, int count, const rsp_spmat_t *mats,
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
        for (int q = 0; q < j; q++)  // a matrix's long-row tickets serve one launch slot
            if (mats[q] == A) return RSP_STATUS_INVALID_VALUE;
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
    // matrix, so the partials stay in d_buffers[j].
    const int64_t R = spmv_resident_tiles(h, compute_type);
    const bool spread_ok = !(h->spmv_variant & 16), c16_ok = !(h->spmv_variant & 32);
    std::vector<TilePlan> plans((size_t)count);
    // layout: per launch [entries | tiles | tile column bases | long rows |
    // 16-bit column offsets of each matrix], each 16-B aligned
    struct Span { int first, count; size_t off_e, off_t, off_c, off_l; std::vector<size_t> off_16; };
    std::vector<Span> spans;
    size_t bytes = 0;
    auto tile_range = [part](const TilePlan &p, int *t0, int *t1) {
        *t0 = part == 2 ? p.nint : 0;
        *t1 = part == 1 ? p.nint : (int)p.blocks.size();
    };
    for (int first = 0; first < count; first += rsp::kSpmvBatchMax) {
        Span sp{first, std::min(rsp::kSpmvBatchMax, count - first), 0, 0, 0, 0, {}};
        std::vector<std::vector<int>> rps((size_t)sp.count), cis((size_t)sp.count);
        int64_t nt_full = 0, nnz_all = 0;
        for (int q = 0; q < sp.count; q++) {
            rsp_spmat_t A = mats[first + q];
            rsp_status_t st = download_pattern(h, A, rps[q], cis[q]);
            if (st != RSP_STATUS_SUCCESS) return st;
            make_tile_plan(rps[q].data(), cis[q].data(), (int)A->rows, A->nnz, compute_type, 0,
                           A->local_cols, c16_ok, plans[first + q], spmv_row_align(h, compute_type));
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
                               spmv_row_align(h, compute_type));
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
        spans.push_back(sp);
    }
    if (bytes > 0) RSP_CHECK_HIP(hipMalloc(&b->d_mem, bytes));
    std::vector<unsigned char> host(bytes);
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
            const char *buf = (const char *)A->d_plan;  // its long-row partials and tickets
            int t0, t1;
            tile_range(p, &t0, &t1);
            const int nlq = part == 1 ? 0 : (int)p.longrows.size();
            rsp::SpmvBatchEntry e{};
            e.rowptr = A->rowptr;
            e.colidx = A->colidx;
            e.vals = A->vals;
            e.x = d_x[sp.first + q];
            e.y = d_y[sp.first + q];
            e.partials = (void *)(buf + A->off_part);
            e.cidx = (const unsigned short *)((char *)b->d_mem + sp.off_16[q]);
            e.cmax = A->cols > 0 ? (int)(A->cols - 1) : 0;
            e.nnz = A->nnz_s;
            e.vector_ok = ((((uintptr_t)A->colidx) | ((uintptr_t)A->vals)) & 15) == 0;
            memcpy(host.data() + sp.off_e + (size_t)q * sizeof(e), &e, sizeof(e));
            a.tiles_at.begin[q] = nt;
            a.longs_at.begin[q] = nl;
            for (int t = t0; t < t1; t++)
                if (p.cbase[(size_t)t] >= 0) b->entries_16bit += p.blocks[(size_t)t].k1 - p.blocks[(size_t)t].k0;
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
            nt += t1 - t0;
            nl += nlq;
        }
        a.tiles_at.begin[sp.count] = nt;
        a.longs_at.begin[sp.count] = nl;
        b->launches.push_back(a);
    }
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
    int **ptrs[] = {&f->d_dpos,     &f->d_hasdiag, &f->L.d_rows,  &f->L.d_ptr,
                    &f->LT.d_rows,  &f->LT.d_ptr,  &f->U.d_rows,  &f->U.d_ptr,
                    &f->d_zero,
                    &f->d_upd_ptr,  &f->d_upd_l,   &f->d_upd_u,   &f->d_lord,
                    &f->d_lend,     &f->d_udiv};
    for (int **p : ptrs) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    for (void **p : {&f->d_sval, &f->d_sx, &f->d_sdg}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    f->fslev.clear();
    for (void **p : {(void **)&f->d_frow, (void **)&f->d_fslots, (void **)&f->d_rchunks, (void **)&f->d_ritems,
                     (void **)&f->d_rpairs, (void **)&f->d_rstaged, (void **)&f->d_rrounds}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    for (rsp_ilu0_info::Dag *d : {&f->L, &f->LT, &f->U}) {
        for (void **p : {(void **)&d->d_tasks, (void **)&d->d_tpos, (void **)&d->d_src,
                         (void **)&d->d_chunks, (void **)&d->d_nshort, (void **)&d->d_trow,
                         (void **)&d->d_sid, (void **)&d->d_stg}) {
            if (*p) (void)hipFree(*p);
            *p = nullptr;
        }
    }
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


static const int kThinThreadsHost = rsp::kThinThreads;

static int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

// fma-chain batch for a mean chain length of total / count
static int chain_batch(long long total, long long count) {
    const double mean = count > 0 ? (double)total / (double)count : 0.0;
    return mean <= 2.5 ? 2 : (mean <= 5.0 ? 4 : 8);
}

}  // extern "C" (C++ helpers)

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
struct SolvePlan {
    std::vector<int> sbase;   // per level: first flat term of its padded short rows, -1 = none
    std::vector<int> nshort;  // per level
    std::vector<int> nwave;   // per level: short + wave rows (the rest: hub rows)
    std::vector<rsp::RowTask> tasks;
    std::vector<int> tpos, src;
    std::vector<rsp::LevelSeg> segs;
    std::vector<rsp::LevelChunk> chunks;
    std::vector<rsp::ThinRowPlan> trow;
    std::vector<int> sid;
    std::vector<rsp::StagedTerm> stg;
};

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
    auto nterms = [&](int i) {
        int cnt = 0;
        row_terms(i, [&](int, int) { cnt++; });
        return cnt;
    };
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

template <typename V>
static hipError_t upload_vec(V **dst, const std::vector<V> &v) {
    size_t bytes = std::max<size_t>(v.size(), 1) * sizeof(V);
    hipError_t e = hipMalloc((void **)dst, bytes);
    if (e != hipSuccess) return e;
    if (!v.empty()) e = hipMemcpy(*dst, v.data(), v.size() * sizeof(V), hipMemcpyHostToDevice);
    return e;
}

// Symbolic ILU(0) data (built by ilu_symbolic below).
struct IluSymbolic {
    std::vector<int> upd_ptr, upd_l, upd_u, lord, lend;
    std::vector<int> stage;  // per lower position: its intra-row stage
};

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
struct FacPlan {
    std::vector<rsp::LevelSeg> segs;
    std::vector<rsp::RndChunk> chunks;
    std::vector<rsp::RndItem> items;
    std::vector<int> pairs, staged, rounds;
};

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
            fp.segs.push_back({l, l + 1, thin, 0, 0, kThinThreadsHost});
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
    std::vector<RItem> ritems;  // a level's items
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
            std::stable_sort(ritems.begin(), ritems.end(),
                             [](const RItem &u, const RItem &v) { return u.round < v.round; });
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

extern "C" {

static hipError_t upload(int **dst, const std::vector<int> &v) {
    size_t bytes = std::max<size_t>(v.size(), 1) * sizeof(int);
    hipError_t e = hipMalloc((void **)dst, bytes);
    if (e != hipSuccess) return e;
    if (!v.empty()) e = hipMemcpy(*dst, v.data(), v.size() * sizeof(int), hipMemcpyHostToDevice);
    return e;
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
}  // extern "C"
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
extern "C" {

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

rsp_status_t rsp_ilu0_analysis(rsp_handle_t h, int n, int nnz, const int *d_row_offsets,
                               const int *d_col_ind, rsp_ilu0_info_t f) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    // diagnostics: RSP_ILU_TIMING=1 prints the wall time of each analysis phase
    const bool timing = env_int("RSP_ILU_TIMING", 0) != 0;
    auto t_last = std::chrono::steady_clock::now();
    auto phase = [&](const char *what) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "rsp_ilu0_analysis n=%d %-14s %8.2f ms\n", n, what,
                std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    if (!f || n < 0 || nnz < 0 || (n > 0 && !d_row_offsets)) return RSP_STATUS_INVALID_VALUE;
    ilu_free_device(f);
    f->analysed = 0;
    f->factored = 0;
    f->structural_zero = -1;
    std::vector<int> rp((size_t)n + 1, 0);
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
    std::vector<int> ci((size_t)nnz_s);
    if (nnz_s > 0) {
        RSP_CHECK_HIP(hipMemcpyAsync(ci.data(), d_col_ind, (size_t)nnz_s * sizeof(int),
                                     hipMemcpyDeviceToHost, h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
    }
    for (int v : ci)
        if (v < 0 || v >= n) return RSP_STATUS_INVALID_VALUE;
    // The diagonal search, update pairs and stages assume each row's columns
    // strictly increasing (the reference loader sorts rows,
    // loadMatrixMarket.cpp:237-242; csrilu02 requires sorted, duplicate-free
    // rows). Unsorted rows or a repeated column are rejected here instead of
    // silently factoring the wrong pattern.
    for (int i = 0; i < n; i++)
        for (int p = rp[(size_t)i] + 1; p < rp[(size_t)i + 1]; p++)
            if (ci[(size_t)p] <= ci[(size_t)p - 1]) return RSP_STATUS_INVALID_VALUE;
    std::vector<int> dpos((size_t)n), hasdiag((size_t)n);
    for (int i = 0; i < n; i++) {
        const int *b = ci.data() + rp[(size_t)i], *e = ci.data() + rp[(size_t)i + 1];
        const int *p = std::lower_bound(b, e, i);
        dpos[(size_t)i] = (int)(p - ci.data());
        hasdiag[(size_t)i] = (p != e && *p == i) ? 1 : 0;
        if (!hasdiag[(size_t)i] && f->structural_zero < 0) f->structural_zero = i;
    }
    // levels of the lower DAG (factor + L solve)
    std::vector<int> lv((size_t)n, 0);
    int nl = n > 0 ? 1 : 0;
    for (int i = 0; i < n; i++) {
        int l = 0;
        for (int p = rp[(size_t)i]; p < dpos[(size_t)i]; p++) l = std::max(l, lv[(size_t)ci[(size_t)p]] + 1);
        lv[(size_t)i] = l;
        nl = std::max(nl, l + 1);
    }
    // transposed strict lower: row k lists (j, pos) for l_jk, j descending
    std::vector<int> ltp((size_t)n + 1, 0);
    for (int j = 0; j < n; j++)
        for (int p = rp[(size_t)j]; p < dpos[(size_t)j]; p++) ltp[(size_t)ci[(size_t)p] + 1]++;
    for (int k = 0; k < n; k++) ltp[(size_t)k + 1] += ltp[(size_t)k];
    std::vector<int> lts((size_t)ltp[(size_t)n]), ltc((size_t)ltp[(size_t)n]);
    {
        std::vector<int> fill(ltp.begin(), ltp.end() - 1);
        for (int j = n - 1; j >= 0; j--)
            for (int p = rp[(size_t)j]; p < dpos[(size_t)j]; p++) {
                int k = ci[(size_t)p];
                int slot = fill[(size_t)k]++;
                lts[(size_t)slot] = p;
                ltc[(size_t)slot] = j;
            }
    }
    // levels of the L^T DAG: row i waits for every j > i with l_ji != 0
    std::vector<int> lvt((size_t)n, 0);
    int nlt = n > 0 ? 1 : 0;
    for (int j = n - 1; j >= 0; j--) {
        nlt = std::max(nlt, lvt[(size_t)j] + 1);
        for (int p = rp[(size_t)j]; p < dpos[(size_t)j]; p++) {
            int k = ci[(size_t)p];
            lvt[(size_t)k] = std::max(lvt[(size_t)k], lvt[(size_t)j] + 1);
        }
    }
    // levels of the U DAG (extension): row i waits for j > i with u_ij != 0
    std::vector<int> lvu((size_t)n, 0);
    int nlu = n > 0 ? 1 : 0;
    for (int i = n - 1; i >= 0; i--) {
        int l = 0;
        for (int p = dpos[(size_t)i] + hasdiag[(size_t)i]; p < rp[(size_t)i + 1]; p++)
            l = std::max(l, lvu[(size_t)ci[(size_t)p]] + 1);
        lvu[(size_t)i] = l;
        nlu = std::max(nlu, l + 1);
    }
    std::vector<int> rows_l, rows_lt, rows_u;
    phase("copy+levels");
    group_levels(lv, nl, f->L.ptr, rows_l);
    group_levels(lvt, nlt, f->LT.ptr, rows_lt);
    group_levels(lvu, nlu, f->U.ptr, rows_u);
    // RSP_ILU_THIN_SOLVE / RSP_ILU_THIN_FACTOR: tuning knobs (0 = no thin runs)
    const int thin_solve = std::min(env_int("RSP_ILU_THIN_SOLVE", rsp::kThinSolveRows), rsp::kThinThreads);
    const int thin_factor = env_int("RSP_ILU_THIN_FACTOR", rsp::kThinFactorRows);
    IluSymbolic sym;
    std::vector<int4> slot_desc;        // fat factor slot rows: {x, rm, qm, 0}
    std::vector<long long> slot_offs;   // ... and their offsets in f->d_fslots
    phase("group");
    if (!ilu_symbolic(n, rp, ci, dpos, hasdiag, sym)) return RSP_STATUS_ALLOC_FAILED;
    phase("symbolic");
    f->n_updates = (long long)sym.upd_l.size();
    {
        long long nl = 0, nu = 0;
        for (int i = 0; i < n; i++) {
            nl += dpos[(size_t)i] - rp[(size_t)i];
            nu += rp[(size_t)i + 1] - dpos[(size_t)i] - hasdiag[(size_t)i];
        }
        f->L.batch = f->LT.batch = chain_batch(nl, n);
        f->U.batch = chain_batch(nu, n);
        for (rsp_ilu0_info::Dag *d : {&f->L, &f->LT, &f->U})  // thin-run term groups
            d->group = env_int("RSP_ILU_GROUP", d->batch == 2 ? 2 : 4) == 2 ? 2 : 4;
        f->fac_batch = chain_batch((long long)sym.upd_l.size(), nnz_s);
    }
    // the factor plan and the three solve plans (flat terms in level order,
    // thin-run chunks, y sources) are independent: built concurrently
    FacPlan fplan;
    SolvePlan sps[3];
    std::vector<int> udiag((size_t)n);
    for (int i = 0; i < n; i++) udiag[(size_t)i] = hasdiag[(size_t)i] ? dpos[(size_t)i] : -1;
    {
        std::vector<std::thread> th;
        th.emplace_back([&] {
            build_factor_plan(n, rp, ci, dpos, hasdiag, sym, f->L.ptr, rows_l, thin_factor, fplan);
        });
        th.emplace_back([&] {
            build_solve_plan(n, f->L.ptr, rows_l, thin_solve, f->L.group, std::vector<int>(),
                             [&](int i, auto emit) {
                                 for (int p = rp[(size_t)i]; p < dpos[(size_t)i]; p++) emit(p, ci[(size_t)p]);
                             }, sps[0]);
        });
        th.emplace_back([&] {
            build_solve_plan(n, f->LT.ptr, rows_lt, thin_solve, f->LT.group, std::vector<int>(),
                             [&](int i, auto emit) {
                                 for (int q = ltp[(size_t)i]; q < ltp[(size_t)i + 1]; q++)
                                     emit(lts[(size_t)q], ltc[(size_t)q]);
                             }, sps[1]);
        });
        th.emplace_back([&] {
            build_solve_plan(n, f->U.ptr, rows_u, thin_solve, f->U.group, udiag, [&](int i, auto emit) {
                for (int p = dpos[(size_t)i] + hasdiag[(size_t)i]; p < rp[(size_t)i + 1]; p++)
                    emit(p, ci[(size_t)p]);
            }, sps[2]);
        });
        for (std::thread &x : th) x.join();
    }
    phase("plans");
    f->fac_segs = fplan.segs;
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = upload_vec(&f->d_rchunks, fplan.chunks);
    if (e == hipSuccess) e = upload_vec(&f->d_ritems, fplan.items);
    if (e == hipSuccess) e = upload_vec(&f->d_rpairs, fplan.pairs);
    if (e == hipSuccess) e = upload_vec(&f->d_rstaged, fplan.staged);
    if (e == hipSuccess) e = upload_vec(&f->d_rrounds, fplan.rounds);
    if (e == hipSuccess) e = upload(&f->d_upd_ptr, sym.upd_ptr);
    if (e == hipSuccess) e = upload(&f->d_upd_l, sym.upd_l);
    if (e == hipSuccess) e = upload(&f->d_upd_u, sym.upd_u);
    if (e == hipSuccess) e = upload(&f->d_lord, sym.lord);
    if (e == hipSuccess) e = upload(&f->d_lend, sym.lend);
    {  // per lower position (i, k): the position of its divisor u_kk (-1: none, or upper)
        std::vector<int> udiv((size_t)nnz_s, -1);
        for (int i = 0; i < n; i++)
            for (int p = rp[(size_t)i]; p < dpos[(size_t)i]; p++) {
                const int k = ci[(size_t)p];
                if (hasdiag[(size_t)k]) udiv[(size_t)p] = dpos[(size_t)k];
            }
        if (e == hipSuccess) e = upload(&f->d_udiv, udiv);
        std::vector<rsp::FacRow> frow(std::max<size_t>(rows_l.size(), 1), rsp::FacRow{});
        for (size_t x = 0; x < rows_l.size(); x++) {
            const int i = rows_l[x], rs = rp[(size_t)i], re = rp[(size_t)i + 1];
            frow[x] = rsp::FacRow{i, rs, dpos[(size_t)i], re, sym.upd_ptr[(size_t)rs], sym.upd_ptr[(size_t)re],
                                  hasdiag[(size_t)i], 0};
        }
        if (e == hipSuccess) e = upload_vec(&f->d_frow, frow);
        // fat factor levels in the slot layout (rsp::FacSlotLevel): each row's
        // structure at a fixed stride, so ilu0_level_slot reads it in one
        // round trip. Levels past RSP_ILU_SLOT_CAP_MB of slots keep FacRow.
        const std::vector<int> &lp = f->L.ptr;
        const int nlev = (int)lp.size() - 1;
        f->fslev.assign((size_t)std::max(nlev, 0), rsp::FacSlotLevel{0, 0, 0, 0, 0});
        // Slot budget (ints): RSP_ILU_SLOT_CAP_MB if set, else the smaller of
        // 2 GB and 1/8 of the device memory free now. A level whose padded
        // slots would take more than twice its rows' own structure (one large
        // row among many small ones) keeps the FacRow path.
        long long cap_mb = env_int("RSP_ILU_SLOT_CAP_MB", -1);
        if (cap_mb < 0) {
            size_t fr = 0, tot = 0;
            cap_mb = 2048;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess) cap_mb = std::min<long long>(cap_mb, (long long)(fr >> 23));
        }
        const long long cap = cap_mb * (1LL << 20) / 4;
        long long total = 0;
        std::vector<int> slot_levels;
        slot_desc.clear();
        slot_offs.clear();
        for (const rsp::LevelSeg &sg : fplan.segs) {
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
                if (total + cnt * stride > cap) continue;
                f->fslev[(size_t)l] = rsp::FacSlotLevel{total, stride, rm, qm, 0};
                total += cnt * stride;
                slot_levels.push_back(l);
            }
        }
        if (total > 0) {  // written on the device from the symbolic arrays (ilu0_build_slots)
            for (int l : slot_levels) {
                const rsp::FacSlotLevel &sl = f->fslev[(size_t)l];
                for (int x = lp[(size_t)l]; x < lp[(size_t)l + 1]; x++) {
                    slot_desc.push_back(int4{x, sl.rm, sl.qm, 0});
                    slot_offs.push_back(sl.off + (long long)(x - lp[(size_t)l]) * sl.stride);
                }
            }
            // the slot layout is an optimisation: without its memory the
            // FacRow path factors every fat level (same bits)
            if (e == hipSuccess && hipMalloc((void **)&f->d_fslots, (size_t)total * sizeof(int)) != hipSuccess) {
                (void)hipGetLastError();
                f->d_fslots = nullptr;
                f->fslev.assign(f->fslev.size(), rsp::FacSlotLevel{0, 0, 0, 0, 0});
                slot_desc.clear();
                slot_offs.clear();
            }
        }
    }
    if (e == hipSuccess) e = upload(&f->d_dpos, dpos);
    if (e == hipSuccess) e = upload(&f->d_hasdiag, hasdiag);
    if (e == hipSuccess) e = upload(&f->L.d_rows, rows_l);
    if (e == hipSuccess) e = upload(&f->L.d_ptr, f->L.ptr);
    if (e == hipSuccess) e = upload(&f->LT.d_rows, rows_lt);
    if (e == hipSuccess) e = upload(&f->LT.d_ptr, f->LT.ptr);
    if (e == hipSuccess) e = upload(&f->U.d_rows, rows_u);
    if (e == hipSuccess) e = upload(&f->U.d_ptr, f->U.ptr);
    for (int kind = 0; kind < 3 && e == hipSuccess; kind++) {
        rsp_ilu0_info::Dag &d = kind == 0 ? f->L : (kind == 1 ? f->LT : f->U);
        SolvePlan &sp = sps[kind];
        d.segs = sp.segs;
        d.nshort = sp.nshort;
        d.nwave = sp.nwave;
        d.sbase = sp.sbase;
        e = upload_vec(&d.d_tasks, sp.tasks);
        if (e == hipSuccess) e = upload_vec(&d.d_nshort, sp.nshort);
        if (e == hipSuccess) e = upload_vec(&d.d_tpos, sp.tpos);
        if (e == hipSuccess) e = upload_vec(&d.d_src, sp.src);
        if (e == hipSuccess) e = upload_vec(&d.d_chunks, sp.chunks);
        if (e == hipSuccess) e = upload_vec(&d.d_trow, sp.trow);
        if (e == hipSuccess) e = upload_vec(&d.d_sid, sp.sid);
        if (e == hipSuccess) e = upload_vec(&d.d_stg, sp.stg);
        d.nterms = (int)sp.tpos.size();
    }
    {  // solve streams: values per flat term, alpha x and u_ii per level-order slot (fp64 size)
        const size_t nt = (size_t)std::max({f->L.nterms, f->LT.nterms, f->U.nterms, 1});
        if (e == hipSuccess) e = hipMalloc(&f->d_sval, nt * sizeof(double));
        if (e == hipSuccess) e = hipMalloc(&f->d_sx, (size_t)std::max(n, 1) * sizeof(double));
        if (e == hipSuccess) e = hipMalloc(&f->d_sdg, (size_t)std::max(n, 1) * sizeof(double));
    }
    if (e == hipSuccess) e = hipMalloc((void **)&f->d_zero, sizeof(int));
    if (e == hipSuccess) e = hipMemsetD32(f->d_zero, INT_MAX, 1);
    if (e == hipSuccess && !slot_desc.empty()) {  // fat factor slots, written on the device
        int4 *d_desc = nullptr;
        long long *d_offs = nullptr;
        hipError_t es = upload_vec(&d_desc, slot_desc);
        if (es == hipSuccess) es = upload_vec(&d_offs, slot_offs);
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
            a.plan.rows = f->L.d_rows;
            es = rsp_k::ilu0_build_slots(a, d_desc, d_offs, (int)slot_desc.size(), f->d_fslots, h->stream);
            if (es == hipSuccess) es = hipStreamSynchronize(h->stream);
        }
        if (d_desc) (void)hipFree(d_desc);
        if (d_offs) (void)hipFree(d_offs);
        if (es != hipSuccess) {  // no slots: fall back to the FacRow path, not a failed analysis
            (void)hipGetLastError();
            (void)hipFree(f->d_fslots);
            f->d_fslots = nullptr;
            f->fslev.assign(f->fslev.size(), rsp::FacSlotLevel{0, 0, 0, 0, 0});
        }
    }
    phase("uploads");
    if (e != hipSuccess) {
        ilu_free_device(f);
        return e == hipErrorOutOfMemory ? RSP_STATUS_ALLOC_FAILED : RSP_STATUS_EXECUTION_FAILED;
    }
    f->n = n;
    f->nnz_s = nnz_s;
    f->rowptr = d_row_offsets;
    f->colidx = d_col_ind;
    f->analysed = 1;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_ilu0_levels(rsp_ilu0_info_t f, int *levels_lower, int *levels_upper) {
    if (!f || !f->analysed) return RSP_STATUS_INVALID_VALUE;
    if (levels_lower) *levels_lower = (int)f->L.ptr.size() - 1;
    if (levels_upper) *levels_upper = (int)f->LT.ptr.size() - 1;
    return RSP_STATUS_SUCCESS;
}

rsp_status_t rsp_ilu0_zero_pivot(rsp_handle_t h, rsp_ilu0_info_t f, int *position) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !position) return RSP_STATUS_INVALID_VALUE;
    *position = -1;
    if (!f->analysed) return RSP_STATUS_INVALID_VALUE;
    int pos = f->structural_zero;
    if (f->factored) {
        int z = INT_MAX;
        RSP_CHECK_HIP(hipMemcpyAsync(&z, f->d_zero, sizeof(int), hipMemcpyDeviceToHost, h->stream));
        RSP_CHECK_HIP(hipStreamSynchronize(h->stream));
        if (z != INT_MAX && (pos < 0 || z < pos)) pos = z;
    }
    if (pos >= 0) {
        *position = pos;
        return RSP_STATUS_ZERO_PIVOT;
    }
    return RSP_STATUS_SUCCESS;
}

static rsp::LevelPlan level_plan(const rsp_ilu0_info::Dag &d, const std::vector<rsp::LevelSeg> &segs,
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
    p.nterms = d.nterms;
    p.nshort = d.d_nshort;
    p.nshort_host = d.nshort.data();
    p.nwave_host = d.nwave.empty() ? nullptr : d.nwave.data();
    return p;
}

rsp_status_t rsp_ilu0_factor(rsp_handle_t h, rsp_ilu0_info_t f, rsp_datatype_t value_type,
                             void *d_values) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !f->analysed || (f->nnz_s > 0 && !d_values)) return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
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
    a.rchunks = f->d_rchunks;
    a.ritems = f->d_ritems;
    a.rpairs = f->d_rpairs;
    a.rstaged = f->d_rstaged;
    a.rrounds = f->d_rrounds;
    a.plan = level_plan(f->L, f->fac_segs, f->fac_batch);
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
        std::vector<unsigned long long> t(trace_cap);
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

static rsp::TrsvArgs trsv_args(rsp_ilu0_info *f, const void *alpha, rsp_datatype_t t,
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
    return a;
}

rsp_status_t rsp_trsv_lower_unit(rsp_handle_t h, rsp_operation_t op, const void *alpha,
                                 rsp_ilu0_info_t f, rsp_datatype_t value_type,
                                 const void *d_values, const void *d_x, void *d_y) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !f->analysed || !alpha) return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    if (f->n > 0 && (!d_x || !d_y || d_x == d_y)) return RSP_STATUS_INVALID_VALUE;
    rsp::TrsvArgs a = trsv_args(f, alpha, value_type, d_values, d_x, d_y);
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
        std::vector<unsigned long long> t(trace_cap);
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

rsp_status_t rsp_trsv_upper(rsp_handle_t h, const void *alpha, rsp_ilu0_info_t f,
                            rsp_datatype_t value_type, const void *d_values, const void *d_x,
                            void *d_y) {
    if (!h) return RSP_STATUS_NOT_INITIALIZED;
    if (!f || !f->analysed || !alpha) return RSP_STATUS_INVALID_VALUE;
    if (value_type != RSP_R_64F && value_type != RSP_R_32F) return RSP_STATUS_INVALID_VALUE;
    if (f->n > 0 && (!d_x || !d_y || d_x == d_y)) return RSP_STATUS_INVALID_VALUE;
    rsp::TrsvArgs a = trsv_args(f, alpha, value_type, d_values, d_x, d_y);
    a.plan = level_plan(f->U, f->U.segs, f->U.batch);
    hipError_t e;
    if (value_type == RSP_R_64F)
        e = rsp_k::trsv_upper_f64(a, h->stream);
    else
        e = h->ftz ? rsp_k_ftz::trsv_upper_f32(a, h->stream) : rsp_k::trsv_upper_f32(a, h->stream);
    return e == hipSuccess ? RSP_STATUS_SUCCESS : RSP_STATUS_EXECUTION_FAILED;
}

}  // extern "C"
