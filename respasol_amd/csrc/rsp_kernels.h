// rsp_kernels.h — internal interface between the C-ABI (rsp_api.cpp) and the
// HIP kernel translation units. The kernel TUs are compiled twice: once as
// namespace rsp_k (IEEE fp32 denormals) and once with
// -fgpu-flush-denormals-to-zero as namespace rsp_k_ftz (the `-ftz=true`
// build of GPU/Makefile:5). fp64 never flushes, so the FTZ namespace carries
// fp32 entry points only.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsp {

// One entry of the SpMV schedule (built by rsp_spmv_preprocess).
//   r1 >= 0       : rows [r0, r1) whose entries [k0, k1) fit one workgroup tile
//                   (every row <= kSpmvLongRow entries);
//   r1 == INT_MIN : the whole long row r0 (kSpmvLongRow < len <= tile cap),
//                   reduced by the 256 threads and written to y directly;
//   other r1 < 0  : chunk [k0, k1) of a row longer than a tile; its partial
//                   goes to slot s = -(r1 + 1) and the chunks are added in
//                   order by the row's last-arriving chunk (or, variant bit 8,
//                   by the separate fixup kernel).
// Partial slot s occupies partials[2 s] (its value) and partials[2 s + 1]
// (the first slot of a row: the row's arrival ticket, an unsigned int kept
// at 0 between calls).
struct alignas(16) SpmvBlock {
    int r0, r1, k0, k1;
};

// Long row: partial slots [first, first + nchunks) belong to `row`.
struct alignas(16) SpmvLongRow {
    int row, first, nchunks, pad;
};

// Tile geometry shared by the planner and the kernels.
#ifndef RSP_SPMV_THREADS
#define RSP_SPMV_THREADS 256  // overridable for tile-geometry experiments (scripts/spmv_probe.py)
#endif
constexpr int kSpmvThreads = RSP_SPMV_THREADS;
#ifndef RSP_SPMV_ITER
#define RSP_SPMV_ITER 4  // overridable for tile-geometry experiments (scripts/spmv_probe.py)
#endif
constexpr int kSpmvIter = RSP_SPMV_ITER;  // vectors per thread per tile
#ifndef RSP_SPMV_MAXROWS
#define RSP_SPMV_MAXROWS 512  // overridable for tile-geometry experiments (scripts/spmv_probe.py)
#endif
constexpr int kSpmvMaxRows = RSP_SPMV_MAXROWS;  // rows per tile (row offsets staged in LDS)
constexpr int kSpmvLongRow = 256;   // rows longer than this get the 256-thread tree
constexpr int kSpmvHeavyMax = 128;  // rows of > 32 entries a tile can hold (<= 4093 / 33)
constexpr int kSpmvWholeRow = -2147483647 - 1;  // SpmvBlock::r1 marker (INT_MIN)
template <typename T>
struct SpmvTile {
    static constexpr int kVec = 16 / sizeof(T);                           // 16-B loads
    static constexpr int kSlots = kSpmvThreads * kSpmvIter * kVec;        // LDS products
    static constexpr int kMaxNnz = kSlots - (kVec - 1);                   // any alignment fits
    // long-row chunk (and longest row reduced whole): fixed by the canonical
    // summation order (oracle_spmv_canon_*), independent of the tile size
    static constexpr int kChunk = kSpmvThreads * 4 * kVec - (kVec - 1);   // 2047 / 4093
    static_assert(kChunk <= kMaxNnz, "a chunk must fit one tile");
    // rows per tile: fp32 tiles hold twice the entries, so twice the rows
    // (fp32 moderate step 0.077 -> 0.0734 ms with 1024; fp64 unchanged by it)
    static constexpr int kMaxRows = sizeof(T) == 8 ? kSpmvMaxRows : 2 * kSpmvMaxRows;
    // staged tiles (round 4): the tile's distinct columns, at most kStageSlots
    // of them, loaded once into the LDS image as contiguous column runs (at
    // most kStageRuns); each entry then reads its x from LDS
    static constexpr int kStageSlots = sizeof(T) == 8 ? 1536 : 2048;
    // list-staged tiles (random-band tiles: too many runs, so an explicit
    // column list): fp64 only — the list's registers fit under fp64's 64-VGPR
    // occupancy step but would cost fp32 a wave per SIMD (71 -> 77 VGPRs)
    static constexpr bool kStageList = sizeof(T) == 8;
};
static_assert(SpmvTile<float>::kMaxNnz / 33 < kSpmvHeavyMax && SpmvTile<double>::kMaxNnz / 33 < kSpmvHeavyMax,
              "every > 32-entry row of a tile fits the heavy-row list");
constexpr int kStageRuns = 254;  // run descriptors per staged tile (+1 sentinel <= 256 threads)

struct SpmvArgs {
    int m;
    const int *rowptr;
    const int *colidx;
    const void *vals;
    const void *x;
    void *y;
    const SpmvBlock *blocks;
    int nblocks;
    // per tile: >= 0 column base of its 16-bit column offsets; -1 int32 colidx;
    // <= -2 a staged tile: code = -2 - cbase, its run descriptors at
    // runs[2 (code >> 8) ..], (code & 255) of them + a sentinel, and its
    // 16-bit values are LDS slot indices of the tile's distinct columns
    const int *cbases;
    const unsigned short *cidx;   // 16-bit column offsets / slot indices (tiles with cbases != -1)
    const int *runs;              // staged tiles: {first column, first slot} per run, {0, slots} last
    int cmax;                     // n - 1 (clamp for neighbour entries of partial vectors)
    const SpmvLongRow *longrows;
    int nlong;
    void *partials;
    double alpha, beta;
    int nnz;        // rowptr[m]: tiles touching the last partial vector go scalar
    int vector_ok;  // colidx/vals 16-B aligned -> vector loads
    int variant;    // bit 0: default-policy (not non-temporal) vals/colidx loads;
                    // bit 4 (plan time): no spreading of a batch's small launches;
                    // bit 9 (plan time): spread single-matrix plans (round-2 rule, A/B);
                    // bit 8: long rows by the separate fixup kernel
};

// Several independent SpMVs in one launch (rsp_spmv_batch_*). The batch
// concatenates the matrices' tiles and long rows; matrix j of a launch owns
// tiles [tiles.begin[j], tiles.begin[j + 1]) and long rows
// [longs.begin[j], longs.begin[j + 1]). The begin tables travel in the kernel
// arguments (entries past `count` hold INT_MAX), so a workgroup finds its
// matrix with scalar compares and loads its entry and its tile in parallel.
constexpr int kSpmvBatchMax = 32;  // matrices per launch
struct alignas(16) SpmvBatchEntry {
    const int *rowptr;
    const int *colidx;
    const void *vals;
    const void *x;
    void *y;
    void *partials;
    const unsigned short *cidx;  // 16-bit column offsets (SpmvArgs::cidx)
    const int *runs;             // staged tiles' run descriptors (SpmvArgs::runs)
    int nnz;        // rowptr[m] (as SpmvArgs::nnz)
    int vector_ok;  // colidx/vals 16-B aligned
    int cmax;       // n - 1
};
struct SpmvBatchTable {
    int begin[kSpmvBatchMax + 1];
};
struct SpmvBatchArgs {
    const SpmvBatchEntry *entries;
    const SpmvBlock *tiles;
    const int *cbases;  // per tile, parallel to `tiles`
    const SpmvLongRow *longrows;
    int count;
    SpmvBatchTable tiles_at, longs_at;
    double alpha, beta;
    int variant;  // bit 0: default-policy loads; bit 3: no per-matrix XCD swizzle;
                  // bit 8: long rows by the separate fixup kernel
};
constexpr int kSpmvVariantFixup = 256;
constexpr int kSpmvVariantNoStage = 1024;  // plan time: no staged tiles (A/B)

// Level schedule of one dependency DAG. Rows are grouped by level
// (rows[ptr[l] .. ptr[l+1])); `segs` (host) cover the levels in order, each
// {lev_begin, lev_end, thin, chunk_begin, chunk_end}: a thin segment is a run
// of small levels that one 1024-thread workgroup walks with workgroup
// barriers between levels (one launch for the whole run; a solve run is cut
// into LDS-staged chunks [c0, c1) of `chunks`); a fat segment is one launch
// per level.
//
// A solve DAG's fat segment of two or more levels is a FLOW segment: c0 / c1
// delimit its work items (FlowItem), which one persistent launch runs in
// order, each item waiting only for the y values it reads (trsv_flow).
struct LevelSeg {
    int lb, le, thin, c0, c1;
    int nth;  // thin solve runs: workgroup size (64 / 256 / 1024, >= the run's widest level)
};
// Solve task of one row, stored in level order: the fma chain runs over the
// flat terms [t0, t1) (term k: matrix value vals[tpos[k]] times the y given
// by src[k]); d = diagonal position for the U solve (-1 = missing).
struct alignas(16) RowTask {
    int i, t0, t1, d;
};
struct alignas(16) LevelChunk {  // levels [l0, l1) of a thin solve run, staged in LDS together
    int l0, l1;
    int x0, x1;    // its level-order slots: ptr[l0], ptr[l1]
    int k0, k1;    // its flat terms: tasks[x0].t0, tasks[x1 - 1].t1
    int st0, st1;  // its staged terms: stg[st0 .. st1)
};
// Work item of a flow segment (level order): n > 0 = short rows x0 .. x0+n-1
// (<= 64, a lane each; t0 >= 0: the padded layout, row r's kFatLongTerms flat
// terms at t0 + r * kFatLongTerms), n == 0 = the one row at slot x0, a wave;
// gate = a row of an earlier level to wait for first (-1 = none; trsv_flow).
struct alignas(16) FlowItem {
    int x0, n, t0, gate;
};
// Static LDS record of a thin-run row (per level-order slot): first term group
// (chunk-relative) | groups << 16, its y window slot, the row, its diagonal.
struct alignas(16) ThinRowPlan {
    int g, out, i, d;
};
// A thin-run term whose y is staged at the chunk start: its chunk-relative
// slot and the row j whose y it needs.
struct alignas(8) StagedTerm {
    int slot, j;
};

struct LevelPlan {
    const int *rows;      // device
    const int *ptr_dev;   // device, nlev + 1
    const int *ptr_host;  // host, nlev + 1
    int nlev;
    const LevelSeg *segs; // host
    int nseg;
    int batch;            // fma-chain load batch (2, 4, 8) from the mean chain length
    int group;            // thin runs: terms padded to groups of this many (2 or 4)
    // solve DAGs only (device):
    const RowTask *tasks; // task of rows[x] at slot x
    const int *tpos;      // flat term -> position in vals
    const int *src;       // flat term -> y source: >= 0 the column (global y, or its value
                          // staged at the chunk start), < 0 slot -(s+1) of the LDS y window
    const LevelChunk *chunks;
    const ThinRowPlan *trow;  // thin runs: static row records (per level-order slot)
    const int *sid;       // thin runs: per term, its y's index in the LDS y buffer
    const StagedTerm *stg;  // thin runs: staged terms, per chunk [st0, st1)
    const FlowItem *fitems; // flow segments: work items, per segment [c0, c1)
    int has_flow;           // the DAG has a flow segment
    int nterms;           // flat terms
    const int *nshort;    // per level: short rows come first (host copy: nshort_host)
    const int *nshort_host;
    const int *nwave_host;  // per level: short + wave rows (fat solve levels; the rest are hub rows)
    const int *sbase_host;  // per level: fat levels whose short rows sit kFatLongTerms flat terms
                            // apart (pads after each row's terms) start at this term; -1 = unpadded
};
constexpr int kLongTerms = 64;       // thin-run solve rows with more terms are done by a whole wave
constexpr int kHubTerms = 256;       // fat-level solve rows with more terms: a workgroup each (RSP_ILU_HUB)
constexpr int kFatLongTerms = 8;     // padded short-row layout: a short row's flat terms (RSP_ILU_FAT_LONG=8)
// fat-level solve rows with more terms than this: a wave each (RSP_ILU_FAT_LONG; round 4: 8 -> 3,
// config-3 solve 42.5 -> 41.6 ms, para-10 -19 %, 2cubes_sphere -22 %, profiles/r04_ilu_fatlong_ab.txt;
// the padded layout needs 8, so it is used only when the knob asks for 8)
constexpr int kFatLongDefault = 3;
constexpr int kYWin = 4096;          // LDS y window of a thin solve run (entries, power of 2)
constexpr int kChunkRows = 1024;     // rows staged per thin-run chunk (<= kYWin)
constexpr int kChunkTerms = 4096;    // terms staged per thin-run chunk
constexpr int kThinThreads = 1024;   // workgroup of a thin segment
constexpr int kGroup = 4;            // thin-run rows: terms padded to whole groups of (at most) this many
constexpr int kPadSrc = -(kYWin + 1); // source of a pad term: the zero slot after the y window
constexpr int kIluWaves = 4;         // rows per 256-thread workgroup (fat factor levels, global path)
constexpr int kFacRow = 256;         // fat factor levels: rows staged in LDS up to this many entries
constexpr int kFacPairs = 1024;      // ... and this many update pairs (else the global path)
constexpr int kThinSolveRows = 512;  // solve levels this small (and <= kThinSolveTerms terms) run thin
constexpr int kThinSolveTerms = 2048; // (padded terms; wider levels run on all CUs: flow segments)
constexpr int kThinFactorRows = 1024; // factor levels this small (and within kRndLevelItems) run thin
// LDS-staged factor chunks (ilu0_chunked): a chunk is a run of levels whose
// rows' positions ("items") and update pairs fit these budgets.
// Round-based thin factor runs (ilu0_rounds): budgets of one LDS chunk, and
// which levels run thin (<= kRndLevelItems positions, every position's update
// list <= kRndItemPairs pairs; RSP_ILU_THIN_FACTOR / _ITEMS knobs).
constexpr int kRndItems = 2048;
constexpr int kRndPairs = 4096;
constexpr int kRndStaged = 4096;
constexpr int kRndRounds = 2048;
// hub levels (a row past the slot layout, so no flow launch) run thin up to this many positions
// (round 4: 2048 -> 32768, config-3 factor 58.8 -> 57.2 ms: dc1 7.38 -> 7.02, ASIC_320ks 2.46 -> 1.92,
// ss1 1.86 -> 1.47; larger gains nothing; profiles/r04_ilu_factor_ab.txt)
constexpr int kRndLevelItems = 1 << 15;
constexpr int kRndFlowItems = 1024;  // ... kRndFlowItems if the level could run in a flow launch
constexpr int kRndItemPairs = 1024;
constexpr int kRndLevelStart = 1 << 15;  // rounds[]: this round opens a level (or a chunk)
struct alignas(16) RndChunk {  // flat ranges of a chunk's items, pairs, staged values, rounds
    int i0, i1, p0, p1, s0, s1, r0, r1;
};
// One position of a thin factor run: its position in vals, its update pairs
// (chunk-relative start | count << 16), its divisor u_kk as an operand index
// (-1: upper, no division), the row if it is that row's diagonal (else -1).
// Operand indices: [0, K) this chunk's slots, [K, 2K) the previous chunk's,
// [2K, 2K + kRndStaged) staged values, 2K + kRndStaged the zero slot
// (K = kRndItems); a pair packs (l_ik | u_kj << 16).
struct alignas(16) RndItem {
    int pos, u, d, zr;
};

// A row of a fat factor level (level-order slot): its row, entry range with
// the diagonal split, its update-pair range, whether it has a diagonal.
struct alignas(16) FacRow {
    int i, rs, di, re, q0, q1, hasdiag, pad;
};

// Fat factor levels, slot layout (ilu0_level_slot): the rows of fat level l
// are fixed-stride slots (stride ints) at fslots + off, row b of the level at
// slot b, so a workgroup finds its row's whole structure without first
// reading a record. Slot: header {i, rs, nlo, nr, nq, hasdiag, global, 0};
// [8, 8 + rm): divisor position of each lower entry (udiv, -1 = none);
// [8 + rm, 8 + 2 rm): up | lo << 11 | le << 20 per entry (upd_ptr, lord,
// lend relative to the row); from kPairsAt(rm): (upd_u, upd_l - rs) per
// update pair. rm / qm = the level's largest LDS-path row / pair count;
// global = 1: the row exceeds kFacRow / kFacPairs (global path). stride 0:
// the level uses the FacRow path.
struct FacSlotLevel {
    long long off;
    int stride, rm, qm, pad;
};
__host__ __device__ constexpr int fac_pairs_at(int rm) { return (8 + 2 * rm + 1) & ~1; }

// Flow runs of the factor: two or more consecutive fat levels, all in the
// slot layout and without global-path rows, run as ONE persistent launch
// (ilu0_flow) over their rows in level order, a row starting when the rows it
// reads are done (per-row flags). A run: levels [lb, le), items [c0, c1).
// An item: its row's slot (fslots offset), the level's rm | qm << 16, and a
// row of an earlier level to wait for first (gate, -1 = none).
struct alignas(16) FacFlowItem {
    long long off;
    int rmqm, gate;
};
struct FacFlowRun {
    int lb, le, c0, c1;
};

// Flow launches (ilu0_flow, trsv_flow): one launch over a run of work items
// in level order; an item waits only for items of lower index.
// Item assignment (FlowCtl::mode):
//  * start tickets (kFlowTickets, the default, RSP_ILU_FLOW_MODE=2): each
//    workgroup takes ONE ticket t when it starts (one agent-scope fetch_add)
//    and its waves walk the static items of t (4 t + wave, + W, ...), so a
//    resident grid runs exactly the static walk. A wave that has waited
//    long (kFlowStealUs) while tickets < G are still unclaimed — some
//    workgroups never started: a co-running kernel holds their CUs — claims
//    one more ticket for its workgroup (a steal) and the workgroup's waves
//    walk all its tickets' items in index order, restarting an item whose
//    wait they abandon (a flow item writes nothing before its waits).
//    Every ticket is then held by a workgroup that has started, and the
//    lowest unfinished item is its owner's next: progress needs no
//    co-residency (ilu0.hip FlowClaims). The tickets come from eight
//    counters of one of two slots (launch sequence number & 1), zeroed by
//    the launch before;
//  * static (RSP_ILU_FLOW_MODE=0): wave w of the grid takes items w, w + W, ... Progress
//    needs every workgroup of the grid resident together: the grid is sized
//    from the occupancy query (one 4-wave workgroup per CU by default), and
//    a wait that outlasts `ticks` gives up and is REPORTED (below), so a
//    co-running kernel that keeps workgroups from being scheduled shows up
//    as EXECUTION_FAILED, never as a hang;
//  * claimed (kFlowClaims, RSP_ILU_FLOW_MODE=1): waves claim items in the
//    order they actually run from one device counter (agent-scope
//    fetch_add, two items ahead), so an item that is waited on is always
//    held by a running wave and no co-residency is needed. Measured on
//    config 3: fp64 factor 59.5 -> 85.8 ms, solve 43.6 -> 53.5 ms (every
//    claim serialises on the one counter), hence opt-in. The counter is
//    never reset: a launch over items [it0, it1) with W waves advances it by
//    exactly (it1 - it0) + 2 W, which the launcher adds to the host mirror,
//    so the next launch knows its base.
// A wait longer than `ticks` (100 MHz wall clock) gives up — never expected;
// a bound instead of a hang — and stores `gen` (the call's generation) into
// *status, which rsp_ilu0_zero_pivot / rsp_trsv_zero_pivot compare with the
// generation of the call they report on.
struct FlowCtl {
    int *status;                      // device word: generation of the last call that gave up
    int gen;                          // this call's generation (>= 1)
    unsigned long long ticks;         // give-up bound (RSP_ILU_FLOW_TIMEOUT_US)
    unsigned long long *claim;        // device claim counter
    unsigned long long *claim_host;   // host: claims issued by the launches enqueued so far
    int mode;                         // RSP_ILU_FLOW_MODE: 0 static items, kFlowClaims claimed items, kFlowTickets start tickets
    unsigned *tickets;                // tickets: two slots of kFlowTicketCtrs counters (launch seq & 1)
    unsigned long long *tk_seq;       // host: ticket launches enqueued so far (a launch's `base`)
    int *done;                        // tickets: per item, the epoch of the call that finished it (after a steal)
    int grid_x;                       // tickets, tests: grid x this past the resident one (RSP_ILU_FLOW_GRID_X)
    unsigned epoch;                   // this call's epoch (unique per call of the info, >= 1)
};
constexpr int kFlowClaims = 1;
constexpr int kFlowTickets = 2;
constexpr int kFlowTicketCtrs = 8;    // tickets: start-claim counters per launch
constexpr int kFlowOwnMax = 1024;     // tickets: the most one workgroup can own (>= the largest flow grid)
#ifndef RSP_TK_STEAL_US
#define RSP_TK_STEAL_US 50
#endif
constexpr int kFlowStealUs = RSP_TK_STEAL_US;      // tickets: a wait this long may steal (2 us once the workgroup has)


struct IluArgs {
    int n;
    const int *rowptr;
    const int *colidx;
    const int *dpos;      // first position with col >= row
    const int *hasdiag;   // 1 if colidx[dpos[i]] == i
    void *vals;
    int *zero_pivot;      // device int, atomicMin target (INT_MAX = none)
    // Update lists (symbolic ILU(0)): position p = (i, j) receives
    // a_ij -= l_ik u_kj for k = the lower columns of row i with u_kj in the
    // pattern, k ascending: pairs (upd_l[u], upd_u[u]) for u in
    // [upd_ptr[p], upd_ptr[p+1]) are the positions of l_ik and u_kj.
    const int *upd_ptr;
    const int *upd_l;
    const int *upd_u;
    // Lower positions of row i, slots [rowptr[i], dpos[i]), grouped by
    // intra-row stage (l_ij waits for the l_ik of its own update list):
    // lord = position, lend = one past the last slot of the slot's stage.
    const int *lord;
    const int *lend;
    const int *udiv;      // lower position (i, k): position of u_kk, -1 if row k has no diagonal
    const FacRow *frow;   // per level-order slot of the L DAG (ilu0_level_lds)
    const int *fslots;    // fat factor levels in the slot layout (ilu0_level_slot), device
    const FacSlotLevel *fslev;  // per level (host), or null
    int fat_slots;        // RSP_ILU_FAT_SLOT (default 1): use the slot layout where built
    int fat_lds;          // fat levels: rows staged in LDS (ilu0_level_lds; RSP_ILU_FAT_LDS=0: global path)
    LevelPlan plan;       // L DAG, factor thresholds
    // round-based thin runs (ilu0_rounds), see RndChunk / RndItem
    const RndChunk *rchunks;
    const RndItem *ritems;
    const int *rpairs, *rstaged, *rrounds;
    unsigned long long *trace;  // diagnostics (RSP_ILU_FTRACE): 4 words per thin-run chunk, or null
    int trace_cap;
    int defer_rounds;  // narrow runs of at least this many rounds flush their items after the run
    int narrow_waves;  // ... and run on this many waves, levels round-robin (RSP_ILU_FNARROW_WAVES)
    // flow runs (ilu0_flow)
    const FacFlowItem *fitems;  // device
    const FacFlowRun *fruns;    // host
    int nfruns;
    const int *lev;             // device: L level of each row
    void *forig;                // device: flow rows' upper input values (ilu0_flow_prep), nnz_s T
    int gen;                    // this factor call's generation (>= 1)
    int flow, flow_grid, flow_sleep;
    int flow_cus;               // CUs of the device (caps a flow grid)
    FlowCtl fc;                 // flow launches: give-up status word, claim counter
    // a pattern without update pairs (rsp_an::IluHostPlan::fac_scale): the
    // whole factor is ilu0_scale_lower, one launch (RSP_ILU_FAC_SCALE=0 at
    // analysis: the one-level plan instead)
    int fac_one;
};

// Block-inverse solve of a deep DAG (round 6; plan: ilu_blocks.cpp, kernels:
// trsv_blocks.hip). The rows in level order ("positions") are cut into
// chunks of kBlkWin positions and, inside a chunk, into blocks of <=
// kBlkRows rows; every row's unknown is a combination (its PATTERN: x
// sources, the block's right-hand sides, then y sources, earlier blocks'
// unknowns, each ascending by position) with coefficients E — the block's
// partitioned inverse, built by the solve from the factor's values
// (trsv_blk_coef). A row's y terms of EARLIER chunks are summed by a parallel
// prologue per chunk (with its x terms); its y terms of its OWN chunk
// (<= kBlkNear for a normal row) are one short fma chain on the chunk's LDS
// window, so a normal block is one dependent step of one wave (lane = row).
// A LONG block is one row whose pattern breaks the caps (a circuit's hub
// row): its terms are summed by a whole wave.
constexpr int kBlkRows = 64, kBlkYMax = 32, kBlkNear = 12, kBlkNearWin = 1 << 30, kBlkWin = 16384;
constexpr int kBlkLongCap = 64 * kBlkNear;  // a long row's in-chunk terms (one record); more start a chunk
constexpr int kBlkPre = 6;  // records in flight in the chunk walk (trsv_blk_seg)
struct alignas(16) BlkDesc {
    int p0, np, kind, kn;     // first position, rows, 0 normal / 1 long, in-chunk terms (rounds: long)
    int eoff, ne, doff, nd;   // its pattern entries (and coefficient slots), its dependencies
    int loff, nlev, ovf, pad; // coefficient build: level ranges at lptr[loff ..], intra-block levels;
                              // ovf: a long block's record overflow offset
};
struct alignas(16) BlkRow {
    int off, nx, ny, nfar;    // pattern entries [off, off + nx + ny): x, far y, near y
};
struct BlkSeg {
    int b0, b1, p0, p1;       // blocks [b0, b1) = positions [p0, p1)
};
struct BlkArgs {
    int n, nb;
    const int *order;         // position -> row
    const BlkDesc *desc;
    const BlkRow *rows;       // per position
    const int *ref;           // per entry: x source -> its row (x index); y source -> its position
    const int *vpos;          // per dependency (block order): position of its value
    const unsigned *eord;     // per coefficient slot (intra-block level order): entry | init 1 << 31
    const int *lptr;          // per block, nlev + 1 slot offsets
    const int *rptr;          // per slot: its recipe items [rptr[k], rptr[k + 1])
    const unsigned *rit;      // recipe item: dependency << 16 | source (0: the constant 1, else entry + 1); long blocks: dependency
    const BlkSeg *segs;       // host
    int nseg;
    int lds_elems;            // coefficient build: LDS values (T) of the largest normal block
    int lds_words;            // ... and LDS words (32-bit) of its slot data
    const void *vals, *x;
    void *y;
    double alpha;
    void *ev, *yp;            // scratch: coefficients (per entry), y by position
    // block records (trsv_blk_pro -> trsv_blk_seg): per block 64 lane records
    // (trsv_blocks.hip BlkLane: the lane's sum so far, its in-chunk
    // coefficients and window slots, its position; 144 / 96 B for fp64 / fp32)
    void *rc;
};

struct TrsvArgs {
    int n;
    const int *rowptr;
    const int *colidx;
    const int *dpos;
    const int *hasdiag;
    const void *vals;
    const void *x;
    void *y;
    double alpha;
    LevelPlan plan;       // the DAG of the solve (L, L^T or U), with its flat terms
    void *sval;           // per flat term: vals[tpos] (0 for a pad), written by trsv_stream
    void *sx;             // per level-order slot: alpha * x_i, written by trsv_stream
    void *sdg;            // per level-order slot: u_ii (U solve), written by trsv_stream
    unsigned long long *trace;  // diagnostics (RSP_ILU_TRACE): 8 timestamps per chunk, or null
    int trace_cap;
    int trace_clk;              // level stamps in shader clock cycles (s_memtime) instead
    int wave_lds;               // fat-level wave rows: chain on LDS broadcast operands (RSP_ILU_WAVE_LDS)
    int narrow_waves;           // thin runs: waves sharing a narrow run, levels round-robin (RSP_ILU_NARROW_WAVES)
    int narrow_split;           // L / L^T narrow runs: one wave, early sums under the late loads (RSP_ILU_NARROW_SPLIT)
    int narrow_pairs;           // L / L^T narrow runs on K waves, two levels per turn (RSP_ILU_NARROW_PAIRS: 1 / 0, -1 auto)
    int loaders;                // thin runs with the pair loop: its waves never load the next chunk (RSP_ILU_LOADERS)
    int flow;                   // run flow segments persistently (RSP_ILU_FLOW, default 1)
    int flow_grid;              // flow launch: 256-thread workgroups (RSP_ILU_FLOW_WPC waves per CU)
    int flow_cus;               // CUs of the device (caps a flow grid)
    FlowCtl fc;                 // flow launches: give-up status word, claim counter
    int flow_sleep;             // flow polls: longest pause, s_sleep units (RSP_ILU_FLOW_SLEEP)
};

}  // namespace rsp

#define RSP_DECLARE_KERNEL_API(NS)                                                              \
    namespace NS {                                                                              \
    hipError_t spmv_f32(const rsp::SpmvArgs &a, hipStream_t s);                                 \
    hipError_t spmv_batch_f32(const rsp::SpmvBatchArgs &a, hipStream_t s);                      \
    hipError_t ilu0_factor_f32(const rsp::IluArgs &a, hipStream_t s);                           \
    hipError_t trsv_lower_n_f32(const rsp::TrsvArgs &a, hipStream_t s);                         \
    hipError_t trsv_lower_t_f32(const rsp::TrsvArgs &a, hipStream_t s);                         \
    hipError_t trsv_upper_f32(const rsp::TrsvArgs &a, hipStream_t s);                           \
    hipError_t trsv_blocks_f32(const rsp::BlkArgs &a, hipStream_t s);                           \
    void warm_spmv();                                                                           \
    void warm_ilu();                                                                            \
    }

RSP_DECLARE_KERNEL_API(rsp_k)
RSP_DECLARE_KERNEL_API(rsp_k_ftz)

namespace rsp_k {
hipError_t gather(int elem_bytes, int64_t n, const int64_t *idx, const void *src, void *dst,
                  hipStream_t s);
hipError_t scatter(int elem_bytes, int64_t n, const int64_t *idx, const void *src, void *dst,
                   hipStream_t s);
hipError_t spmv_f64(const rsp::SpmvArgs &a, hipStream_t s);
hipError_t spmv_batch_f64(const rsp::SpmvBatchArgs &a, hipStream_t s);
int spmv_tiles_per_cu(int elem_bytes);  // resident spmv_tiles workgroups per CU
// warm_*: load the translation unit's code object on the current device now
// (HIP loads a code object at the first use of one of its kernels; without
// this, the first timed call of a run pays it: ~1.2-1.5 ms, measured).
void warm_analysis();
hipError_t ilu0_factor_f64(const rsp::IluArgs &a, hipStream_t s);
hipError_t trsv_lower_n_f64(const rsp::TrsvArgs &a, hipStream_t s);
hipError_t trsv_lower_t_f64(const rsp::TrsvArgs &a, hipStream_t s);
hipError_t trsv_upper_f64(const rsp::TrsvArgs &a, hipStream_t s);
hipError_t trsv_blocks_f64(const rsp::BlkArgs &a, hipStream_t s);
// Writes the slots of the fat factor levels (rsp::FacSlotLevel layout) from
// the symbolic arrays already on the device: one workgroup per slot row,
// desc[t] = {level-order slot x, rm, qm, 0}, offs[t] = its slot's offset.
hipError_t ilu0_build_slots(const rsp::IluArgs &a, const int4 *desc, const long long *offs, int nrows,
                            int *slots, hipStream_t s);
// ILU(0) analysis on the device (ilu_analysis.hip): diagonal positions +
// structural zero of a pattern the host has validated (flags[1] = atomicMin
// of the rows without a diagonal); the symbolic factor's update lists (count,
// exclusive scan, fill; rows_c / n_c: the rows of each length class, see
// ilu_analysis.hip; cap0 >= the longest row of class 0, <= 1024), then
// stages, stage order (lord / lend) and divisor positions (udiv; scratch: one
// int per position) of the rows of <= maxlen entries, one thread each, and of
// the nwrows rows listed in wrows (maxlen < length <= 1024), one wave each.
hipError_t ilu_an_rows(int n, const int *rp, const int *ci, int *dpos, int *hasdiag, int *flags, hipStream_t s);
hipError_t ilu_an_count(const int *const rows_c[3], const int n_c[3], int cap0, const int *rp, const int *ci,
                        const int *dpos, const int *hasdiag, int *cnt, int *gcur, hipStream_t s);
hipError_t ilu_an_scan(const int *cnt, int *ptr, int count, void *temp, size_t *temp_bytes, hipStream_t s);
hipError_t ilu_an_gather_pairs(const int *rows, int nrows, const int *rp, const int *ptr, const int *cbase,
                               const int *upd_l, const int *upd_u, int *out_l, int *out_u, hipStream_t s);
hipError_t ilu_an_fill(const int *const rows_c[3], const int n_c[3], int cap0, const int *rp, const int *ci,
                       const int *dpos, const int *hasdiag, const int *ptr, int *gcur, int *upd_l, int *upd_u,
                       hipStream_t s);
hipError_t ilu_an_stages(int n, int maxlen, const int *rp, const int *ci, const int *dpos, const int *hasdiag,
                         const int *ptr, const int *upd_l, int *stage, int *lord, int *lend, int *udiv,
                         int *scratch, const int *wrows, int nwrows, hipStream_t s);
// The per-term half of a solve plan (ilu_analysis.cpp solve_plan_terms, same
// arrays bit for bit) from its per-row half already on the device: flat term
// positions and y sources, the thin runs' window remap, row records, y
// indices, staged terms and the chunks' staged ranges. Row i's terms, in the
// split order (early, then late): kind 0 (L) positions lpos[rp[i] .. dpos[i])
// (column ci[p]); kind 1 (L^T) entries [ltp[i], ltp[i+1]) of the transposed
// lower part (position lts[q], column ltc[q]); ne[i] of them early. stg holds room for every thin-run term (>= 1 entry); scratch:
// slot_of (n ints), nst / nst_ptr (nch + 1 ints each), scan (temp bytes of
// ilu_an_scan over nch + 1). nstg_out (device, may be null): staged terms.
struct SolveTermsArgs {
    int kind, n, nx, total, nch, group;
    const rsp::RowTask *tasks;
    const int *ptr;  // level pointers
    const int *rp, *ci, *dpos;
    const int *ltp, *lts, *ltc;
    const int *lpos;  // kind 0: the split term order (position of term o of row i at lpos[rp[i] + o])
    const int *ne;    // per row: its early terms (split order; ilu_analysis.cpp split_padded)
    rsp::LevelChunk *chunks;
    const int *cbase;  // per chunk: its thin run's first slot
    int *tpos, *src, *sid;
    rsp::ThinRowPlan *trow;
    rsp::StagedTerm *stg;
    int *slot_of, *nst, *nst_ptr;
    void *scan;
};
hipError_t ilu_an_solve_terms(const SolveTermsArgs &a, hipStream_t s);
}  // namespace rsp_k
