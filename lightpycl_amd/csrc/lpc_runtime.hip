// lpc_runtime.hip -- host runtime behind the C ABI of include/lpc.h.
//
// One lpc_handle per GPU: a HIP stream, the uploaded scene (filter / exact /
// vertex records + mesh tables), a chunk workspace and the device-resident ray
// population of a trace.  All launches go to the handle's stream.
#include "lpc_kernels.hip"
#include "lpc.h"
#include "lpc_comm.hpp"
#include "lpc_build.hpp"
#include <hip/hip_ext.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <limits>
#include <map>
#include <string>
#include <vector>

using namespace lpck;

static double host_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

namespace {

struct DBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

// 8 SoA arrays (ox oy oz dx dy dz pw | pmid) in one allocation.
struct Pop {
    DBuf buf;
    int64_t cap = 0;
    float *f(int k) const { return (float *)buf.p + (size_t)k * cap; }
    int32_t *pmid() const { return (int32_t *)((float *)buf.p + (size_t)7 * cap); }
    RaysIn in(int64_t off = 0) const {
        RaysIn r;
        r.ox = f(0) + off; r.oy = f(1) + off; r.oz = f(2) + off;
        r.dx = f(3) + off; r.dy = f(4) + off; r.dz = f(5) + off;
        r.pw = f(6) + off; r.pmid = pmid() + off;
        return r;
    }
    RaysOut out(int64_t off = 0) const {
        RaysOut r;
        r.ox = f(0) + off; r.oy = f(1) + off; r.oz = f(2) + off;
        r.dx = f(3) + off; r.dy = f(4) + off; r.dz = f(5) + off;
        r.pw = f(6) + off; r.pmid = pmid() + off;
        return r;
    }
};

struct PieceTable {
    DBuf pieces, spieces;              // hierarchy pieces (k_roots_s / k_rootwalk), sliver pieces (k_slivers)
    int32_t npieces = 0, nspieces = 0;
    DBuf groups;                       // k_roots_s gate: the runs' root records, s_lo/s_hi = their pieces
    int32_t ngroups = 0;               // 0: no gate (pieces are the run roots, or > 64 runs)
    std::vector<float> sdmin;          // per sliver piece (ascending): min dmin of its slivers
};

const int kShadeF = 12;   // float arrays of the shade outputs
const int kShadeI = 8;    // int arrays
const int kAccRing = 8;   // mapped counter slots (iterations in flight: at most 2)

// Launch policy.  Each value won its A/B (DESIGN.md sections 5 and 7; the losing
// alternatives and their knobs were removed in round 5, the tables there keep the
// record).  None of them changes a result: every path flushes with
// order-independent atomics and the filters are supersets of the exact test.
const int64_t kSortMin = 4096;          // populations below this are traced unsorted
const int64_t kOnesweepMin = 500000;    // rocPRIM onesweep radix sort from this many rays (merge sort below)
const int kRootsPerBlock = 16;          // k_roots_s packets per block (one task per packet)
#ifndef LPC_Q_TARGET
#define LPC_Q_TARGET 65536               // compile-time A/B builds (tools/build_variant.py)
#endif
const int64_t kQTarget = LPC_Q_TARGET;  // (packet, piece) root tests to aim for: the piece level
#ifndef LPC_CHAIN_PIECES
#define LPC_CHAIN_PIECES 4              // compile-time A/B builds (tools/build_variant.py)
#endif
// chained populations up to kChainPiecesMax rays whose target gives the run roots
// (g = 1) in a scene of fewer than kChainPiecesRuns live mesh runs take the pieces
// of g = kChainPieces instead (round 5 A/B, DESIGN.md section 5: lens 10 M -21 %;
// the eye's >= 38 M-ray iterations +1-2 %, hence the size cap; the 10-run
// synthetic scene's config 5 +5 % (dense -3 %), hence the run bound)
const int32_t kChainPieces = LPC_CHAIN_PIECES;
const int64_t kChainPiecesMax = (int64_t)32 << 20;
const int64_t kChainPiecesRuns = 8;
#ifndef LPC_WALK_GRID
#define LPC_WALK_GRID 65536             // compile-time A/B builds (tools/build_variant.py)
#endif
const int64_t kWalkWaves = LPC_WALK_GRID;   // k_rootwalk grid (single-wave blocks, grid-stride)
const int64_t kSliverMergePpw = 4;      // packets per merged sliver unit (k_rootwalk's tail)
const int64_t kSliverWaves = 16384;     // k_slivers: (packet, piece) waves to aim for
#ifndef LPC_SPILL_LEVELS
#define LPC_SPILL_LEVELS 3               // compile-time A/B builds (tools/build_variant.py)
#endif
const int kSpillLevels = LPC_SPILL_LEVELS;  // k_spill levels (hand-over depth) for populations >= kSpillSmallN
const int kSpillLevelsSmall = 1;        // ... below (round 5 A/B: 4 levels, level budgets 10 or 14 / 8, two
                                        //   levels below: neutral or slower)
const int64_t kSpillSmallN = 262144;
#ifndef LPC_SPILL_BLOCKS
#define LPC_SPILL_BLOCKS 4096            // compile-time A/B builds (tools/build_variant.py)
#endif
const int64_t kSpillBlocks = LPC_SPILL_BLOCKS;  // k_spill level l grid: max(kSpillMinBlocks, kSpillBlocks >> l) x 4 waves
const int64_t kSpillMinBlocks = 256;
const int kSpillPairShift = 5;          // exact pairs per node visit in the hand-over budget (log2; round 5
                                        //   A/B with the pair list: 4 and 6 equal)
const int kKeyObits = 6;                // re-sorted populations: origin bits per axis of the 5-D Morton key
const double kThin = 1.0;               // thin-triangle rule factor (thin_axis; 0.25 / 2 measured slower)

}  // namespace

// The timing events of lpc_prof_enable skip the system-scope fence of an event
// record (cache writeback + invalidate: ~7 us of GPU idle per walk launch with
// it, ~0 without; round 5 A/B).  The side stream's fork /
// join events keep it (a device-scope release measured equal).
static const unsigned kEvTimingFlags = hipEventDisableSystemFence;

struct lpc_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    char name[256] = {0};
    int cus = 0;
    // scene
    int32_t M = 0, K = 0, Mpad = 0;
    std::vector<float> hv0, hv1, hv2;               // host copies, made on demand from d_raw (record rebuilds, profiling)
    const float *src_v[3] = {nullptr, nullptr, nullptr};   // the scene's (n,4) rows: the caller's during
                                                    //   lpc_scene_upload, hv0..2 after host_vertices()
    DBuf d_raw;                                     // the scene's v0 | v1 | v2 rows on the device ((M,4) each)
    std::vector<int32_t> run_lo, run_hi;
    std::vector<std::vector<int32_t>> run_levels;    // per run: (first node, count) per level, root first
    std::vector<FiltRec> node_self;                  // each node's own test (piece roots)
    std::vector<float> sliver_dmin_host;             // SliverRec::dmin, host copy
    double pop_dmax2 = INFINITY, init_dmax2 = INFINITY;   // max |D|^2 of the trace population / emitted rays
    std::vector<int32_t> run_slo, run_shi;           // sliver records per run
    int64_t n_slivers = 0;
    int64_t n_thin = 0;                              // of them thin triangles (thin_axis, k = 1)
    float box_lo[3] = {0, 0, 0}, box_scale[3] = {1, 1, 1};
    double scene_scale = 1.0;                        // half diagonal of the scene box (filter h)
    std::vector<int32_t> slot_run;
    std::vector<int32_t> meas_meshes;
    DBuf d_nodes, d_srec, d_xrec, d_verts, d_mat, d_ior, d_refl, d_diss;
    double dcap = 16.0;
    double dcap_init = 16.0;                        // LPC_DCAP_MILLI / 1000 (tests: a rebuild inside a trace)
    std::map<std::vector<int32_t>, PieceTable> ptabs;   // by the hierarchy level each live run is cut at
    // workspace
    int64_t chunk = 0;                              // rays per chunk (0 -> default)
    int64_t ws_rays = 0;
    DBuf w_key, w_sc, w_rs, w_shf, w_shi, w_blk_cnt, w_blk_off, w_blk_pow;
    DBuf w_soa, w_stage, w_sort, w_sort_tmp;
    DBuf w_aos;                                     // rays as 32-byte rows for the coherence gather
    DBuf w_tm;                                      // per ray: the slots a flush wrote (traced path, K <= 32)
    DBuf w_bhist;                                   // its per-block hi-digit counts + digit totals
    bool acc_pending = false;                       // next slot reset also resets the iteration counters
    int64_t acc_pending_total = 0;
    int64_t m_inflight = 0;                         // populations of the iterations enqueued, not yet read
    int64_t walk_grid = kWalkWaves;                 // k_rootwalk blocks (lpc_set_walk_grid, LPC_WALK_GRID)
    int64_t sliver_merge = 0;                       // LPC_SLIVER_MERGE: sliver units in k_rootwalk's grid from
                                                    // this population size (0: always; -1: never,
                                                    // k_slivers on the side stream)
    DBuf w_fc;                                      // k_shade_stage tile counts / power / max |dir|^2
    DBuf w_gsum;                                    // per 256-tile group counts, two buffers (zero when unused)
    int64_t gcap = 0;
    int gpar = 0;                                   // the buffer the next traced launch uses
    int64_t gdirty[2] = {0, 0};                     // groups a launch left non-zero in each buffer
    bool slots_clean = false;                       // every slot (max_ray_len slots_mrl, idx -1, count 0)
    float slots_mrl = 0.0f;
    bool misc_clean = false;                        // the launch words were reset for the next launch
    int half = 3;                                   // LPC_HALF: 3 = half-line cull at the piece roots of chained
                                                    //   populations (run_intersect), 0 = off
    bool half_roots = false;                        // ... at the piece roots (k_roots)
    bool in_trace = false;                          // run_intersect called from lpc_trace_iterate
    DBuf d_live;                                    // [K] slot written by some run
    DBuf w_pk;                                      // PacketRec per 128-ray wave (k_slivers)
    DBuf d_misc;                                    // LPC_MISC_WORDS per-launch words
    size_t sort_tmp_bytes = 0;
    int64_t resort_min = 2000000;                   // chained traced populations from this size are sorted again
    uint32_t *tm_cur = nullptr;                     // this launch's masks (the walk writes, k_shade_stage reads)
    // work hand-over (LPC_BUDGET, LPC_SPILL_CAP, LPC_LARGE_PER_TRI: tests drive the
    // queue-overflow and budget paths at small sizes)
    int spill_budget = 20;                          // node visits before a wave hands over (0 off)
    int64_t spill_large_per_tri = 16;
    int64_t spill_cap = (int64_t)1 << 22;           // k_spill queue capacity (items)
    DBuf w_spill;                                   // k_spill queue
    bool pop_traced = false;                        // the population is in its parents' traced order
    bool pop_emitted = false;                       // the population is the emitted rays (set_rays)
    int init_key_lo = 0, init_key_hi = 32;          // key bits that vary over the emitted rays (set_rays)
    bool init_bsort = false;                        // their sort may be the counting sort (bsort_fits)
    DBuf w_qroots;                                  // root items
    DevAcc *acc_host = nullptr;                     // pinned copy of d_acc (one read per iteration)
    DevAcc *acc_map = nullptr, *acc_map_dev = nullptr;   // mapped pinned ring k_scan / k_stage_move publish into
                                                    // (slot seq % kAccRing; + device address)
    // speculative iterations (trace_run, LPC_SPEC): iteration i + 1 is enqueued
    // device-sized (IterCtl) before iteration i's counters are read
    bool spec = true;
    DBuf d_ctl;                                     // IterCtl
    int ctl_par = 0;                                // the parity the next enqueued iteration reads
    double ds_thr = -INFINITY;                      // trace_run's power threshold (k_stage_move's stop rule)
    bool mat_passive = false;                       // no material can raise a ray's power (lpc_scene_upload)
    bool pow_nonneg = false;                        // every emitted power >= 0 (set_rays)
    std::vector<double> hist_r;                     // the last trace_run's populations / its first (the
    int32_t hist_iter = -1;                         //   speculation's prediction) and its iteration limit
    bool dcap_rebuilt = false;                      // check_dcap rebuilt the records (a speculative iteration is void)
    unsigned int acc_seq = 0;
    int host_prof = 0;                              // LPC_HOSTPROF: host-side timing of each iteration (stderr);
                                                    //   2: also each launch's hand-over queue lengths (synchronising)
    hipStream_t stream2 = nullptr;                  // side stream: the sliver kernels beside the hierarchy stage
    bool side_tried = false;                        // stream2 / ev_side created on first use (side_stream)
    // results export (lpc_trace_iterate_export): k_export packs a chunk's part of
    // the results tuple into xst[par] on the main stream, the export stream copies
    // it to the caller's host block while the next kernels run
    hipStream_t xstream = nullptr;
    hipEvent_t ev_xready[2] = {nullptr, nullptr}, ev_xdone[2] = {nullptr, nullptr};
    bool xdone_rec[2] = {false, false};             // ev_xdone[par] recorded (the staging may still be read)
    DBuf xst[2];
    int xpar = 0;
    bool x_inflight = false;                        // copies queued on xstream
    hipEvent_t ev_side[2] = {nullptr, nullptr};     // rays ready (main -> side), slivers done (side -> main)
    double host_last = 0.0;
    bool pop_init = false;                          // the population is I (the emitted rays, set_rays)
    bool mp_valid = false;                          // mp_last = the trace's measured power per measure mesh
    DBuf d_mrun;                                    // its running sums on the device (k_stage_move)
    DBuf d_cbase;                                   // chunked traced iterations: running row bases (ping-pong)
    DBuf w_tbox, d_pbox;                            // per-tile boxes (k_shade_stage), the population's box (k_stage_move)
    bool pbox_ok = false;                           // d_pbox holds the current population's origin box
    double mp_last[LPC_MP_MAX] = {0, 0, 0, 0};
    // trace
    Pop A, B, T, I;
    int64_t n_cur = 0, n_init = 0;
    float max_ray_len = 1e3f, ior_env = 1.0f;
    bool traced_ready = false;
    bool inflight = false;                          // the stream may still run a trace's last kernels (settle)
    DBuf m_buf;                                     // measured: x y z pw | mesh
    int64_t m_cap = 0, m_total = 0;
    DBuf d_acc;
    DBuf d_tmp;                                     // misc small device scratch
    DBuf d_scan;                                    // RayScan of set_rays (k_ray_scan)
    DBuf d_stats;                                   // walk counters (profiling)
    DBuf d_fan;                                     // profiling: fan-triangle flags (SpillArgs::fan)
    // profiling
    bool prof = false, prof_stats = false, prof_light = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_isect, ev_rest, ev_kern;
    std::vector<hipEvent_t> ev_pool;
    double prof_isect_ms = 0.0, prof_rest_ms = 0.0, prof_kern_ms = 0.0;
    int64_t prof_launches = 0, prof_pairs = 0;
    int prof_every = 1;                              // light mode: events on every prof_every-th walk launch
    int64_t prof_seq = 0;                            // ... walk launches seen
    bool prof_sampled = false;                       // the last run_queue's walk launch carries events
    // ray-sharded trace (lpc_set_allreduce): the termination decisions and the
    // trace-end aggregates over all ranks
    lpc_allreduce_fn xchg = nullptr;
    void *xchg_ctx = nullptr;
    std::vector<lpc_iter_stats> gstats;             // all-reduced per-iteration stats of the last lpc_trace_run
    double xchg_us = 0.0;                           // host time inside the hook (lpc_prof)
    int64_t xchg_calls = 0;
    // streamed batches of new rays (lpc_trace_stage_rays / lpc_trace_run_staged_async):
    // a FIFO of up to two staged batches, each copied to the device by a helper
    // thread on the copy stream while the handle traces the batch before it
    struct RaySlot {
        Pop P;                                      // the batch as SoA rows (swapped with I when it is traced)
        DBuf aos;                                   // its (n,4) origin / direction rows (stage modes 0, 1)
        void *pin = nullptr;                        // pinned host staging of the caller's rows
        size_t pin_bytes = 0;
        DBuf scan;                                  // k_ray_scan of the batch (device) ...
        RayScan *scan_host = nullptr;               // ... and its pinned copy
        hipEvent_t ev = nullptr;                    // the batch's copies, unpacks and scan done (cstream)
        std::thread th;
        int rc = 0;
        std::string err;
        int64_t n = 0;
        float max_ray_len = 1e3f, ior_env = 1.0f;
        int64_t scan_gen = -1;                      // the scene generation its scan keyed to (-1: none)
    } rslot[2];
    int64_t scene_gen = 0;                          // lpc_scene_upload count (the scan's key box)
    int rs_head = 0, rs_count = 0;
    hipStream_t cstream = nullptr;                  // copy stream of the staged batches
    int stage_mode = 0;                             // LPC_STAGE_MODE: 0 pageable DMA (round 6 A/B: 1.23-1.28 G
                                                    //   fresh rays), 1 pinned rows (0.83-0.93), 2 pinned SoA chunks (0.77-1.0)
    hipEvent_t ev_stage = nullptr;                  // main-stream work before a stage call (cstream waits)
};

static std::string g_open_err;

static int set_err(lpc_handle *h, int code, const std::string &msg)
{
    if (h) h->err = msg; else g_open_err = msg;
    return code;
}

#define HIPCHK(h, expr)                                                                     \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return set_err(h, LPC_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define RETIF(x)                  \
    do {                          \
        int rc_ = (x);            \
        if (rc_) return rc_;      \
    } while (0)

// Shading kernels templated on the register-resident slot count KU (shade_eval):
// the smallest of 4, 8, 12, 16 that holds the scene's K meshes, 0 = slots read
// from memory as postproc needs them (K > 16).
#define LPC_KU_LAUNCH(h, KERN, grid, block, stream, ...)                                          \
    do {                                                                                         \
        const int K_ = (h)->K;                                                                   \
        if (K_ <= 4) hipLaunchKernelGGL(KERN<4>, grid, block, 0, stream, __VA_ARGS__);           \
        else if (K_ <= 8) hipLaunchKernelGGL(KERN<8>, grid, block, 0, stream, __VA_ARGS__);      \
        else if (K_ <= 12) hipLaunchKernelGGL(KERN<12>, grid, block, 0, stream, __VA_ARGS__);    \
        else if (K_ <= 16) hipLaunchKernelGGL(KERN<16>, grid, block, 0, stream, __VA_ARGS__);    \
        else hipLaunchKernelGGL(KERN<0>, grid, block, 0, stream, __VA_ARGS__);                   \
    } while (0)

#define LPC_KU_LAUNCH2(h, KERN, B, grid, block, stream, ...)                                      \
    do {                                                                                         \
        const int K_ = (h)->K;                                                                   \
        if (K_ <= 4) hipLaunchKernelGGL((KERN<4, B>), grid, block, 0, stream, __VA_ARGS__);      \
        else if (K_ <= 8) hipLaunchKernelGGL((KERN<8, B>), grid, block, 0, stream, __VA_ARGS__); \
        else if (K_ <= 12) hipLaunchKernelGGL((KERN<12, B>), grid, block, 0, stream, __VA_ARGS__); \
        else if (K_ <= 16) hipLaunchKernelGGL((KERN<16, B>), grid, block, 0, stream, __VA_ARGS__); \
        else hipLaunchKernelGGL((KERN<0, B>), grid, block, 0, stream, __VA_ARGS__);              \
    } while (0)

// Wait for a trace's kernels still queued on the stream: lpc_trace_iterate and
// lpc_trace_run_async return once the iteration counters are published, while
// the rows of the next population still move.  Every entry point that copies
// device data to the host or reuses the caller's buffers calls this first.
static int settle(lpc_handle *h)
{
    if (h && h->inflight) {
        h->inflight = false;
        if (h->stream) HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    if (h && h->x_inflight) {                       // results-export copies to the caller's host blocks
        h->x_inflight = false;
        if (h->xstream) HIPCHK(h, hipStreamSynchronize(h->xstream));
    }
    return 0;
}

static int dalloc(lpc_handle *h, DBuf &b, size_t bytes, bool keep = false)
{
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return 0;
    void *p = nullptr;
    // the stream may still use the old buffer (iterations return before their
    // last kernel ends): let it finish before the buffer goes
    if (b.p && h && h->stream) (void)hipStreamSynchronize(h->stream);
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess)
        return set_err(h, LPC_E_NOMEM, "hipMalloc(" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
    if (keep && b.p && b.bytes) {
        HIPCHK(h, hipMemcpyAsync(p, b.p, b.bytes, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    if (b.p) (void)hipFree(b.p);
    b.p = p;
    b.bytes = bytes;
    return 0;
}

static void dfree(DBuf &b)
{
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

static int pop_reserve(lpc_handle *h, Pop &P, int64_t n)
{
    if (P.cap >= n && P.buf.p) return 0;
    int64_t cap = std::max<int64_t>(n, 1024);
    if (P.buf.p && h->stream) (void)hipStreamSynchronize(h->stream);   // see dalloc
    dfree(P.buf);
    RETIF(dalloc(h, P.buf, (size_t)cap * 8 * 4));
    P.cap = cap;
    return 0;
}

static inline unsigned grid1(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

// ---------------------------------------------------------------------------
// scene records: lpc_build.hpp builds them on the host (runs on host threads)
static void drop_piece_tables(lpc_handle *h)
{
    for (auto &kv : h->ptabs) { dfree(kv.second.pieces); dfree(kv.second.spieces); dfree(kv.second.groups); }
    h->ptabs.clear();
}

static int host_threads();
static void host_parts(int64_t n, int T, const std::function<void(int64_t, int64_t, int)> &fn);
static void host_pool_run(int n, const std::function<void(int)> &fn);
static void stage_drop(lpc_handle *h);

// Per mesh run: an 8-wide sphere hierarchy over its triangles in a top-down
// median-split order, every node's test node_record() of ALL triangles below it
// (so the slack does not compound from level to level); triangles whose sphere
// test is degenerate (slivers) or far wider than the triangle (thin) go to the
// run's line-filter list; triangles that can never be hit are dropped.  Results
// do not depend on the order (ties are resolved by triangle index).
static int host_vertices(lpc_handle *h);

static int build_records(lpc_handle *h)
{
    drop_piece_tables(h);   // pieces index the records built here
    if (!h->src_v[0]) RETIF(host_vertices(h));       // a rebuild after the upload: the rows from the device
    SceneBuildIn in;
    in.v0 = h->src_v[0]; in.v1 = h->src_v[1]; in.v2 = h->src_v[2];
    in.run_lo = h->run_lo.data(); in.run_hi = h->run_hi.data(); in.nr = h->run_lo.size();
    in.dcap = h->dcap; in.scene_scale = h->scene_scale; in.thin_k = kThin; in.stack_max = LPC_STACK;
    SceneBuildOut out;
    const double t0 = h->host_prof ? host_us() : 0.0;
    const std::string err = build_scene_records(in, out, [](int n, const std::function<void(int)> &fn) {
        host_pool_run(n, fn);
    });
    if (!err.empty()) return set_err(h, LPC_E_ARG, err);
    if (h->host_prof)
        fprintf(stderr, "[lpc host] scene records %.1f us (%zu nodes, %zu slivers, %d threads)\n", host_us() - t0,
                out.nodes.size(), out.slivers.size(), host_threads());
    h->run_levels.swap(out.run_levels);
    h->node_self.swap(out.node_self);
    h->run_slo.swap(out.run_slo);
    h->run_shi.swap(out.run_shi);
    h->n_slivers = out.n_slivers;
    h->n_thin = out.n_thin;
    // spare records so no buffer is empty
    if (out.nodes.empty()) { Node8 z; memset(&z, 0, sizeof(z)); out.nodes.push_back(z); }
    if (out.slivers.empty()) {
        SliverRec ss;
        memset(&ss, 0, sizeof(ss));
        ss.a = NAN; ss.idx = -1; ss.dmin = INFINITY;
        out.slivers.push_back(ss);
    }
    h->sliver_dmin_host.clear();
    for (const SliverRec &q : out.slivers) h->sliver_dmin_host.push_back(q.dmin);
    h->Mpad = (int32_t)out.nodes.size();
    // exact records in leaf order (a leaf's 8 records are 384 contiguous bytes:
    // the walk stages them into LDS with one LDS-DMA load), each with its
    // triangle index; 8 spare records at the end, so the last leaf's load stays
    // inside the buffer (round 6; by triangle index before, A/B neutral)
    // (k_exact_records from the rows on the device and the leaf order)
    const double tb0 = h->host_prof ? host_us() : 0.0;
    const size_t nx = out.xorder.size();
    RETIF(dalloc(h, h->d_xrec, (nx + 8) * sizeof(ExactRec)));
    RETIF(dalloc(h, h->d_tmp, std::max<size_t>(nx, 1) * 4));
    if (nx) HIPCHK(h, hipMemcpy(h->d_tmp.p, out.xorder.data(), nx * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemsetAsync((ExactRec *)h->d_xrec.p + nx, 0, 8 * sizeof(ExactRec), h->stream));
    if (nx) {
        const float4 *raw = (const float4 *)h->d_raw.p;
        hipLaunchKernelGGL(k_exact_records, dim3(grid1((int64_t)nx)), dim3(256), 0, h->stream, (int64_t)nx,
                           (const int32_t *)h->d_tmp.p, raw, raw + h->M, raw + 2 * (size_t)h->M,
                           (ExactRec *)h->d_xrec.p);
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));      // d_tmp is reused
    const double tb1 = h->host_prof ? host_us() : 0.0;
    RETIF(dalloc(h, h->d_nodes, out.nodes.size() * sizeof(Node8)));
    RETIF(dalloc(h, h->d_srec, out.slivers.size() * sizeof(SliverRec)));
    HIPCHK(h, hipMemcpy(h->d_nodes.p, out.nodes.data(), out.nodes.size() * sizeof(Node8), hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->d_srec.p, out.slivers.data(), out.slivers.size() * sizeof(SliverRec),
                        hipMemcpyHostToDevice));
    if (h->host_prof)
        fprintf(stderr, "[lpc host] records upload: exact records %.1f us, nodes %.1f us\n", tb1 - tb0, host_us() - tb1);
    return 0;
}

// Host copies of the scene's rows, from the device (a filter-record rebuild or
// the profiling fan flags after lpc_scene_upload returned).
static int host_vertices(lpc_handle *h)
{
    if (h->hv0.size() != 4 * (size_t)h->M) {
        std::vector<float> *hv[3] = {&h->hv0, &h->hv1, &h->hv2};
        for (int k = 0; k < 3; ++k) {
            hv[k]->resize(4 * (size_t)h->M);
            HIPCHK(h, hipMemcpy(hv[k]->data(), (const float *)h->d_raw.p + (size_t)k * 4 * h->M, (size_t)h->M * 16,
                                hipMemcpyDeviceToHost));
        }
    }
    for (int k = 0; k < 3; ++k) h->src_v[k] = (k == 0 ? h->hv0 : k == 1 ? h->hv1 : h->hv2).data();
    return 0;
}

// Piece table: hierarchy pieces = subtrees of the runs that own a slot (a run
// whose slot a later run overwrites is skipped, as its results are): all nodes
// of the shallowest level with >= g nodes (g = 1: the run roots; q_level picks
// g for a launch).  Sliver pieces = the runs' slivers in blocks of <= 64 (one
// lane each).
static int piece_table(lpc_handle *h, PieceTable **out, int32_t g)
{
    const size_t nr = h->run_levels.size();
    std::vector<int32_t> run_slot(nr, -1);
    for (int32_t j = 0; j < h->K; ++j)
        if (h->slot_run[(size_t)j] >= 0) run_slot[(size_t)h->slot_run[(size_t)j]] = j;
    // the level each live run is cut at: the shallowest with >= g nodes (many g
    // give the same cut, so a scene builds only a few tables)
    std::vector<int32_t> cut(nr, -1);
    for (size_t r = 0; r < nr; ++r) {
        if (run_slot[r] < 0) continue;
        const std::vector<int32_t> &L = h->run_levels[r];
        size_t lv = 0;
        while (lv + 1 < L.size() / 2 && L[2 * lv + 1] < g) ++lv;
        cut[r] = L.empty() ? -2 : (int32_t)lv;
    }
    auto it = h->ptabs.find(cut);
    if (it != h->ptabs.end()) { *out = &it->second; return 0; }
    std::vector<Piece> pcs, spc, grp;
    std::vector<float> sdm;
    for (size_t r = 0; r < nr; ++r) {
        if (run_slot[r] < 0) continue;
        const std::vector<int32_t> &L = h->run_levels[r];
        if (!L.empty()) {
            const size_t lv = (size_t)cut[r];
            Piece gp;                   // the run root's own test over the run's pieces
            memset(&gp, 0, sizeof(gp));
            gp.root = L[0];
            const FiltRec &gt = h->node_self[(size_t)gp.root];
            gp.cx = gt.cx; gp.cy = gt.cy; gp.cz = gt.cz; gp.negB = gt.negB; gp.negA = gt.negA;
            gp.slot = run_slot[r];
            gp.s_lo = (int32_t)pcs.size();
            gp.s_hi = gp.s_lo + L[2 * lv + 1];
            grp.push_back(gp);
            for (int32_t i = 0; i < L[2 * lv + 1]; ++i) {
                Piece p;
                memset(&p, 0, sizeof(p));
                p.root = L[2 * lv] + i;
                const FiltRec &t = h->node_self[(size_t)p.root];
                p.cx = t.cx; p.cy = t.cy; p.cz = t.cz; p.negB = t.negB; p.negA = t.negA;
                p.slot = run_slot[r];
                pcs.push_back(p);
            }
        }
        for (int32_t a = h->run_slo[r]; a < h->run_shi[r]; a += 64) {
            Piece p;
            memset(&p, 0, sizeof(p));
            p.root = -1;
            p.s_lo = a;
            p.s_hi = std::min(a + 64, h->run_shi[r]);
            p.slot = run_slot[r];
            spc.push_back(p);
            sdm.push_back(h->sliver_dmin_host[(size_t)a]);     // the run's slivers ascend in dmin
        }
    }
    if (pcs.size() > 65535 || spc.size() > 65535) return set_err(h, LPC_E_ARG, "too many triangle pieces");
    PieceTable &t = h->ptabs[cut];
    t.npieces = (int32_t)pcs.size();
    t.nspieces = (int32_t)spc.size();
    {   // sliver pieces in ascending dmin: a launch takes the prefix its rays can reach
        std::vector<size_t> o(spc.size());
        for (size_t i = 0; i < o.size(); ++i) o[i] = i;
        std::stable_sort(o.begin(), o.end(), [&](size_t x, size_t y) { return sdm[x] < sdm[y]; });
        std::vector<Piece> s2;
        t.sdmin.clear();
        for (size_t i : o) { s2.push_back(spc[i]); t.sdmin.push_back(sdm[i]); }
        spc.swap(s2);
    }
    if (!pcs.empty()) {
        RETIF(dalloc(h, t.pieces, pcs.size() * sizeof(Piece)));
        HIPCHK(h, hipMemcpy(t.pieces.p, pcs.data(), pcs.size() * sizeof(Piece), hipMemcpyHostToDevice));
    }
    if (!spc.empty()) {
        RETIF(dalloc(h, t.spieces, spc.size() * sizeof(Piece)));
        HIPCHK(h, hipMemcpy(t.spieces.p, spc.data(), spc.size() * sizeof(Piece), hipMemcpyHostToDevice));
    }
    // the gate pays when the runs are cut below their roots (<= 64 runs: one mask)
    t.ngroups = 0;
    if (grp.size() <= 64 && grp.size() < pcs.size()) {
        RETIF(dalloc(h, t.groups, grp.size() * sizeof(Piece)));
        HIPCHK(h, hipMemcpy(t.groups.p, grp.data(), grp.size() * sizeof(Piece), hipMemcpyHostToDevice));
        t.ngroups = (int32_t)grp.size();
    }
    *out = &t;
    return 0;
}

// Coherence sort: rocPRIM's default algorithm choice (block merge sort up to
// 1 Mi items, onesweep above) below onesweep_min rays, onesweep from there
// (RaySortOnesweep: 8-bit digit passes; forcing it at every size measured slower,
// 189 vs 131 us per 1 M-ray iteration incl. k_raykey/k_gather).
using RaySortCfg = rocprim::default_config;
using RaySortOnesweep = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                   rocprim::default_config, 0>;


// Rays per chunk.  Default: as many as ~32 GB of per-chunk workspace holds (slots
// 12 B per mesh + ~200 B of coherence copies, shade outputs and sort buffers per
// ray), at most 128 Mi: a chunk is also the unit of the coherence sort, and large
// populations (the eye's grow past 100 M rays) trace up to 1.5x faster in 128 Mi
// chunks than in 8 Mi ones.
static int64_t chunk_rays(const lpc_handle *h)
{
    if (h->chunk > 0) return h->chunk;
    const int64_t per_ray = (int64_t)12 * std::max(h->K, 1) + 200;
    const int64_t c = ((int64_t)32 << 30) / per_ray;
    return std::max<int64_t>((int64_t)1 << 20, std::min<int64_t>((int64_t)128 << 20, c));
}

// The largest population a device-sized iteration may hold: below the re-sort
// size (a device-sized iteration keeps its parents' order), one chunk, the
// root-item encoding's packet bound.  k_stage_move sizes the next iteration 0
// (it runs empty) when more children are kept, and the host re-runs it.
static int64_t ds_cap(const lpc_handle *h)
{
    return std::max<int64_t>(0, std::min<int64_t>({h->resort_min - 1, chunk_rays(h), (int64_t)LPC_Q_MAX_PACKETS * 64}));
}

// Workspace for a chunk of `n` rays.
static int ensure_ws(lpc_handle *h, int64_t n)
{
    if (n <= h->ws_rays) return 0;
    {
        const int64_t C = n;
        RETIF(dalloc(h, h->w_key, (size_t)h->K * C * 8));
        RETIF(dalloc(h, h->w_sc, (size_t)h->K * C * 4));
        RETIF(dalloc(h, h->w_rs, (size_t)8 * C * 4));
        RETIF(dalloc(h, h->w_pk, (size_t)((C + 127) / 128) * sizeof(PacketRec)));
        RETIF(dalloc(h, h->d_misc, LPC_MISC_WORDS * 4));
        RETIF(dalloc(h, h->w_shf, (size_t)kShadeF * C * 4));
        RETIF(dalloc(h, h->w_shi, (size_t)kShadeI * C * 4));
        const int64_t nb = (C + 1023) / 1024;
        RETIF(dalloc(h, h->w_blk_cnt, (size_t)3 * nb * 4));
        RETIF(dalloc(h, h->w_blk_off, (size_t)3 * nb * 8));
        RETIF(dalloc(h, h->w_blk_pow, (size_t)nb * 8));
        RETIF(dalloc(h, h->w_soa, (size_t)8 * C * 4));
        RETIF(dalloc(h, h->w_stage, (size_t)C * 16));
        RETIF(dalloc(h, h->w_aos, (size_t)C * 32));
        RETIF(dalloc(h, h->w_tm, (size_t)C * 4));
        RETIF(dalloc(h, h->w_tbox, (size_t)((C + LPC_ST_TILE - 1) / LPC_ST_TILE + 1) * 6 * 4));
        RETIF(dalloc(h, h->d_pbox, 6 * 4));
        HIPCHK(h, hipMemsetAsync(h->w_tm.p, 0, h->w_tm.bytes, h->stream));
        RETIF(dalloc(h, h->w_sort, (size_t)C * 16));    // keys in/out, values in/out
        RETIF(dalloc(h, h->w_bhist, ((size_t)LPC_BS_ND * ((C + LPC_BS_RPB - 1) / LPC_BS_RPB) + 2 * LPC_BS_ND + 8) * 4));
        size_t tb = 0;
        HIPCHK(h, rocprim::radix_sort_pairs<RaySortCfg>(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                                        (const int32_t *)nullptr, (int32_t *)nullptr, (size_t)C, 0,
                                                        32, h->stream));
        size_t tb1 = 0;
        HIPCHK(h, rocprim::radix_sort_pairs<RaySortOnesweep>(nullptr, tb1, (const uint32_t *)nullptr,
                                                             (uint32_t *)nullptr, (const int32_t *)nullptr,
                                                             (int32_t *)nullptr, (size_t)C, 0, 32, h->stream));
        tb = std::max(tb, tb1);
        RETIF(dalloc(h, h->w_sort_tmp, tb));
        const int64_t nt = (C + LPC_ST_TILE - 1) / LPC_ST_TILE;
        RETIF(dalloc(h, h->w_fc, (size_t)nt * (8 + 4 + 4 + 8 * LPC_MP_MAX) + 64));   // staging tiles' power, counts,
                                                                                      // max |dir|^2, measured power
        h->gcap = (nt + LPC_ST_GROUP - 1) / LPC_ST_GROUP + 1;                        // group counts, two launches'
        RETIF(dalloc(h, h->w_gsum, (size_t)2 * h->gcap * 8));
        HIPCHK(h, hipMemsetAsync(h->w_gsum.p, 0, h->w_gsum.bytes, h->stream));
        h->gpar = 0;
        h->gdirty[0] = h->gdirty[1] = 0;

        h->slots_clean = h->misc_clean = false;         // fresh slot arrays
        h->sort_tmp_bytes = tb;
        h->ws_rays = C;
    }
    return 0;
}

static ShadeOutPtrs shade_ptrs(lpc_handle *h, bool extra)
{
    const size_t C = (size_t)h->ws_rays;
    float *f = (float *)h->w_shf.p;
    int32_t *i = (int32_t *)h->w_shi.p;
    ShadeOutPtrs o;
    o.destx = f + 0 * C; o.desty = f + 1 * C; o.destz = f + 2 * C; o.pw = f + 3 * C;
    o.rdx = f + 4 * C; o.rdy = f + 5 * C; o.rdz = f + 6 * C; o.rpw = f + 7 * C;
    o.tdx = f + 8 * C; o.tdy = f + 9 * C; o.tdz = f + 10 * C; o.tpw = f + 11 * C;
    o.imid = i + 0 * C; o.meas = i + 1 * C; o.rms = i + 2 * C; o.tms = i + 3 * C;
    if (extra) { o.iidx = i + 4 * C; o.n1 = i + 5 * C; o.n2 = i + 6 * C; o.ent = i + 7 * C; }
    else { o.iidx = o.n1 = o.n2 = o.ent = nullptr; }
    return o;
}

static hipEvent_t ev_get(lpc_handle *h)
{
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, kEvTimingFlags) != hipSuccess) return nullptr;
    return e;
}

// Resolve recorded event pairs (after a stream sync).
static void prof_resolve(lpc_handle *h)
{
    // pairs whose end has not happened yet (a speculative iteration still queued)
    // stay for a later call
    auto drain = [&](std::vector<std::pair<hipEvent_t, hipEvent_t>> &v, double &acc) {
        size_t keep = 0;
        for (auto &pr : v) {
            if (hipEventQuery(pr.second) == hipErrorNotReady) { v[keep++] = pr; continue; }
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) acc += ms;
            h->ev_pool.push_back(pr.first);
            h->ev_pool.push_back(pr.second);
        }
        v.resize(keep);
    };
    drain(h->ev_isect, h->prof_isect_ms);
    drain(h->ev_kern, h->prof_kern_ms);
    drain(h->ev_rest, h->prof_rest_ms);
}

// Device-sized launch of a population whose size the previous iteration left in
// IterCtl (run_intersect / run_queue / run_spill_levels; NULL: host-sized).
struct DevSize {
    const long long *nd;        // population size (device)
    const unsigned *dm2;        // its max |D|^2 (float bits, device)
    int64_t pred;               // expected size: piece level, budgets, grids
    int64_t bound;              // capacity bound: workspaces, root-item shards
};

// Work hand-over (k_spill levels): queue, budget by population size.
static int spill_setup(lpc_handle *h, int64_t n, SpillArgs *SP)
{
    *SP = SpillArgs{nullptr, nullptr, 0u, 0, 31, h->tm_cur, nullptr};
    if (h->prof_stats) {                // diagnostic: the fan triangles (apex valence >= 32), built once
        if (!h->d_fan.p) {
            RETIF(host_vertices(h));
            std::map<std::array<uint32_t, 3>, int32_t> val;
            auto key = [&](const std::vector<float> &v, int32_t i) {
                std::array<uint32_t, 3> k;
                memcpy(k.data(), &v[4 * (size_t)i], 12);
                return k;
            };
            for (int32_t i = 0; i < h->M; ++i) { ++val[key(h->hv0, i)]; ++val[key(h->hv1, i)]; ++val[key(h->hv2, i)]; }
            std::vector<uint8_t> f((size_t)h->M, 0);
            for (int32_t i = 0; i < h->M; ++i)
                f[(size_t)i] = val[key(h->hv0, i)] >= 32 || val[key(h->hv1, i)] >= 32 || val[key(h->hv2, i)] >= 32;
            RETIF(dalloc(h, h->d_fan, (size_t)h->M));
            HIPCHK(h, hipMemcpy(h->d_fan.p, f.data(), (size_t)h->M, hipMemcpyHostToDevice));
        }
        SP->fan = (const uint8_t *)h->d_fan.p;
    }
    if (h->spill_budget <= 0) return 0;
    RETIF(dalloc(h, h->w_spill, (size_t)2 * h->spill_cap * sizeof(SpillItem)));
    SP->items = (SpillItem *)h->w_spill.p;
    SP->ctr = (uint32_t *)h->d_misc.p + LPC_MISC_SPILL;
    SP->cap = (uint32_t)std::min<int64_t>(h->spill_cap, 0x7fffffff);
    // no hand-over once a population fills the chip many times over (from
    // LPC_LARGE_PER_TRI rays per triangle)
    SP->budget = n >= h->spill_large_per_tri * (int64_t)h->M ? 0 : h->spill_budget;
    SP->pair_shift = kSpillPairShift;
    return 0;
}

// The rays of a launch as one base of 8 equally spaced arrays (RayBase): the
// coherence copy (stride n) or a population / staging buffer (stride = its
// capacity).  Every RaysIn the runtime builds has this shape.
static int ray_base(lpc_handle *h, const RaysIn &in, const float *rs, int64_t n, RayBase *out)
{
    if (rs) { *out = RayBase{rs, n}; return 0; }
    const int64_t st = in.oy - in.ox;
    if (in.oz - in.oy != st || in.dx - in.oz != st || in.dy - in.dx != st || in.dz - in.dy != st)
        return set_err(h, LPC_E_ARG, "internal: ray arrays not equally spaced");
    *out = RayBase{in.ox, st};
    return 0;
}

// hand-over levels of a launch of n rays (0: none)
static int spill_level_count(const lpc_handle *h, int64_t n, const SpillArgs &SP)
{
    const int lv = n >= kSpillSmallN ? kSpillLevels : kSpillLevelsSmall;
    return SP.budget > 0 ? std::max(1, std::min(lv, 7)) : 0;
}

// level l's input (queue l % 2, length misc[6 + l]) and output (level l + 1)
static void spill_level_args(lpc_handle *h, const SpillArgs &SP, int l, int levels, SpillArgs *I, SpillArgs *O)
{
    uint32_t *misc = (uint32_t *)h->d_misc.p;
    *I = SP; *O = SP;
    I->items = (SpillItem *)h->w_spill.p + (size_t)(l % 2) * (size_t)h->spill_cap;
    I->ctr = misc + LPC_MISC_SPILL + l;
    O->items = (SpillItem *)h->w_spill.p + (size_t)((l + 1) % 2) * (size_t)h->spill_cap;
    O->ctr = misc + LPC_MISC_SPILL + l + 1;
    O->budget = l + 1 < levels ? SP.budget : 0;
}

// hand-over levels: level l reads queue l % 2 (length misc[6 + l]) and queues
// what exceeds the budget for level l + 1; the last level finishes
static int run_spill_levels(lpc_handle *h, const RaysIn &in, const float *rs, int64_t n, const int32_t *perm,
                            float eps, float max_ray_len, unsigned long long *skey, int32_t *scnt,
                            unsigned long long *stats, const SpillArgs &SP, const long long *nd = nullptr)
{
    uint32_t *misc = (uint32_t *)h->d_misc.p;
    RayBase ray;
    RETIF(ray_base(h, in, rs, n, &ray));
    const int levels = spill_level_count(h, n, SP);
    for (int l = 0; l < levels; ++l) {
        SpillArgs I, O;
        spill_level_args(h, SP, l, levels, &I, &O);
        // later levels hold fewer items (and often none): smaller grids, in
        // 4-wave units, launched as single-wave blocks
        const unsigned g = (unsigned)std::max<int64_t>(kSpillMinBlocks, kSpillBlocks >> l) * 4u;
        // profiling counters only in the PROF instantiation (fewer live registers without)
        if (stats)
            hipLaunchKernelGGL((k_spill<8, true>), dim3(g), dim3(64), 0, h->stream, ray, n, perm,
                               (const Node8 *)h->d_nodes.p, (const ExactRec *)h->d_xrec.p, eps, max_ray_len, skey,
                               scnt, stats, I, O, nd);
        else
            hipLaunchKernelGGL((k_spill<8, false>), dim3(g), dim3(64), 0, h->stream, ray, n, perm,
                               (const Node8 *)h->d_nodes.p, (const ExactRec *)h->d_xrec.p, eps, max_ray_len, skey,
                               scnt, stats, I, O, nd);
    }
    HIPCHK(h, hipGetLastError());
    return 0;
}

// Piece level of the work queue: pieces per run so that (packets x pieces) root
// tests reach q_target (mesh run roots for large populations, finer pieces for
// small ones, whose few packets would otherwise be few items).
static int32_t q_level(const lpc_handle *h, int64_t n, bool chained)
{
    int64_t live_runs = 0;
    for (int32_t j = 0; j < h->K; ++j) live_runs += h->slot_run[(size_t)j] >= 0;
    live_runs = std::max<int64_t>(live_runs, 1);
    const int64_t npk = (n + 63) / 64;
    const int32_t g = (int32_t)std::min<int64_t>(4096, std::max<int64_t>(1, (kQTarget + npk * live_runs - 1) /
                                                                               (npk * live_runs)));
    return (g == 1 && chained && n <= kChainPiecesMax && live_runs < kChainPiecesRuns) ? kChainPieces : g;
}

// A device-side consistency check failed (QueueArgs::err / the compaction's
// prefix check, kept in DevAcc::qerr): the launch's results are incomplete.
// Clear the flag and report.  Never expected; the checks keep a sizing error from
// silently losing intersections.
static int q_failed(lpc_handle *h)
{
    (void)hipStreamSynchronize(h->stream);
    (void)hipMemset((char *)h->d_acc.p + offsetof(DevAcc, qerr), 0, sizeof(uint32_t));
    return set_err(h, LPC_E_HIP, "device-side consistency check failed (root-item capacity or compaction prefix): "
                                 "results incomplete");
}

static int check_qerr(lpc_handle *h)
{
    uint32_t e = 0;
    HIPCHK(h, hipMemcpy(&e, (char *)h->d_acc.p + offsetof(DevAcc, qerr), sizeof(e), hipMemcpyDeviceToHost));
    return e ? q_failed(h) : 0;
}

// The root-item queue of a launch of n rays: shard capacity, buffer, arguments.
// k_roots_s holds at most 64 LPC_ROOTS_TASKS pieces in LDS: a table with more
// (more than 1 024 live mesh runs, cut at their roots, no gate) is tested in
// batches of that many pieces, one k_roots_s launch each, into the same queue.
#define LPC_ROOTS_BATCH (64 * LPC_ROOTS_TASKS)
struct RootsBatch {
    int S, pb;
    int64_t blocks, vblocks;
};
static RootsBatch roots_batch(int64_t npk, const DevSize *ds, int32_t npieces)
{
    RootsBatch b;
    b.S = (int)((npieces + 63) / 64);           // S tasks per packet (npieces <= 64 S)
    b.pb = b.S >= 3 ? 1 : b.S == 2 ? 2 : kRootsPerBlock;   // pb packets per block
    b.blocks = (npk + b.pb - 1) / b.pb;
    b.vblocks = !ds ? b.blocks : (((ds->bound + 63) / 64) + b.pb - 1) / b.pb;
    return b;
}
struct QueueShape {
    int64_t npk, rs_blocks;
    int rs_S, rs_pb;
    int nbatch;                                 // k_roots_s launches (pieces in batches of LPC_ROOTS_BATCH)
};
static int queue_args(lpc_handle *h, int64_t n, const PieceTable *pt, const DevSize *ds, QueueArgs *Qo,
                      QueueShape *sh)
{
    // device-sized (ds): n is the expected size (grids), the bound sizes the shards
    const int64_t npk = (n + 63) / 64;
    const int nbatch = std::max(1, (int)((pt->npieces + LPC_ROOTS_BATCH - 1) / LPC_ROOTS_BATCH));
    if (nbatch > 1 && pt->ngroups > 0) return set_err(h, LPC_E_STATE, "internal: gated pieces in several batches");
    const RootsBatch b0 = roots_batch(npk, ds, std::min<int32_t>(pt->npieces, LPC_ROOTS_BATCH));
    // per shard: at most its blocks' packets x pieces items, summed over the batches
    // (k_roots_s / k_gather_roots flag an overflow through Q.err instead of dropping
    // items silently)
    int64_t rcap = 0;
    for (int k = 0; k < nbatch; ++k) {
        const int32_t np = std::min<int32_t>(pt->npieces - k * LPC_ROOTS_BATCH, LPC_ROOTS_BATCH);
        const RootsBatch b = roots_batch(npk, ds, np);
        rcap += ((b.vblocks + LPC_Q_CSHARDS - 1) / LPC_Q_CSHARDS) * b.pb * (int64_t)np;
    }
    const int rs_S = b0.S, rs_pb = b0.pb;
    const int64_t rs_blocks = b0.blocks;
    // k_gather_roots: 16 packets per block
    rcap = std::max<int64_t>(rcap, ((((npk + 15) / 16) + LPC_Q_CSHARDS - 1) / LPC_Q_CSHARDS) * 16 *
                                       (int64_t)pt->npieces);
    if (rcap >= 0xffffffffLL) return set_err(h, LPC_E_ARG, "root items: too many per shard");
    RETIF(dalloc(h, h->w_qroots, (size_t)LPC_Q_CSHARDS * (size_t)rcap * 8));
    QueueArgs Q;
    Q.roots = (uint64_t *)h->w_qroots.p;
    Q.ctl = (uint32_t *)h->d_misc.p;
    Q.err = (uint32_t *)((char *)h->d_acc.p + offsetof(DevAcc, qerr));
    Q.rcap = (uint32_t)rcap;
    *Qo = Q;
    sh->npk = npk; sh->rs_blocks = rs_blocks; sh->rs_S = rs_S; sh->rs_pb = rs_pb;
    sh->nbatch = nbatch;
    return 0;
}

// The hierarchy stage: k_roots_s writes the (packet, piece) items whose root test
// passes, k_rootwalk walks them grid-stride and hands heavy subtrees to the
// k_spill levels.  roots_done: k_gather_roots already wrote
// the items (same queue arguments).
static int run_queue(lpc_handle *h, const RaysIn &in, const float *rs, int64_t n, const int32_t *perm,
                     const PieceTable *pt, float eps, float max_ray_len, unsigned long long *skey, int32_t *scnt,
                     unsigned long long *stats, const DevSize *ds = nullptr, const SliverArgs *merged = nullptr,
                     bool roots_done = false)
{
    QueueArgs Q;
    QueueShape sh;
    RETIF(queue_args(h, n, pt, ds, &Q, &sh));
    if (h->host_prof)
        fprintf(stderr, "[lpc host] roots: n %lld packets %lld pieces %d groups %d S %d pb %d blocks %lld rcap %lld\n",
                (long long)n, (long long)sh.npk, (int)pt->npieces, (int)pt->ngroups, sh.rs_S, sh.rs_pb,
                (long long)sh.rs_blocks, (long long)Q.rcap);
    for (int k = 0; !roots_done && k < sh.nbatch; ++k) {
        const int32_t np = std::min<int32_t>(pt->npieces - k * LPC_ROOTS_BATCH, LPC_ROOTS_BATCH);
        const RootsBatch b = roots_batch(sh.npk, ds, np);
        const Piece *pc = (const Piece *)pt->pieces.p + (size_t)k * LPC_ROOTS_BATCH;
        const dim3 rg((unsigned)std::max<int64_t>(b.blocks, 1));
        if (h->half_roots)
            hipLaunchKernelGGL(k_roots_s<true>, rg, dim3(256), 0, h->stream, in, rs, n, pc, (int)np,
                               (const Piece *)pt->groups.p, (int)pt->ngroups, Q, b.S, b.pb, ds ? ds->nd : nullptr);
        else
            hipLaunchKernelGGL(k_roots_s<false>, rg, dim3(256), 0, h->stream, in, rs, n, pc, (int)np,
                               (const Piece *)pt->groups.p, (int)pt->ngroups, Q, b.S, b.pb, ds ? ds->nd : nullptr);
    }
    // merged sliver tests (LPC_SLIVER_MERGE): the packet bounds before the walk,
    // on this stream; the walk's waves take the (packet group, piece) units
    SliverArgs SA;
    memset(&SA, 0, sizeof(SA));
    if (merged) {
        SA = *merged;
        const int64_t npkx = (n + 127) / 128;
        hipLaunchKernelGGL(k_packet<2>, dim3((unsigned)((npkx + 3) / 4)), dim3(256), 0, h->stream, in, rs, n,
                           (PacketRec *)h->w_pk.p, ds ? ds->nd : nullptr);
    }
    RayBase ray;
    RETIF(ray_base(h, in, rs, n, &ray));
    SpillArgs SP;
    RETIF(spill_setup(h, n, &SP));
    const unsigned grid = (unsigned)h->walk_grid;      // single-wave blocks
    // profiling: the launch's own start/stop timestamps (hipExtLaunchKernel), no
    // event packets between the kernels
    hipEvent_t k0 = nullptr, k1 = nullptr;
    // light mode samples every prof_every-th launch: a launch with events costs
    // ~7 us more (bench A/B)
    h->prof_sampled = h->prof && (!h->prof_light || h->prof_seq++ % h->prof_every == 0);
    if (h->prof_sampled) { k0 = ev_get(h); k1 = ev_get(h); }
    // profiling counters only in the PROF instantiation, the merged sliver units
    // only in the MERGED one (fewer live registers without: the plain walk holds
    // 7 waves per SIMD, the merged one 6)
#define LPC_LAUNCH_WALK(PF, MG)                                                                                     \
    hipExtLaunchKernelGGL((k_rootwalk<8, PF, MG>), dim3(grid), dim3(64), 0, h->stream, k0, k1, 0, ray, n, perm,      \
                          (const Node8 *)h->d_nodes.p, (const ExactRec *)h->d_xrec.p, eps, max_ray_len, skey, scnt, \
                          stats, Q, SP, ds ? ds->nd : nullptr, SA)
    if (stats) {
        if (merged) LPC_LAUNCH_WALK(true, true);
        else LPC_LAUNCH_WALK(true, false);
    } else if (merged) {
        LPC_LAUNCH_WALK(false, true);
    } else {
        LPC_LAUNCH_WALK(false, false);
    }
#undef LPC_LAUNCH_WALK
    if (h->prof_sampled) h->ev_kern.push_back({k0, k1});
    RETIF(run_spill_levels(h, in, rs, n, perm, eps, max_ray_len, skey, scnt, stats, SP, ds ? ds->nd : nullptr));
    if (h->host_prof >= 2) {                          // diagnostic: this launch's hand-over queue lengths
        uint32_t q[8] = {0};
        HIPCHK(h, hipStreamSynchronize(h->stream));
        HIPCHK(h, hipMemcpy(q, (uint32_t *)h->d_misc.p + LPC_MISC_SPILL, sizeof(q), hipMemcpyDeviceToHost));
        fprintf(stderr, "[lpc host] hand-over: n %lld items per level %u %u %u %u\n", (long long)n, q[0], q[1], q[2],
                q[3]);
    }
    return 0;
}

// intersect for n rays of `in` into the slot arrays, and optionally into a
// caller's [ray][mesh] buffers (st_user != NULL, the reference's scratch layout).
// traced != NULL (trace iterations without per-ray exports): the launch works in
// its coherence order and *traced receives the rays in that order.
// ds != NULL (a speculative trace iteration, chained traced population): n is
// the bound, the kernels read the population size on the device and the
// launch shapes follow ds->pred.
// the side stream of the sliver kernels and its fork / join events, created on
// first use (a handle whose slivers run in the walk's grid holds one stream, so
// several handles in flight each keep a hardware queue of their own); false:
// all on the main stream
static bool side_stream(lpc_handle *h)
{
    if (!h->side_tried) {
        h->side_tried = true;
        const unsigned evf = hipEventDisableTiming;
        if (hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&h->ev_side[0], evf) != hipSuccess ||
            hipEventCreateWithFlags(&h->ev_side[1], evf) != hipSuccess) {
            (void)hipGetLastError();
            if (h->stream2) (void)hipStreamDestroy(h->stream2);
            for (hipEvent_t &e : h->ev_side)
                if (e) { (void)hipEventDestroy(e); e = nullptr; }
            h->stream2 = nullptr;
        }
    }
    return h->stream2 && h->ev_side[0] && h->ev_side[1];
}

static int run_intersect(lpc_handle *h, const RaysIn &in, int64_t n, float max_ray_len,
                         float *st_user, int32_t *si_user, int32_t *sc_user,
                         double dmax2 = INFINITY, RaysIn *traced = nullptr, const DevSize *ds = nullptr)
{
    RETIF(ensure_ws(h, n));
    const int64_t nb = n;                          // capacity
    if (ds) n = std::max<int64_t>(1, std::min(ds->pred, nb));   // launch shapes
    if ((nb + 63) / 64 > (int64_t)LPC_Q_MAX_PACKETS)
        return set_err(h, LPC_E_STATE, "internal: chunk above the root items' packet bound");
    // the pieces of the root items: q_level's cut (the same sliver pieces at every
    // cut), coarser while k_roots_s cannot hold them (tiny populations)
    PieceTable *pt;
    int32_t g = q_level(h, n, traced && h->pop_traced);
    RETIF(piece_table(h, &pt, g));
    // (a table of more than 1 024 run roots, g = 1, goes to k_roots_s in batches)
    while (pt->npieces > LPC_ROOTS_BATCH && g > 1) {
        g = std::max(1, g / 8);
        RETIF(piece_table(h, &pt, g));
    }
    const float eps = 0.000001f * max_ray_len;   // .cl:245, single-precision constant
    unsigned long long *skey = (unsigned long long *)h->w_key.p;
    int32_t *scnt = (int32_t *)h->w_sc.p;
    uint32_t *misc = (uint32_t *)h->d_misc.p;
    SlotInit SI;
    SI.K = h->K; SI.live = (const int32_t *)h->d_live.p; SI.max_ray_len = max_ray_len;
    SI.skey = skey; SI.scnt = scnt; SI.misc = misc;
    SI.acc = h->acc_pending ? (DevAcc *)h->d_acc.p : nullptr;
    SI.m_total = (unsigned long long)h->acc_pending_total;
    SI.uniform = 0;
    SI.tmask = nullptr;
    h->acc_pending = false;
    // traced mode: the children come out in their parents' traced order and need
    // no sort of their own
    const bool chained_pop = traced && h->pop_traced;
    // a chained population keeps its parents' order, except a large one
    // (LPC_RESORT_MIN): after many generations that order has lost its coherence
    const bool sorted = n >= kSortMin && (!chained_pop || (!ds && n >= h->resort_min));
    // the slot reset rides on k_raykey when it runs before everything that reads misc
    const bool fold_init = sorted && n >= LPC_MISC_WORDS;
    // Traced iterations (k_shade_stage) leave every slot they read in the clean
    // state (max_ray_len, idx -1, count 0), so once the whole slot array is clean
    // no slot needs a reset; only the launch words do (k_stage_move reset them for
    // the next launch; the emitted rays' k_raykey does).
    // LPC_HALF 3 (default): the half-line cull at the piece roots (k_roots_s items)
    // of a trace's chained populations; "emitted" = the trace's first population,
    // whatever the export mode; the drop-in kernels (lpc_intersect,
    // lpc_bounce_host: no trace population) are never culled.  0: off.
    h->half_roots = h->in_trace && h->half == 3 && !h->pop_emitted;
    const bool restore = traced != nullptr;
    const bool clean = restore && h->slots_clean && h->slots_mrl == max_ray_len;
    // written-slot masks: kept by every flush of this launch, read by its
    // k_shade_stage (restore path only; a mask bit may be stale, never missing:
    // the masks are cleared with the slots, and only the restore path reads them)
    h->tm_cur = (restore && h->K <= 32) ? (uint32_t *)h->w_tm.p : nullptr;
    const bool misc_clean = restore && h->misc_clean;
    h->slots_clean = h->misc_clean = false;
    SlotInit SIk = SI;
    SIk.skey = nullptr; SIk.misc = nullptr; SIk.acc = nullptr;
    if (restore && !clean) {            // the whole array to the clean state (stride-independent)
        SI.uniform = 1;
        SI.tmask = (uint32_t *)h->w_tm.p;
        const int64_t all = h->ws_rays;
        hipLaunchKernelGGL(k_slot_init, dim3(grid1(std::max<int64_t>(all, LPC_MISC_WORDS))), dim3(256), 0,
                           h->stream, all, SI);
    } else if (restore) {               // slots clean: the launch words only (k_stage_move writes all counters)
        SI.skey = nullptr;
        SI.acc = nullptr;
        if (fold_init) SIk = SI;
        else if (!misc_clean)
            hipLaunchKernelGGL(k_slot_init, dim3(grid1(LPC_MISC_WORDS)), dim3(256), 0, h->stream, (int64_t)0, SI);
    } else if (fold_init) {
        SIk = SI;
    } else {
        hipLaunchKernelGGL(k_slot_init, dim3(grid1(std::max<int64_t>(n, LPC_MISC_WORDS))), dim3(256), 0, h->stream,
                           n, SI);
    }
    const int32_t *perm = nullptr;
    const float *rs = nullptr;
    bool roots_done = false;                    // k_gather_roots wrote the root items
    if (sorted) {
        // coherence order: rays of one wave share origin cell and direction
        // (key [scene-box origin cell | direction], k_raykey), gathered from the
        // 32-byte rows k_raykey wrote
        const size_t C = (size_t)h->ws_rays;
        uint32_t *kin = (uint32_t *)h->w_sort.p, *kout = kin + C;
        int32_t *vin = (int32_t *)(kout + C), *vout = vin + C;
        // the emitted rays' varying key bits (set_rays)
        int b0 = 0, b1 = 32;
        if (traced && h->pop_emitted) { b0 = h->init_key_lo; b1 = h->init_key_hi; }
        const int nbits = b1 - b0;
        if (traced && h->pop_emitted && h->init_bsort && nbits >= 1 && nbits <= 16 && n >= LPC_MISC_WORDS) {
            // counting sort (MSD, two 8-bit digits, stable), then the gather
            const int hb = std::min(nbits, LPC_BS_HB), lb = nbits - hb;
            const int64_t nblk = (n + LPC_BS_RPB - 1) / LPC_BS_RPB;
            uint32_t *hist = (uint32_t *)h->w_bhist.p, *tot = hist + (size_t)LPC_BS_ND * nblk;
            uint32_t *bst = tot + LPC_BS_ND;
            hipLaunchKernelGGL(k_bkey, dim3((unsigned)nblk), dim3(LPC_BS_T), 0, h->stream, in, n, h->box_lo[0],
                               h->box_lo[1], h->box_lo[2], h->box_scale[0], h->box_scale[1], h->box_scale[2], kin,
                               (float4 *)h->w_aos.p, SIk, b0, lb, hb, hist, nblk);
            hipLaunchKernelGGL(k_bprefix, dim3(1u << hb), dim3(256), 0, h->stream, hist, nblk, tot);
            hipLaunchKernelGGL(k_bscatter, dim3((unsigned)nblk), dim3(LPC_BS_T), 0, h->stream, (const uint32_t *)kin,
                               n, b0, lb, hb, (const uint32_t *)hist, nblk, (const uint32_t *)tot, bst,
                               (uint8_t *)kout, vin, vout);
            if (lb > 0)
                hipLaunchKernelGGL(k_bsort2, dim3(1u << hb, LPC_BS_MAXB / LPC_BS_RPB), dim3(LPC_BS_T), 0, h->stream,
                                   (const uint8_t *)kout,
                                   (const int32_t *)vin, lb, (const uint32_t *)bst, vout);
        } else {
            // a re-sorted chained population: the key (5-D Morton) spans its own box
            // (k_stage_move of the iteration that made it), not the scene's
            const uint32_t *pbox = (traced && chained_pop && h->pbox_ok) ? (const uint32_t *)h->d_pbox.p : nullptr;
            hipLaunchKernelGGL(k_raykey, dim3(grid1(n)), dim3(256), 0, h->stream, in, n, h->box_lo[0], h->box_lo[1],
                               h->box_lo[2], h->box_scale[0], h->box_scale[1], h->box_scale[2], kin, vin,
                               (float4 *)h->w_aos.p, SIk, pbox, pbox ? kKeyObits : 5, pbox ? 1 : 0);
            size_t tb = h->sort_tmp_bytes;
            if (n >= kOnesweepMin)          // large populations: onesweep (one pass per 8 key bits)
                HIPCHK(h, rocprim::radix_sort_pairs<RaySortOnesweep>(h->w_sort_tmp.p, tb, kin, kout, vin, vout,
                                                                     (size_t)n, b0, b1, h->stream));
            else
                HIPCHK(h, rocprim::radix_sort_pairs<RaySortCfg>(h->w_sort_tmp.p, tb, kin, kout, vin, vout, (size_t)n,
                                                                b0, b1, h->stream));
        }
        perm = vout;
        // the gather with the root tests fused in (k_gather_roots), when the
        // launch has one root-test task per packet and no run gate
        if (!ds && pt->npieces > 0 && pt->npieces <= 64 && pt->ngroups == 0) {
            QueueArgs Qf;
            QueueShape shf;
            RETIF(queue_args(h, n, pt, nullptr, &Qf, &shf));
            const dim3 gg((unsigned)((n + 1023) / 1024));
            if (h->half_roots)
                hipLaunchKernelGGL(k_gather_roots<true>, gg, dim3(1024), 0, h->stream, (const float4 *)h->w_aos.p,
                                   n, perm, (float *)h->w_rs.p, traced ? 1 : 0, (const Piece *)pt->pieces.p,
                                   (int)pt->npieces, Qf);
            else
                hipLaunchKernelGGL(k_gather_roots<false>, gg, dim3(1024), 0, h->stream, (const float4 *)h->w_aos.p,
                                   n, perm, (float *)h->w_rs.p, traced ? 1 : 0, (const Piece *)pt->pieces.p,
                                   (int)pt->npieces, Qf);
            roots_done = true;
        } else {
            hipLaunchKernelGGL(k_gather_aos, dim3(grid1(n)), dim3(256), 0, h->stream, (const float4 *)h->w_aos.p, n,
                               perm, (float *)h->w_rs.p, traced ? 1 : 0);
        }
        rs = (const float *)h->w_rs.p;
    }
    if (traced) {
        // positions of the coherence order are the rays' indices from here on
        if (rs) {
            const float *f = rs;
            RaysIn t;
            t.ox = f; t.oy = f + n; t.oz = f + 2 * n; t.dx = f + 3 * n; t.dy = f + 4 * n; t.dz = f + 5 * n;
            t.pw = f + 6 * n; t.pmid = (const int32_t *)(f + 7 * n);
            *traced = t;
        } else {
            *traced = in;
        }
        perm = nullptr;
    }
    unsigned long long *stats = h->prof_stats ? (unsigned long long *)h->d_stats.p : nullptr;
    // sliver pieces the launch's rays can reach: dmin <= max |D| (sliver_dmin)
    if (!(dmax2 >= 0.0)) dmax2 = INFINITY;          // NaN bound (a NaN direction): no culling
    const float dmax = (float)std::min<double>(sqrt(dmax2 * (1.0 + 1e-5)), (double)INFINITY);
    int32_t nsp = 0;
    while (nsp < pt->nspieces && (ds || pt->sdmin[(size_t)nsp] <= dmax)) ++nsp;
    // device-sized: the population's max |D| read on the device (every sliver piece
    // in the grid, culled there)
    const unsigned *dm2_dev = ds ? ds->dm2 : nullptr;
    const long long *nd_dev = ds ? ds->nd : nullptr;
    // LPC_SLIVER_MERGE: from this population size (default 0: every size) the
    // sliver units run in the walk's own grid (k_rootwalk's tail) on this stream;
    // below, k_slivers runs beside the hierarchy stage on a second stream (both
    // only add to the slots with order-independent atomics; joined at the end),
    // launched after the hierarchy stage's kernels (the host reaches k_roots_s /
    // k_rootwalk sooner).  One stream per trace keeps several traces in flight
    // from interleaving fork / join events
    const bool merge_try = h->sliver_merge >= 0 && n >= h->sliver_merge && nsp > 0 && pt->npieces > 0;
    const bool side = !merge_try && nsp > 0 && side_stream(h);
    hipStream_t ss = h->stream;
    if (side) {
        ss = h->stream2;
        HIPCHK(h, hipEventRecord(h->ev_side[0], h->stream));
    }
    auto sliver_args = [&](int64_t ppw) {
        SliverArgs A;
        memset(&A, 0, sizeof(A));
        A.R = in; A.rs = rs; A.n = n; A.perm = perm; A.pk = (const PacketRec *)h->w_pk.p;
        A.srec = (const SliverRec *)h->d_srec.p; A.pieces = (const Piece *)pt->spieces.p; A.nsp = nsp;
        A.ppw = (int)ppw; A.eps = eps; A.max_ray_len = max_ray_len; A.dmax = dmax;
        A.skey = skey; A.scnt = scnt; A.stats = stats; A.nd = nd_dev; A.dm2d = dm2_dev; A.tmask = h->tm_cur;
        return A;
    };
    auto launch_slivers = [&]() -> int {
        if (side) HIPCHK(h, hipStreamWaitEvent(h->stream2, h->ev_side[0], 0));
        if (nsp > 0) {
            // packets per wave: enough (packet, piece) waves to fill the GPU, no more
            const int64_t npkx = (n + 127) / 128;
            const int64_t ppw = std::max<int64_t>(1, npkx * nsp / kSliverWaves);
            const dim3 sg((unsigned)((npkx + 4 * ppw - 1) / (4 * ppw)), (unsigned)nsp);
            hipLaunchKernelGGL(k_packet<2>, dim3((unsigned)((npkx + 3) / 4)), dim3(256), 0, ss, in, rs, n,
                               (PacketRec *)h->w_pk.p, nd_dev);
            hipLaunchKernelGGL(k_slivers, sg, dim3(256), 0, ss, sliver_args(ppw));
            HIPCHK(h, hipGetLastError());
        }
        if (side) HIPCHK(h, hipEventRecord(h->ev_side[1], h->stream2));
        return 0;
    };
    if (!side && !merge_try) RETIF(launch_slivers());       // no side stream: before the walk, this stream
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->prof && !h->prof_light) { e0 = ev_get(h); e1 = ev_get(h); (void)hipEventRecord(e0, h->stream); }
    h->prof_sampled = false;
    if (pt->npieces > 0) {
        const SliverArgs SAm = sliver_args(kSliverMergePpw);
        RETIF(run_queue(h, in, rs, n, perm, pt, eps, max_ray_len, skey, scnt, stats, ds, merge_try ? &SAm : nullptr,
                        roots_done));
    }
    if (h->prof) {      // the intersect stage: the walk (+ k_packet, k_slivers)
        if (!h->prof_light) {
            (void)hipEventRecord(e1, h->stream);
            h->ev_isect.push_back({e0, e1});
        }
        if (!h->prof_light || h->prof_sampled) {
            h->prof_launches += 1;
            h->prof_pairs += n * (int64_t)h->M;
        }
    }
    if (side) RETIF(launch_slivers());
    if (side) HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_side[1], 0));
    if (st_user) {
        hipLaunchKernelGGL(k_slot_export, dim3(grid1(n)), dim3(256), 0, h->stream, n, h->K,
                           (const int32_t *)h->d_live.p, (const unsigned long long *)skey,
                           (const int32_t *)scnt, st_user, si_user, sc_user, 1);
    }
    HIPCHK(h, hipGetLastError());
    return 0;
}

static ShadeArgs shade_args(lpc_handle *h, const RaysIn &in, const int32_t *meas_in, int64_t n, float max_ray_len,
                            float ior_env, bool extra)
{
    ShadeArgs A;
    A.in = in; A.meas_in = meas_in; A.n = n; A.K = h->K;
    A.skey = (const unsigned long long *)h->w_key.p; A.sc = (const int32_t *)h->w_sc.p;
    A.mat_type = (const int32_t *)h->d_mat.p; A.ior = (const float *)h->d_ior.p;
    A.refl = (const float *)h->d_refl.p; A.diss = (const float *)h->d_diss.p;
    A.verts = (const float *)h->d_verts.p;
    A.max_ray_len = max_ray_len; A.ior_env = ior_env;
    A.o = shade_ptrs(h, extra);
    return A;
}

static int run_shade(lpc_handle *h, const RaysIn &in, const int32_t *meas_in, int64_t n,
                     float max_ray_len, float ior_env, bool extra)
{
    ShadeArgs A;
    A.in = in; A.meas_in = meas_in; A.n = n; A.K = h->K;
    A.skey = (const unsigned long long *)h->w_key.p; A.sc = (const int32_t *)h->w_sc.p;
    A.mat_type = (const int32_t *)h->d_mat.p; A.ior = (const float *)h->d_ior.p;
    A.refl = (const float *)h->d_refl.p; A.diss = (const float *)h->d_diss.p;
    A.verts = (const float *)h->d_verts.p;
    A.max_ray_len = max_ray_len; A.ior_env = ior_env;
    A.o = shade_ptrs(h, extra);
    LPC_KU_LAUNCH(h, k_shade, dim3(grid1(n)), dim3(256), h->stream, A);
    HIPCHK(h, hipGetLastError());
    return 0;
}

// If |D| of any upcoming ray exceeds the filter's Dcap, rebuild the filter
// records without the tiny-triangle culling (Dcap = inf).
static int check_dcap(lpc_handle *h, double dmax2)
{
    if (dmax2 <= h->dcap * h->dcap * (1.0 - 1e-6)) return 0;
    h->dcap = INFINITY;
    h->dcap_rebuilt = true;
    return build_records(h);
}

extern "C" {

int lpc_abi_version(void) { return LPC_ABI_VERSION; }

int lpc_device_count(int *count)
{
    if (!count) return set_err(nullptr, LPC_E_ARG, "count is NULL");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return 0;
}

int lpc_device_query(int device, char *name, int name_len, char *arch, int arch_len, int *cu_count)
{
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || device < 0 || device >= c)
        return set_err(nullptr, LPC_E_ARG, "no HIP device " + std::to_string(device));
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return set_err(nullptr, LPC_E_HIP, "hipGetDeviceProperties");
    if (name && name_len > 0) { strncpy(name, p.name, (size_t)name_len - 1); name[name_len - 1] = 0; }
    if (arch && arch_len > 0) { strncpy(arch, p.gcnArchName, (size_t)arch_len - 1); arch[arch_len - 1] = 0; }
    if (cu_count) *cu_count = p.multiProcessorCount;
    return 0;
}

int lpc_open(int device, lpc_handle **out)
{
    if (!out) return set_err(nullptr, LPC_E_ARG, "out is NULL");
    *out = nullptr;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess || c == 0)
        return set_err(nullptr, LPC_E_HIP, std::string("no HIP device: ") + hipGetErrorString(e));
    if (device < 0 || device >= c)
        return set_err(nullptr, LPC_E_ARG, "device ordinal " + std::to_string(device) + " out of range");
    lpc_handle *h = new lpc_handle();
    h->device = device;
    e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete h;
        return set_err(nullptr, LPC_E_HIP, std::string("stream: ") + hipGetErrorString(e));
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        snprintf(h->name, sizeof(h->name), "%s (%s)", prop.name, prop.gcnArchName);
        h->cus = prop.multiProcessorCount;
    }
    int rc = dalloc(h, h->d_acc, sizeof(DevAcc));
    if (rc) { g_open_err = h->err; lpc_close(h); return rc; }
    rc = dalloc(h, h->d_mrun, LPC_MP_MAX * sizeof(double));
    if (rc) { g_open_err = h->err; lpc_close(h); return rc; }
    rc = dalloc(h, h->d_ctl, sizeof(IterCtl));
    if (rc) { g_open_err = h->err; lpc_close(h); return rc; }
    if (hipMemset(h->d_acc.p, 0, sizeof(DevAcc)) != hipSuccess ||   // counters start empty (qerr 0)
        hipMemset(h->d_ctl.p, 0, sizeof(IterCtl)) != hipSuccess) {
        g_open_err = "counter init";
        lpc_close(h);
        return LPC_E_HIP;
    }
    // size switches and test hooks (results do not depend on them; DESIGN.md
    // section 5): the tests drive the re-sort, the merged sliver units, the work
    // hand-over and its queue overflow, chunked iterations and a filter-record
    // rebuild inside a trace at small sizes
    auto env_int = [](const char *k, int64_t dflt) -> int64_t {
        const char *v = getenv(k);
        return (v && *v) ? strtoll(v, nullptr, 10) : dflt;
    };
    h->half = env_int("LPC_HALF", h->half) == 0 ? 0 : 3;
    h->chunk = std::max<int64_t>(0, env_int("LPC_CHUNK", h->chunk));
    h->resort_min = std::max<int64_t>(1, env_int("LPC_RESORT_MIN", h->resort_min));
    h->sliver_merge = env_int("LPC_SLIVER_MERGE", h->sliver_merge);
    h->walk_grid = std::min<int64_t>(std::max<int64_t>(env_int("LPC_WALK_GRID", h->walk_grid), 64), 1 << 22);
    h->spec = env_int("LPC_SPEC", h->spec) != 0;
    h->dcap_init = (double)env_int("LPC_DCAP_MILLI", 16000) / 1000.0;
    h->spill_budget = (int)env_int("LPC_BUDGET", h->spill_budget);
    h->spill_large_per_tri = env_int("LPC_LARGE_PER_TRI", h->spill_large_per_tri);
    h->spill_cap = std::max<int64_t>(env_int("LPC_SPILL_CAP", h->spill_cap), 64);
    h->host_prof = (int)env_int("LPC_HOSTPROF", 0);
    h->stage_mode = (int)std::min<int64_t>(2, std::max<int64_t>(0, env_int("LPC_STAGE_MODE", h->stage_mode)));
    if (hipHostMalloc((void **)&h->acc_map, kAccRing * sizeof(DevAcc), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void **)&h->acc_map_dev, h->acc_map, 0) != hipSuccess) {
        h->acc_map = h->acc_map_dev = nullptr;       // counters then come by copy + stream sync
    } else {
        memset(h->acc_map, 0, kAccRing * sizeof(DevAcc));
    }
    if (hipHostMalloc((void **)&h->acc_host, sizeof(DevAcc), hipHostMallocDefault) != hipSuccess) {
        g_open_err = "pinned host buffer";
        lpc_close(h);
        return LPC_E_HIP;
    }
    *out = h;
    return 0;
}

int lpc_close(lpc_handle *h)
{
    if (!h) return 0;
    (void)settle(h);                     // a trace still running (lpc_trace_iterate / _run_async)
    (void)hipSetDevice(h->device);
    stage_drop(h);
    for (auto &rs : h->rslot) {
        dfree(rs.P.buf); dfree(rs.aos); dfree(rs.scan);
        if (rs.pin) (void)hipHostFree(rs.pin);
        if (rs.scan_host) (void)hipHostFree(rs.scan_host);
        if (rs.ev) (void)hipEventDestroy(rs.ev);
    }
    if (h->ev_stage) (void)hipEventDestroy(h->ev_stage);
    if (h->cstream) (void)hipStreamDestroy(h->cstream);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    DBuf *bufs[] = {&h->d_raw, &h->d_nodes, &h->w_pk, &h->d_xrec, &h->d_verts, &h->d_mat, &h->d_ior, &h->d_refl,
                    &h->d_diss, &h->w_key, &h->w_sc, &h->w_rs, &h->d_live,
                    &h->w_shf, &h->w_shi, &h->w_blk_cnt, &h->w_blk_off, &h->w_blk_pow, &h->w_soa,
                    &h->w_stage, &h->w_sort, &h->w_sort_tmp, &h->w_bhist, &h->d_srec, &h->A.buf, &h->B.buf, &h->T.buf, &h->I.buf, &h->m_buf,
                    &h->d_acc, &h->d_tmp, &h->d_scan, &h->d_stats, &h->d_misc, &h->w_spill, &h->w_qroots,
                    &h->w_aos, &h->w_fc, &h->d_mrun, &h->w_gsum, &h->d_ctl, &h->d_cbase, &h->w_tbox, &h->d_pbox};
    for (DBuf *b : bufs) dfree(*b);
    if (h->acc_host) (void)hipHostFree(h->acc_host);
    h->acc_host = nullptr;
    if (h->acc_map) (void)hipHostFree(h->acc_map);
    h->acc_map = h->acc_map_dev = nullptr;
    for (auto &kv : h->ptabs) { dfree(kv.second.pieces); dfree(kv.second.spieces); dfree(kv.second.groups); }
    prof_resolve(h);
    for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
    if (h->stream2) { (void)hipStreamSynchronize(h->stream2); (void)hipStreamDestroy(h->stream2); }
    if (h->xstream) { (void)hipStreamSynchronize(h->xstream); (void)hipStreamDestroy(h->xstream); }
    for (int k = 0; k < 2; ++k) {
        if (h->ev_xready[k]) (void)hipEventDestroy(h->ev_xready[k]);
        if (h->ev_xdone[k]) (void)hipEventDestroy(h->ev_xdone[k]);
        dfree(h->xst[k]);
    }
    for (hipEvent_t e : h->ev_side) if (e) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return 0;
}

const char *lpc_last_error(const lpc_handle *h) { return h ? h->err.c_str() : g_open_err.c_str(); }

int lpc_device_info(lpc_handle *h, char *name, int name_len, int *cu_count)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (name && name_len > 0) { strncpy(name, h->name, (size_t)name_len - 1); name[name_len - 1] = 0; }
    if (cu_count) *cu_count = h->cus;
    return 0;
}

int lpc_scene_upload(lpc_handle *h, int32_t tri_count, const float *v0, const float *v1,
                     const float *v2, const int32_t *mesh_id, int32_t mesh_count,
                     const int32_t *mat_type, const float *ior, const float *refl,
                     const float *diss)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    if (tri_count <= 0 || mesh_count <= 0 || !v0 || !v1 || !v2 || !mesh_id || !mat_type || !ior ||
        !refl || !diss)
        return set_err(h, LPC_E_ARG, "scene needs >= 1 triangle, >= 1 mesh and all tables");
    // the walk's sparse exact-test pairs hold a triangle index in 26 bits (and root
    // items node ids in 28, LPC_Q_MAX_NODES)
    if (tri_count >= (1 << 26))
        return set_err(h, LPC_E_ARG, "scene has too many triangles (limit 2^26 - 1)");
    // the root items carry a mesh's scratch slot in 12 bits (q_item)
    if (mesh_count > LPC_Q_MAX_SLOTS + 1)
        return set_err(h, LPC_E_ARG, "scene has too many meshes (limit " + std::to_string(LPC_Q_MAX_SLOTS + 1) + ")");
    const double tu0 = h->host_prof ? host_us() : 0.0;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    ++h->scene_gen;                     // staged batches' scans keyed to the old box are redone when traced
    const int32_t M = tri_count, K = mesh_count;
    for (int32_t i = 0; i < M; ++i)
        if (mesh_id[i] < 0 || mesh_id[i] >= K)
            return set_err(h, LPC_E_ARG, "mesh_id[" + std::to_string(i) + "] out of range");
    h->M = M; h->K = K;
    dfree(h->d_fan);                                // profiling flags of the previous scene
    // the rows go to the device as they are (the vertex and exact records are
    // built there); the host reads the caller's arrays during this call and keeps
    // no copy (host_vertices fetches one for a later rebuild)
    h->hv0.clear(); h->hv1.clear(); h->hv2.clear();
    h->src_v[0] = v0; h->src_v[1] = v1; h->src_v[2] = v2;
    RETIF(dalloc(h, h->d_raw, (size_t)M * 48));
    for (int k = 0; k < 3; ++k)
        HIPCHK(h, hipMemcpyAsync((float *)h->d_raw.p + (size_t)k * 4 * M, k == 0 ? v0 : k == 1 ? v1 : v2,
                                 (size_t)M * 16, hipMemcpyHostToDevice, h->stream));
    // runs of equal mesh_id and the slot each one flushes into (.cl:260-265, 286)
    h->run_lo.clear(); h->run_hi.clear();
    for (int32_t i = 0; i < M; ++i) {
        if (i == 0 || mesh_id[i] != mesh_id[i - 1]) { h->run_lo.push_back(i); h->run_hi.push_back(i + 1); }
        else h->run_hi.back() = i + 1;
    }
    const size_t nr = h->run_lo.size();
    h->slot_run.assign((size_t)K, -1);
    for (size_t r = 0; r < nr; ++r) {
        int32_t slot = (r + 1 < nr) ? mesh_id[h->run_lo[r + 1]] - 1 : mesh_id[h->run_lo[r]];
        if (slot < 0)
            return set_err(h, LPC_E_ARG, "mesh_id sequence writes below slot 0 (reference would "
                                         "corrupt another ray's scratch); mesh ids must not decrease to 0");
        h->slot_run[slot] = (int32_t)r;   // a later run overwrites, as the sequential loop does
    }
    {
        std::vector<int32_t> live((size_t)K);
        for (int32_t j = 0; j < K; ++j) live[(size_t)j] = h->slot_run[(size_t)j] >= 0;
        RETIF(dalloc(h, h->d_live, (size_t)K * 4));
        HIPCHK(h, hipMemcpy(h->d_live.p, live.data(), (size_t)K * 4, hipMemcpyHostToDevice));
    }
    h->meas_meshes.clear();
    for (int32_t j = 0; j < K; ++j) if (mat_type[j] == 3) h->meas_meshes.push_back(j);
    // passive materials: the children of a ray never carry more power than it
    // (refractive: R, T = 1 - R in [0, 1] for finite positive indices,
    // .cl:313-326; mirror: P R with 0 <= R <= 1, .cl:443 -- a negative R flips the
    // sign, so a population's summed power could grow; dissipation only
    // attenuates, .cl:385-394)
    h->mat_passive = true;
    for (int32_t j = 0; j < K; ++j) {
        if ((mat_type[j] == 0 || mat_type[j] == 4) && !(ior[j] > 0.0f && std::isfinite(ior[j])))
            h->mat_passive = false;
        if (mat_type[j] == 1 && !(refl[j] >= 0.0f && refl[j] <= 1.0f)) h->mat_passive = false;
    }
    // vertices (the hit triangle's normal in the shading), from the rows on the device
    RETIF(dalloc(h, h->d_verts, (size_t)M * 36));
    {
        const float4 *raw = (const float4 *)h->d_raw.p;
        hipLaunchKernelGGL(k_vertex_rows, dim3(grid1(M)), dim3(256), 0, h->stream, (int64_t)M, raw, raw + M,
                           raw + 2 * (size_t)M, (float *)h->d_verts.p);
        HIPCHK(h, hipGetLastError());
    }
    {   // scene box for the ray coherence key
        float lo3[3] = {INFINITY, INFINITY, INFINITY}, hi3[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (const float *vs : {v0, v1, v2})
            for (int32_t i = 0; i < M; ++i)
                for (int k = 0; k < 3; ++k) {
                    const float v = vs[4 * (size_t)i + k];
                    if (std::isfinite(v)) { lo3[k] = std::min(lo3[k], v); hi3[k] = std::max(hi3[k], v); }
                }
        double diag2 = 0.0;
        for (int k = 0; k < 3; ++k) {
            const float ext = hi3[k] - lo3[k];
            h->box_lo[k] = std::isfinite(lo3[k]) ? lo3[k] : 0.0f;
            h->box_scale[k] = (std::isfinite(ext) && ext > 0.0f) ? 32.0f / ext : 1.0f;
            if (std::isfinite(ext)) diag2 += (double)ext * ext;
        }
        h->scene_scale = diag2 > 0.0 ? 0.5 * sqrt(diag2) : 1.0;
    }
    h->dcap = h->dcap_init;
    const double tu1 = h->host_prof ? host_us() : 0.0;
    const int brc = build_records(h);
    h->src_v[0] = h->src_v[1] = h->src_v[2] = nullptr;     // the caller's arrays are theirs again
    RETIF(brc);
    const double tu2 = h->host_prof ? host_us() : 0.0;
    RETIF(dalloc(h, h->d_mat, (size_t)K * 4));
    RETIF(dalloc(h, h->d_ior, (size_t)K * 4));
    RETIF(dalloc(h, h->d_refl, (size_t)K * 4));
    RETIF(dalloc(h, h->d_diss, (size_t)K * 4));
    HIPCHK(h, hipMemcpy(h->d_mat.p, mat_type, (size_t)K * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->d_ior.p, ior, (size_t)K * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->d_refl.p, refl, (size_t)K * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->d_diss.p, diss, (size_t)K * 4, hipMemcpyHostToDevice));
    h->ws_rays = 0;   // K may have changed
    h->traced_ready = false;
    if (h->host_prof)
        fprintf(stderr, "[lpc host] scene upload: tables %.1f us, records %.1f us, device copies %.1f us\n", tu1 - tu0,
                tu2 - tu1, host_us() - tu2);
    return 0;
}

// The process's host worker threads (host_threads() - 1 of them beside the
// caller), created at first use and kept: a thread start costs tens of us on
// the GPU boxes, which a scene upload or a ray pass would otherwise pay per call.
// One caller at a time; a concurrent caller (a staging helper thread) runs its
// tasks itself.
namespace {
class HostPool {
public:
    explicit HostPool(int workers)
    {
        for (int k = 0; k < workers; ++k) th_.emplace_back([this]() { loop(); });
    }
    ~HostPool()
    {
        { std::lock_guard<std::mutex> lk(m_); stop_ = true; }
        cv_.notify_all();
        for (std::thread &t : th_) t.join();
    }
    void run(int n, const std::function<void(int)> &fn)
    {
        std::unique_lock<std::mutex> busy(call_, std::try_to_lock);
        if (!busy.owns_lock() || th_.empty() || n <= 1) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &fn;
            n_ = n;
            next_.store(0);
            active_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        for (int i; (i = next_.fetch_add(1)) < n;) fn(i);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this]() { return active_ == 0; });
        job_ = nullptr;
    }

private:
    void loop()
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)> *job;
            int n;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&]() { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
                n = n_;
            }
            for (int i; (i = next_.fetch_add(1)) < n;) (*job)(i);
            std::lock_guard<std::mutex> lk(m_);
            if (--active_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_, call_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int n_ = 0, active_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
    std::atomic<int> next_{0};
};
}  // namespace

static void host_pool_run(int n, const std::function<void(int)> &fn)
{
    static HostPool pool(std::max(0, host_threads() - 1));
    pool.run(n, fn);
}

// Host passes over the caller's rays (set_rays, bounce_host) split over threads:
// fn(lo, hi, part) for T contiguous parts, results combined by the caller in
// part order (so every combine is deterministic).
static void host_parts(int64_t n, int T, const std::function<void(int64_t, int64_t, int)> &fn)
{
    if (T <= 1 || n < (1 << 16)) { fn(0, n, 0); return; }
    host_pool_run(T, [&](int t) { fn(n * t / T, n * (t + 1) / T, t); });
}

static int host_threads()
{
    static int t = [] {
        const char *v = getenv("LPC_HOST_THREADS");
        int k = v && *v ? atoi(v) : (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(k, 16));
    }();
    return t;
}

static double host_dmax2(int64_t n, const float *dir4)
{
    const int T = host_threads();
    std::vector<double> part((size_t)T, 0.0);
    host_parts(n, T, [&](int64_t lo, int64_t hi, int t) {
        double m = 0.0;
        for (int64_t i = lo; i < hi; ++i) {
            const float *d = dir4 + 4 * i;
            double q = (double)d[0] * d[0] + (double)d[1] * d[1] + (double)d[2] * d[2];
            if (!(q <= m)) m = q;   // NaN propagates as "large"
        }
        part[(size_t)t] = m;
    });
    double m = 0.0;
    for (double q : part)
        if (!(q <= m)) m = q;
    return m;
}

// Upload (n,4) host rows into SoA arrays of a population (rows 0..n): both row
// arrays into one staging buffer (the copies return once the host arrays are
// read), then the unpacks on the stream; `sync`: wait for them (the caller may
// reuse the staging buffer at once otherwise).
static int upload_rays(lpc_handle *h, Pop &P, int64_t n, const float *origin4, const float *dir4,
                       const float *pow, const int32_t *prev_mid, bool sync = true)
{
    RETIF(dalloc(h, h->w_stage, (size_t)n * 32));
    float4 *so = (float4 *)h->w_stage.p, *sd = so + n;
    HIPCHK(h, hipMemcpy(so, origin4, (size_t)n * 16, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(sd, dir4, (size_t)n * 16, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(P.f(6), pow, (size_t)n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_unpack4, dim3(grid1(n)), dim3(256), 0, h->stream, n, (const float4 *)so, P.f(0), P.f(1),
                       P.f(2));
    hipLaunchKernelGGL(k_unpack4, dim3(grid1(n)), dim3(256), 0, h->stream, n, (const float4 *)sd, P.f(3), P.f(4),
                       P.f(5));
    if (prev_mid) HIPCHK(h, hipMemcpy(P.pmid(), prev_mid, (size_t)n * 4, hipMemcpyHostToDevice));
    else                                        // just emitted (-2, iterative_tracer.py:118), filled on the device
        HIPCHK(h, hipMemsetD32Async((hipDeviceptr_t)P.pmid(), -2, (size_t)n, h->stream));
    HIPCHK(h, hipGetLastError());
    if (sync) HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

static int copy_pop(lpc_handle *h, Pop &dst, const Pop &src, int64_t n)
{
    for (int k = 0; k < 7; ++k)
        HIPCHK(h, hipMemcpyAsync(dst.f(k), src.f(k), (size_t)n * 4, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(dst.pmid(), src.pmid(), (size_t)n * 4, hipMemcpyDeviceToDevice, h->stream));
    return 0;
}

int lpc_bounce_host(lpc_handle *h, int64_t n, const float *origin4, const float *dir4,
                    float *pow, int32_t *meas, const int32_t *prev_mid, float max_ray_len,
                    float ior_env, float *dest4, int32_t *isect_mid, float *r_dir4, float *r_pow,
                    int32_t *r_meas, float *t_dir4, float *t_pow, int32_t *t_meas,
                    int32_t *n1_mid, int32_t *n2_mid, int32_t *entering, int32_t *isect_idx)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    if (!h->M) return set_err(h, LPC_E_STATE, "no scene uploaded");
    if (n < 0 || !origin4 || !dir4 || !pow || !meas || !prev_mid || !dest4 || !isect_mid ||
        !r_dir4 || !r_pow || !r_meas || !t_dir4 || !t_pow || !t_meas)
        return set_err(h, LPC_E_ARG, "bounce_host: missing buffer");
    if (n == 0) return 0;
    HIPCHK(h, hipSetDevice(h->device));
    const double bdmax2 = host_dmax2(n, dir4);
    RETIF(check_dcap(h, bdmax2));
    const int64_t C = std::min(n, chunk_rays(h));
    RETIF(ensure_ws(h, C));
    Pop P;
    RETIF(pop_reserve(h, P, C));
    DBuf dmeas;
    RETIF(dalloc(h, dmeas, (size_t)C * 4));
    int rc = 0;
    for (int64_t base = 0; base < n && !rc; base += C) {
        const int64_t nc = std::min(C, n - base);
        rc = upload_rays(h, P, nc, origin4 + 4 * base, dir4 + 4 * base, pow + base, prev_mid + base);
        if (rc) break;
        if (hipMemcpy(dmeas.p, meas + base, (size_t)nc * 4, hipMemcpyHostToDevice) != hipSuccess) { rc = set_err(h, LPC_E_HIP, "meas upload"); break; }
        rc = run_intersect(h, P.in(), nc, max_ray_len, nullptr, nullptr, nullptr, bdmax2);
        if (!rc) rc = run_shade(h, P.in(), (const int32_t *)dmeas.p, nc, max_ray_len, ior_env, true);
        if (rc) break;
        ShadeOutPtrs o = shade_ptrs(h, true);
        hipError_t e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) { rc = set_err(h, LPC_E_HIP, std::string("bounce: ") + hipGetErrorString(e)); break; }
        if ((rc = check_qerr(h)) != 0) break;
        auto d2h = [&](void *dst, const void *src, size_t bytes) {
            if (!rc && dst && hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) != hipSuccess)
                rc = set_err(h, LPC_E_HIP, "bounce: D2H");
        };
        auto pack = [&](float *dst4, const float *x, const float *y, const float *z) {
            hipLaunchKernelGGL(k_pack4, dim3(grid1(nc)), dim3(256), 0, h->stream, nc, x, y, z,
                               (float4 *)h->w_stage.p);
            if (hipStreamSynchronize(h->stream) != hipSuccess) { rc = set_err(h, LPC_E_HIP, "pack"); return; }
            d2h(dst4 + 4 * base, h->w_stage.p, (size_t)nc * 16);
        };
        RETIF(dalloc(h, h->w_stage, (size_t)nc * 16));
        pack(dest4, o.destx, o.desty, o.destz);
        pack(r_dir4, o.rdx, o.rdy, o.rdz);
        pack(t_dir4, o.tdx, o.tdy, o.tdz);
        d2h(pow + base, o.pw, (size_t)nc * 4);
        d2h(meas + base, o.meas, (size_t)nc * 4);
        d2h(isect_mid + base, o.imid, (size_t)nc * 4);
        d2h(r_pow + base, o.rpw, (size_t)nc * 4);
        d2h(r_meas + base, o.rms, (size_t)nc * 4);
        d2h(t_pow + base, o.tpw, (size_t)nc * 4);
        d2h(t_meas + base, o.tms, (size_t)nc * 4);
        if (n1_mid) d2h(n1_mid + base, o.n1, (size_t)nc * 4);
        if (n2_mid) d2h(n2_mid + base, o.n2, (size_t)nc * 4);
        if (entering) d2h(entering + base, o.ent, (size_t)nc * 4);
        if (isect_idx) d2h(isect_idx + base, o.iidx, (size_t)nc * 4);
    }
    dfree(P.buf);
    dfree(dmeas);
    if (h->prof) { (void)hipStreamSynchronize(h->stream); prof_resolve(h); }
    return rc;
}

// ---- reference-kernel drop-ins ------------------------------------------------
int lpc_intersect(lpc_handle *h, int64_t n, const float *dev_origin4, const float *dev_dir4,
                  float max_ray_len, float *dev_tmin, int32_t *dev_cnt, int32_t *dev_itmp)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    if (!h->M) return set_err(h, LPC_E_STATE, "no scene uploaded");
    if (n < 0 || !dev_origin4 || !dev_dir4 || !dev_tmin || !dev_cnt || !dev_itmp)
        return set_err(h, LPC_E_ARG, "intersect: missing buffer");
    if (n == 0) return 0;
    HIPCHK(h, hipSetDevice(h->device));
    const int64_t C = std::min(n, chunk_rays(h));
    RETIF(ensure_ws(h, C));
    float *s = (float *)h->w_soa.p;
    const size_t Cw = (size_t)h->ws_rays;
    for (int64_t base = 0; base < n; base += C) {
        const int64_t nc = std::min(C, n - base);
        hipLaunchKernelGGL(k_unpack4, dim3(grid1(nc)), dim3(256), 0, h->stream, nc,
                           (const float4 *)dev_origin4 + base, s, s + Cw, s + 2 * Cw);
        hipLaunchKernelGGL(k_unpack4, dim3(grid1(nc)), dim3(256), 0, h->stream, nc,
                           (const float4 *)dev_dir4 + base, s + 3 * Cw, s + 4 * Cw, s + 5 * Cw);
        RaysIn in;
        in.ox = s; in.oy = s + Cw; in.oz = s + 2 * Cw; in.dx = s + 3 * Cw; in.dy = s + 4 * Cw;
        in.dz = s + 5 * Cw; in.pw = nullptr; in.pmid = nullptr;
        RETIF(run_intersect(h, in, nc, max_ray_len, dev_tmin + base * h->K, dev_itmp + base * h->K,
                            dev_cnt + base * h->K));
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    RETIF(check_qerr(h));
    if (h->prof) prof_resolve(h);
    return 0;
}

int lpc_intersect_postproc(lpc_handle *h, int64_t n, const float *dev_origin4,
                           const float *dev_dir4, float *dev_dest4, const int32_t *dev_prev_mid,
                           int32_t *dev_n1_mid, int32_t *dev_n2_mid, int32_t *dev_entering,
                           int32_t *dev_isect_mid, int32_t *dev_isect_idx,
                           const float *dev_tmin, const int32_t *dev_cnt,
                           const int32_t *dev_itmp, float max_ray_len)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    if (!h->M) return set_err(h, LPC_E_STATE, "no scene uploaded");
    if (n < 0 || !dev_origin4 || !dev_dir4 || !dev_dest4 || !dev_prev_mid || !dev_n1_mid ||
        !dev_n2_mid || !dev_entering || !dev_isect_mid || !dev_isect_idx || !dev_tmin ||
        !dev_cnt || !dev_itmp)
        return set_err(h, LPC_E_ARG, "intersect_postproc: missing buffer");
    if (n == 0) return 0;
    HIPCHK(h, hipSetDevice(h->device));
    PostprocAosArgs A;
    A.n = n; A.K = h->K;
    A.origin = (const float4 *)dev_origin4; A.dir = (const float4 *)dev_dir4;
    A.dest = (float4 *)dev_dest4; A.prev_mid = dev_prev_mid;
    A.n1 = dev_n1_mid; A.n2 = dev_n2_mid; A.entering = dev_entering;
    A.imid = dev_isect_mid; A.iidx = dev_isect_idx;
    A.tmin = dev_tmin; A.cnt = dev_cnt; A.itmp = dev_itmp;
    A.mat_type = (const int32_t *)h->d_mat.p; A.max_ray_len = max_ray_len;
    hipLaunchKernelGGL(k_postproc_aos, dim3(grid1(n)), dim3(256), 0, h->stream, A);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lpc_reflect_refract_rays(lpc_handle *h, int64_t n, const float *dev_origin4,
                             const float *dev_dest4, const float *dev_dir4, float *dev_pow,
                             int32_t *dev_meas, const int32_t *dev_n1_mid,
                             const int32_t *dev_n2_mid, float *dev_r_origin4, float *dev_r_dir4,
                             float *dev_r_pow, int32_t *dev_r_meas, float *dev_t_origin4,
                             float *dev_t_dir4, float *dev_t_pow, int32_t *dev_t_meas,
                             const int32_t *dev_isect_mid, const int32_t *dev_isect_idx,
                             float ior_env)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    if (!h->M) return set_err(h, LPC_E_STATE, "no scene uploaded");
    if (n < 0 || !dev_origin4 || !dev_dest4 || !dev_dir4 || !dev_pow || !dev_meas ||
        !dev_n1_mid || !dev_n2_mid || !dev_r_origin4 || !dev_r_dir4 || !dev_r_pow ||
        !dev_r_meas || !dev_t_origin4 || !dev_t_dir4 || !dev_t_pow || !dev_t_meas ||
        !dev_isect_mid || !dev_isect_idx)
        return set_err(h, LPC_E_ARG, "reflect_refract_rays: missing buffer");
    if (n == 0) return 0;
    HIPCHK(h, hipSetDevice(h->device));
    FresnelAosArgs A;
    A.n = n;
    A.origin = (const float4 *)dev_origin4; A.dest = (const float4 *)dev_dest4;
    A.dir = (const float4 *)dev_dir4; A.pow = dev_pow; A.meas = dev_meas;
    A.n1 = dev_n1_mid; A.n2 = dev_n2_mid; A.imid = dev_isect_mid; A.iidx = dev_isect_idx;
    A.r_origin = (float4 *)dev_r_origin4; A.r_dir = (float4 *)dev_r_dir4;
    A.t_origin = (float4 *)dev_t_origin4; A.t_dir = (float4 *)dev_t_dir4;
    A.r_pow = dev_r_pow; A.t_pow = dev_t_pow; A.r_meas = dev_r_meas; A.t_meas = dev_t_meas;
    A.mat_type = (const int32_t *)h->d_mat.p; A.ior = (const float *)h->d_ior.p;
    A.refl = (const float *)h->d_refl.p; A.diss = (const float *)h->d_diss.p;
    A.verts = (const float *)h->d_verts.p; A.ior_env = ior_env;
    hipLaunchKernelGGL(k_fresnel_aos, dim3(grid1(n)), dim3(256), 0, h->stream, A);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

// ---- device-resident trace ------------------------------------------------------
int lpc_set_walk_grid(lpc_handle *h, int64_t blocks)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (blocks != 0 && (blocks < 64 || blocks > (1 << 22))) return set_err(h, LPC_E_ARG, "walk grid out of range");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    h->walk_grid = blocks ? blocks : kWalkWaves;
    return 0;
}

int lpc_set_chunk(lpc_handle *h, int64_t rays_per_chunk)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (rays_per_chunk < 0) return set_err(h, LPC_E_ARG, "negative chunk");
    h->chunk = rays_per_chunk;
    return 0;
}

static int reset_measured(lpc_handle *h)
{
    h->m_total = 0;
    DevAcc z;
    memset(&z, 0, sizeof(z));
    HIPCHK(h, hipMemcpy(h->d_acc.p, &z, sizeof(z), hipMemcpyHostToDevice));
    return 0;
}

// May the emitted rays' coherence sort be the counting sort (k_bkey..k_bsort2)?
// Its second level runs one block per hi bucket, so it pays only when no bucket
// is large: the hi-digit counts of k_raykey's key that k_ray_scan counted for
// the key window in use.  A collimated beam's few origin cells, or a narrow
// cone's few direction cells, go to rocPRIM (the sort is exact either way).
static bool bsort_fits(const lpc_handle *h, int64_t n, const RayScan &S)
{
    const int nbits = h->init_key_hi - h->init_key_lo;
    if (nbits < 1 || nbits > 16 || n < LPC_MISC_WORDS) return false;
    const int hb = std::min(nbits, LPC_BS_HB), lb = nbits - hb;
    if (lb == 0) return true;                              // one level: no per-bucket pass
    const int w = h->init_key_lo + lb == 8 ? 0 : h->init_key_lo + lb == 23 ? 1 : -1;
    if (w < 0 || hb != 8) return false;                   // windows k_ray_scan did not count
    uint32_t mx = 0;
    for (int b = 0; b < 256; ++b) mx = std::max(mx, S.hist[w][b]);
    return mx <= (uint32_t)LPC_BS_MAXB;
}

static int emitted_rays(lpc_handle *h, int64_t n, const RayScan &S, float max_ray_len, float ior_env);

int lpc_trace_set_rays(lpc_handle *h, int64_t n, const float *origin4, const float *dir4,
                       const float *pow, float max_ray_len, float ior_env)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    if (!h->M) return set_err(h, LPC_E_STATE, "no scene uploaded");
    if (n < 0 || (n > 0 && (!origin4 || !dir4 || !pow))) return set_err(h, LPC_E_ARG, "set_rays: missing buffer");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    RETIF(pop_reserve(h, h->I, std::max<int64_t>(n, 1)));
    // the rays, then their analysis on the device (k_ray_scan, one 2 KB read-back)
    RayScan S;
    memset(&S, 0, sizeof(S));
    if (n > 0) {
        RETIF(upload_rays(h, h->I, n, origin4, dir4, pow, nullptr, false));
        RETIF(dalloc(h, h->d_scan, sizeof(RayScan)));
        HIPCHK(h, hipMemsetAsync(h->d_scan.p, 0, sizeof(RayScan), h->stream));
        hipLaunchKernelGGL(k_ray_scan, dim3((unsigned)std::min<int64_t>(grid1(n), 2048)), dim3(256), 0, h->stream,
                           h->I.in(), n, h->box_lo[0], h->box_lo[1], h->box_lo[2], h->box_scale[0], h->box_scale[1],
                           h->box_scale[2], (RayScan *)h->d_scan.p);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipMemcpyAsync(&S, h->d_scan.p, sizeof(RayScan), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    return emitted_rays(h, n, S, max_ray_len, ior_env);
}

// The emitted rays' analysis (k_ray_scan) into the trace state, as the rays in
// I: lpc_trace_set_rays and a staged batch that becomes current.
static int emitted_rays(lpc_handle *h, int64_t n, const RayScan &S, float max_ray_len, float ior_env)
{
    memcpy(&h->init_dmax2, &S.dmax2_bits, sizeof(double));
    h->pow_nonneg = S.neg_pow == 0u;
    // coherence key bits that can vary over these rays (k_raykey: [origin cell 15 |
    // direction 16]): a point source has one origin cell, a collimated beam one
    // direction, and the sort skips the rest
    const bool same_o = S.diff_o == 0u, same_d = S.diff_d == 0u;
    h->init_key_lo = 0;
    h->init_key_hi = 31;
    if (same_o) h->init_key_hi = 16;
    if (same_d) h->init_key_lo = 16;
    if (same_o && same_d) { h->init_key_lo = 0; h->init_key_hi = 8; }   // one digit pass
    h->init_bsort = bsort_fits(h, n, S);
    RETIF(check_dcap(h, h->init_dmax2));
    h->n_init = n;
    h->max_ray_len = max_ray_len;
    h->ior_env = ior_env;
    h->traced_ready = true;
    return lpc_trace_reset(h);
}

int lpc_trace_reset(lpc_handle *h)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (!h->traced_ready) return set_err(h, LPC_E_STATE, "trace_reset before trace_set_rays");
    HIPCHK(h, hipSetDevice(h->device));
    // the first iteration reads the emitted rays where set_rays put them (I is
    // never written by an iteration: no copy)
    h->pop_init = true;
    h->mp_valid = true;                             // until an iteration does not sum it
    h->n_cur = h->n_init;
    h->pop_traced = false;
    h->pop_emitted = true;
    h->pop_dmax2 = h->init_dmax2;
    h->pbox_ok = false;
    h->m_total = 0;                             // measured record emptied (the first iteration resets the counters)
    h->m_inflight = 0;
    return 0;
}

// ---- streamed batches of new rays ------------------------------------------
// A staged batch is copied by a helper thread: the caller's (n,4) rows
// transposed into the slot's pinned staging as the population's SoA arrays (a
// few host threads, chunk by chunk, each chunk's DMAs queued as soon as it is
// ready: 28 B per ray cross PCIe), the emitted rays' fills and k_ray_scan, all on
// the copy stream, which first
// waits for the main-stream work queued when the batch was staged (the slot's
// buffers may hold an earlier batch's emitted rays).  The main thread meanwhile
// traces the batch before it.
static void stage_worker(lpc_handle *h, lpc_handle::RaySlot *s, const float *origin4, const float *dir4,
                         const float *pow, const float box_lo[3], const float box_scale[3], bool scan)
{
    auto fail = [&](hipError_t e, const char *what) {
        s->rc = LPC_E_HIP;
        s->err = std::string("stage_rays: ") + what + ": " + hipGetErrorString(e);
    };
    const double t0 = h->host_prof ? host_us() : 0.0;
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) { fail(e, "hipSetDevice"); return; }
    const int64_t n = s->n;
    hipStream_t cs = h->cstream;
    const int mode = h->stage_mode;
    if (mode == 2) {
        // chunks: the host transposes chunk c + 1 into the pinned SoA arrays while
        // the DMAs of chunk c run (28 B per ray cross PCIe)
        float *pin = (float *)s->pin;
        const int64_t CH = (int64_t)1 << 18;
        const int T = std::max(1, std::min(4, host_threads()));
        for (int64_t lo = 0; lo < n; lo += CH) {
            const int64_t hi = std::min(n, lo + CH);
            host_parts(hi - lo, T, [&](int64_t a, int64_t b, int) {
                for (int64_t i = lo + a; i < lo + b; ++i) {
                    const float *o = origin4 + 4 * i, *d = dir4 + 4 * i;
                    pin[i] = o[0]; pin[n + i] = o[1]; pin[2 * n + i] = o[2];
                    pin[3 * n + i] = d[0]; pin[4 * n + i] = d[1]; pin[5 * n + i] = d[2];
                }
                memcpy(pin + 6 * n + lo + a, pow + lo + a, (size_t)(b - a) * 4);
            });
            for (int k = 0; k < 7; ++k)
                if ((e = hipMemcpyAsync(s->P.f(k) + lo, pin + (size_t)k * n + lo, (size_t)(hi - lo) * 4,
                                        hipMemcpyHostToDevice, cs)) != hipSuccess) {
                    fail(e, "copy");
                    return;
                }
        }
    } else {
        // the (n,4) rows as they are: from the caller's memory (mode 0: the
        // runtime's own staging of a pageable copy) or through the slot's pinned
        // block (mode 1: host threads copy, one DMA), unpacked on the device
        float4 *so = (float4 *)s->aos.p, *sd = so + n;
        const char *src_o = (const char *)origin4, *src_d = (const char *)dir4, *src_p = (const char *)pow;
        if (mode == 1) {
            char *pin = (char *)s->pin;
            host_parts(n, host_threads(), [&](int64_t lo, int64_t hi, int) {
                memcpy(pin + (size_t)lo * 16, origin4 + 4 * lo, (size_t)(hi - lo) * 16);
                memcpy(pin + (size_t)n * 16 + (size_t)lo * 16, dir4 + 4 * lo, (size_t)(hi - lo) * 16);
                memcpy(pin + (size_t)n * 32 + (size_t)lo * 4, pow + lo, (size_t)(hi - lo) * 4);
            });
            src_o = pin; src_d = pin + (size_t)n * 16; src_p = pin + (size_t)n * 32;
        }
        if ((e = hipMemcpyAsync(so, src_o, (size_t)n * 16, hipMemcpyHostToDevice, cs)) != hipSuccess ||
            (e = hipMemcpyAsync(sd, src_d, (size_t)n * 16, hipMemcpyHostToDevice, cs)) != hipSuccess ||
            (e = hipMemcpyAsync(s->P.f(6), src_p, (size_t)n * 4, hipMemcpyHostToDevice, cs)) != hipSuccess) {
            fail(e, "copy");
            return;
        }
        hipLaunchKernelGGL(k_unpack4, dim3(grid1(n)), dim3(256), 0, cs, n, (const float4 *)so, s->P.f(0), s->P.f(1),
                           s->P.f(2));
        hipLaunchKernelGGL(k_unpack4, dim3(grid1(n)), dim3(256), 0, cs, n, (const float4 *)sd, s->P.f(3), s->P.f(4),
                           s->P.f(5));
    }
    if ((e = hipMemsetD32Async((hipDeviceptr_t)s->P.pmid(), -2, (size_t)n, cs)) != hipSuccess) { fail(e, "fill"); return; }
    if (scan) {                                     // the scene's key box is known: the analysis rides along
        if ((e = hipMemsetAsync(s->scan.p, 0, sizeof(RayScan), cs)) != hipSuccess) { fail(e, "fill"); return; }
        hipLaunchKernelGGL(k_ray_scan, dim3((unsigned)std::min<int64_t>(grid1(n), 2048)), dim3(256), 0, cs, s->P.in(),
                           n, box_lo[0], box_lo[1], box_lo[2], box_scale[0], box_scale[1], box_scale[2],
                           (RayScan *)s->scan.p);
        if ((e = hipGetLastError()) != hipSuccess) { fail(e, "launch"); return; }
        if ((e = hipMemcpyAsync(s->scan_host, s->scan.p, sizeof(RayScan), hipMemcpyDeviceToHost, cs)) != hipSuccess) {
            fail(e, "copy");
            return;
        }
    }
    if ((e = hipEventRecord(s->ev, cs)) != hipSuccess) fail(e, "event");
    if (h->host_prof) {
        const double t1 = host_us();
        (void)hipEventSynchronize(s->ev);
        fprintf(stderr, "[lpc host] stage mode %d: %lld rays, enqueued %.1f us, done %.1f us\n", mode, (long long)n,
                t1 - t0, host_us() - t0);
    }
}

// Join the helpers and forget the staged batches (lpc_close).
static void stage_drop(lpc_handle *h)
{
    for (auto &s : h->rslot)
        if (s.th.joinable()) s.th.join();
    h->rs_count = 0;
    if (h->cstream) (void)hipStreamSynchronize(h->cstream);
}

int lpc_trace_stage_rays(lpc_handle *h, int64_t n, const float *origin4, const float *dir4, const float *pow,
                         float max_ray_len, float ior_env)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (n <= 0 || !origin4 || !dir4 || !pow) return set_err(h, LPC_E_ARG, "stage_rays: need n > 0 rays and all buffers");
    if (h->rs_count >= 2) return set_err(h, LPC_E_STATE, "stage_rays: two batches are staged already");
    HIPCHK(h, hipSetDevice(h->device));
    if (!h->cstream) {
        HIPCHK(h, hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking));
        HIPCHK(h, hipEventCreateWithFlags(&h->ev_stage, hipEventDisableTiming));
    }
    lpc_handle::RaySlot &s = h->rslot[(h->rs_head + h->rs_count) % 2];
    if (s.th.joinable()) s.th.join();
    if (!s.ev) HIPCHK(h, hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
    if (!s.scan_host) HIPCHK(h, hipHostMalloc((void **)&s.scan_host, sizeof(RayScan), hipHostMallocDefault));
    // buffers (allocations synchronise; they grow only with the batch size)
    RETIF(pop_reserve(h, s.P, n));
    RETIF(dalloc(h, s.scan, sizeof(RayScan)));
    if (h->stage_mode != 2) RETIF(dalloc(h, s.aos, (size_t)n * 32));
    const size_t pb = (size_t)n * (h->stage_mode == 2 ? 28 : 36);
    if (h->stage_mode != 0 && s.pin_bytes < pb) {
        if (s.pin) { (void)hipStreamSynchronize(h->cstream); (void)hipHostFree(s.pin); s.pin = nullptr; s.pin_bytes = 0; }
        HIPCHK(h, hipHostMalloc(&s.pin, pb, hipHostMallocDefault));
        s.pin_bytes = pb;
    }
    s.n = n;
    s.max_ray_len = max_ray_len;
    s.ior_env = ior_env;
    s.rc = 0;
    s.err.clear();
    s.scan_gen = h->M ? h->scene_gen : -1;      // no scene yet: the scan runs when the batch is traced
    // the slot's device buffers may hold an earlier batch's emitted rays: the copy
    // stream starts after the main-stream work queued so far
    HIPCHK(h, hipEventRecord(h->ev_stage, h->stream));
    HIPCHK(h, hipStreamWaitEvent(h->cstream, h->ev_stage, 0));
    const float lo[3] = {h->box_lo[0], h->box_lo[1], h->box_lo[2]};
    const float sc[3] = {h->box_scale[0], h->box_scale[1], h->box_scale[2]};
    s.th = std::thread(stage_worker, h, &s, origin4, dir4, pow, lo, sc, s.scan_gen >= 0);
    ++h->rs_count;
    return 0;
}

static int trace_run(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                     int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap,
                     bool wait);

int lpc_trace_run_staged_async(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                               int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (!h->rs_count) return set_err(h, LPC_E_STATE, "run_staged: no batch staged (lpc_trace_stage_rays)");
    if (!h->M) return set_err(h, LPC_E_STATE, "no scene uploaded");
    if (mesh_power && mesh_power_cap < h->K)
        return set_err(h, LPC_E_ARG, "trace: mesh_power capacity below the scene's mesh count");
    if (!n_iter || (max_iter > 0 && !per_iter)) return set_err(h, LPC_E_ARG, "trace_run: null output");
    HIPCHK(h, hipSetDevice(h->device));
    lpc_handle::RaySlot &s = h->rslot[h->rs_head];
    if (s.th.joinable()) s.th.join();
    h->rs_head ^= 1;
    --h->rs_count;
    if (s.rc) return set_err(h, s.rc, s.err);
    // the analysis is read on the host (the copy ran during the previous trace);
    // the trace's first kernels wait for the batch on the device
    HIPCHK(h, hipEventSynchronize(s.ev));
    HIPCHK(h, hipStreamWaitEvent(h->stream, s.ev, 0));
    if (s.scan_gen != h->scene_gen) {           // staged before this scene: its analysis now, on the stream
        RETIF(dalloc(h, s.scan, sizeof(RayScan)));
        HIPCHK(h, hipMemsetAsync(s.scan.p, 0, sizeof(RayScan), h->stream));
        hipLaunchKernelGGL(k_ray_scan, dim3((unsigned)std::min<int64_t>(grid1(s.n), 2048)), dim3(256), 0, h->stream,
                           s.P.in(), s.n, h->box_lo[0], h->box_lo[1], h->box_lo[2], h->box_scale[0],
                           h->box_scale[1], h->box_scale[2], (RayScan *)s.scan.p);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipMemcpyAsync(s.scan_host, s.scan.p, sizeof(RayScan), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    std::swap(h->I, s.P);
    RETIF(emitted_rays(h, s.n, *s.scan_host, s.max_ray_len, s.ior_env));
    return trace_run(h, max_iter, power_threshold, per_iter, n_iter, measured_count, mesh_power, mesh_power_cap,
                     false);
}

// All-reduce (sum) of the iteration's stats over the ranks of a sharded trace.
// Slot 0 of every exchange is a failure flag (0 from a healthy rank, 1 from a
// rank that failed locally: xchg_poison), so the data values are free to hold
// NaN -- a trace whose ray powers are NaN keeps iterating exactly as a single
// device (and the reference: NaN < thr is false) does.
#define LPC_XCHG_STATS 6
static int xchg_stats(lpc_handle *h, const lpc_iter_stats &S, lpc_iter_stats *G)
{
    double v[LPC_XCHG_STATS] = {0.0, (double)S.n_in, (double)S.n_reflect, (double)S.n_refract,
                                (double)S.n_measured, S.power_next};
    const double t0 = host_us();
    const int rc = h->xchg(h->xchg_ctx, v, LPC_XCHG_STATS);
    h->xchg_us += host_us() - t0;
    h->xchg_calls += 1;
    if (rc != 0) return set_err(h, LPC_E_STATE, "trace: all-reduce hook failed");
    if (v[0] != 0.0) return set_err(h, LPC_E_STATE, "trace: a peer rank failed (failure flag in the all-reduced stats)");
    G->n_in = (int64_t)v[1]; G->n_reflect = (int64_t)v[2]; G->n_refract = (int64_t)v[3];
    G->n_measured = (int64_t)v[4]; G->power_next = v[5];
    return 0;
}

static int trace_run(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                     int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap,
                     bool wait);

// A rank that fails locally still takes part in the exchange its peers wait in,
// with the failure flag (slot 0) set: they see it in the sums and fail at once
// (xchg_stats, the trace-end sums) instead of waiting for a rank that left, and
// every rank has made the same number of exchanges.  The flag sits in slot 0 of
// every exchange shape, so the peers see it whichever exchange they are in.  The
// local error stays the one reported.
static void xchg_poison(lpc_handle *h, int32_t n)
{
    if (!h->xchg) return;
    std::vector<double> v((size_t)n, std::numeric_limits<double>::quiet_NaN());
    v[0] = 1.0;
    const std::string keep = h->err;
    (void)h->xchg(h->xchg_ctx, v.data(), n);
    h->err = keep;
}

int lpc_trace_run(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                  int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap)
{
    return trace_run(h, max_iter, power_threshold, per_iter, n_iter, measured_count, mesh_power, mesh_power_cap,
                     true);
}

int lpc_trace_run_async(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                        int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap)
{
    return trace_run(h, max_iter, power_threshold, per_iter, n_iter, measured_count, mesh_power, mesh_power_cap,
                     false);
}

int lpc_trace_rerun_async(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                          int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap)
{
    if (h && mesh_power && mesh_power_cap < h->K)       // before the reset: nothing changed on error
        return set_err(h, LPC_E_ARG, "trace: mesh_power capacity below the scene's mesh count");
    RETIF(lpc_trace_reset(h));
    return trace_run(h, max_iter, power_threshold, per_iter, n_iter, measured_count, mesh_power, mesh_power_cap,
                     false);
}

int lpc_set_allreduce(lpc_handle *h, lpc_allreduce_fn fn, void *ctx)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    h->xchg = fn;
    h->xchg_ctx = ctx;
    return 0;
}

int lpc_trace_global_stats(lpc_handle *h, lpc_iter_stats *per_iter, int32_t cap, int32_t *n_iter)
{
    if (!h || !n_iter) return set_err(h, LPC_E_ARG, "null argument");
    *n_iter = (int32_t)h->gstats.size();
    if (per_iter)
        for (int32_t i = 0; i < std::min(cap, *n_iter); ++i) per_iter[i] = h->gstats[(size_t)i];
    return 0;
}

int lpc_shm_comm_open(const char *name, int32_t rank, int32_t world, int32_t create, lpc_shm_comm **out)
{
    if (!out) return set_err(nullptr, LPC_E_ARG, "shm comm: null output");
    std::string err;
    lpcc::ShmComm *c = nullptr;
    if (lpcc::shm_open_comm(name, rank, world, create, &c, &err) != 0) return set_err(nullptr, LPC_E_ARG, err);
    *out = (lpc_shm_comm *)c;
    return 0;
}

int lpc_shm_comm_unlink(lpc_shm_comm *c)
{
    if (!c) return set_err(nullptr, LPC_E_ARG, "shm comm: null");
    lpcc::shm_unlink_comm((lpcc::ShmComm *)c);
    return 0;
}

int lpc_shm_allreduce(void *comm, double *vals, int32_t n)
{
    lpcc::ShmComm *c = (lpcc::ShmComm *)comm;
    if (!c) return set_err(nullptr, LPC_E_ARG, "shm comm: null");
    if (lpcc::shm_allreduce(c, vals, n) != 0)
        return set_err(nullptr, LPC_E_STATE, c->err.empty() ? "shm comm: bad argument" : c->err);
    return 0;
}

int lpc_shm_comm_abort(lpc_shm_comm *c)
{
    if (!c) return set_err(nullptr, LPC_E_ARG, "shm comm: null");
    lpcc::shm_abort((lpcc::ShmComm *)c, "shm comm: aborted by this rank");
    return 0;
}

int lpc_shm_comm_close(lpc_shm_comm *c)
{
    lpcc::shm_close_comm((lpcc::ShmComm *)c);
    return 0;
}

int lpc_sync(lpc_handle *h)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    return settle(h);
}

int lpc_trace_population(lpc_handle *h, int64_t *n)
{
    if (!h || !n) return set_err(h, LPC_E_ARG, "null argument");
    *n = h->n_cur;
    return 0;
}

static int ensure_measured(lpc_handle *h, int64_t need)
{
    if (need <= h->m_cap) return 0;
    // the first reservation takes twice the need: a trace's next iterations then
    // append without the growth copy (which waits for the stream)
    int64_t cap = std::max<int64_t>(h->m_cap ? need : 2 * need, std::max<int64_t>(2 * h->m_cap, 1 << 16));
    DBuf nb;
    RETIF(dalloc(h, nb, (size_t)cap * 5 * 4));
    if (h->m_cap > 0) {         // all old rows: an iteration still in flight may append past m_total
        for (int k = 0; k < 5; ++k)
            HIPCHK(h, hipMemcpyAsync((char *)nb.p + (size_t)k * cap * 4,
                                     (char *)h->m_buf.p + (size_t)k * h->m_cap * 4,
                                     (size_t)h->m_cap * 4, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    dfree(h->m_buf);
    h->m_buf = nb;
    h->m_cap = cap;
    return 0;
}

// Wait (spinning) until k_scan / k_stage_move has published the counters of the
// iteration with sequence number `seq` in its mapped ring slot; the stream keeps
// running.  A stream that fails or finishes without publishing is reported.
static int wait_mapped_acc(lpc_handle *h, unsigned seq, DevAcc *out)
{
    DevAcc *slot = h->acc_map + seq % kAccRing;
    volatile DevAcc *m = slot;
    for (uint64_t i = 1;; ++i) {
        if (__atomic_load_n(&slot->seq, __ATOMIC_ACQUIRE) == seq) break;
        if ((i & 255u) == 0u) {
            const hipError_t e = hipStreamQuery(h->stream);
            if (e == hipSuccess) {
                if (__atomic_load_n(&slot->seq, __ATOMIC_ACQUIRE) == seq) break;
                return set_err(h, LPC_E_HIP, "iteration counters were not published");
            }
            if (e != hipErrorNotReady) return set_err(h, LPC_E_HIP, std::string("trace: ") + hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
    out->nR = m->nR; out->nT = m->nT; out->m_total = m->m_total; out->nM_iter = m->nM_iter;
    out->pow_next = m->pow_next; out->dmax2_bits = m->dmax2_bits; out->qerr = m->qerr;
    out->seq = m->seq; out->pneg = m->pneg;
    for (int k = 0; k < LPC_MP_MAX; ++k) out->mpow[k] = m->mpow[k];
    return 0;
}

// An enqueued iteration whose counters have not been read yet.
struct Pending {
    int64_t n_in = 0;           // its population (-1: device-sized, known once the iteration before is read)
    unsigned seq = 0;           // mapped ring slot / sequence number (early)
    bool early = false;         // counters through the mapped ring (else copy + sync)
    bool traced = false;        // its children come out in traced order
    bool fused = false;         // k_shade_stage + k_stage_move: it wrote the next IterCtl entry
    bool mp_fused = false;      // it summed the measured power per measure mesh
    bool ds = false;            // device-sized (speculative)
    bool empty = false;         // nothing to do (n_in 0, host-sized)
    int64_t n_bound = 0;        // device-sized: population bound
    double thr = -INFINITY;     // fused: the stop threshold its k_stage_move applied (ds_thr)
    // host state before its enqueue (undo of a discarded speculative iteration)
    bool was_init = false, was_traced = false, was_emitted = false, was_pbox = false;
};

// A results export (lpc_trace_iterate_export): the caller's host block and
// whether it holds the origins.  Host layout over the iteration's N rays:
// [origin (N,4) if org][dest (N,4)][pow (N)][meas (N)].
struct ExportSpec {
    char *host = nullptr;
    int org = 0;
};

// One chunk's export: k_export packs it into a staging buffer in the host
// layout, the export stream copies it to the caller's block (one DMA when the
// chunk is the whole population) while the main stream runs on.  Two staging
// buffers alternate; the main stream waits for a buffer's last copy before
// packing into it again.
static int export_chunk(lpc_handle *h, const RaysIn &in, const ShadeOutPtrs &o, int64_t nc, int64_t base,
                        int64_t N, const ExportSpec &X)
{
    if (!h->xstream) {
        HIPCHK(h, hipStreamCreateWithFlags(&h->xstream, hipStreamNonBlocking));
        for (int k = 0; k < 2; ++k) {
            HIPCHK(h, hipEventCreateWithFlags(&h->ev_xready[k], hipEventDisableTiming));
            HIPCHK(h, hipEventCreateWithFlags(&h->ev_xdone[k], hipEventDisableTiming));
        }
    }
    const int par = h->xpar;
    h->xpar ^= 1;
    const size_t orow = X.org ? 16 : 0;
    const size_t row = orow + 16 + 4 + 4;
    if (h->xst[par].bytes < (size_t)nc * row && h->xdone_rec[par])
        HIPCHK(h, hipEventSynchronize(h->ev_xdone[par]));      // its last copy ends before it is freed
    RETIF(dalloc(h, h->xst[par], (size_t)nc * row));
    if (h->xdone_rec[par]) HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_xdone[par], 0));
    char *d = (char *)h->xst[par].p;
    float4 *xo = (float4 *)d;
    float4 *xd = (float4 *)(d + (size_t)nc * orow);
    float *xp = (float *)(d + (size_t)nc * (orow + 16));
    int32_t *xm = (int32_t *)(d + (size_t)nc * (orow + 20));
    hipLaunchKernelGGL(k_export, dim3(grid1(nc)), dim3(256), 0, h->stream, nc, in, o, X.org, xo, xd, xp, xm);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->ev_xready[par], h->stream));
    HIPCHK(h, hipStreamWaitEvent(h->xstream, h->ev_xready[par], 0));
    const double hm = h->host_prof ? host_us() : 0.0;
    // the copy into the caller's pinned block: a copy kernel writing the mapped
    // block over PCIe (round 5: hipMemcpyAsync into a block stalled the host 4-15 ms
    // on the block's first asynchronous copy, whatever primed it, DESIGN.md
    // section 7e), or a DMA copy when the block is not device-mapped / aligned
    auto copy_out = [&](char *host, const char *dev, size_t bytes) -> int {
        void *hdev = nullptr;
        if (hipHostGetDevicePointer(&hdev, host, 0) == hipSuccess && hdev && (((uintptr_t)hdev | (uintptr_t)dev) & 15u) == 0) {
            hipLaunchKernelGGL(k_copy_host, dim3(1024), dim3(256), 0, h->xstream, (const lpc_u4 *)dev, (lpc_u4 *)hdev,
                               (int64_t)(bytes / 16), (int64_t)bytes);
            HIPCHK(h, hipGetLastError());
        } else {
            HIPCHK(h, hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, h->xstream));
        }
        return 0;
    };
    if (nc == N) {
        RETIF(copy_out(X.host, d, (size_t)nc * row));
        if (h->host_prof)
            fprintf(stderr, "[lpc host]   export copy %.1f us (host %p, %zu B)\n", host_us() - hm, (void *)X.host,
                    (size_t)nc * row);
    } else {                                                    // chunk: each section at its rays' offset
        size_t hoff = 0, doff = 0;
        const size_t elt[4] = {orow, 16, 4, 4};
        for (int k = 0; k < 4; ++k) {
            if (elt[k] == 0) continue;
            RETIF(copy_out(X.host + hoff + (size_t)base * elt[k], d + doff, (size_t)nc * elt[k]));
            hoff += (size_t)N * elt[k];
            doff += (size_t)nc * elt[k];
        }
    }
    HIPCHK(h, hipEventRecord(h->ev_xdone[par], h->xstream));
    h->xdone_rec[par] = true;
    h->x_inflight = true;
    return 0;
}

// Enqueue one iteration over the current population (host-sized: h->n_cur rays;
// ds != NULL: device-sized, traced single-chunk only).  Host bookkeeping that
// needs no counters (population roles) happens here; iter_collect the rest.
static int iter_enqueue(lpc_handle *h, float *out_origin4, float *out_dest4, float *out_pow, int32_t *out_meas,
                        float *out_next_pow, const DevSize *ds, Pending *P, const ExportSpec *X = nullptr)
{
    *P = Pending();
    P->was_init = h->pop_init; P->was_traced = h->pop_traced; P->was_emitted = h->pop_emitted;
    P->was_pbox = h->pbox_ok;
    const int64_t N = ds ? ds->bound : h->n_cur;
    P->n_in = ds ? -1 : N;
    P->ds = ds != nullptr;
    P->n_bound = N;
    if (N == 0) { P->empty = true; return 0; }
    const int64_t C = std::min(N, chunk_rays(h));
    if (ds && C < N) return set_err(h, LPC_E_STATE, "internal: device-sized iteration over one chunk only");
    const double hp0 = h->host_prof ? host_us() : 0.0;
    RETIF(ensure_ws(h, C));
    RETIF(pop_reserve(h, h->B, 2 * N));
    if (!ds) RETIF(pop_reserve(h, h->T, N));
    // measured rows: the iterations still in flight may append up to their populations
    RETIF(ensure_measured(h, h->m_total + h->m_inflight + N));
    if (h->host_prof)
        fprintf(stderr, "[lpc host]   buffers %.1f us (m_total %lld inflight %lld m_cap %lld)\n", host_us() - hp0,
                (long long)h->m_total, (long long)h->m_inflight, (long long)h->m_cap);
    h->m_inflight += N;
    if (ds) {
        h->acc_pending = false;         // k_stage_move writes every counter
    } else if (C >= N) {                // one chunk: the counters reset rides on the slot reset
        h->acc_pending = true;
        h->acc_pending_total = h->m_total;
    } else {
        hipLaunchKernelGGL(k_acc_init, dim3(1), dim3(64), 0, h->stream, (DevAcc *)h->d_acc.p,
                           (unsigned long long)h->m_total);
    }
    const size_t mc = (size_t)h->m_cap;
    float *mf = (float *)h->m_buf.p;
    // traced mode: one chunk, no per-ray export (the population then comes out in
    // its parents' coherence order; measured rays per iteration likewise)
    const bool exports = out_origin4 || out_dest4 || out_pow || out_meas || out_next_pow || X;
    const bool traced = !exports;
    // the counters come back through the mapped host ring k_scan / k_stage_move
    // write, so the host decides and launches the next iteration while the rows
    // still move (profiling: only the light level, whose events end before)
    const bool early = h->acc_map_dev && (C >= N || traced) && !out_next_pow && (!h->prof || h->prof_light);
    ++h->acc_seq;
    P->seq = h->acc_seq;
    P->early = early;
    P->traced = traced;
    // traced: k_shade_stage + k_stage_move (several chunks: each places its rows
    // after the earlier chunks', refracted rows staged in T, k_append at the end)
    const bool fused = traced;
    if (fused && C < N) RETIF(dalloc(h, h->d_cbase, 8 * sizeof(unsigned long long)));
    if (ds && !(fused && early)) return set_err(h, LPC_E_STATE, "internal: device-sized iteration off the fused path");
    P->fused = fused;
    P->thr = h->ds_thr;
    const size_t Cs = (size_t)h->ws_rays;
    const int64_t ntc = (int64_t)((Cs + LPC_ST_TILE - 1) / LPC_ST_TILE);   // staging tile arrays' stride
    IterCtl *ctl = (IterCtl *)h->d_ctl.p;
    const int par = h->ctl_par;
    bool box_made = false;                  // the fused chunks wrote the children's box (d_pbox)
    for (int64_t base = 0; base < N; base += C) {
        const int64_t nc = std::min(C, N - base);
        RaysIn in = (h->pop_init ? h->I : h->A).in(base);
        RaysIn tin;
        h->in_trace = true;
        const int rc_i = run_intersect(h, in, nc, h->max_ray_len, nullptr, nullptr, nullptr, h->pop_dmax2,
                                       traced ? &tin : nullptr, ds);
        h->in_trace = false;
        RETIF(rc_i);
        if (traced) in = tin;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (h->prof && !h->prof_light) { e0 = ev_get(h); e1 = ev_get(h); (void)hipEventRecord(e0, h->stream); }
        ShadeOutPtrs o = shade_ptrs(h, false);
        CompactArgs A;
        A.n = nc; A.nb = (nc + 1023) / 1024; A.o = o;
        A.blk_cnt = (int32_t *)h->w_blk_cnt.p; A.blk_off = (long long *)h->w_blk_off.p;
        A.blk_pow = (double *)h->w_blk_pow.p; A.acc = (DevAcc *)h->d_acc.p;
        A.nR = h->B.out(); A.nT = h->T.out();
        A.direct_t = (C >= N) ? 1 : 0;                      // one chunk: no refracted staging
        if (A.direct_t) A.nT = A.nR;
        A.mx = mf; A.my = mf + mc; A.mz = mf + 2 * mc; A.mp = mf + 3 * mc;
        A.mm = (int32_t *)(mf + 4 * mc);
        A.host_acc = early ? h->acc_map_dev + P->seq % kAccRing : nullptr;
        A.seq = P->seq;
        if (fused) {                  // shade + staged compaction, two kernels (k_shade_stage, k_stage_move)
            // device-sized: grid from the expected size (grid-stride over the actual tiles)
            const int64_t ng_rays = ds ? std::max<int64_t>(1, std::min(ds->pred, nc)) : nc;
            const int64_t nt = (ng_rays + LPC_ST_TILE - 1) / LPC_ST_TILE;
            const int64_t nt_max = (nc + LPC_ST_TILE - 1) / LPC_ST_TILE;     // tiles the launch may touch
            StageArgs G;
            G.S = shade_args(h, in, nullptr, nc, h->max_ray_len, h->ior_env, false);
            G.nd = ds ? ds->nd : nullptr;
            G.stR = (float *)h->w_shf.p;                // the 20 shade-output arrays hold the staging rows
            G.stT = (float *)h->w_shi.p;
            G.stM = (float *)h->w_soa.p;
            G.cst = (int64_t)Cs;
            G.tpow = (double *)h->w_fc.p;
            G.tcnt = (uint32_t *)(G.tpow + ntc);
            G.tdm = G.tcnt + ntc;
            G.skey = (unsigned long long *)h->w_key.p;
            G.scnt = (int32_t *)h->w_sc.p;
            // measured power per measure mesh summed on the way (no k_mesh_sum at the trace end)
            G.nmp = h->meas_meshes.size() <= (size_t)LPC_MP_MAX ? (int)h->meas_meshes.size() : 0;
            for (int m = 0; m < LPC_MP_MAX; ++m) G.mpm[m] = m < G.nmp ? h->meas_meshes[(size_t)m] : -1;
            G.tmp = (double *)(G.tdm + ntc);            // 16 ntc bytes in: 8-aligned
            const int64_t ng = (nt_max + LPC_ST_GROUP - 1) / LPC_ST_GROUP;
            unsigned long long *gs = (unsigned long long *)h->w_gsum.p;
            G.gsum = gs + (size_t)h->gpar * (size_t)h->gcap;
            G.tmask = h->tm_cur;            // set by this chunk's run_intersect
            // the children's origin box when they may be re-sorted (population >= LPC_RESORT_MIN)
            const bool want_box = !ds && 2 * N >= h->resort_min;
            G.tbox = want_box ? (uint32_t *)h->w_tbox.p : nullptr;

            if (ds) LPC_KU_LAUNCH2(h, k_shade_stage, true, dim3((unsigned)nt), dim3(LPC_ST_TILE), h->stream, G);
            else LPC_KU_LAUNCH2(h, k_shade_stage, false, dim3((unsigned)nt), dim3(LPC_ST_TILE), h->stream, G);
            MoveArgs M;
            M.ntiles = nt_max;
            M.stR = G.stR; M.stT = G.stT; M.stM = G.stM; M.cst = G.cst;
            M.tcnt = G.tcnt; M.tpow = G.tpow; M.tdm = G.tdm;
            M.popR = h->B.f(0); M.capR = h->B.cap;
            M.mrec = mf; M.capM = (int64_t)mc;
            M.m_base = (unsigned long long)h->m_total;
            M.acc = (DevAcc *)h->d_acc.p;
            M.host_acc = A.host_acc;
            M.seq = A.seq;
            M.misc = (uint32_t *)h->d_misc.p;
            M.nmp = G.nmp;
            M.tmp = G.tmp;
            M.mrun = (double *)h->d_mrun.p;
            M.gsum = G.gsum;
            M.ngroups = ng;
            M.gsum_next = gs + (size_t)(1 - h->gpar) * (size_t)h->gcap;
            M.gdirty_next = h->gdirty[1 - h->gpar];
            M.ctl = ctl;
            M.par = par;
            M.thr = h->ds_thr;
            M.nmax = ds_cap(h);
            M.dcap2 = h->dcap * h->dcap * (1.0 - 1e-6);
            M.tbox = G.tbox;
            M.pbox = G.tbox ? (uint32_t *)h->d_pbox.p : nullptr;
            box_made = G.tbox != nullptr;
            M.popT = nullptr; M.capT = 0; M.cbase_in = nullptr; M.cbase_out = nullptr;
            M.first = 1; M.last = 1;
            if (C < N) {                        // chunk base / C of several
                const int64_t k = base / C;
                unsigned long long *cb = (unsigned long long *)h->d_cbase.p;
                M.popT = h->T.f(0); M.capT = h->T.cap;
                M.cbase_in = cb + (k & 1) * 3; M.cbase_out = cb + ((k & 1) ^ 1) * 3;
                M.first = base == 0 ? 1 : 0;
                M.last = base + nc >= N ? 1 : 0;
                if (!M.last) { M.host_acc = nullptr; M.ctl = nullptr; }   // the last chunk publishes the totals
            }
            h->gdirty[1 - h->gpar] = 0;
            h->gdirty[h->gpar] = ng;            // this launch's k_shade_stage adds into its first ng groups
            h->gpar = 1 - h->gpar;
            P->mp_fused = G.nmp > 0 || h->meas_meshes.empty();
            if (ds) hipLaunchKernelGGL(k_stage_move<true>, dim3((unsigned)nt), dim3(LPC_ST_TILE), 0, h->stream, M);
            else hipLaunchKernelGGL(k_stage_move<false>, dim3((unsigned)nt), dim3(LPC_ST_TILE), 0, h->stream, M);
            h->slots_clean = true;              // k_shade_stage restored what it read
            h->slots_mrl = h->max_ray_len;
            h->misc_clean = true;               // k_stage_move reset the next launch's words
            HIPCHK(h, hipGetLastError());
            if (h->prof && !h->prof_light) { (void)hipEventRecord(e1, h->stream); h->ev_rest.push_back({e0, e1}); }
            continue;
        }
        RETIF(run_shade(h, in, nullptr, nc, h->max_ray_len, h->ior_env, false));
        hipLaunchKernelGGL(k_count, dim3((unsigned)A.nb), dim3(256), 0, h->stream, A);
        if (X) {
            const double hx = h->host_prof ? host_us() : 0.0;
            RETIF(export_chunk(h, in, o, nc, base, N, *X));
            if (h->host_prof) fprintf(stderr, "[lpc host]   export chunk %.1f us\n", host_us() - hx);
        }
        if (out_origin4 || out_dest4 || out_pow || out_meas) {
            // the copies below run on the null stream: the shading on h->stream first
            HIPCHK(h, hipStreamSynchronize(h->stream));
            auto pack = [&](float *dst4, const float *x, const float *y, const float *z) -> int {
                hipLaunchKernelGGL(k_pack4, dim3(grid1(nc)), dim3(256), 0, h->stream, nc, x, y, z,
                                   (float4 *)h->w_stage.p);
                HIPCHK(h, hipStreamSynchronize(h->stream));
                HIPCHK(h, hipMemcpy(dst4 + 4 * base, h->w_stage.p, (size_t)nc * 16, hipMemcpyDeviceToHost));
                return 0;
            };
            if (out_origin4) RETIF(pack(out_origin4, in.ox, in.oy, in.oz));
            if (out_dest4) RETIF(pack(out_dest4, o.destx, o.desty, o.destz));
            if (out_pow) HIPCHK(h, hipMemcpy(out_pow + base, o.pw, (size_t)nc * 4, hipMemcpyDeviceToHost));
            if (out_meas) HIPCHK(h, hipMemcpy(out_meas + base, o.meas, (size_t)nc * 4, hipMemcpyDeviceToHost));
        }
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, h->stream, A);
        hipLaunchKernelGGL(k_scatter, dim3((unsigned)A.nb), dim3(256), 0, h->stream, A);
        HIPCHK(h, hipGetLastError());
        if (h->prof && !h->prof_light) { (void)hipEventRecord(e1, h->stream); h->ev_rest.push_back({e0, e1}); }
    }
    // refracted block after the reflected one (k_append reads the counts on the
    // device), then the counters to the pinned copy: one host sync per iteration
    if (C < N) {
        hipLaunchKernelGGL(k_append, dim3((unsigned)std::min<int64_t>(grid1(N), 8192)), dim3(256), 0, h->stream,
                           h->B.out(), h->T.in(), (const DevAcc *)h->d_acc.p, h->B.cap, h->T.cap);
        HIPCHK(h, hipGetLastError());
    }
    h->ctl_par ^= 1;                    // the next iteration reads the entry this one's k_stage_move writes
    // the children are the next population (their counts come with iter_collect)
    h->pbox_ok = box_made;
    std::swap(h->A, h->B);
    h->pop_init = false;
    h->pop_traced = traced;
    h->pop_emitted = false;
    h->inflight = true;                 // k_stage_move / k_scatter may still run
    return 0;
}

// Read an enqueued iteration's counters (in enqueue order) and finish its host
// bookkeeping.  out_next_pow: the kept children's power (the population after it).
static int iter_collect(lpc_handle *h, const Pending &P, float *out_next_pow, lpc_iter_stats *st)
{
    lpc_iter_stats S;
    memset(&S, 0, sizeof(S));
    S.n_in = P.n_in;
    S.power_nonneg = 1;
    if (P.empty) { if (st) *st = S; return 0; }
    DevAcc acc;
    const double t_wait = h->host_prof ? host_us() : 0.0;
    if (P.early) {
        RETIF(wait_mapped_acc(h, P.seq, &acc));
    } else {
        HIPCHK(h, hipMemcpyAsync(h->acc_host, h->d_acc.p, sizeof(DevAcc), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        acc = *h->acc_host;
    }
    h->m_inflight -= P.n_bound;
    if (acc.qerr) return q_failed(h);
    if (h->host_prof) {
        const double t_got = host_us();
        fprintf(stderr, "[lpc host] n %lld%s  since last %.1f us  wait %.1f us\n", (long long)P.n_in,
                P.ds ? " (device-sized)" : "", t_wait - h->host_last, t_got - t_wait);
        h->host_last = t_got;
    }
    const int64_t nR = (int64_t)acc.nR, nT = (int64_t)acc.nT;
    if (out_next_pow && nR + nT > 0) {   // the population after the swap (iter_enqueue)
        HIPCHK(h, hipMemcpyAsync(out_next_pow, h->A.f(6), (size_t)(nR + nT) * 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    if (h->prof) prof_resolve(h);
    h->n_cur = nR + nT;
    h->m_total = (int64_t)acc.m_total;
    // the running per-mesh measured power stays valid while every iteration sums it
    h->mp_valid = h->mp_valid && P.mp_fused;
    if (h->mp_valid) memcpy(h->mp_last, acc.mpow, sizeof(h->mp_last));
    S.n_reflect = nR; S.n_refract = nT; S.n_measured = (int64_t)acc.nM_iter;
    S.power_next = acc.pow_next;
    S.power_nonneg = P.fused ? -1 : (acc.pneg ? 0 : 1);
    float dm2;
    memcpy(&dm2, &acc.dmax2_bits, 4);
    RETIF(check_dcap(h, (double)dm2));
    h->pop_dmax2 = (double)dm2;                 // the next population's max |D|^2 (float, see run_intersect)
    if (st) *st = S;
    return 0;
}

// A sharded trace's dropped speculative iteration may have run non-empty: its
// k_stage_move added its measured power to the trace's running sums on the
// device; they go back to the last read iteration's (the host copy).  Its
// measured rows lie past m_total and its children in the scratch population,
// both ignored.
static int restore_mrun(lpc_handle *h)
{
    if (!h->mp_valid || !h->d_mrun.p) return 0;
    // rare (a misprediction at the trace's end): after the dropped iteration's
    // kernels, a synchronous copy from the handle's host copy
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(h->d_mrun.p, h->mp_last, sizeof(h->mp_last), hipMemcpyHostToDevice));
    return 0;
}

// A speculative iteration the trace did not need (it ran empty on the device:
// IterCtl said 0): the population roles go back to before its enqueue.
static void iter_discard(lpc_handle *h, const Pending &P)
{
    h->m_inflight -= P.n_bound;
    if (P.empty) return;
    std::swap(h->A, h->B);
    h->pop_init = P.was_init;
    h->pop_traced = P.was_traced;
    h->pop_emitted = P.was_emitted;
    h->pbox_ok = P.was_pbox;
}

int lpc_trace_iterate(lpc_handle *h, float *out_origin4, float *out_dest4, float *out_pow,
                      int32_t *out_meas, float *out_next_pow, lpc_iter_stats *st)
{
    const double t_enter = h && h->host_prof ? host_us() : 0.0;
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (!h->traced_ready) return set_err(h, LPC_E_STATE, "trace_iterate before trace_set_rays");
    HIPCHK(h, hipSetDevice(h->device));
    Pending P;
    RETIF(iter_enqueue(h, out_origin4, out_dest4, out_pow, out_meas, out_next_pow, nullptr, &P));
    if (h->host_prof && !P.empty)
        fprintf(stderr, "[lpc host] n %lld  launch %.1f us\n", (long long)P.n_in, host_us() - t_enter);
    return iter_collect(h, P, out_next_pow, st);
}

int lpc_trace_iterate_export(lpc_handle *h, void *host, int32_t flags, lpc_iter_stats *st)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (!host) return set_err(h, LPC_E_ARG, "trace_iterate_export: null host block");
    if (!h->traced_ready) return set_err(h, LPC_E_STATE, "trace_iterate_export before trace_set_rays");
    HIPCHK(h, hipSetDevice(h->device));
    const double t_enter = h->host_prof ? host_us() : 0.0;
    ExportSpec X;
    X.host = (char *)host;
    X.org = (flags & 1) ? 1 : 0;
    Pending P;
    RETIF(iter_enqueue(h, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &P, &X));
    if (h->host_prof && !P.empty)
        fprintf(stderr, "[lpc host] n %lld  export launch %.1f us\n", (long long)P.n_in, host_us() - t_enter);
    return iter_collect(h, P, nullptr, st);
}

int lpc_trace_population_power(lpc_handle *h, float *out)
{
    if (!h || !out) return set_err(h, LPC_E_ARG, "null argument");
    RETIF(settle(h));
    if (h->n_cur > 0) {
        const Pop &P = h->pop_init ? h->I : h->A;
        HIPCHK(h, hipMemcpy(out, P.f(6), (size_t)h->n_cur * 4, hipMemcpyDeviceToHost));
    }
    return 0;
}

int lpc_host_alloc(size_t bytes, void **out)
{
    if (!out) return set_err(nullptr, LPC_E_ARG, "host_alloc: null output");
    *out = nullptr;
    const hipError_t e = hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault);
    if (e != hipSuccess) return set_err(nullptr, LPC_E_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    return 0;
}

int lpc_host_free(void *p)
{
    if (p) (void)hipHostFree(p);
    return 0;
}

int lpc_host_seq_sum_f32(const float *x, int64_t n, float *out)
{
    if (!out || (n > 0 && !x) || n < 0) return set_err(nullptr, LPC_E_ARG, "host_seq_sum_f32: bad argument");
    // np.add.accumulate's order: x[0], then + x[1], ... (no reassociation: the
    // build has no fast-math; the adds form one dependent chain)
    float s = n > 0 ? x[0] : 0.0f;
    for (int64_t i = 1; i < n; ++i) s += x[i];
    *out = s;
    return 0;
}

// May the iteration after the one in flight (population <= bound rays, chained
// traced) be enqueued device-sized?  Single chunk, fused compaction, mapped
// counters, root-item path, no per-kernel profiling.  A sharded trace (all-reduce
// hook) speculates too: the device then stops only on an empty local population,
// and the host drops the iteration when the ranks' sums end the trace.
static bool ds_ok(const lpc_handle *h, int64_t bound)
{
    return h->spec && h->acc_map_dev && (!h->prof || h->prof_light) && bound > 0 && bound <= chunk_rays(h) &&
           bound < h->resort_min && (bound + 63) / 64 <= (int64_t)LPC_Q_MAX_PACKETS;
}

// The trace loop (iterative_tracer.py:383-391).  With speculation (LPC_SPEC, and
// a previous trace of the same first population, limit and threshold that
// reached the next iteration), iteration i + 1 is enqueued device-sized
// (IterCtl: its size and the stop rule evaluated by iteration i's k_stage_move)
// before iteration i's counters are read, so the GPU never waits for the host
// between iterations.  The results are the same bits: the device applies the
// host's rules; an iteration the trace turns out not to need runs empty and is
// dropped (iter_discard); a Dcap overflow (records rebuilt) re-runs it host-sized.
static int trace_run(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                     int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap,
                     bool wait)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (!n_iter || (max_iter > 0 && !per_iter)) return set_err(h, LPC_E_ARG, "trace_run: null output");
    // mesh_power receives one double per mesh of the CURRENT scene: a buffer sized
    // for an earlier scene with fewer meshes is refused, not overrun
    if (mesh_power && mesh_power_cap < h->K)
        return set_err(h, LPC_E_ARG, "trace: mesh_power capacity below the scene's mesh count");
    if (!h->traced_ready) return set_err(h, LPC_E_STATE, "trace_run before trace_set_rays");
    if (h->host_prof)                           // the caller's time between traces
        fprintf(stderr, "[lpc host] trace enter  since last %.1f us\n", host_us() - h->host_last);
    HIPCHK(h, hipSetDevice(h->device));
    *n_iter = 0;
    h->gstats.clear();
    // the prediction: the last trace from emitted rays with this iteration limit
    // (which iterations it reached, populations relative to the first)
    const int64_t n0 = h->pop_emitted ? h->n_cur : -1;
    const bool hist_ok = n0 > 0 && h->hist_iter == max_iter && !h->hist_r.empty();
    h->dcap_rebuilt = false;
    std::vector<int64_t> seen;
    // the device's stop rule for speculative iterations (k_stage_move): the
    // threshold on this device's own power left -- or, in a sharded trace, none:
    // the power left is a sum over all ranks, only the host sees it after the
    // exchange, and a speculative iteration the ranks' sums end is dropped
    h->ds_thr = h->xchg ? -INFINITY : power_threshold;
    // sharded: a conservative local rule.  The device may stop the trace only when
    // the ranks' sum is certain to fall below the threshold: with passive
    // materials and non-negative powers a population's power never grows, so the
    // other ranks' power left after the last exchanged iteration j bounds theirs
    // at every later iteration (slack for the float32 children sums), and this
    // rank's power below threshold - that bound ends the global trace too.
    const bool mono = h->xchg && h->mat_passive && h->pow_nonneg && h->ior_env > 0.0f && std::isfinite(h->ior_env);
    double others = INFINITY;           // upper bound of the other ranks' power left (last exchange)
    int32_t others_it = -1;
    auto local_thr = [&](int32_t it) {  // k_stage_move's stop threshold of iteration `it`
        if (!h->xchg) return power_threshold;
        if (!mono || others_it < 0 || !(others < INFINITY)) return -(double)INFINITY;
        return power_threshold - others * (1.0 + 1e-5 * (double)(it - others_it + 1));
    };
    int rc = 0;
    bool exchanged = false;             // rc came from the exchange itself (no poison owed)
    int32_t post_fail = -1;             // failed after this iteration's exchange: the shape the peers wait in next
    Pending cur, nxt;
    bool have_cur = false, have_nxt = false;
    for (int32_t i = 0; i < max_iter; ++i) {
        if (!have_cur) {
            h->ds_thr = local_thr(i);
            if ((rc = iter_enqueue(h, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &cur))) break;
            have_cur = true;
        }
        // iteration i + 1, device-sized, while iteration i runs (its population is
        // known: host-sized, or the kept children of iteration i - 1)
        if (hist_ok && i + 1 < max_iter && (int64_t)h->hist_r.size() > i + 1 && cur.fused && !cur.empty &&
            cur.n_in > 0) {
            // its bound: all children of the current population, capped at
            // ds_cap (more kept children: it runs empty and is re-run host-sized)
            const int64_t bound = std::min<int64_t>(2 * cur.n_in, ds_cap(h));
            const int64_t pred_n = (int64_t)llround(h->hist_r[(size_t)i + 1] * (double)n0);
            if (pred_n <= bound && ds_ok(h, bound)) {
                IterCtl *ctl = (IterCtl *)h->d_ctl.p;
                DevSize D;
                D.nd = &ctl->n[h->ctl_par];
                D.dm2 = &ctl->dm2[h->ctl_par];
                D.pred = std::max<int64_t>(1, std::min(pred_n, bound));
                D.bound = bound;
                h->ds_thr = local_thr(i + 1);
                if ((rc = iter_enqueue(h, nullptr, nullptr, nullptr, nullptr, nullptr, &D, &nxt))) break;
                have_nxt = true;
            }
        }
        lpc_iter_stats S;
        const double cur_thr = cur.thr;     // the stop rule cur's k_stage_move sized nxt with
        rc = iter_collect(h, cur, nullptr, &S);
        have_cur = false;
        if (rc) break;
        per_iter[i] = S;
        *n_iter = i + 1;
        seen.push_back(S.n_in);
        // sharded trace: every rank decides on the sums over all ranks (the
        // identical bits everywhere), so all stop at the iteration a single
        // device would (iterative_tracer.py:383-391)
        lpc_iter_stats G = S;
        if (h->xchg && (rc = xchg_stats(h, S, &G))) { exchanged = true; break; }
        h->gstats.push_back(G);
        if (h->xchg) {
            others = std::max(0.0, G.power_next - S.power_next) * (1.0 + 1e-9);
            others_it = i;
        }
        const bool stop = G.power_next < power_threshold || G.n_reflect + G.n_refract == 0;   // :383, :389
        if (have_nxt) {
            const bool rebuilt = h->dcap_rebuilt;
            h->dcap_rebuilt = false;
            if (stop || rebuilt || i + 1 >= max_iter) {
                // not part of the trace: it ran empty on the device (its IterCtl
                // size was 0) -- or, sharded, it may have run on this rank's kept
                // children when the ranks' sums stopped the trace; after a Dcap
                // rebuild its measured power must not count either
                iter_discard(h, nxt);
                have_nxt = false;
                if ((h->xchg || rebuilt) && (rc = restore_mrun(h))) {
                    // this iteration's exchange is done: the peers wait next in
                    // the trace-end sums (stop) or the next iteration's stats
                    post_fail = stop ? ((measured_count || mesh_power) ? h->K + 2 : 0) : LPC_XCHG_STATS;
                    break;
                }
            } else if (S.n_reflect + S.n_refract > nxt.n_bound || S.power_next < cur_thr) {
                // more children than it was sized for, or this device's stop rule
                // fired where the trace goes on (a sharded rank's local bound,
                // should its premise fail): it ran empty on the device; the next
                // pass of the loop runs the iteration host-sized
                iter_discard(h, nxt);
                have_nxt = false;
                if (h->xchg && (rc = restore_mrun(h))) { post_fail = LPC_XCHG_STATS; break; }
            } else {
                nxt.n_in = S.n_reflect + S.n_refract;           // this rank's population
                cur = nxt;
                have_cur = true;
                have_nxt = false;
            }
        }
        if (stop) break;
    }
    if (have_nxt) iter_discard(h, nxt);
    if (have_cur) {                                         // an error with one still queued
        (void)hipStreamSynchronize(h->stream);
        iter_discard(h, cur);
    }
    if (rc && !exchanged) {
        if (post_fail < 0) xchg_poison(h, LPC_XCHG_STATS);               // the peers wait in this iteration's exchange
        else if (post_fail > 0) xchg_poison(h, post_fail);
    }
    RETIF(rc);
    // this trace's populations (relative to the first) predict the next trace's
    if (n0 > 0) {
        h->hist_r.clear();
        for (int64_t v : seen) h->hist_r.push_back((double)v / (double)n0);
        h->hist_iter = max_iter;
    }
    if (measured_count || mesh_power) {                     // the trace's aggregates, same call
        // [failure flag, per-mesh power (K), measured count]
        int64_t c = 0;
        std::vector<double> mp((size_t)h->K + 2, 0.0);
        if ((rc = lpc_trace_measured(h, &c, mp.data() + 1, h->K))) {
            xchg_poison(h, h->K + 2);
            return rc;
        }
        if (h->xchg) {                                      // trace-end sums over the ranks
            mp[(size_t)h->K + 1] = (double)c;
            if (h->xchg(h->xchg_ctx, mp.data(), h->K + 2) != 0)
                return set_err(h, LPC_E_STATE, "trace: all-reduce hook failed");
            if (mp[0] != 0.0) return set_err(h, LPC_E_STATE, "trace: a peer rank failed (failure flag in the trace-end sums)");
            c = (int64_t)mp[(size_t)h->K + 1];
        }
        if (measured_count) *measured_count = c;
        if (mesh_power) memcpy(mesh_power, mp.data() + 1, (size_t)h->K * 8);
    }
    if (wait) RETIF(settle(h));                             // the trace's last kernels too
    if (h->host_prof) {
        const double t = host_us();
        fprintf(stderr, "[lpc host] trace leave  since last %.1f us\n", t - h->host_last);
        h->host_last = t;
    }
    return 0;
}

static int mesh_power(lpc_handle *h, double *out)
{
    for (int32_t j = 0; j < h->K; ++j) out[j] = 0.0;
    if (h->m_total == 0) return 0;
    if (h->mp_valid && h->meas_meshes.size() <= (size_t)LPC_MP_MAX) {   // summed per tile by the traced iterations
        for (size_t m = 0; m < h->meas_meshes.size(); ++m) out[h->meas_meshes[m]] = h->mp_last[m];
        return 0;
    }
    const int64_t nb = (h->m_total + LPC_MSUM_TILE - 1) / LPC_MSUM_TILE;
    RETIF(dalloc(h, h->d_tmp, (size_t)nb * 8));
    std::vector<double> part((size_t)nb);
    const size_t mc = (size_t)h->m_cap;
    const float *mf = (const float *)h->m_buf.p;
    for (int32_t j : h->meas_meshes) {
        hipLaunchKernelGGL(k_mesh_sum, dim3((unsigned)nb), dim3(256), 0, h->stream, h->m_total,
                           mf + 3 * mc, (const int32_t *)(mf + 4 * mc), j, (double *)h->d_tmp.p);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipMemcpyAsync(part.data(), h->d_tmp.p, (size_t)nb * 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        double s = 0.0;
        for (double v : part) s += v;
        out[j] = s;
    }
    return 0;
}

int lpc_trace_measured(lpc_handle *h, int64_t *count, double *mesh_pow, int32_t mesh_pow_cap)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (mesh_pow && mesh_pow_cap < h->K)
        return set_err(h, LPC_E_ARG, "trace_measured: mesh_power capacity below the scene's mesh count");
    HIPCHK(h, hipSetDevice(h->device));
    if (count) *count = h->m_total;
    if (mesh_pow) RETIF(mesh_power(h, mesh_pow));
    return 0;
}

int lpc_trace_fetch_measured(lpc_handle *h, float *pos4, float *pow, int32_t *mesh)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    HIPCHK(h, hipSetDevice(h->device));
    const int64_t n = h->m_total;
    if (n == 0) return 0;
    const size_t mc = (size_t)h->m_cap;
    const float *mf = (const float *)h->m_buf.p;
    if (pos4) {
        RETIF(dalloc(h, h->w_stage, (size_t)n * 16));
        hipLaunchKernelGGL(k_pack4, dim3(grid1(n)), dim3(256), 0, h->stream, n, mf, mf + mc,
                           mf + 2 * mc, (float4 *)h->w_stage.p);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipStreamSynchronize(h->stream));
        HIPCHK(h, hipMemcpy(pos4, h->w_stage.p, (size_t)n * 16, hipMemcpyDeviceToHost));
    }
    if (pow) HIPCHK(h, hipMemcpy(pow, mf + 3 * mc, (size_t)n * 4, hipMemcpyDeviceToHost));
    if (mesh) HIPCHK(h, hipMemcpy(mesh, mf + 4 * mc, (size_t)n * 4, hipMemcpyDeviceToHost));
    return 0;
}

int lpc_project_hist(lpc_handle *h, int mode, int64_t n, const float *pos4, const float *pwr,
                     const float *rot4, const float *pivot4, const double *xedges, int nx,
                     const double *yedges, int ny, double weight_div, double *H, float *x,
                     float *y, float *pwr_cor)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    if ((mode != 0 && mode != 1) || nx <= 0 || ny <= 0 || !rot4 || !pivot4 || !xedges || !yedges || !H)
        return set_err(h, LPC_E_ARG, "project_hist: bad argument");
    if (pos4 && !pwr) return set_err(h, LPC_E_ARG, "project_hist: pwr is NULL");
    HIPCHK(h, hipSetDevice(h->device));
    if (!pos4) n = h->m_total;
    if (n < 0) return set_err(h, LPC_E_ARG, "project_hist: negative n");
    // device scratch: [rot 16 f | piv 4 f | xe | ye | H | (pos4, pwr) | (x, y, pc)]
    const size_t o_rot = 0, o_xe = 128, o_ye = o_xe + (size_t)(nx + 1) * 8;
    const size_t o_H = (o_ye + (size_t)(ny + 1) * 8 + 255) / 256 * 256;
    const size_t o_in = (o_H + (size_t)nx * ny * 8 + 255) / 256 * 256;
    const size_t in_bytes = pos4 ? (size_t)n * 20 : 0;
    const size_t o_out = (o_in + in_bytes + 255) / 256 * 256;
    const size_t out_bytes = x ? (size_t)n * 12 : 0;
    RETIF(dalloc(h, h->d_tmp, o_out + out_bytes + 16));
    char *d = (char *)h->d_tmp.p;
    float rp[20];
    memcpy(rp, rot4, 16 * 4);
    memcpy(rp + 16, pivot4, 4 * 4);
    HIPCHK(h, hipMemcpy(d + o_rot, rp, sizeof(rp), hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(d + o_xe, xedges, (size_t)(nx + 1) * 8, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(d + o_ye, yedges, (size_t)(ny + 1) * 8, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemsetAsync(d + o_H, 0, (size_t)nx * ny * 8, h->stream));
    ProjArgs A;
    memset(&A, 0, sizeof(A));
    A.n = n; A.mode = mode;
    if (pos4) {
        HIPCHK(h, hipMemcpy(d + o_in, pos4, (size_t)n * 16, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(d + o_in + (size_t)n * 16, pwr, (size_t)n * 4, hipMemcpyHostToDevice));
        A.pos4 = (const float4 *)(d + o_in);
        A.pwr = (const float *)(d + o_in + (size_t)n * 16);
    } else {
        const size_t mc = (size_t)h->m_cap;
        const float *mf = (const float *)h->m_buf.p;
        A.px = mf; A.py = mf + mc; A.pz = mf + 2 * mc; A.pwr = mf + 3 * mc;
    }
    A.rot = (const float *)(d + o_rot);
    A.piv = (const float *)(d + o_rot) + 16;
    if (x) { A.x = (float *)(d + o_out); A.y = A.x + n; A.pc = A.y + n; }
    A.xe = (const double *)(d + o_xe); A.ye = (const double *)(d + o_ye);
    A.nx = nx; A.ny = ny; A.div = weight_div; A.H = (double *)(d + o_H);
    if (n > 0) {
        hipLaunchKernelGGL(k_project_hist, dim3(grid1(n)), dim3(256), 0, h->stream, A);
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(H, d + o_H, (size_t)nx * ny * 8, hipMemcpyDeviceToHost));
    if (x && n > 0) {
        HIPCHK(h, hipMemcpy(x, A.x, (size_t)n * 4, hipMemcpyDeviceToHost));
        if (y) HIPCHK(h, hipMemcpy(y, A.y, (size_t)n * 4, hipMemcpyDeviceToHost));
        if (pwr_cor) HIPCHK(h, hipMemcpy(pwr_cor, A.pc, (size_t)n * 4, hipMemcpyDeviceToHost));
    }
    return 0;
}

int lpc_filter_eval(lpc_handle *h, int64_t n, const float *origin3, const float *dir3, const float *rec5,
                    int mode, float *out_d)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    if (n < 0 || mode < 0 || mode > 3 || (n > 0 && (!origin3 || !dir3 || !rec5 || !out_d)))
        return set_err(h, LPC_E_ARG, "filter_eval: bad argument");
    RETIF(settle(h));
    HIPCHK(h, hipSetDevice(h->device));
    if (n == 0) return 0;
    RETIF(dalloc(h, h->d_tmp, (size_t)n * 48));
    float *dO = (float *)h->d_tmp.p, *dD = dO + 3 * n, *dR = dD + 3 * n, *dOut = dR + 5 * n;
    HIPCHK(h, hipMemcpy(dO, origin3, (size_t)n * 12, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(dD, dir3, (size_t)n * 12, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(dR, rec5, (size_t)n * 20, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_filter_eval, dim3(grid1(n)), dim3(256), 0, h->stream, n, (const float *)dO,
                       (const float *)dD, (const float *)dR, mode, dOut);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(out_d, dOut, (size_t)n * 4, hipMemcpyDeviceToHost));
    return 0;
}

int lpc_prof_enable(lpc_handle *h, int on)
{
    if (!h) return set_err(nullptr, LPC_E_ARG, "null handle");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    h->prof_every = std::max(1, on >> 8);           // 4 + 256 k: light, every k-th walk launch
    on &= 0xff;
    h->prof_seq = 0;
    h->prof = on != 0;
    h->prof_stats = on == 2;
    h->prof_light = on == 4;                        // k_rootwalk events only (bench timed region)
    if (h->prof_stats && !h->d_stats.p) {
        RETIF(dalloc(h, h->d_stats, LPC_STATS_WORDS * 8));
        HIPCHK(h, hipMemset(h->d_stats.p, 0, LPC_STATS_WORDS * 8));
    }
    return 0;
}

int lpc_prof_read(lpc_handle *h, lpc_prof *out, int reset)
{
    if (!h || !out) return set_err(h, LPC_E_ARG, "null argument");
    RETIF(settle(h));                   // a trace still running (lpc_trace_iterate / _run_async)
    (void)hipStreamSynchronize(h->stream);
    prof_resolve(h);
    out->intersect_ms = h->prof_isect_ms;
    out->kernel_ms = h->prof_kern_ms;
    out->shade_ms = h->prof_rest_ms;
    out->intersect_launches = h->prof_launches;
    out->xchg_us = h->xchg_us;
    out->xchg_calls = h->xchg_calls;
    out->pairs = h->prof_pairs;
    std::vector<unsigned long long> st(LPC_STATS_WORDS, 0ull);
    if (h->d_stats.p) HIPCHK(h, hipMemcpy(st.data(), h->d_stats.p, LPC_STATS_WORDS * 8, hipMemcpyDeviceToHost));
    out->node_visits = (int64_t)st[0];
    out->group_tests = (int64_t)st[1];
    out->wave_traversals = (int64_t)st[2];
    out->exact_tests = (int64_t)st[3];
    for (int b = 0; b < 24; ++b) out->wave_hist[b] = (int64_t)st[LPC_STATS_HIST + b];
    out->tail_waves = (int64_t)st[4]; out->tail_nodes = (int64_t)st[5];
    out->tail_spread_urad = (int64_t)st[6]; out->tail_exact = (int64_t)st[7];
    out->walk_cycles = (int64_t)st[LPC_STATS_CYC]; out->drain_cycles = (int64_t)st[LPC_STATS_CYC + 1];
    out->fan_exact = (int64_t)st[LPC_STATS_CYC + 2];
    out->behind_exact = (int64_t)st[LPC_STATS_CYC + 3];
    out->hit_exact = (int64_t)st[LPC_STATS_CYC + 4];
    out->heavy_piece = -1; out->heavy_piece_ticks = 0; out->piece_ticks = 0;
    for (int p = 0; p < LPC_STATS_PIECES; ++p) {
        const int64_t v = (int64_t)st[LPC_STATS_PIECE + p];
        out->piece_ticks += v;
        if (v > out->heavy_piece_ticks) { out->heavy_piece_ticks = v; out->heavy_piece = p; }
    }
    if (reset) {
        h->prof_isect_ms = h->prof_rest_ms = h->prof_kern_ms = 0.0; h->prof_launches = h->prof_pairs = 0;
        h->xchg_us = 0.0; h->xchg_calls = 0;
        if (h->d_stats.p) HIPCHK(h, hipMemset(h->d_stats.p, 0, LPC_STATS_WORDS * 8));
    }
    return 0;
}

}  // extern "C"
