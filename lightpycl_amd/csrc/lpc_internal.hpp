// lpc_internal.hpp -- argument structs shared by the kernels and the host runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lpck {

struct Piece {                       // part of one mesh run
    int32_t root;                     // subtree root node (k_intersect)
    int32_t s_lo, s_hi;               // sliver records [s_lo, s_hi) (k_slivers)
    int32_t slot;                     // per-mesh scratch slot the run flushes into
    float cx, cy, cz, negB, negA;     // the root's own test
    int32_t pad[3];
};

// Per (slot, ray) nearest hit as one 64-bit key: order-preserving float bits of
// t above the triangle index, so atomicMin gives the minimal t and, among equal
// t, the lowest index (the reference's first-minimum rule, .cl:277-283).
__host__ __device__ inline unsigned long long slot_key(float t, int32_t idx)
{
    uint32_t u = __builtin_bit_cast(uint32_t, t);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (uint32_t)idx;
}
__host__ __device__ inline float slot_key_t(unsigned long long k)
{
    uint32_t u = (uint32_t)(k >> 32);
    u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
    return __builtin_bit_cast(float, u);
}
__host__ __device__ inline int32_t slot_key_idx(unsigned long long k) { return (int32_t)(uint32_t)k; }

// Profiling counters (lpc_prof_enable(h, 2)): [0..3] traversal counters,
// [HIST..HIST+24) k_intersect wave-duration histogram (log2 of 100 MHz ticks),
// [PIECE..PIECE+PIECES) summed wave ticks per piece.
#define LPC_STATS_HIST 8
#define LPC_STATS_PIECE 32
#define LPC_STATS_PIECES 4096
#define LPC_STATS_WORDS (LPC_STATS_PIECE + LPC_STATS_PIECES)

// Per-launch device words of the intersect stage (uint32, reset by k_slot_init):
// [0..5] population origin box (k_bbox, coherence key modes 1-2), [6..13]
// hand-over queue lengths (k_intersect -> k_spill level 0 -> level 1 ...),
// from word 32 the work queue's control words (k_roots / k_trav), every group on
// a 128-byte line of its own: a device-scope atomic evicts its line from the
// L2, and one word serialises its atomics (~11 ns each), so counters are sharded.
#define LPC_MISC_SPILL 6                  // [6 + l]: items queued for hand-over level l (l < 8)
#define LPC_Q_CSHARDS 8                   // root-item shards (k_roots block b -> b % 8, or packet-range eighths)
#define LPC_Q_DSHARDS 32                  // hand-over queue shards (k_trav block b -> b % 32)
#define LPC_Q_NINIT(c) (32 * (1 + (c)))   // root items k_roots wrote into shard c
#define LPC_Q_CHEAD(c) (32 * (9 + (c)))   // claim head of root shard c
// Hand-over shard d: a 64-bit word TP = slots reserved (low half) | items
// handed over and not finished (high half), so one returning atomic reserves
// slots and counts them before they are published; tickets taken by waiting
// waves; and, on a line of its own, the shard's waves still in the root phase.
#define LPC_Q_TP(d) (32 * (17 + 2 * (d)))
#define LPC_Q_DHEAD(d) (32 * (17 + 2 * (d)) + 2)
#define LPC_Q_RBUSY(d) (32 * (18 + 2 * (d)))
#define LPC_MISC_WORDS (32 * (17 + 2 * LPC_Q_DSHARDS))

// Work queue of the intersect stage (k_roots -> k_trav).  An item is one packet
// (64 rays of the coherence order) against one subtree of a mesh run, packed in
// 64 bits: packet (24 bits) | node (28 bits) | slot (12 bits).  k_roots writes the
// (packet, piece root) pairs whose root test some ray passes (the test
// k_intersect's waves start with); k_trav's waves claim them in batches and walk
// them, and while waves of their shard wait for work they hand the bottom of
// their stack over through the shard's queue.  A queue slot holds LPC_QEMPTY
// until an item is published into it (8-byte agent-scope atomic store: data and
// flag in one granule); its consumer writes LPC_QEMPTY back, so the queue is
// empty again between launches.
#define LPC_QEMPTY 0xffffffffffffffffull
__host__ __device__ inline uint64_t q_item(uint32_t w, uint32_t node, uint32_t slot)
{
    return ((uint64_t)w << 40) | ((uint64_t)node << 12) | (uint64_t)slot;
}
__host__ __device__ inline uint32_t q_w(uint64_t it) { return (uint32_t)(it >> 40); }
__host__ __device__ inline uint32_t q_node(uint64_t it) { return (uint32_t)(it >> 12) & 0x0fffffffu; }
__host__ __device__ inline uint32_t q_slot(uint64_t it) { return (uint32_t)it & 0xfffu; }
#define LPC_Q_MAX_PACKETS ((1u << 24) - 1u)
#define LPC_Q_MAX_NODES ((1u << 28) - 1u)
#define LPC_Q_MAX_SLOTS 4095

struct QueueArgs {
    uint64_t *roots;                  // [LPC_Q_CSHARDS][rcap] root items
    uint64_t *dq;                     // [LPC_Q_DSHARDS][dcap] hand-over slots (LPC_QEMPTY when free)
    uint32_t *ctl;                    // misc words (LPC_Q_*)
    uint32_t *err;                    // set when a wave gives up waiting (a bug: never expected)
    uint32_t rcap, dcap;
    uint32_t spin_max;                // polls before a waiting wave gives up
    int32_t batch;                    // root items per claim
    int32_t hunger;                   // hand work over to waiting waves (0: never, A/B only)
    int32_t dshard;                   // set per wave by k_trav (-1: no hand-over)
    uint32_t *irec;                   // per-item records (profiling, lpc_prof_enable(h, 5)) or NULL
    uint32_t irec_cap;
    // XCD-local walk (LPC_XCD_WALK): the root shards are contiguous eighths of the
    // packet range (k_roots*), and k_rootwalk's waves on XCD x (blocks b % 8 == x,
    // the hardware's round-robin dispatch) walk the x-th eighth of the item list,
    // so each XCD's L2 holds the scene records of one eighth of the directions.
    int32_t xcd;
    int64_t npk;                      // packets of the launch (range shards)
};
// root shard of a k_roots* block whose first packet is w0
__host__ __device__ inline int q_shard(const QueueArgs &Q, int64_t w0, uint32_t block)
{
    if (!Q.xcd) return (int)(block % LPC_Q_CSHARDS);
    const int64_t c = (w0 * LPC_Q_CSHARDS) / (Q.npk > 0 ? Q.npk : 1);
    return (int)(c < LPC_Q_CSHARDS - 1 ? c : LPC_Q_CSHARDS - 1);
}
#define LPC_Q_IREC_N 16                   // misc word: item records written this launch

// Work hand-over: a k_intersect wave that has visited `budget` nodes with two or
// more subtrees still on its stack queues each of them as one item; k_spill
// runs the items, one wave each (per-ray results flush with the same
// order-independent atomics, so the split does not change the result).
struct SpillItem {
    int32_t w, node, slot, piece;     // packet, subtree root, slot, piece (stats)
};
struct SpillArgs {
    SpillItem *items;
    uint32_t *ctr;                    // misc + LPC_MISC_SPILL
    uint32_t cap;
    int budget;                       // cost before hand-over (0: never), in node visits
    int pair_shift;                   // exact pairs per node visit = 1 << pair_shift (31: not counted)
};

// A fan group met by a k_intersect wave (packet, piece): group id and the rays
// that passed the group's test; k_groups processes them.
struct GItem {
    int32_t g, pad;
    uint64_t m;
};

struct RaysIn {                       // a ray population (SoA)
    const float *ox, *oy, *oz, *dx, *dy, *dz, *pw;
    const int32_t *pmid;              // previous intersected mesh (-2 emitted, -1 outside)
};
struct RaysOut {
    float *ox, *oy, *oz, *dx, *dy, *dz, *pw;
    int32_t *pmid;
};

struct ShadeOutPtrs {                 // per-ray outputs of k_shade (SoA)
    float *destx, *desty, *destz, *pw;
    int32_t *imid, *meas;
    float *rdx, *rdy, *rdz, *rpw;
    int32_t *rms;
    float *tdx, *tdy, *tdz, *tpw;
    int32_t *tms;
    int32_t *iidx, *n1, *n2, *ent;    // optional (NULL iidx disables all four)
};

struct ShadeArgs {
    RaysIn in;
    const int32_t *meas_in;           // NULL -> 0 (device loop population)
    int64_t n;
    int32_t K;
    const unsigned long long *skey;   // [K][n] per-slot nearest hit (slot_key)
    const int32_t *sc;                // [K][n] hit count
    const int32_t *mat_type;
    const float *ior, *refl, *diss, *verts;
    float max_ray_len, ior_env;
    ShadeOutPtrs o;
    // counts first (LPC_SHADE_CFIRST, traced iterations only, whose slots start in
    // the uniform clean state): a slot's key is read only when its count is not 0
    // (a count of 0 means the key is still slot_key(max_ray_len, -1))
    int32_t cfirst;
};

#define LPC_MP_MAX 4                      // measure meshes whose power the traced path sums per tile
struct DevAcc {                       // device-side counters of one iteration
    unsigned long long nR, nT;        // kept reflected / refracted (running within iteration)
    unsigned long long m_total;       // measured record length (persistent)
    unsigned long long nM_iter;       // measured this iteration
    double pow_next;                  // float64 sum of kept children power
    unsigned int dmax2_bits;          // max |dir|^2 of kept children (float bits)
    unsigned int qerr;                // k_trav gave up waiting on its work queue (QueueArgs::err)
    unsigned int seq;                 // host copy only: iteration number, written last (k_scan)
    unsigned int pad;
    double mpow[LPC_MP_MAX];          // traced path: measured power of the trace so far per measure mesh
};

struct SlotInit {                     // per-mesh slot initial state of a launch (k_slot_init)
    int32_t K;
    const int32_t *live;
    float max_ray_len;
    unsigned long long *skey;
    int32_t *scnt;
    uint32_t *misc;                   // LPC_MISC_WORDS per-launch words (reset), may be NULL
    DevAcc *acc;                      // iteration counters to reset, may be NULL
    unsigned long long m_total;
    int uniform;                      // every slot (max_ray_len, idx -1): the traced path's clean state
};

struct CompactArgs {
    int64_t n, nb;                    // rays in chunk, 1024-ray tiles
    ShadeOutPtrs o;
    int32_t *blk_cnt;                 // [3][nb]
    long long *blk_off;               // [3][nb]
    double *blk_pow;                  // [nb]
    DevAcc *acc;
    RaysOut nR, nT;                   // next population: reflected block, refracted staging
    int32_t *childR, *childT;         // order chaining: each parent's children's positions (or NULL)
    int direct_t;                     // single chunk: refracted children go straight after the
                                      // reflected block (offset acc->nR), no staging / k_append
    float *mx, *my, *mz, *mp;         // measured record
    int32_t *mm;
    DevAcc *host_acc;                 // mapped pinned host copy k_scan publishes (or NULL)
    unsigned int seq;                 // ... with this sequence number, written last
};

// Two-kernel compaction of a traced single-chunk iteration (k_shade_stage ->
// k_stage_move, see lpc_kernels.hip).  Tile counts are packed in one word:
// reflected | refracted << 9 | measured << 18 (each <= LPC_ST_TILE).
#define LPC_ST_TILE 256                   // rays per staging tile (k_shade_stage / k_stage_move block)
struct StageArgs {
    ShadeArgs S;                      // shading inputs (S.o unused)
    float *stR, *stT;                 // staged kept children: 8 arrays each (ox..pw | pmid), stride cst
    float *stM;                       // staged measured rays: x y z pw | mesh, stride cst
    int64_t cst;
    uint32_t *tcnt;                   // [ntiles] packed counts
    double *tpow;                     // [ntiles] kept children power
    uint32_t *tdm;                    // [ntiles] max |dir|^2 (float bits) of kept children
    unsigned long long *skey;         // the slots read by the shading, restored to the clean state
    int32_t *scnt;                    //   (key slot_key(max_ray_len, -1), count 0) after the read
    int nmp;                          // measure meshes summed per tile (<= LPC_MP_MAX; 0: none)
    int32_t mpm[LPC_MP_MAX];          // their mesh ids
    double *tmp;                      // [ntiles][LPC_MP_MAX] measured power per tile and measure mesh
    unsigned long long *gsum;         // per group of LPC_ST_GROUP tiles: counts (21 bits each), zero before
};
#define LPC_ST_GROUP 256                  // tiles per count group (k_stage_move prefixes: groups, then tiles)
__host__ __device__ inline unsigned long long gsum_pack(uint32_t r, uint32_t t, uint32_t m)
{
    return (unsigned long long)r | ((unsigned long long)t << 21) | ((unsigned long long)m << 42);
}
struct MoveArgs {
    int64_t ntiles;
    const float *stR, *stT, *stM;
    int64_t cst;
    const uint32_t *tcnt;
    const double *tpow;
    const uint32_t *tdm;
    float *popR;                      // next population: 8 arrays, stride capR
    int64_t capR;
    float *mrec;                      // measured record: x y z pw | mesh, stride capM
    int64_t capM;
    unsigned long long m_base;        // measured record length before this iteration
    DevAcc *acc;
    DevAcc *host_acc;                 // mapped pinned host copy (or NULL)
    unsigned int seq;
    uint32_t *misc;                   // the next launch's words (LPC_MISC_WORDS), reset here
    int nmp;                          // measure meshes summed per tile (StageArgs)
    const double *tmp;
    double *mrun;                     // [LPC_MP_MAX] the trace's running sums (own buffer: counter resets keep it)
    const unsigned long long *gsum;   // group counts of this launch (StageArgs::gsum)
    int64_t ngroups;
    unsigned long long *gsum_next;    // the next launch's group counts: its first gdirty_next (left by the
    int64_t gdirty_next;              //   launch before this one) zeroed here
};

// Order chaining (k_ocount / k_oscan / k_oscatter): the next population's
// coherence order = the kept children in their parents' traced order
// ([reflected ; refracted]), with the rays copied into that order.
struct OrderArgs {
    int64_t n, nb;                    // parents, 1024-parent tiles
    const int32_t *perm;              // traced order of the parents (position -> index)
    const int32_t *childR, *childT;   // parent index -> child position (-1 none)
    ShadeOutPtrs o;                   // parents' shade outputs (child rays)
    int32_t *blk;                     // [2][nb] counts, then offsets
    long long *totR;                  // reflected children total (device)
    const DevAcc *acc;                // n_next = acc->nR + acc->nT
    int32_t *perm_next;               // [n_next]
    float *rs_next;                   // [6][n_next]
};

struct PostprocAosArgs {
    int64_t n;
    int32_t K;
    const float4 *origin, *dir;
    float4 *dest;
    const int32_t *prev_mid;
    int32_t *n1, *n2, *entering, *imid, *iidx;
    const float *tmin;
    const int32_t *cnt, *itmp;
    const int32_t *mat_type;
    float max_ray_len;
};

struct FresnelAosArgs {
    int64_t n;
    const float4 *origin, *dest, *dir;
    float *pow;
    int32_t *meas;
    const int32_t *n1, *n2, *imid, *iidx;
    float4 *r_origin, *r_dir, *t_origin, *t_dir;
    float *r_pow, *t_pow;
    int32_t *r_meas, *t_meas;
    const int32_t *mat_type;
    const float *ior, *refl, *diss, *verts;
    float ior_env;
};

struct ProjArgs {
    int64_t n;
    int mode;                         // 0 angular, 1 stereographic
    const float4 *pos4;               // either pos4 or px/py/pz
    const float *px, *py, *pz, *pwr;
    const float *rot, *piv;           // device copies: rot 4x4 rows, pivot 4
    float *x, *y, *pc;                // optional outputs
    const double *xe, *ye;
    int nx, ny;
    double div;                       // H += pc / div  (dx*dy, float64)
    double *H;
};

}  // namespace lpck
