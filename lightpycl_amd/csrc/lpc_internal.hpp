// lpc_internal.hpp -- argument structs shared by the kernels and the host runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lpck {

struct Piece {                       // part of one mesh run
    int32_t root;                     // subtree root node (the root items' start)
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
// [HIST..HIST+24) walk item duration histogram (log2 of 100 MHz ticks),
// [PIECE..PIECE+PIECES) summed wave ticks per piece.
#define LPC_STATS_HIST 8
#define LPC_STATS_PIECE 32
#define LPC_STATS_PIECES 4096
#define LPC_STATS_CYC (LPC_STATS_PIECE + LPC_STATS_PIECES)   // [CYC]: walk cycles, [CYC + 1]: drain cycles
#define LPC_STATS_WORDS (LPC_STATS_CYC + 8)

// Per-launch device words of the intersect stage (uint32, reset by k_slot_init
// or k_stage_move): [6..13] hand-over queue lengths (k_rootwalk ->
// k_spill level 0 -> level 1 ...), from word 32 the root-item shard counters
// (k_roots*), each on a 128-byte line of its own: a device-scope atomic evicts its
// line from the L2, and one word serialises its atomics (~11 ns each).
#define LPC_MISC_SPILL 6                  // [6 + l]: items queued for hand-over level l (l < 8)
#define LPC_Q_CSHARDS 8                   // root-item shards (k_roots* block b -> b % 8)
#define LPC_Q_NINIT(c) (32 * (1 + (c)))   // root items k_roots* wrote into shard c
#define LPC_MISC_WORDS (32 * (1 + LPC_Q_CSHARDS))

// Root items of the intersect stage (k_roots* -> k_rootwalk).  An item is one
// packet (64 rays of the coherence order) against one subtree of a mesh run,
// packed in 64 bits: packet (24 bits) | node (28 bits) | slot (12 bits).  k_roots*
// write the (packet, piece root) pairs whose root test some ray passes (the test
// each walk item starts with); k_rootwalk walks them grid-stride.
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
    uint32_t *ctl;                    // misc words (LPC_Q_NINIT)
    uint32_t *err;                    // DevAcc::qerr: set if a shard overflows rcap (never expected; the
                                      //   host then reports the launch as incomplete instead of losing hits)
    uint32_t rcap;
};
// root shard of a k_roots* block
__host__ __device__ inline int q_shard(uint32_t block) { return (int)(block % LPC_Q_CSHARDS); }

// Work hand-over: a walk wave that has visited `budget` nodes with two or
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
    uint32_t *tmask;                  // per ray: bit j set when a flush wrote slot j (NULL: not kept)
    const uint8_t *fan;               // profiling (PROF): triangles with a vertex shared by >= 32 others
};

struct RaysIn {                       // a ray population (SoA)
    const float *ox, *oy, *oz, *dx, *dy, *dz, *pw;
    const int32_t *pmid;              // previous intersected mesh (-2 emitted, -1 outside)
};
struct RaysOut {
    float *ox, *oy, *oz, *dx, *dy, *dz, *pw;
    int32_t *pmid;
};

// The sliver-list tests of one launch (k_slivers, or k_rootwalk's tail when
// merged: LPC_SLIVER_MERGE).  Device-sized launches (nd) read n and max |D|^2
// (dm2d) on the device.  nsp = 0: no sliver work.
struct SliverArgs {
    RaysIn R;
    const float *rs;
    int64_t n;
    const int32_t *perm;
    const lpc::PacketRec *pk;
    const lpc::SliverRec *srec;
    const Piece *pieces;
    int nsp;                          // sliver pieces of the launch (the prefix its rays can reach)
    int ppw;                          // packets per (wave, piece) unit
    float eps, max_ray_len, dmax;
    unsigned long long *skey;
    int32_t *scnt;
    unsigned long long *stats;
    const long long *nd;
    const unsigned *dm2d;
    uint32_t *tmask;
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
};

#define LPC_MP_MAX 4                      // measure meshes whose power the traced path sums per tile
struct DevAcc {                       // device-side counters of one iteration
    unsigned long long nR, nT;        // kept reflected / refracted (running within iteration)
    unsigned long long m_total;       // measured record length (persistent)
    unsigned long long nM_iter;       // measured this iteration
    double pow_next;                  // float64 sum of kept children power
    unsigned int dmax2_bits;          // max |dir|^2 of kept children (float bits)
    unsigned int qerr;                // a consistency check failed on the device (QueueArgs::err)
    unsigned int seq;                 // host copy only: iteration number, written last (k_scan)
    unsigned int pneg;                // != 0: some kept child's power is negative or NaN (k_count)
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
    uint32_t *tmask;                  // the written-slot masks to clear with the slots (or NULL)
};

struct CompactArgs {
    int64_t n, nb;                    // rays in chunk, 1024-ray tiles
    ShadeOutPtrs o;
    int32_t *blk_cnt;                 // [3][nb]
    long long *blk_off;               // [3][nb]
    double *blk_pow;                  // [nb]
    DevAcc *acc;
    RaysOut nR, nT;                   // next population: reflected block, refracted staging
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
// Device-sized iterations (trace_run's speculative enqueue):
// what the iteration of sequence parity p reads -- its population size, the
// measured record's length before it, its rays' max |D|^2 -- written by the
// previous iteration's k_stage_move (n 0: the trace ended, or a kept direction
// exceeded Dcap: dcap_hit, the host rebuilds the records and re-runs).
struct IterCtl {
    long long n[2];
    unsigned long long m[2];
    unsigned int dm2[2];
    unsigned int dcap_hit;
    unsigned int pad;
};

struct StageArgs {
    ShadeArgs S;                      // shading inputs (S.o unused)
    const long long *nd;              // device-sized launch: S.n read here (NULL: S.n)
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
    uint32_t *tmask;                  // the walk's written-slot masks (only those slots are read), or NULL
    uint32_t *tbox;                   // [ntiles][6] box of the tile's kept children origins (ord_f32 min xyz,
                                      //   max xyz), or NULL: the next population's coherence key box
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
    IterCtl *ctl;                     // NULL, or the next iteration's size is written here
    int par;                          // this iteration's parity in ctl (k_stage_move<true>: ntiles,
                                      //   ngroups and m_base from ctl[par] as well)
    double thr;                       // trace_run's power threshold (-inf: none)
    long long nmax;                   // a device-sized next iteration holds at most this many rays: more
                                      //   kept children -> its size 0 (the host re-runs it host-sized)
    double dcap2;                     // Dcap^2 (1 - 1e-6), check_dcap's bound
    // an iteration in several chunks (population > one chunk): each chunk's launch
    // places its rows after the earlier chunks' -- reflected into popR, refracted
    // into the staging popT (k_append moves them behind all reflected), measured
    // rays after the record -- from the running bases of cbase_in (written by the
    // previous chunk's block 0, ping-pong), and block 0 adds the chunk's counters
    // to the iteration's (acc).  popT == NULL: one chunk, refracted after reflected.
    float *popT;
    int64_t capT;
    const unsigned long long *cbase_in;   // [3] R, T, M bases (first chunk: 0, 0, m_base)
    unsigned long long *cbase_out;
    int first, last;
    const uint32_t *tbox;             // StageArgs::tbox (NULL: no box)
    uint32_t *pbox;                   // [6] the next population's origin box (block 0; chunks combine)
};
// Order-preserving float bits (min / max of the uint = of the float).
__host__ __device__ inline uint32_t ord_f32(float f)
{
    const uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float ord_f32_inv(uint32_t u)
{
    return __builtin_bit_cast(float, (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

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

// set_rays' analysis of the emitted rays (k_ray_scan), read back once.
struct RayScan {
    unsigned long long dmax2_bits;    // max |D|^2 (float64, NaN as +inf): the bits of a non-negative double
    uint32_t diff_o, diff_d;          // != 0: some origin / direction differs from ray 0's
    uint32_t neg_pow;                 // != 0: some power is negative or NaN
    uint32_t pad;
    uint32_t hist[2][256];            // counting-sort hi digits: key bits [8, 16) and [23, 31)
};

}  // namespace lpck
