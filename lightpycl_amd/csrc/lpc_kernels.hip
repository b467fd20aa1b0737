// lpc_kernels.hip -- gfx950 kernels of the LightPyCL per-bounce path.
//
//   k_packet         per-wave bound (origin ball + direction cone) of 64 or 128 rays.
//   k_roots*, k_rootwalk, k_spill
//                    the hot loop (replaces __kernel intersect, .cl:243-289):
//                    (packet, piece) items whose root test passes, walked one
//                    wave each through the piece's sphere hierarchy for 64 rays
//                    at once, per-ray conservative tests, exact Moller-Trumbore
//                    only for candidates -> per-slot nearest hit (64-bit
//                    atomicMin) and hit count; heavy items hand subtrees over
//                    to k_spill levels.
//   k_packet, k_slivers
//                    degenerate "sliver" triangles by a line filter.
//   k_raykey, k_gather_aos
//                    rays into coherence order (key + rocPRIM radix sort).
//   k_slot_init/k_slot_export
//                    per-mesh scratch slots (.cl:260-288): pieces flush their
//                    nearest hit with 64-bit atomicMin (slot_key) and counts
//                    with atomicAdd, so the result is order independent.
//   k_shade          intersect_postproc (.cl:105-240) + reflect_refract_rays
//                    (.cl:346-474) fused, one lane per ray, SoA in / SoA out.
//   k_count/k_scan/k_scatter
//                    on-device compaction of the kept children in the
//                    reference order [reflected ; refracted] (iterative_tracer.py
//                    :366-373), measured-ray record and float64 power sums.
//   k_project_hist   angular/stereographic projection (.cl:488-538) and
//                    np.histogram2d-compatible binning (iterative_tracer.py:534-562).
// Layout in HBM: SoA float/int32 arrays per ray; triangle records AoS (32 B
// filter record, 48 B exact record, 36 B vertices), see DESIGN.md.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "lpc_math.hpp"
#include "lpc_internal.hpp"

using namespace lpc;

typedef float f2 __attribute__((ext_vector_type(2)));

namespace lpck {

// Drain entries whose ray mask has at least this many rays are tested
// triangle-uniform (the record by scalar loads, each lane its own ray, results
// in registers); sparser ones are queued as (triangle, ray) pairs at the leaf
// (round 5 A/B with the pair list: 32 and 40 beat 24 by 1.5 %, 16 lost 4 %).
#ifndef LPC_DRAIN_U
#define LPC_DRAIN_U 32
#endif
// The hierarchy kernels' launch bounds in waves per SIMD (compile-time A/B
// builds, tools/build_variant.py; 5 and 7 measured equal or slower).
#ifndef LPC_WALK_MINB
#define LPC_WALK_MINB 6
#endif

// ---------------------------------------------------------------------------
// Intersection.  Rays are processed in the coherence order (k_raykey + radix
// sort + k_gather); every kernel flushes its per-ray nearest hit and count into
// the per-mesh slots with order-independent atomics (slot_flush), so the kernels
// and their pieces may run in any order:
//   k_rootwalk   a mesh run's sphere hierarchy (filter_test), 64-ray packets;
//   k_packet     per-wave bound of 128 rays (origin ball + direction cone);
//   k_slivers    the runs' slivers: lane-parallel packet_sliver_test, then the
//                per-ray line filter.
// Every filter level is implied by the one below it and the lowest one by the
// exact test (tests/test_filter_superset.py), so the exact Moller-Trumbore test
// sees every pair it would accept: results are bit-exact.
static __device__ __forceinline__ bool any_lane(bool b)
{
    return __builtin_amdgcn_ballot_w64(b) != 0;
}
static __device__ __forceinline__ float bcast(float v, int l)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
static __device__ __forceinline__ int bcasti(int v, int l) { return __builtin_amdgcn_readlane(v, l); }


template <class T>
static __device__ __forceinline__ T wave_red(T v, int op)   // 0 min, 1 max, 2 sum
{
    for (int o = 32; o >= 1; o >>= 1) {
        const T u = __shfl_xor(v, o, 64);
        v = op == 0 ? (u < v ? u : v) : op == 1 ? (u > v ? u : v) : v + u;
    }
    return v;
}

// Packet bound of each wave of 64 * RPL rays (one wave per packet; ray
// w*64*RPL + r*64 + lane on lane `lane`: k_slivers' map for RPL 2).
template <int RPL>
static __device__ __forceinline__ void packet_bound(const RaysIn &R, const float *__restrict__ rs, int64_t n,
                                                    PacketRec *__restrict__ pk, int64_t w, int lane)
{
    int64_t q[RPL];
    for (int r = 0; r < RPL; ++r) {
        const int64_t s = w * 64 * RPL + r * 64 + lane;
        q[r] = s < n ? s : n - 1;
    }
    float o[RPL][3], d[RPL][3];
    for (int r = 0; r < RPL; ++r) {
        if (rs) {
            for (int k = 0; k < 3; ++k) { o[r][k] = rs[k * n + q[r]]; d[r][k] = rs[(3 + k) * n + q[r]]; }
        } else {
            o[r][0] = R.ox[q[r]]; o[r][1] = R.oy[q[r]]; o[r][2] = R.oz[q[r]];
            d[r][0] = R.dx[q[r]]; d[r][1] = R.dy[q[r]]; d[r][2] = R.dz[q[r]];
        }
    }
    float mn[3], mx[3], nrm[RPL][3];
    int fin = 1;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;
    for (int k = 0; k < 3; ++k) {
        mn[k] = o[0][k]; mx[k] = o[0][k];
        for (int r = 1; r < RPL; ++r) { mn[k] = fminf(mn[k], o[r][k]); mx[k] = fmaxf(mx[k], o[r][k]); }
    }
    for (int r = 0; r < RPL; ++r) {
        const float l = sqrtf(d[r][0] * d[r][0] + d[r][1] * d[r][1] + d[r][2] * d[r][2]);
        fin &= (l > 0.0f && l < INFINITY && fabsf(o[r][0] + o[r][1] + o[r][2]) < INFINITY) ? 1 : 0;
        for (int k = 0; k < 3; ++k) nrm[r][k] = d[r][k] / l;
        sx += nrm[r][0]; sy += nrm[r][1]; sz += nrm[r][2];
    }
    for (int k = 0; k < 3; ++k) { mn[k] = wave_red(mn[k], 0); mx[k] = wave_red(mx[k], 1); }
    fin = wave_red(fin, 0);
    sx = wave_red(sx, 2); sy = wave_red(sy, 2); sz = wave_red(sz, 2);
    PacketRec Q;
    packet_centre(mn, mx, Q);
    float rr = 0.0f;
    for (int r = 0; r < RPL; ++r) {
        const float x = o[r][0] - Q.ox, y = o[r][1] - Q.oy, z = o[r][2] - Q.oz;
        rr = fmaxf(rr, sqrtf(x * x + y * y + z * z));
    }
    rr = wave_red(rr, 1);
    packet_finish(rr, sx, sy, sz, Q);
    float ang = packet_angle(nrm[0][0], nrm[0][1], nrm[0][2], Q.ax, Q.ay, Q.az);
    for (int r = 1; r < RPL; ++r)
        ang = fmaxf(ang, packet_angle(nrm[r][0], nrm[r][1], nrm[r][2], Q.ax, Q.ay, Q.az));
    if (!(ang == ang)) ang = INFINITY;
    ang = wave_red(ang, 1);
    packet_angle_finish(ang, fin != 0, Q);
    for (int k = 0; k < 5; ++k) Q.pad[k] = 0;
    if (lane == 0) pk[w] = Q;
}

// nd != NULL: a device-sized launch (the population size read on the device,
// grid-stride over the packets; trace_run's speculative iterations).
template <int RPL>
__global__ __launch_bounds__(256) void k_packet(RaysIn R, const float *__restrict__ rs, int64_t n,
                                                PacketRec *__restrict__ pk, const long long *__restrict__ nd)
{
    if (nd) n = *nd;
    const int lane = threadIdx.x & 63;
    for (int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); w * 64 * RPL < n; w += (int64_t)gridDim.x * 4)
        packet_bound<RPL>(R, rs, n, pk, w, lane);
}

// Per-ray nearest-hit state and its flush into the run's slot (original ray
// index q): only pieces with hits write; atomicMin on slot_key keeps the minimal
// t and, among equal t, the lowest triangle index, so the flush order is free.
// tmask (traced path): the ray's written-slot mask gets the slot's bit, so the
// shading reads only the slots a flush wrote.
static __device__ __forceinline__ void slot_flush(unsigned long long *skey, int32_t *scnt, int64_t o, int64_t q,
                                                  float t, int32_t i, int32_t c, uint32_t *tmask, int32_t slot)
{
    if (c) atomicAdd(&scnt[o + q], c);
    if (i >= 0) atomicMin(&skey[o + q], slot_key(t, i));
    if (tmask && (c || i >= 0)) atomicOr(&tmask[q], 1u << slot);
}

static __device__ __forceinline__ void load_ray(const RaysIn &R, const float *__restrict__ rs, int64_t n, int64_t q,
                                                f3 &O, f3 &D)
{
    if (rs) {
        O = mk3(rs[q], rs[n + q], rs[2 * n + q]);
        D = mk3(rs[3 * n + q], rs[4 * n + q], rs[5 * n + q]);
    } else {
        O = mk3(R.ox[q], R.oy[q], R.oz[q]);
        D = mk3(R.dx[q], R.dy[q], R.dz[q]);
    }
}

// The traversal's rays: one base of 8 equally spaced arrays (a population or
// the coherence copy; fewer kernel arguments and live registers in k_rootwalk /
// k_spill than separate pointers).
struct RayBase {
    const float *b;                   // ox at b, oy at b + s, ... dz at b + 5 s
    int64_t s;
    __device__ __forceinline__ void load(int64_t q, f3 &O, f3 &D) const
    {
        O = mk3(b[q], b[s + q], b[2 * s + q]);
        D = mk3(b[3 * s + q], b[4 * s + q], b[5 * s + q]);
    }
};

// Unit direction for the filter tests (its rounding is inside the filter's
// margin); one definition for every kernel that filters, and k_filter_eval.
static __device__ __forceinline__ void unit_dir(const f3 &D, float &nx, float &ny, float &nz)
{
    const float u = 1.0f / sqrtf(D.x * D.x + D.y * D.y + D.z * D.z);
    nx = D.x * u; ny = D.y * u; nz = D.z * u;
}

// Stack depth per wave (node refs); the host checks every hierarchy fits:
// (W - 1) per level + 1.
#define LPC_STACK 64

// LDS of one wave's traversal: the node stack, the deferred exact tests -- dense
// entries (a triangle and the mask of its >= LPC_DRAIN_U rays) and sparse pairs
// (record << 6 | ray lane, appended at the leaf) -- and the per-ray state.
// LPC_PAIRS keeps the wave at 5376 bytes (6 waves per SIMD are VGPR-bound).
#ifndef LPC_PAIRS
#define LPC_PAIRS 512
#endif
struct WaveLds {
    int32_t stack[LPC_STACK];
    int32_t qidx[64];
    uint64_t qmask[64];
    uint32_t pairs[LPC_PAIRS];
    float ray[6][64];                  // the packet's rays (O, D) for the pairs
    unsigned long long lkey[64];       // per-ray nearest hit (slot_key)
    int32_t lcnt[64];                  // per-ray hit count
};

// Drain a wave's deferred exact tests, folding the results into the per-ray
// accumulators L.lkey / L.lcnt (minimal slot_key(t, idx) for t < max_ray_len, a
// count for every accepted t > eps: mt_accumulate's rule).  Dense entries
// (L.qidx / L.qmask [0, nq)) are tested triangle-uniform (the record by scalar
// loads, each lane its own ray in registers), the sparse pairs (L.pairs [0, np))
// 64 per step, one per lane (record gathered, ray read from L.ray).
// PROF: an exact test's class -- on a fan triangle, wholly behind the ray origin
// (all three vertices at (V - O).D < 0), an accepted hit (t > eps).
struct ExactClass {
    uint32_t fan, behind, hit;
};
static __device__ __forceinline__ void exact_class(ExactClass &c, const uint8_t *__restrict__ fan, int32_t idx,
                                                   const f3 &O, const f3 &D, const ExactRec &x, bool hit)
{
    if (fan && fan[idx]) ++c.fan;
    const float a0 = (x.v0x - O.x) * D.x + (x.v0y - O.y) * D.y + (x.v0z - O.z) * D.z;
    const float a1 = a0 + (x.e1x * D.x + x.e1y * D.y + x.e1z * D.z);
    const float a2 = a0 + (x.e2x * D.x + x.e2y * D.y + x.e2z * D.z);
    if (a0 < 0.0f && a1 < 0.0f && a2 < 0.0f) ++c.behind;
    if (hit) ++c.hit;
}

template <bool PROF>
static __device__ __forceinline__ void drain_queue(WaveLds &L, int32_t &nq, int32_t &np, const bool final,
                                                   const int lane, const uint8_t *__restrict__ fan, ExactClass &xc,
                                                   const ExactRec *__restrict__ xrec, const float eps,
                                                   const float max_ray_len, const unsigned long long key0,
                                                   const f3 &O, const f3 &D, uint32_t &n_pairs, uint32_t &n_exact)
{
    if (nq) {
        const bool ve = lane < nq;
        const int32_t my_idx = ve ? L.qidx[lane] : 0;
        const uint64_t my_mask = ve ? L.qmask[lane] : 0ull;
        auto rl64 = [](uint64_t v, int l) -> uint64_t {
            return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
        };
        // this lane's own ray against each dense triangle, accumulated in
        // registers with the same rule, then into its LDS accumulators (only this
        // lane writes them here; the pairs' LDS atomics come later in this wave's
        // program order)
        unsigned long long ukey = key0;
        int32_t ucnt = 0;
        int32_t idx = __builtin_amdgcn_readfirstlane(my_idx);
        ExactRec x = xrec[idx];
        for (int e = 0; e < nq; ++e) {
            const uint64_t m = rl64(my_mask, e);
            // the next dense entry's record, loaded while this one is tested
            const int32_t nidx = e + 1 < nq ? __builtin_amdgcn_readlane(my_idx, e + 1) : idx;
            const ExactRec nx = xrec[nidx];
            if ((m >> lane) & 1ull) {
                float t;
                const bool hit = mt_exact(O, D, mk3(x.v0x, x.v0y, x.v0z), mk3(x.e1x, x.e1y, x.e1z),
                                          mk3(x.e2x, x.e2y, x.e2z), &t) && t > eps;
                if (hit) {
                    ++ucnt;
                    if (t < max_ray_len) {
                        const unsigned long long k = slot_key(t, x.idx);
                        ukey = k < ukey ? k : ukey;
                    }
                }
                if (PROF) { ++n_exact; exact_class(xc, fan, x.idx, O, D, x, hit); }
            }
            n_pairs += (uint32_t)__builtin_popcountll(m);
            idx = nidx;
            x = nx;
        }
        if (ucnt) {
            L.lcnt[lane] += ucnt;
            const unsigned long long kl = L.lkey[lane];
            L.lkey[lane] = ukey < kl ? ukey : kl;
        }
        nq = 0;
    }
    // a drain inside the walk tests whole steps of 64 pairs and keeps the rest
    // (< 64) for the next one; the final drain tests them all
    const int todo = final ? np : (np & ~63);
    n_pairs += (uint32_t)todo;
    auto pair_test = [&](uint32_t pr, const ExactRec &x) {
        const int32_t idx = x.idx;
        const int r = (int)(pr & 63u);
        const f3 Or = mk3(L.ray[0][r], L.ray[1][r], L.ray[2][r]);
        const f3 Dr = mk3(L.ray[3][r], L.ray[4][r], L.ray[5][r]);
        float t;
        const bool hit = mt_exact(Or, Dr, mk3(x.v0x, x.v0y, x.v0z), mk3(x.e1x, x.e1y, x.e1z),
                                  mk3(x.e2x, x.e2y, x.e2z), &t) && t > eps;
        if (hit) {
            atomicAdd(&L.lcnt[r], 1);
            if (t < max_ray_len) atomicMin(&L.lkey[r], slot_key(t, idx));
        }
        if (PROF) { ++n_exact; exact_class(xc, fan, idx, Or, Dr, x, hit); }
    };
    for (int base = 0; base < todo; base += 64) {
        const int q = base + lane;
        if (q < todo) {
            const uint32_t pr = L.pairs[q];
            pair_test(pr, xrec[(int32_t)(pr >> 6)]);
        }
    }
    const int rest = np - todo;
    if (rest > 0 && todo > 0) {
        const uint32_t v = lane < rest ? L.pairs[todo + lane] : 0u;
        if (lane < rest) L.pairs[lane] = v;
    }
    np = rest;
}

// One packet (64 rays of the coherence order from w*64, one per lane) against
// one piece (a subtree of one mesh run).  The wave walks the subtree with a
// wave-uniform stack in LDS: a node's four children are tested against all 64
// rays (filter form d <= 0, see filter_record; node data wave-uniform through
// the scalar cache); a child node is pushed when any ray passes it, a child
// triangle's (index, lane mask) is queued for the exact test.
// PROF: the profiling counters (compiled out of the default launches: fewer
// live registers in the hot loop).  start: the subtree root (a root item's
// piece, or a k_spill item whose parent passed).
template <int W, bool PROF = false>
static __device__ __forceinline__ void trav_packet(WaveLds &L, const RayBase &ray,
                                                   int64_t n, const int32_t *__restrict__ perm,
                                                   const NodeW<W> *__restrict__ nodes,
                                                   const ExactRec *__restrict__ xrec,
                                                   const int32_t slot, int64_t w, int piece_id, float eps,
                                                   float max_ray_len,
                                                   unsigned long long *__restrict__ skey,
                                                   int32_t *__restrict__ scnt,
                                                   unsigned long long *__restrict__ stats,
                                                   SpillArgs SP, int32_t start)
{
    const int lane = threadIdx.x & 63;
    const int64_t s = w * 64 + lane;
    f3 O, D;
    ray.load(s < n ? s : n - 1, O, D);
    float nx, ny, nz;
    unit_dir(D, nx, ny, nz);
    L.ray[0][lane] = O.x; L.ray[1][lane] = O.y; L.ray[2][lane] = O.z;
    L.ray[3][lane] = D.x; L.ray[4][lane] = D.y; L.ray[5][lane] = D.z;
    const unsigned long long key0 = slot_key(max_ray_len, -1);
    L.lkey[lane] = key0;
    L.lcnt[lane] = 0;

    const uint64_t clk0 = (PROF && stats) ? wall_clock64() : 0;
    int32_t top = 0, nq = 0, np = 0;
    uint32_t n_nodes = 0, n_exact = 0;              // profiling counters (stats != NULL)
    uint32_t n_pairs = 0;                           // exact pairs drained (wave-uniform; hand-over cost)
    ExactClass xc = {0u, 0u, 0u};                   // PROF: exact tests by class (exact_class)
    // Exact tests are deferred: candidate (triangle, ray lanes) entries queue up
    // in LDS; a drain expands them into (triangle, ray) pairs, runs 64 pairs at a
    // time one per lane (exact record gathered, ray read from LDS) and folds the
    // results into the per-ray accumulators with LDS atomics: atomicMin on
    // slot_key(t, idx) for t < max_ray_len and a count for every accepted t > eps,
    // which is mt_accumulate's rule (minimal t, lowest index among equal t).
    uint64_t cyc_drain = 0;                         // PROF: shader-clock cycles in the drains
    const uint64_t cyc0 = (PROF && stats) ? clock64() : 0;
    auto drain = [&](bool final) {
        const uint64_t c0 = (PROF && stats) ? clock64() : 0;
        drain_queue<PROF>(L, nq, np, final, lane, PROF ? SP.fan : nullptr, xc, xrec, eps, max_ray_len, key0, O, D,
                          n_pairs, n_exact);
        if (PROF && stats) cyc_drain += clock64() - c0;
    };
    int budget = SP.budget;
    L.stack[top++] = start;
    while (top > 0) {
        // work hand-over: after `budget` nodes the subtrees left on the stack go
        // to k_spill, one wave each (a wave stuck in a dense region would
        // otherwise be the launch's critical path)
        // cost so far in node-visit units: one visit ~ 32 exact pairs
        if (budget > 0 && (int)(n_nodes + (n_pairs >> SP.pair_shift)) >= budget && top >= 2) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(SP.ctr, (uint32_t)top);
            base = (uint32_t)__builtin_amdgcn_readlane((int)base, 0);
            // top <= LPC_STACK = 64 (the host's depth check): one entry per lane
            if (base + (uint32_t)top <= SP.cap) {
                if (lane < top) {
                    SpillItem it;
                    it.w = (int32_t)w; it.node = L.stack[lane]; it.slot = slot; it.piece = piece_id;
                    SP.items[base + lane] = it;
                }
                top = 0;
                break;
            }
            // queue full: void the part of the range inside it, carry on here
            if (lane < top && base + (uint32_t)lane < SP.cap) SP.items[base + lane].node = -1;
            budget = 0;
        }
        const int32_t node = __builtin_amdgcn_readfirstlane(L.stack[--top]);
        const NodeW<W> N = nodes[node];
        ++n_nodes;
        // the W child tests as packed pairs
        float d[W];
#pragma unroll
        for (int k = 0; k < W; k += 2) {
            const lpc_f2 r = filter_test2(lpc_f2{N.cx[k], N.cx[k + 1]}, lpc_f2{N.cy[k], N.cy[k + 1]},
                                          lpc_f2{N.cz[k], N.cz[k + 1]}, lpc_f2{N.negB[k], N.negB[k + 1]},
                                          lpc_f2{N.negA[k], N.negA[k + 1]}, O.x, O.y, O.z, nx, ny, nz);
            d[k] = r.x;
            d[k + 1] = r.y;
        }
        if (N.ref[0] >= 0) {                       // internal node: children are nodes
#pragma unroll
            for (int k = 0; k < W; ++k)
                if (any_lane(d[k] <= 0.0f)) L.stack[top++] = N.ref[k];
        } else {                                   // leaf: exact records ~ref -> deferred exact tests
            // room for the leaf's W entries / pairs (one drain site per node)
            if (nq > 64 - W || np > LPC_PAIRS - W * (LPC_DRAIN_U - 1)) drain(false);
#pragma unroll
            for (int k = 0; k < W; ++k) {
                const bool pass = d[k] <= 0.0f;
                const uint64_t m = __builtin_amdgcn_ballot_w64(pass);
                if (!m) continue;
                const int c = __builtin_popcountll(m);
                if (c >= LPC_DRAIN_U) {            // dense: one entry, tested triangle-uniform
                    if (lane == 0) { L.qidx[nq] = ~N.ref[k]; L.qmask[nq] = m; }
                    ++nq;
                } else {                           // sparse: one pair per passing ray
                    if (pass)
                        L.pairs[np + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                            ((uint32_t)(~N.ref[k]) << 6) | (uint32_t)lane;
                    np += c;
                }
            }
        }
    }
    drain(true);
    if (PROF && stats) {
        for (int o = 32; o >= 1; o >>= 1) {
            n_exact += __shfl_xor(n_exact, o, 64);
            xc.fan += __shfl_xor(xc.fan, o, 64);
            xc.behind += __shfl_xor(xc.behind, o, 64);
            xc.hit += __shfl_xor(xc.hit, o, 64);
        }
        // packet spread: max angle between a lane's direction and lane 0's
        const float cs = nx * bcast(nx, 0) + ny * bcast(ny, 0) + nz * bcast(nz, 0);
        const float cmin = wave_red(cs, 0);
        if (lane == 0) {
            const uint64_t dt = wall_clock64() - clk0;
            const int b = dt ? min(23, 63 - __builtin_clzll(dt)) : 0;
            if (dt >= (1ull << 16)) {           // tail wave (>= 655 us)
                atomicAdd(&stats[4], 1ull);
                atomicAdd(&stats[5], (unsigned long long)n_nodes);
                atomicAdd(&stats[6], (unsigned long long)(acosf(fminf(1.0f, fmaxf(-1.0f, cmin))) * 1e6f));
                atomicAdd(&stats[7], (unsigned long long)n_exact);
            }
            atomicAdd(&stats[0], (unsigned long long)n_nodes);
            atomicAdd(&stats[LPC_STATS_CYC], (unsigned long long)(clock64() - cyc0));
            atomicAdd(&stats[LPC_STATS_CYC + 1], (unsigned long long)cyc_drain);
            if (xc.fan) atomicAdd(&stats[LPC_STATS_CYC + 2], (unsigned long long)xc.fan);
            if (xc.behind) atomicAdd(&stats[LPC_STATS_CYC + 3], (unsigned long long)xc.behind);
            if (xc.hit) atomicAdd(&stats[LPC_STATS_CYC + 4], (unsigned long long)xc.hit);
            atomicAdd(&stats[2], 1ull);
            atomicAdd(&stats[3], (unsigned long long)n_exact);
            atomicAdd(&stats[LPC_STATS_HIST + b], 1ull);
            if (piece_id < LPC_STATS_PIECES) atomicAdd(&stats[LPC_STATS_PIECE + piece_id], (unsigned long long)dt);
        }
    }
    if (s < n) {
        const unsigned long long k = L.lkey[lane];
        const int32_t c = L.lcnt[lane];
        const int64_t o = (int64_t)slot * n, q = perm ? perm[s] : s;
        if (c) atomicAdd(&scnt[o + q], c);
        if (k != key0) atomicMin(&skey[o + q], k);
        if (SP.tmask && (c || k != key0)) atomicOr(&SP.tmask[q], 1u << slot);
    }
}

// k_spill: the subtrees handed over by the previous level (queue `in`), one item
// per wave, grid-stride over the queue (its length is read on the device).  An
// item that again exceeds the budget hands its remaining subtrees to the next
// level's queue (`out`; budget 0 on the last level).  One wave per block (a
// wave's slot frees when its items end, see k_rootwalk).
template <int W, bool PROF = false>
__global__ __launch_bounds__(64, LPC_WALK_MINB) void k_spill(RayBase ray, int64_t n,
                                               const int32_t *__restrict__ perm, const NodeW<W> *__restrict__ nodes,
                                               const ExactRec *__restrict__ xrec, float eps, float max_ray_len,
                                               unsigned long long *__restrict__ skey, int32_t *__restrict__ scnt,
                                               unsigned long long *__restrict__ stats, SpillArgs SP,
                                               SpillArgs out, const long long *__restrict__ nd)
{
    __shared__ WaveLds lds;
    if (nd) n = *nd;
    const uint32_t total = min(*SP.ctr, SP.cap);
    const uint32_t stride = gridDim.x;
    for (uint32_t it = blockIdx.x; it < total; it += stride) {
        const SpillItem I = SP.items[it];
        if (I.node < 0) continue;
        trav_packet<W, PROF>(lds, ray, n, perm, nodes, xrec, I.slot, I.w, I.piece, eps, max_ray_len, skey, scnt,
                             stats, out, I.node);
    }
}

// k_roots_s: the root items, one per (packet, piece) whose root test some ray of
// the packet passes (lanes = a packet's rays), as tasks: a block takes
// pb packets, task t = (packet t / S, piece class t % S) tests the pieces
// p = class + S k (npieces <= 64 S), the block's 4 waves take the tasks in turn,
// and the block reserves all its items with one atomic.  Small populations (few
// packets) get S = 2..4 waves per packet instead of one wave looping over every
// piece; large ones several packets per atomic.
// Gated form (ngroups > 0: pieces cut below the run roots): a task first tests
// the runs' root records (`groups`, s_lo/s_hi = the run's range of pieces) and
// then only the pieces of runs some ray of the packet passes.  Exact: a ray whose
// line Moller-Trumbore accepts against a triangle passes every test above it
// (node_record of all triangles below), the run root's included, so a piece of a
// run no ray passes holds no accepted pair for the packet.
// Piece records are wave-uniform (scalar loads); a lane accumulates its own
// pass bits and the wave ORs them once per task (no ballot per test).
#define LPC_ROOTS_TASKS 16
static __device__ __forceinline__ uint64_t wave_or64(uint64_t v)
{
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    for (int o = 32; o >= 1; o >>= 1) {
        lo |= (uint32_t)__shfl_xor((int)lo, o, 64);
        hi |= (uint32_t)__shfl_xor((int)hi, o, 64);
    }
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)hi) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)lo);
}

// Grid-stride over the virtual blocks (pb packets each; device-sized launches
// read n on the device, nd != NULL).
// The root tests' records in LDS (cx cy cz negB | negA): the piece loop reads
// them with broadcast LDS loads instead of one scalar-load round trip per piece.
struct RootsLds {
    float4 pc[LPC_ROOTS_TASKS * 64];
    float pa[LPC_ROOTS_TASKS * 64];
    float4 gc[64];
    float ga[64];
};

template <bool HALF>
static __device__ __forceinline__ void roots_block(const RaysIn &R, const float *__restrict__ rs, int64_t n,
                                                   const Piece *__restrict__ pieces, int npieces,
                                                   const Piece *__restrict__ groups, int ngroups, const QueueArgs &Q,
                                                   int S, int pb, int64_t vb, unsigned long long *s_m,
                                                   uint32_t *s_off, const RootsLds &L);

template <bool HALF>
__global__ __launch_bounds__(256) void k_roots_s(RaysIn R, const float *__restrict__ rs, int64_t n,
                                                 const Piece *__restrict__ pieces, int npieces,
                                                 const Piece *__restrict__ groups, int ngroups, QueueArgs Q,
                                                 int S, int pb, const long long *__restrict__ nd)
{
    __shared__ unsigned long long s_m[LPC_ROOTS_TASKS];
    __shared__ uint32_t s_off[LPC_ROOTS_TASKS + 1];
    __shared__ RootsLds L;
    if (nd) n = *nd;
    for (int i = threadIdx.x; i < npieces; i += 256) {
        const Piece &P = pieces[i];
        L.pc[i] = make_float4(P.cx, P.cy, P.cz, P.negB);
        L.pa[i] = P.negA;
    }
    for (int i = threadIdx.x; i < ngroups; i += 256) {
        const Piece &G = groups[i];
        L.gc[i] = make_float4(G.cx, G.cy, G.cz, G.negB);
        L.ga[i] = G.negA;
    }
    __syncthreads();
    const int64_t nvb = ((n + 63) / 64 + pb - 1) / pb;
    for (int64_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
        roots_block<HALF>(R, rs, n, pieces, npieces, groups, ngroups, Q, S, pb, vb, s_m, s_off, L);
        __syncthreads();                          // s_m / s_off reused by the next virtual block
    }
}

template <bool HALF>
static __device__ __forceinline__ void roots_block(const RaysIn &R, const float *__restrict__ rs, int64_t n,
                                                   const Piece *__restrict__ pieces, int npieces,
                                                   const Piece *__restrict__ groups, int ngroups, const QueueArgs &Q,
                                                   int S, int pb, int64_t vb, unsigned long long *s_m,
                                                   uint32_t *s_off, const RootsLds &L)
{
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int c = q_shard((uint32_t)vb);
    const int ntask = S * pb;
    for (int t = wv; t < ntask; t += 4) {
        const int64_t w = vb * pb + t / S;
        const int cls = t % S;
        uint64_t m = 0;
        if (w * 64 < n) {
            const int64_t s = w * 64 + lane;
            f3 O, D;
            load_ray(R, rs, n, s < n ? s : n - 1, O, D);
            float nx, ny, nz;
            unit_dir(D, nx, ny, nz);
            uint64_t ml = 0;                    // this lane's ray: bit k = piece cls + S k passes
            auto test = [&](int lo, int hi) {   // the class's pieces in [lo, hi)
                const int p0 = lo + ((cls - lo % S) % S + S) % S;
                int p = p0, k = p0 / S;
                // two pieces per packed-FP32 test (each half one evaluation of the
                // scalar test's formula: the same conservative filter)
#pragma unroll 2
                for (; p + S < hi; p += 2 * S, k += 2) {
                    const float4 c0 = L.pc[p], c1 = L.pc[p + S];
                    const lpc_f2 cx = {c0.x, c1.x}, cy = {c0.y, c1.y}, cz = {c0.z, c1.z}, nb = {c0.w, c1.w};
                    const lpc_f2 na = {L.pa[p], L.pa[p + S]};
                    const lpc_f2 d = HALF ? filter_test2h(cx, cy, cz, nb, na, O.x, O.y, O.z, nx, ny, nz)
                                          : filter_test2(cx, cy, cz, nb, na, O.x, O.y, O.z, nx, ny, nz);
                    ml |= ((uint64_t)(d.x <= 0.0f) << k) | ((uint64_t)(d.y <= 0.0f) << (k + 1));
                }
                if (p < hi) {
                    const float4 c = L.pc[p];
                    const float a = L.pa[p];
                    const float d = HALF ? filter_testh(c.x, c.y, c.z, c.w, a, O.x, O.y, O.z, nx, ny, nz)
                                         : filter_test(c.x, c.y, c.z, c.w, a, O.x, O.y, O.z, nx, ny, nz);
                    ml |= (uint64_t)(d <= 0.0f) << k;
                }
            };
            if (ngroups > 0) {
                uint64_t gl = 0;
#pragma unroll 4
                for (int g = 0; g < ngroups; ++g) {
                    const float4 c = L.gc[g];
                    const float d = filter_test(c.x, c.y, c.z, c.w, L.ga[g], O.x, O.y, O.z, nx, ny, nz);
                    gl |= (uint64_t)(d <= 0.0f) << g;
                }
                for (uint64_t gm = wave_or64(gl); gm; gm &= gm - 1) {
                    const int g = __builtin_ctzll(gm);
                    test(groups[g].s_lo, groups[g].s_hi);
                }
            } else {
                test(0, npieces);
            }
            m = wave_or64(ml);
        }
        if (lane == 0) s_m[t] = m;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int t = 0; t < ntask; ++t) { s_off[t] = tot; tot += (uint32_t)__builtin_popcountll(s_m[t]); }
        s_off[ntask] = tot ? atomicAdd(Q.ctl + LPC_Q_NINIT(c), tot) : 0u;
    }
    __syncthreads();
    const uint32_t base = s_off[ntask];
    for (int t = wv; t < ntask; t += 4) {
        const uint64_t m = s_m[t];
        if (!((m >> lane) & 1ull)) continue;
        const int64_t w = vb * pb + t / S;
        const int p = t % S + S * lane;
        const uint32_t pos = base + s_off[t] + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (pos < Q.rcap)
            Q.roots[(size_t)c * Q.rcap + pos] = q_item((uint32_t)w, (uint32_t)pieces[p].root, (uint32_t)pieces[p].slot);
        else
            atomicOr(Q.err, 2u);                  // would be lost: the host reports the launch
    }
}

static __device__ __forceinline__ void sliver_group(const SliverArgs &A, int64_t n, float dmax, int64_t w0,
                                                    int64_t w1, int piece);
static __device__ __forceinline__ void sliver_launch_size(const SliverArgs &A, int64_t &n, float &dmax);

// k_rootwalk: the root items (k_roots_s / k_gather_roots: the (packet, piece)
// pairs whose root test some ray of the packet passes), grid-stride, one item per
// wave at a time.  A wave that exceeds the hand-over budget queues its remaining
// subtrees for k_spill (`out`).
// One wave per block: a block's slots free as soon as its item ends, where a
// 4-wave block holds its LDS until its slowest item ends (round 2 per-item
// records: ~2 800 of 6 144 wave slots walking on average with 4).
template <int W, bool PROF = false, bool MERGED = false>
__global__ __launch_bounds__(64, LPC_WALK_MINB) void k_rootwalk(RayBase ray, int64_t n,
                                                     const int32_t *__restrict__ perm,
                                                     const NodeW<W> *__restrict__ nodes,
                                                     const ExactRec *__restrict__ xrec, float eps, float max_ray_len,
                                                     unsigned long long *__restrict__ skey, int32_t *__restrict__ scnt,
                                                     unsigned long long *__restrict__ stats, QueueArgs Q,
                                                     SpillArgs out, const long long *__restrict__ nd,
                                                     SliverArgs SA)
{
    __shared__ WaveLds lds;
    if (nd) n = *nd;
    // the shards' item prefix in LDS: a register array indexed by a loop variable
    // would hold 9 VGPRs for the whole walk (the walk then spills at 6 waves/SIMD)
    __shared__ uint32_t s_pre[LPC_Q_CSHARDS + 1];
    if (threadIdx.x == 0) {
        uint32_t p = 0;
        s_pre[0] = 0;
#pragma unroll
        for (int c = 0; c < LPC_Q_CSHARDS; ++c) { p += min(Q.ctl[LPC_Q_NINIT(c)], Q.rcap); s_pre[c + 1] = p; }
    }
    __syncthreads();
    const uint32_t stride = gridDim.x, iend = s_pre[LPC_Q_CSHARDS];
    for (uint32_t i = blockIdx.x; i < iend; i += stride) {
        int c = 0;
        while (i >= s_pre[c + 1]) ++c;
        const uint64_t it = Q.roots[(size_t)c * Q.rcap + (i - s_pre[c])];
        const int32_t slot = (int32_t)q_slot(it);
        trav_packet<W, PROF>(lds, ray, n, perm, nodes, xrec, slot, (int64_t)q_w(it), slot, eps, max_ray_len, skey,
                             scnt, stats, out, (int32_t)q_node(it));
    }
    // merged sliver tests (LPC_SLIVER_MERGE): (packet group, sliver piece) units
    // grid-stride after the root items, so the waves whose items end early take
    // them -- no second stream whose long-lived waves would hold the CUs
    if (MERGED && SA.nsp > 0) {
        int64_t ns;
        float dmax;
        sliver_launch_size(SA, ns, dmax);
        const int64_t npk = (ns + 127) / 128, ppw = SA.ppw;
        const int64_t units = ((npk + ppw - 1) / ppw) * SA.nsp;
        for (int64_t u = blockIdx.x; u < units; u += stride) {
            const int64_t g = u / SA.nsp;
            const int64_t w0 = g * ppw;
            sliver_group(SA, ns, dmax, w0, min(w0 + ppw, npk), (int)(u - g * SA.nsp));
        }
    }
}

// k_slivers: the run's slivers (line filter) for packets of 128 rays (two per
// lane), grid = (ceil(n / (512 ppw)), sliver pieces of <= 64 slivers): a wave
// holds its piece's slivers one per lane and takes ppw consecutive packets in
// turn: lane-parallel packet_sliver_test against the packet's PacketRec (scalar
// loads), then, for the slivers that pass, the per-ray line filter and the exact
// test.  Most (packet, piece) pairs fail the packet test, so a wave's fixed cost
// (sliver records, loop setup) is spread over ppw packets.
// Device-sized launch (nd != NULL): the population size and its max |D|^2 (dm2d,
// float bits) read on the device, ppw = the packets over the grid's waves, and
// every sliver piece in grid.y (a piece whose slivers no ray can pass exits).
// One wave: packets [w0, w1) of 128 rays against sliver piece `piece`.
static __device__ __forceinline__ void sliver_group(const SliverArgs &A, int64_t n, float dmax, int64_t w0,
                                                    int64_t w1, int piece)
{
    const int lane = threadIdx.x & 63;
    const Piece P = A.pieces[piece];
    const int32_t j = P.s_lo + lane;
    SliverRec S;
    if (j < P.s_hi) S = A.srec[j];
    else { memset(&S, 0, sizeof(S)); S.a = NAN; S.idx = -1; }
    if (!(S.dmin <= dmax)) S.a = NAN;             // no ray of the launch can pass its DEN test
    if (!any_lane(S.a == S.a)) return;            // the whole piece culled
    const int64_t o = (int64_t)P.slot * n;
    const float eps = A.eps, max_ray_len = A.max_ray_len;
    uint32_t n_tests = 0, n_exact = 0;
    for (int64_t w = w0; w < w1; ++w) {
        const PacketRec Q = A.pk[w];
        uint64_t m = __builtin_amdgcn_ballot_w64(packet_sliver_test(Q, S));
        if (!m) continue;
        const int64_t s0 = w * 128 + lane, s1 = s0 + 64;
        f3 O0, O1, D0, D1;
        load_ray(A.R, A.rs, n, s0 < n ? s0 : n - 1, O0, D0);
        load_ray(A.R, A.rs, n, s1 < n ? s1 : n - 1, O1, D1);
        const f2 ox = {O0.x, O1.x}, oy = {O0.y, O1.y}, oz = {O0.z, O1.z};
        const f2 dx = {D0.x, D1.x}, dy = {D0.y, D1.y}, dz = {D0.z, D1.z};
        const f2 dl = {sqrtf(D0.x * D0.x + D0.y * D0.y + D0.z * D0.z), sqrtf(D1.x * D1.x + D1.y * D1.y + D1.z * D1.z)};
        float t0 = max_ray_len, t1 = max_ray_len;
        int32_t i0 = -1, i1 = -1, c0 = 0, c1 = 0;
        while (m) {
            const int k = __builtin_ctzll(m);
            m &= m - 1;
            const float v0x = bcast(S.v0x, k), v0y = bcast(S.v0y, k), v0z = bcast(S.v0z, k);
            const float e2x = bcast(S.e2x, k), e2y = bcast(S.e2y, k), e2z = bcast(S.e2z, k);
            const float sa = bcast(S.a, k), sbb = bcast(S.b, k);
            const f2 tx = ox - v0x, ty = oy - v0y, tz = oz - v0z;
            const f2 cx = e2y * tz - e2z * ty;
            const f2 cy = e2z * tx - e2x * tz;
            const f2 cz = e2x * ty - e2y * tx;
            const f2 x = dx * cx + dy * cy + dz * cz;
            const f2 tm = {fmaxf(fmaxf(fabsf(tx.x), fabsf(ty.x)), fabsf(tz.x)),
                           fmaxf(fmaxf(fabsf(tx.y), fabsf(ty.y)), fabsf(tz.y))};
            const f2 rhs = dl * (sa + sbb * tm);
            const f2 d = x * x - rhs * rhs;
            ++n_tests;
            const bool r0 = d.x <= 0.0f, r1 = d.y <= 0.0f;
            if (!any_lane(r0 || r1)) continue;
            const int32_t idx = bcasti(S.idx, k);
            const f3 V0 = mk3(v0x, v0y, v0z);
            // a thin triangle's filter edge is E1 (ax1): the exact record in its order
            const f3 Ea = mk3(e2x, e2y, e2z), Eb = mk3(bcast(S.e1x, k), bcast(S.e1y, k), bcast(S.e1z, k));
            const bool ax1 = bcasti(S.ax1, k) != 0;
            const f3 E1 = ax1 ? Ea : Eb, E2 = ax1 ? Eb : Ea;
            if (r0) mt_accumulate(O0, D0, V0, E1, E2, idx, eps, t0, i0, c0);
            if (r1) mt_accumulate(O1, D1, V0, E1, E2, idx, eps, t1, i1, c1);
            n_exact += (uint32_t)r0 + (uint32_t)r1;
        }
        if (s0 < n) slot_flush(A.skey, A.scnt, o, A.perm ? A.perm[s0] : s0, t0, i0, c0, A.tmask, P.slot);
        if (s1 < n) slot_flush(A.skey, A.scnt, o, A.perm ? A.perm[s1] : s1, t1, i1, c1, A.tmask, P.slot);
    }
    if (A.stats) {
        for (int q = 32; q >= 1; q >>= 1) n_exact += __shfl_xor(n_exact, q, 64);
        if (lane == 0) {
            atomicAdd(&A.stats[1], (unsigned long long)n_tests);
            atomicAdd(&A.stats[3], (unsigned long long)n_exact);
        }
    }
}

// The launch's n and max |D| (device-sized: from the device, as run_intersect
// computes them on the host).
static __device__ __forceinline__ void sliver_launch_size(const SliverArgs &A, int64_t &n, float &dmax)
{
    n = A.n;
    dmax = A.dmax;
    if (A.nd) {
        n = *A.nd;
        const double d2 = (double)__uint_as_float(*A.dm2d);
        dmax = d2 >= 0.0 ? (float)fmin(sqrt(d2 * (1.0 + 1e-5)), (double)INFINITY) : INFINITY;
    }
}

__global__ __launch_bounds__(256) void k_slivers(SliverArgs A)
{
    int64_t n;
    float dmax;
    sliver_launch_size(A, n, dmax);
    int64_t ppw = A.ppw;
    if (A.nd) ppw = max((int64_t)1, ((n + 127) / 128 + (int64_t)gridDim.x * 4 - 1) / ((int64_t)gridDim.x * 4));
    const int64_t npk = (n + 127) / 128;
    const int64_t w0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * ppw;
    if (w0 >= npk) return;
    sliver_group(A, n, dmax, w0, min(w0 + ppw, npk), (int)blockIdx.y);
}

// k_gather from the 32-byte rows k_raykey wrote: one cache line per ray instead
// of one per component (the permutation is random with respect to memory).
// full: also the power and previous mesh (the rows' last two words, k_raykey),
// so the copy is a whole population in coherence order (traced mode).
__global__ __launch_bounds__(256) void k_gather_aos(const float4 *__restrict__ aos, int64_t n,
                                                    const int32_t *__restrict__ perm, float *__restrict__ rs, int full)
{
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const int64_t q = perm[s];
    const float4 a = aos[2 * q], b = aos[2 * q + 1];
    rs[s] = a.x; rs[n + s] = a.y; rs[2 * n + s] = a.z;
    rs[3 * n + s] = a.w; rs[4 * n + s] = b.x; rs[5 * n + s] = b.y;
    if (full) { rs[6 * n + s] = b.z; rs[7 * n + s] = b.w; }
}

// k_gather_aos with the root tests of k_roots_s fused in (one task per packet:
// at most 64 pieces, no run gate): 16 packets per 1024-thread block, each wave
// gathers its packet's 64 rays and tests them against the pieces from the rows
// it just read (the values k_roots_s would load from the gathered copy), then the
// block reserves its items with one atomic, as k_roots_s does.  Lanes past n add
// nothing (k_roots_s tests ray n - 1 there, which its own lane already covers).
template <bool HALF>
__global__ __launch_bounds__(1024) void k_gather_roots(const float4 *__restrict__ aos, int64_t n,
                                                       const int32_t *__restrict__ perm, float *__restrict__ rs,
                                                       int full, const Piece *__restrict__ pieces, int npieces,
                                                       QueueArgs Q)
{
    __shared__ float4 s_pc[64];
    __shared__ float s_pa[64];
    __shared__ unsigned long long s_m[16];
    __shared__ uint32_t s_off[17];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((int)threadIdx.x < npieces) {
        const Piece &P = pieces[threadIdx.x];
        s_pc[threadIdx.x] = make_float4(P.cx, P.cy, P.cz, P.negB);
        s_pa[threadIdx.x] = P.negA;
    }
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = s < n;
    float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b = a;
    if (in) {
        const int64_t q = perm[s];
        a = aos[2 * q];
        b = aos[2 * q + 1];
        rs[s] = a.x; rs[n + s] = a.y; rs[2 * n + s] = a.z;
        rs[3 * n + s] = a.w; rs[4 * n + s] = b.x; rs[5 * n + s] = b.y;
        if (full) { rs[6 * n + s] = b.z; rs[7 * n + s] = b.w; }
    }
    __syncthreads();
    const int64_t w = (int64_t)blockIdx.x * nw + wv;       // this wave's packet
    uint64_t ml = 0;
    if (in) {
        const f3 O = mk3(a.x, a.y, a.z), D = mk3(a.w, b.x, b.y);
        float nx, ny, nz;
        unit_dir(D, nx, ny, nz);
        int p = 0;
        for (; p + 1 < npieces; p += 2) {
            const float4 c0 = s_pc[p], c1 = s_pc[p + 1];
            const lpc_f2 cx = {c0.x, c1.x}, cy = {c0.y, c1.y}, cz = {c0.z, c1.z}, nb = {c0.w, c1.w};
            const lpc_f2 na = {s_pa[p], s_pa[p + 1]};
            const lpc_f2 d = HALF ? filter_test2h(cx, cy, cz, nb, na, O.x, O.y, O.z, nx, ny, nz)
                                  : filter_test2(cx, cy, cz, nb, na, O.x, O.y, O.z, nx, ny, nz);
            ml |= ((uint64_t)(d.x <= 0.0f) << p) | ((uint64_t)(d.y <= 0.0f) << (p + 1));
        }
        if (p < npieces) {
            const float4 c = s_pc[p];
            const float d = HALF ? filter_testh(c.x, c.y, c.z, c.w, s_pa[p], O.x, O.y, O.z, nx, ny, nz)
                                 : filter_test(c.x, c.y, c.z, c.w, s_pa[p], O.x, O.y, O.z, nx, ny, nz);
            ml |= (uint64_t)(d <= 0.0f) << p;
        }
    }
    const uint64_t m = wave_or64(ml);
    if (lane == 0) s_m[wv] = m;
    __syncthreads();
    const int c = q_shard((uint32_t)blockIdx.x);
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int k = 0; k < nw; ++k) { s_off[k] = tot; tot += (uint32_t)__builtin_popcountll(s_m[k]); }
        s_off[nw] = tot ? atomicAdd(Q.ctl + LPC_Q_NINIT(c), tot) : 0u;
    }
    __syncthreads();
    if ((m >> lane) & 1ull) {
        const uint32_t pos = s_off[nw] + s_off[wv] + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (pos < Q.rcap)
            Q.roots[(size_t)c * Q.rcap + pos] = q_item((uint32_t)w, (uint32_t)pieces[lane].root,
                                                       (uint32_t)pieces[lane].slot);
        else
            atomicOr(Q.err, 2u);
    }
}

// Slot initial state: slots a run flushes into start at (max_ray_len, idx -1,
// count 0); slots no run writes keep the reference's initial scratch
// (max_ray_len, idx 0, count 0).  Also empties the launch's origin box (misc).
// (also, when SI.acc != NULL, the iteration counters: k_acc_init folded in)
static __device__ __forceinline__ void slot_init_ray(const SlotInit &SI, int64_t n, int64_t r)
{
    if (SI.misc && r < LPC_MISC_WORDS) SI.misc[r] = r < 3 ? 0xffffffffu : 0u;
    if (SI.acc && r == 0) {
        DevAcc z;
        memset(&z, 0, sizeof(z));
        z.m_total = SI.m_total;
        *SI.acc = z;
    }
    if (r >= n || !SI.skey) return;
    if (SI.tmask) SI.tmask[r] = 0u;
    for (int32_t j = 0; j < SI.K; ++j) {
        SI.skey[(int64_t)j * n + r] = slot_key(SI.max_ray_len, (SI.uniform || SI.live[j]) ? -1 : 0);
        SI.scnt[(int64_t)j * n + r] = 0;
    }
}

__global__ __launch_bounds__(256) void k_slot_init(int64_t n, SlotInit SI)
{
    slot_init_ray(SI, n, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// Drop-in export of the slots to the reference's scratch buffers
// (isect_min_ray_len / ray_isect_mesh_idx_tmp / isects_count, [ray][mesh]).
// keep_unwritten: slots no run writes are left as the caller had them.
__global__ __launch_bounds__(256) void k_slot_export(int64_t n, int32_t K, const int32_t *__restrict__ live,
                                                     const unsigned long long *__restrict__ skey,
                                                     const int32_t *__restrict__ scnt, float *__restrict__ st,
                                                     int32_t *__restrict__ si, int32_t *__restrict__ sc,
                                                     int keep_unwritten)
{
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    for (int32_t j = 0; j < K; ++j) {
        if (!live[j] && keep_unwritten) continue;
        const unsigned long long k = skey[(int64_t)j * n + r];
        const int64_t a = r * K + j;
        st[a] = slot_key_t(k); si[a] = slot_key_idx(k); sc[a] = scnt[(int64_t)j * n + r];
    }
}

// Ray coherence key: 15-bit Morton code of the origin cell (32^3 grid) above a
// 16-bit Morton code of the octahedral-mapped direction.
static __device__ __forceinline__ uint32_t spread2(uint32_t x)   // 8 bits -> even bits
{
    x &= 0xff;
    x = (x | (x << 4)) & 0x0f0f;
    x = (x | (x << 2)) & 0x3333;
    x = (x | (x << 1)) & 0x5555;
    return x;
}
static __device__ __forceinline__ uint32_t spread3(uint32_t x)   // 5 bits -> every third bit
{
    x &= 0x1f;
    x = (x | (x << 8)) & 0x100f;
    x = (x | (x << 4)) & 0x10c3;
    x = (x | (x << 2)) & 0x1249;
    return x;
}

// Key = [origin cell 15 bits][direction 16 bits] over the scene box (bx0.., sx..).
static __device__ __forceinline__ uint32_t raykey_ray(const RaysIn &R, int64_t i, float bx0, float by0, float bz0,
                                                      float sx, float sy, float sz, float4 *__restrict__ aos)
{
    if (aos) {          // the ray as one 32-byte row: k_gather_aos reads it with one line per ray
        aos[2 * i] = make_float4(R.ox[i], R.oy[i], R.oz[i], R.dx[i]);
        aos[2 * i + 1] = make_float4(R.dy[i], R.dz[i], R.pw ? R.pw[i] : 0.0f,
                                     R.pmid ? __int_as_float(R.pmid[i]) : 0.0f);
    }
    const float dx = R.dx[i], dy = R.dy[i], dz = R.dz[i];
    const float l1 = fabsf(dx) + fabsf(dy) + fabsf(dz);
    float px = l1 > 0.0f ? dx / l1 : 0.0f, py = l1 > 0.0f ? dy / l1 : 0.0f;
    if (dz < 0.0f) {
        const float tx = (1.0f - fabsf(py)) * (px >= 0.0f ? 1.0f : -1.0f);
        const float ty = (1.0f - fabsf(px)) * (py >= 0.0f ? 1.0f : -1.0f);
        px = tx; py = ty;
    }
    const uint32_t du = (uint32_t)fminf(fmaxf((px * 0.5f + 0.5f) * 256.0f, 0.0f), 255.0f);
    const uint32_t dv = (uint32_t)fminf(fmaxf((py * 0.5f + 0.5f) * 256.0f, 0.0f), 255.0f);
    const uint32_t ox = (uint32_t)fminf(fmaxf((R.ox[i] - bx0) * sx, 0.0f), 31.0f);
    const uint32_t oy = (uint32_t)fminf(fmaxf((R.oy[i] - by0) * sy, 0.0f), 31.0f);
    const uint32_t oz = (uint32_t)fminf(fmaxf((R.oz[i] - bz0) * sz, 0.0f), 31.0f);
    const uint32_t okey = spread3(ox) | (spread3(oy) << 1) | (spread3(oz) << 2);
    const uint32_t dkey = spread2(du) | (spread2(dv) << 1);
    return (okey << 16) | dkey;
}

// Key with ob origin bits per axis and db direction bits per octahedral axis
// (3 ob + 2 db <= 32), Morton-interleaved, origin cells above direction: the
// re-sorted chained populations' key in their own box (LPC_KEY_OBITS).
static __device__ __forceinline__ uint32_t raykey_ray_bits(const RaysIn &R, int64_t i, float bx0, float by0,
                                                           float bz0, float sx, float sy, float sz, int ob, int db,
                                                           int mode)
{
    const float dx = R.dx[i], dy = R.dy[i], dz = R.dz[i];
    const float l1 = fabsf(dx) + fabsf(dy) + fabsf(dz);
    float px = l1 > 0.0f ? dx / l1 : 0.0f, py = l1 > 0.0f ? dy / l1 : 0.0f;
    if (dz < 0.0f) {
        const float tx = (1.0f - fabsf(py)) * (px >= 0.0f ? 1.0f : -1.0f);
        const float ty = (1.0f - fabsf(px)) * (py >= 0.0f ? 1.0f : -1.0f);
        px = tx; py = ty;
    }
    const float dn = (float)(1 << db), on = (float)(1 << ob), sc = on / 32.0f;
    const uint32_t du = (uint32_t)fminf(fmaxf((px * 0.5f + 0.5f) * dn, 0.0f), dn - 1.0f);
    const uint32_t dv = (uint32_t)fminf(fmaxf((py * 0.5f + 0.5f) * dn, 0.0f), dn - 1.0f);
    const uint32_t o[3] = {(uint32_t)fminf(fmaxf((R.ox[i] - bx0) * sx * sc, 0.0f), on - 1.0f),
                           (uint32_t)fminf(fmaxf((R.oy[i] - by0) * sy * sc, 0.0f), on - 1.0f),
                           (uint32_t)fminf(fmaxf((R.oz[i] - bz0) * sz * sc, 0.0f), on - 1.0f)};
    if (mode == 1) {    // 5-D Morton: origin and direction bits interleaved from the top
        uint32_t key = 0;
        int pos = 3 * ob + 2 * db;
        const int top = ob > db ? ob : db;
        for (int b = top - 1; b >= 0; --b) {
            if (b < ob)
                for (int k = 0; k < 3; ++k) key |= ((o[k] >> b) & 1u) << --pos;
            if (b < db) { key |= ((du >> b) & 1u) << --pos; key |= ((dv >> b) & 1u) << --pos; }
        }
        return key;
    }
    uint32_t okey = 0, dkey = 0;
    for (int b = 0; b < ob; ++b)
        for (int k = 0; k < 3; ++k) okey |= ((o[k] >> b) & 1u) << (3 * b + k);
    for (int b = 0; b < db; ++b) dkey |= (((du >> b) & 1u) << (2 * b)) | (((dv >> b) & 1u) << (2 * b + 1));
    if (mode == 2) return (dkey << (3 * ob)) | okey;             // direction-major
    return (okey << (2 * db)) | dkey;
}

__global__ __launch_bounds__(256) void k_raykey(RaysIn R, int64_t n, float bx0, float by0, float bz0,
                                                float sx, float sy, float sz, uint32_t *__restrict__ keys,
                                                int32_t *__restrict__ vals, float4 *__restrict__ aos,
                                                SlotInit SI, const uint32_t *__restrict__ pbox, int obits,
                                                int kmode)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pbox) {         // the population's own origin box (the previous k_stage_move), per axis
        float *b0[3] = {&bx0, &by0, &bz0}, *sc[3] = {&sx, &sy, &sz};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t a = pbox[k], b = pbox[3 + k];
            if (a > b) continue;                 // empty: the scene box
            const float lo = ord_f32_inv(a), ext = ord_f32_inv(b) - lo;
            *b0[k] = lo;
            *sc[k] = (ext > 0.0f && isfinite(ext)) ? 32.0f / ext : 1.0f;
        }
    }
    if (SI.skey || SI.misc || SI.acc) slot_init_ray(SI, n, i);     // k_slot_init folded in (one launch fewer)
    if (i >= n) return;
    uint32_t key = raykey_ray(R, i, bx0, by0, bz0, sx, sy, sz, aos);
    if (obits != 5 || kmode != 0)               // another origin / direction split (pbox populations)
        key = raykey_ray_bits(R, i, bx0, by0, bz0, sx, sy, sz, obits, (32 - 3 * obits) / 2, kmode);
    keys[i] = key;
    vals[i] = (int32_t)i;
}

// set_rays' analysis of the emitted rays, one pass over the uploaded population
// (replaces host passes over the caller's arrays): max |D|^2 (float64, NaN as
// +inf; the filter records' Dcap check), whether every origin / direction equals
// ray 0's (float compares: the coherence key's varying bits), whether every power
// is >= 0 (the sharded stop rule), and the hi-digit counts of the counting sort's
// two possible key windows -- k_raykey's own key, so the bucket estimate is exact:
// bits [8, 16) (a point source: 16 direction bits, hi digit 8) and [23, 31) (a
// collimated beam: 15 origin bits, hi digit 8).
__global__ __launch_bounds__(256) void k_ray_scan(RaysIn R, int64_t n, float bx0, float by0, float bz0, float sx,
                                                  float sy, float sz, RayScan *__restrict__ out)
{
    __shared__ uint32_t h[2][256];
    __shared__ uint32_t s_f[3];
    __shared__ unsigned long long s_m;
    for (int i = threadIdx.x; i < 512; i += 256) h[i >> 8][i & 255] = 0u;
    if (threadIdx.x < 3) s_f[threadIdx.x] = 0u;
    if (threadIdx.x == 0) s_m = 0ull;
    __syncthreads();
    const float o0x = R.ox[0], o0y = R.oy[0], o0z = R.oz[0], d0x = R.dx[0], d0y = R.dy[0], d0z = R.dz[0];
    double m = 0.0;
    uint32_t fo = 0u, fd = 0u, fp = 0u;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float ox = R.ox[i], oy = R.oy[i], oz = R.oz[i], dx = R.dx[i], dy = R.dy[i], dz = R.dz[i];
        double q = (double)dx * dx + (double)dy * dy + (double)dz * dz;
        if (q != q) q = INFINITY;
        m = q > m ? q : m;
        fo |= (ox != o0x || oy != o0y || oz != o0z) ? 1u : 0u;
        fd |= (dx != d0x || dy != d0y || dz != d0z) ? 1u : 0u;
        fp |= !(R.pw[i] >= 0.0f) ? 1u : 0u;
        const uint32_t key = raykey_ray(R, i, bx0, by0, bz0, sx, sy, sz, nullptr);
        atomicAdd(&h[0][(key >> 8) & 255u], 1u);
        atomicAdd(&h[1][(key >> 23) & 255u], 1u);
    }
    const unsigned long long mb = (unsigned long long)__double_as_longlong(m);   // m >= 0: bits order as values
    if (fo) atomicOr(&s_f[0], 1u);
    if (fd) atomicOr(&s_f[1], 1u);
    if (fp) atomicOr(&s_f[2], 1u);
    atomicMax(&s_m, mb);
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 256)
        if (h[i >> 8][i & 255]) atomicAdd(&out->hist[i >> 8][i & 255], h[i >> 8][i & 255]);
    if (threadIdx.x == 0) {
        atomicMax(&out->dmax2_bits, s_m);
        if (s_f[0]) atomicOr(&out->diff_o, 1u);
        if (s_f[1]) atomicOr(&out->diff_d, 1u);
        if (s_f[2]) atomicOr(&out->neg_pow, 1u);
    }
}

// ---------------------------------------------------------------------------
// Counting sort of the coherence keys when the key bits that vary span <= 16
// (the emitted rays of a traced trace from a point source or a collimated beam,
// set_rays): MSD with two 8-bit digits, every rank taken in index order (wave
// match ballots, waves and rounds in order), so the permutation is the stable
// sort's and identical from run to run.
//   k_bkey      key (+ 32-byte row, + slot reset), the block's hi-digit counts
//   k_bprefix   per hi digit: exclusive prefix of the block counts, digit total
//   k_bscatter  stable scatter by hi digit: (lo digit, ray) into bucket order;
//               block 0 writes the bucket starts.  One level (lb = 0): perm
//   k_bsort2    one block per hi bucket: stable order by lo digit in LDS, perm
//               written in order
// then k_gather_aos as after rocPRIM.  Replaces key + rocPRIM onesweep (4 fills,
// 2 histogram and 2 look-back pass kernels for 1 M rays).  set_rays takes this
// path only when a host estimate puts at most LPC_BS_MAXB rays into a hi bucket.
#define LPC_BS_T 1024                      // threads per block
#ifndef LPC_BS_RPB
#define LPC_BS_RPB 4096                    // rays per k_bkey / k_bscatter block (-D: compile-time A/B)
#endif
#define LPC_BS_HB 8                        // hi digit bits (at most); lo digit <= 8 bits
#define LPC_BS_ND (1 << LPC_BS_HB)
#define LPC_BS_MAXB 16384                  // largest hi bucket the host estimate admits (k_bsort2 chunks)

// Rank of each lane's digit among the lower lanes with the same digit, and the
// number of valid lanes with it (`valid` lanes only).
static __device__ __forceinline__ void wave_match(uint32_t d, bool valid, int nbits, int &rank, int &cnt, bool &last)
{
    uint64_t peers = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (k >= nbits) break;
        const bool b = (d >> k) & 1u;
        const uint64_t m = __builtin_amdgcn_ballot_w64(b);
        peers &= b ? m : ~m;
    }
    const int lane = threadIdx.x & 63;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    rank = __builtin_popcountll(peers & lt);
    cnt = __builtin_popcountll(peers);
    last = valid && (peers >> lane) == 1ull;           // highest lane of its digit
}

struct BSortLds {
    uint16_t wc[LPC_BS_T / 64][LPC_BS_ND];   // per wave, per digit: the round's count (zero between rounds)
    uint32_t off[LPC_BS_T / 64][LPC_BS_ND];  // per wave, per digit: the wave's first position
    uint32_t run[LPC_BS_ND + 1];             // running position per digit
};

// One round of LPC_BS_T items (item j of the round on thread j): stable
// positions from the running per-digit positions; `run` advances by the round's
// counts.  The per-digit prefix over the 16 waves: 4 threads per digit (4 waves
// each), combined with two shuffles.
static __device__ __forceinline__ uint32_t bs_round(BSortLds &S, uint32_t d, bool valid, int nbits, int nd)
{
    const int t = threadIdx.x, w = t >> 6;
    int rank, cnt;
    bool last;
    wave_match(d, valid, nbits, rank, cnt, last);
    if (last) S.wc[w][d] = (uint16_t)cnt;
    __syncthreads();
    {
        const int e = t >> 2, g = t & 3;                // digit e, waves 4 g .. 4 g + 3
        uint32_t c[4], p = 0;
        if (e < nd) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                c[v] = S.wc[4 * g + v][e];
                S.wc[4 * g + v][e] = 0;
                p += c[v];
            }
        }
        uint32_t incl = p;                              // inclusive scan over the 4 threads of the digit
        const uint32_t u1 = __shfl_up(incl, 1, 64);
        if (g >= 1) incl += u1;
        const uint32_t u2 = __shfl_up(incl, 2, 64);
        if (g >= 2) incl += u2;
        if (e < nd) {
            uint32_t o = S.run[e] + incl - p;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                S.off[4 * g + v][e] = o;
                o += c[v];
            }
        }
        // the digit's 4 threads are lanes of one wave: their reads of run[e] above
        // are done before this write
        if (e < nd && g == 3) S.run[e] += incl;
    }
    __syncthreads();
    return valid ? S.off[w][d] + (uint32_t)rank : 0u;
}

// dst[d] = base + sum of src[0 .. d) for d <= nd (nd < LPC_BS_T), block-wide; the
// caller synchronises before reading dst.
static __device__ __forceinline__ void bs_excl_scan(const uint32_t *src, int nd, uint32_t base, uint32_t *dst,
                                                    uint32_t *ws)
{
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t v = t < nd ? src[t] : 0u;
    uint32_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    uint32_t e = base + incl - v;
    for (int k = 0; k < w; ++k) e += ws[k];
    if (t <= nd) dst[t] = e;
}

// Keys of rays [b * RPB, (b + 1) * RPB) and their 32-byte rows (k_raykey), the
// window's hi digit counted per block into hist[digit * nblk + b].
__global__ __launch_bounds__(LPC_BS_T) void k_bkey(RaysIn R, int64_t n, float bx0, float by0, float bz0, float sx,
                                                   float sy, float sz, uint32_t *__restrict__ keys,
                                                   float4 *__restrict__ aos, SlotInit SI, int b0, int lb, int hb,
                                                   uint32_t *__restrict__ hist, int64_t nblk)
{
    __shared__ uint32_t hcnt[LPC_BS_ND];
    const int nd = 1 << hb;
    if ((int)threadIdx.x < nd) hcnt[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * LPC_BS_RPB;
#pragma unroll
    for (int j = 0; j < LPC_BS_RPB / LPC_BS_T; ++j) {
        const int64_t i = base + j * LPC_BS_T + threadIdx.x;
        if (SI.skey || SI.misc || SI.acc) slot_init_ray(SI, n, i);
        if (i < n) {
            const uint32_t k = raykey_ray(R, i, bx0, by0, bz0, sx, sy, sz, aos);
            keys[i] = k;
            atomicAdd(&hcnt[(k >> (b0 + lb)) & (uint32_t)(nd - 1)], 1u);
        }
    }
    __syncthreads();
    if ((int)threadIdx.x < nd) hist[(int64_t)threadIdx.x * nblk + blockIdx.x] = hcnt[threadIdx.x];
}

// One block per hi digit: exclusive prefix of its per-block counts (in place),
// the digit's total into tot[digit].
__global__ __launch_bounds__(256) void k_bprefix(uint32_t *__restrict__ hist, int64_t nblk, uint32_t *__restrict__ tot)
{
    __shared__ uint32_t ws[4];
    uint32_t *row = hist + (int64_t)blockIdx.x * nblk;
    uint32_t carry = 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t c0 = 0; c0 < nblk; c0 += 256) {
        const int64_t c = c0 + threadIdx.x;
        const uint32_t v = c < nblk ? row[c] : 0u;
        uint32_t incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        if (lane == 63) ws[w] = incl;
        __syncthreads();
        uint32_t wbase = 0, all = 0;
        for (int v2 = 0; v2 < 4; ++v2) {
            if (v2 < w) wbase += ws[v2];
            all += ws[v2];
        }
        if (c < nblk) row[c] = carry + wbase + incl - v;
        carry += all;
        __syncthreads();
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

// Stable scatter by hi digit: (lo digit, ray) pairs into bucket order, or for
// one level (lb == 0) the final permutation.  Block 0 writes the bucket starts
// (bst[0 .. nd]).
__global__ __launch_bounds__(LPC_BS_T) void k_bscatter(const uint32_t *__restrict__ keys, int64_t n, int b0, int lb,
                                                       int hb, const uint32_t *__restrict__ hist, int64_t nblk,
                                                       const uint32_t *__restrict__ tot, uint32_t *__restrict__ bst,
                                                       uint8_t *__restrict__ mlo, int32_t *__restrict__ midx,
                                                       int32_t *__restrict__ perm)
{
    __shared__ BSortLds S;
    __shared__ uint32_t st[LPC_BS_ND + 1];
    __shared__ uint32_t ws[LPC_BS_T / 64];
    const int nd = 1 << hb;
    const int t = threadIdx.x;
    bs_excl_scan(tot, nd, 0u, st, ws);
    for (int i = t; i < (LPC_BS_T / 64) * LPC_BS_ND; i += LPC_BS_T) (&S.wc[0][0])[i] = 0;
    __syncthreads();
    if (t < nd) S.run[t] = st[t] + hist[(int64_t)t * nblk + blockIdx.x];
    if (blockIdx.x == 0 && t <= nd) bst[t] = st[t];
    const int64_t base = (int64_t)blockIdx.x * LPC_BS_RPB;
    constexpr int NR = LPC_BS_RPB / LPC_BS_T;
    uint32_t k[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        const int64_t i = base + j * LPC_BS_T + t;
        k[j] = i < n ? keys[i] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        const int64_t i = base + j * LPC_BS_T + t;
        const bool valid = i < n;
        const uint32_t d = (k[j] >> (b0 + lb)) & (uint32_t)(nd - 1);
        const uint32_t pos = bs_round(S, d, valid, hb, nd);
        if (valid) {
            if (lb == 0) {
                perm[pos] = (int32_t)i;
            } else {
                mlo[pos] = (uint8_t)((k[j] >> b0) & ((1u << lb) - 1u));
                midx[pos] = (int32_t)i;
            }
        }
    }
}

// Second level: block (bucket b = blockIdx.x, chunk c = blockIdx.y) orders the
// c-th LPC_BS_RPB entries of hi bucket b by the lo digit, stably: an entry's
// place is the bucket start + the bucket's entries of smaller lo digits (counted
// over the whole bucket) + the entries of its digit in earlier chunks (counted
// over those chunks) + its rank inside the chunk.  Chunks past the bucket's end
// exit; a bucket needs at most LPC_BS_MAXB / LPC_BS_RPB chunks (the host's estimate),
// a larger one is ordered by its last block, serially over its remaining chunks.
__global__ __launch_bounds__(LPC_BS_T) void k_bsort2(const uint8_t *__restrict__ mlo,
                                                     const int32_t *__restrict__ midx, int lb,
                                                     const uint32_t *__restrict__ bst, int32_t *__restrict__ perm)
{
    __shared__ BSortLds S;
    __shared__ uint32_t hl[LPC_BS_ND], hb4[LPC_BS_ND], lst[LPC_BS_ND + 1];
    __shared__ uint32_t ws[LPC_BS_T / 64];
    const int nl = 1 << lb;
    const int t = threadIdx.x;
    const int64_t s0 = bst[blockIdx.x], s1 = bst[blockIdx.x + 1];
    const int64_t c0 = s0 + (int64_t)blockIdx.y * LPC_BS_RPB;
    if (c0 >= s1) return;                               // block-uniform
    // the last chunk block takes every chunk from its own to the bucket's end
    const bool last = blockIdx.y + 1 == gridDim.y;
    const int64_t c1 = last ? s1 : min(s1, c0 + LPC_BS_RPB);
    if (t < nl) { hl[t] = 0; hb4[t] = 0; }
    for (int i = t; i < (LPC_BS_T / 64) * LPC_BS_ND; i += LPC_BS_T) (&S.wc[0][0])[i] = 0;
    __syncthreads();
    constexpr int IPT = LPC_BS_RPB / LPC_BS_T;
    for (int64_t e0 = s0; e0 < s1; e0 += LPC_BS_RPB) {  // lo-digit counts: the bucket, and before c0
        uint32_t d[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int64_t i = e0 + j * LPC_BS_T + t;
            d[j] = i < s1 ? mlo[i] : 0xffffffffu;
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            if (d[j] == 0xffffffffu) continue;
            atomicAdd(&hl[d[j]], 1u);
            if (e0 + j * LPC_BS_T + t < c0) atomicAdd(&hb4[d[j]], 1u);
        }
    }
    __syncthreads();
    bs_excl_scan(hl, nl, (uint32_t)s0, lst, ws);
    __syncthreads();
    if (t < nl) S.run[t] = lst[t] + hb4[t];
    for (int64_t e0 = c0; e0 < c1; e0 += LPC_BS_RPB) {
        uint32_t d[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int64_t i = e0 + j * LPC_BS_T + t;
            d[j] = i < c1 ? mlo[i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int64_t i = e0 + j * LPC_BS_T + t;
            const bool valid = i < c1;
            const uint32_t pos = bs_round(S, d[j], valid, lb, nl);
            if (valid) perm[pos] = midx[i];
        }
    }
}

// Test entry (lpc_filter_eval, tests/test_gpu_filter.py): the device's own
// filter code paths on given (ray, record) pairs, so the superset property
// (every pair Moller-Trumbore accepts passes the filter) is checked on the code
// the GPU runs.  mode 0: filter_test (k_roots_s / k_gather_roots root tests
// without the cull, a lone last piece); 1: filter_test2 (the packed child tests
// of the walk and the packed root tests), record i packed with record i ^ 1
// against ray i; 2: filter_test2h (the packed root tests with the half-line cull,
// LPC_HALF 3, the default); 3: filter_testh (the same for a lone last piece).
// rec: cx cy cz negB negA per pair.
__global__ __launch_bounds__(256) void k_filter_eval(int64_t n, const float *__restrict__ O,
                                                     const float *__restrict__ D, const float *__restrict__ rec,
                                                     int mode, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f3 o = mk3(O[3 * i], O[3 * i + 1], O[3 * i + 2]);
    const f3 d = mk3(D[3 * i], D[3 * i + 1], D[3 * i + 2]);
    float nx, ny, nz;
    unit_dir(d, nx, ny, nz);
    const int64_t j = (i ^ 1) < n ? (i ^ 1) : i;
    const float *a = rec + 5 * i, *b = rec + 5 * j;
    float r;
    if (mode == 1 || mode == 2) {
        const lpc_f2 cx = {a[0], b[0]}, cy = {a[1], b[1]}, cz = {a[2], b[2]}, nb = {a[3], b[3]}, na = {a[4], b[4]};
        r = mode == 1 ? filter_test2(cx, cy, cz, nb, na, o.x, o.y, o.z, nx, ny, nz).x
                      : filter_test2h(cx, cy, cz, nb, na, o.x, o.y, o.z, nx, ny, nz).x;
    } else if (mode == 3) {
        r = filter_testh(a[0], a[1], a[2], a[3], a[4], o.x, o.y, o.z, nx, ny, nz);
    } else {
        r = filter_test(a[0], a[1], a[2], a[3], a[4], o.x, o.y, o.z, nx, ny, nz);
    }
    out[i] = r;
}

// ---------------------------------------------------------------------------
// k_shade: postproc + Fresnel for one ray per lane (exact arithmetic).
// touched (optional): bit j set for slots j < 64 that hold anything but the clean
// state (max_ray_len, idx -1, count 0), noted as postproc reads them
// KU > 0 (A.K <= KU): the ray's K slots are loaded up front into registers (one
// memory round trip instead of one per mesh and loop).
template <int KU = 0>
static __device__ __forceinline__ ShadeOut shade_eval(const ShadeArgs &A, int64_t r, PostOut &po, f3 &dest,
                                                      uint64_t *touched = nullptr, uint32_t lmask = 0xffffffffu)
{
    const f3 O = mk3(A.in.ox[r], A.in.oy[r], A.in.oz[r]);
    const f3 D = mk3(A.in.dx[r], A.in.dy[r], A.in.dz[r]);
    const int32_t prev = A.in.pmid[r];
    const int64_t n = A.n;
    const unsigned long long k0 = slot_key(A.max_ray_len, -1);
    if constexpr (KU > 0) {
        unsigned long long kr[KU];
        int32_t cr[KU];
        {
#pragma unroll
            for (int j = 0; j < KU; ++j) {
                kr[j] = k0; cr[j] = 0;
                // lmask: the slots a flush wrote (the others hold the clean state)
                if (j < A.K && ((lmask >> (j & 31)) & 1u)) {
                    kr[j] = A.skey[(int64_t)j * n + r];
                    cr[j] = A.sc[(int64_t)j * n + r];
                }
            }
        }
        if (touched) {
            uint64_t m = 0;
#pragma unroll
            for (int j = 0; j < KU; ++j) m |= (kr[j] != k0 || cr[j] != 0) ? 1ull << j : 0ull;
            *touched = m;
        }
        auto slot = [&](int32_t j, float &t, int32_t &c, int32_t &i) {
            t = slot_key_t(kr[j]); i = slot_key_idx(kr[j]); c = cr[j];
        };
        po = postproc<KU>(A.K, prev, A.mat_type, A.max_ray_len, slot);
    } else {
        auto slot = [&](int32_t j, float &t, int32_t &c, int32_t &i) {
            // lmask: the slots a flush wrote (the others hold the clean state)
            if (j < 32 && !((lmask >> j) & 1u)) { t = A.max_ray_len; i = -1; c = 0; return; }
            const int64_t a = (int64_t)j * n + r;
            const unsigned long long k = A.skey[a];
            t = slot_key_t(k); i = slot_key_idx(k); c = A.sc[a];
            if (touched && j < 64 && (k != k0 || c != 0)) *touched |= 1ull << j;
        };
        po = postproc(A.K, prev, A.mat_type, A.max_ray_len, slot);
    }
    dest = ray_dest(O, D, po.t_min);
    const int32_t meas_in = A.meas_in ? A.meas_in[r] : 0;
    auto tri = [&](int32_t idx, f3 &v0, f3 &v1, f3 &v2) {
        const float *v = A.verts + (int64_t)idx * 9;
        v0 = mk3(v[0], v[1], v[2]); v1 = mk3(v[3], v[4], v[5]); v2 = mk3(v[6], v[7], v[8]);
    };
    return shade(O, D, dest, A.in.pw[r], meas_in, po.hit_mesh, po.hit_idx, po.n1, po.n2, A.mat_type, A.ior,
                 A.refl, A.diss, A.ior_env, tri);
}

template <int KU = 0>
static __device__ __forceinline__ ShadeOut shade_ray(const ShadeArgs &A, int64_t r)
{
    PostOut po;
    f3 dest;
    const ShadeOut s = shade_eval<KU>(A, r, po, dest);
    A.o.destx[r] = dest.x; A.o.desty[r] = dest.y; A.o.destz[r] = dest.z;
    A.o.imid[r] = po.hit_mesh;
    A.o.pw[r] = s.pow;
    A.o.meas[r] = s.meas;
    A.o.rdx[r] = s.r_dir.x; A.o.rdy[r] = s.r_dir.y; A.o.rdz[r] = s.r_dir.z;
    A.o.rpw[r] = s.r_pow; A.o.rms[r] = s.r_meas;
    A.o.tdx[r] = s.t_dir.x; A.o.tdy[r] = s.t_dir.y; A.o.tdz[r] = s.t_dir.z;
    A.o.tpw[r] = s.t_pow; A.o.tms[r] = s.t_meas;
    if (A.o.iidx) {
        A.o.iidx[r] = po.hit_idx; A.o.n1[r] = po.n1; A.o.n2[r] = po.n2;
        A.o.ent[r] = po.hit_mesh >= 0 ? po.entering : 0;   // no hit: the reference's zeroed buffer (iterative_tracer.py:230)
    }
    return s;
}

template <int KU>
__global__ __launch_bounds__(256) void k_shade(ShadeArgs A)
{
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= A.n) return;
    (void)shade_ray<KU>(A, r);
}

// ---------------------------------------------------------------------------
// Compaction.  A tile is 1024 rays = 4 sub-tiles of 256 (one lane per ray).
static __device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
static __device__ __forceinline__ float wave_max(float v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ __launch_bounds__(256) void k_count(CompactArgs A)
{
    __shared__ int32_t s_cnt[3][4];
    __shared__ double s_pow[4];
    __shared__ float s_dm[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t tile = (int64_t)blockIdx.x * 1024;
    int32_t cR = 0, cT = 0, cM = 0;
    double pk = 0.0;
    float dm = 0.0f;
    bool neg = false;                    // a kept child's power < 0 or NaN (the host's sum bound needs >= 0)
    for (int sub = 0; sub < 4; ++sub) {
        const int64_t r = tile + sub * 256 + threadIdx.x;
        if (r < A.n) {
            const bool fR = A.o.rms[r] == 0, fT = A.o.tms[r] == 0, fM = A.o.meas[r] == 1;
            cR += fR; cT += fT; cM += fM;
            neg = neg || (fR && !(A.o.rpw[r] >= 0.0f)) || (fT && !(A.o.tpw[r] >= 0.0f));
            if (fR) {
                pk += (double)A.o.rpw[r];
                dm = fmaxf(dm, A.o.rdx[r] * A.o.rdx[r] + A.o.rdy[r] * A.o.rdy[r] + A.o.rdz[r] * A.o.rdz[r]);
            }
            if (fT) {
                pk += (double)A.o.tpw[r];
                dm = fmaxf(dm, A.o.tdx[r] * A.o.tdx[r] + A.o.tdy[r] * A.o.tdy[r] + A.o.tdz[r] * A.o.tdz[r]);
            }
        }
    }
    // wave reductions (fixed order -> deterministic)
    for (int o = 32; o >= 1; o >>= 1) {
        cR += __shfl_xor(cR, o, 64); cT += __shfl_xor(cT, o, 64); cM += __shfl_xor(cM, o, 64);
    }
    pk = wave_sum(pk);
    dm = wave_max(dm);
    if (any_lane(neg) && lane == 0) atomicOr(&A.acc->pneg, 1u);
    if (lane == 0) {
        s_cnt[0][wv] = cR; s_cnt[1][wv] = cT; s_cnt[2][wv] = cM; s_pow[wv] = pk; s_dm[wv] = dm;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int64_t b = blockIdx.x, nb = A.nb;
        A.blk_cnt[0 * nb + b] = s_cnt[0][0] + s_cnt[0][1] + s_cnt[0][2] + s_cnt[0][3];
        A.blk_cnt[1 * nb + b] = s_cnt[1][0] + s_cnt[1][1] + s_cnt[1][2] + s_cnt[1][3];
        A.blk_cnt[2 * nb + b] = s_cnt[2][0] + s_cnt[2][1] + s_cnt[2][2] + s_cnt[2][3];
        A.blk_pow[b] = ((s_pow[0] + s_pow[1]) + s_pow[2]) + s_pow[3];
        const float m = fmaxf(fmaxf(s_dm[0], s_dm[1]), fmaxf(s_dm[2], s_dm[3]));
        atomicMax(&A.acc->dmax2_bits, __float_as_uint(m));
    }
}

// Single-block exclusive scan of the per-tile counts + fixed-order sums.
__global__ __launch_bounds__(1024) void k_scan(CompactArgs A)
{
    __shared__ long long s_sc[3][1024];
    __shared__ double s_d[1024];
    __shared__ long long s_base[3];
    const int t = threadIdx.x;
    const int64_t nb = A.nb;
    const int64_t per = (nb + 1023) / 1024;
    const int64_t lo = t * per, hi = (lo + per < nb) ? lo + per : nb;
    if (t == 0) {
        s_base[0] = (long long)A.acc->nR;
        s_base[1] = (long long)A.acc->nT;
        s_base[2] = (long long)A.acc->m_total;
    }
    long long loc[3] = {0, 0, 0};
    double lp = 0.0;
    for (int64_t i = lo; i < hi; ++i) {
        loc[0] += A.blk_cnt[i]; loc[1] += A.blk_cnt[nb + i]; loc[2] += A.blk_cnt[2 * nb + i];
        lp += A.blk_pow[i];
    }
    for (int f = 0; f < 3; ++f) s_sc[f][t] = loc[f];
    s_d[t] = lp;
    __syncthreads();
    // inclusive Hillis-Steele scan over 1024 thread totals
    for (int off = 1; off < 1024; off <<= 1) {
        long long v0 = 0, v1 = 0, v2 = 0;
        if (t >= off) { v0 = s_sc[0][t - off]; v1 = s_sc[1][t - off]; v2 = s_sc[2][t - off]; }
        __syncthreads();
        s_sc[0][t] += v0; s_sc[1][t] += v1; s_sc[2][t] += v2;
        __syncthreads();
    }
    long long run[3];
    for (int f = 0; f < 3; ++f) run[f] = s_base[f] + s_sc[f][t] - loc[f];
    for (int64_t i = lo; i < hi; ++i) {
        for (int f = 0; f < 3; ++f) {
            A.blk_off[f * nb + i] = run[f];
            run[f] += A.blk_cnt[f * nb + i];
        }
    }
    // fixed-order tree sum of the kept power
    for (int off = 512; off >= 1; off >>= 1) {
        __syncthreads();
        if (t < off) s_d[t] += s_d[t + off];
    }
    __syncthreads();
    const double pow_next = s_d[0];
    if (t == 1023) {
        A.acc->nR = (unsigned long long)(s_base[0] + s_sc[0][1023]);
        A.acc->nT = (unsigned long long)(s_base[1] + s_sc[1][1023]);
        const long long mt = s_sc[2][1023];
        A.acc->m_total = (unsigned long long)(s_base[2] + mt);
        A.acc->nM_iter += (unsigned long long)mt;
    }
    if (t == 0) A.acc->pow_next += pow_next;
    if (A.host_acc) {
        // publish the iteration's counters to the mapped host copy, the sequence
        // number last: the host reads them while k_scatter still runs
        __syncthreads();
        if (t == 0) {
            const DevAcc a = *A.acc;
            DevAcc *o = A.host_acc;
            __hip_atomic_store(&o->nR, a.nR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&o->nT, a.nT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&o->m_total, a.m_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&o->nM_iter, a.nM_iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store((unsigned long long *)&o->pow_next, __double_as_longlong(a.pow_next),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&o->dmax2_bits, a.dmax2_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&o->qerr, a.qerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&o->pneg, a.pneg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // every counter store acknowledged before the sequence number is sent
            // (a release fence would also write back the whole L2)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&o->seq, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ __launch_bounds__(256) void k_scatter(CompactArgs A)
{
    __shared__ int32_t s_w[3][4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t tile = (int64_t)blockIdx.x * 1024;
    const int64_t nb = A.nb;
    int64_t base[3] = {A.blk_off[blockIdx.x], A.blk_off[nb + blockIdx.x], A.blk_off[2 * nb + blockIdx.x]};
    if (A.direct_t) base[1] += (int64_t)A.acc->nR;          // k_scan wrote the final reflected count
    for (int sub = 0; sub < 4; ++sub) {
        const int64_t r = tile + sub * 256 + threadIdx.x;
        const bool in = r < A.n;
        const bool fR = in && A.o.rms[r] == 0;
        const bool fT = in && A.o.tms[r] == 0;
        const bool fM = in && A.o.meas[r] == 1;
        const uint64_t bR = __ballot(fR), bT = __ballot(fT), bM = __ballot(fM);
        const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
        const int pR = __popcll(bR & below), pT = __popcll(bT & below), pM = __popcll(bM & below);
        if (lane == 0) { s_w[0][wv] = __popcll(bR); s_w[1][wv] = __popcll(bT); s_w[2][wv] = __popcll(bM); }
        __syncthreads();
        int32_t wo[3] = {0, 0, 0}, tot[3] = {0, 0, 0};
        for (int w = 0; w < 4; ++w)
            for (int f = 0; f < 3; ++f) {
                if (w < wv) wo[f] += s_w[f][w];
                tot[f] += s_w[f][w];
            }
        if (fR || fT || fM) {
            const float dx = A.o.destx[r], dy = A.o.desty[r], dz = A.o.destz[r];
            const int32_t mid = A.o.imid[r];
            if (fR) {
                const int64_t q = base[0] + wo[0] + pR;
                A.nR.ox[q] = dx; A.nR.oy[q] = dy; A.nR.oz[q] = dz;
                A.nR.dx[q] = A.o.rdx[r]; A.nR.dy[q] = A.o.rdy[r]; A.nR.dz[q] = A.o.rdz[r];
                A.nR.pw[q] = A.o.rpw[r]; A.nR.pmid[q] = mid;
            }
            if (fT) {
                const int64_t q = base[1] + wo[1] + pT;
                A.nT.ox[q] = dx; A.nT.oy[q] = dy; A.nT.oz[q] = dz;
                A.nT.dx[q] = A.o.tdx[r]; A.nT.dy[q] = A.o.tdy[r]; A.nT.dz[q] = A.o.tdz[r];
                A.nT.pw[q] = A.o.tpw[r]; A.nT.pmid[q] = mid;
            }
            if (fM) {
                const int64_t q = base[2] + wo[2] + pM;
                A.mx[q] = dx; A.my[q] = dy; A.mz[q] = dz; A.mp[q] = A.o.pw[r]; A.mm[q] = mid;
            }
        }
        for (int f = 0; f < 3; ++f) base[f] += tot[f];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Two-kernel compaction of a traced single-chunk iteration (StageArgs /
// MoveArgs), replacing k_shade + k_count + k_scan + k_scatter + k_append:
//   k_shade_stage  shading, one ray per thread; a 256-ray tile's kept children
//                  and measured rays are written compacted into the tile's own
//                  staging rows, with the tile's counts, kept power and max |dir|^2;
//   k_stage_move   every block sums the tile counts (its tile's prefix and the
//                  totals, so the refracted block goes straight after the
//                  reflected one) and moves its tile's staged rows into place;
//                  block 0 also writes the iteration counters (fixed-order power
//                  sum) and publishes them to the host.
// Children and measured rays land at the same positions as with the four
// kernels ([reflected ; refracted], each in parent order).
template <int KU, bool DS>
__global__ __launch_bounds__(LPC_ST_TILE) void k_shade_stage(StageArgs A)
{
    __shared__ double s_mp[LPC_MP_MAX][LPC_ST_TILE / 64];
    __shared__ int32_t s_w[3][LPC_ST_TILE / 64];
    __shared__ double s_pow[LPC_ST_TILE / 64];
    __shared__ float s_dm[LPC_ST_TILE / 64];
    __shared__ uint32_t s_bx[LPC_ST_TILE / 64][6];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // the shading inputs as a local (a device-sized launch sets its n; writing the
    // kernel argument itself would put the whole argument block in scratch)
    ShadeArgs S = A.S;
    if constexpr (DS) S.n = *A.nd;
    auto tile_body = [&](const int64_t tile) {
    const int64_t r = tile * LPC_ST_TILE + threadIdx.x;
    const bool in = r < S.n;
    PostOut po;
    po.hit_mesh = -1;
    f3 dest = mk3(0.0f, 0.0f, 0.0f);
    ShadeOut s;
    memset(&s, 0, sizeof(s));
    s.r_meas = -1; s.t_meas = -1;
    if (in) {
        uint64_t touched = 0;
        // the walk's written-slot mask (K <= 32): only those slots are read, and
        // the mask goes back to 0 with them
        uint32_t lm = 0xffffffffu;
        if (A.tmask) {
            lm = A.tmask[r];
            if (lm) A.tmask[r] = 0u;
        }
        s = shade_eval<KU>(S, r, po, dest, &touched, lm);
        // the slots just read back to the clean state: those a flush wrote (noted
        // while postproc read them; slots 64 and up are read again)
        const unsigned long long k0 = slot_key(S.max_ray_len, -1);
        while (touched) {
            const int j = __builtin_ctzll(touched);
            touched &= touched - 1;
            const int64_t a = (int64_t)j * S.n + r;
            A.skey[a] = k0;
            A.scnt[a] = 0;
        }
        for (int32_t j = 64; j < S.K; ++j) {
            const int64_t a = (int64_t)j * S.n + r;
            if (A.skey[a] != k0) A.skey[a] = k0;
            if (A.scnt[a] != 0) A.scnt[a] = 0;
        }
    }
    const bool fR = in && s.r_meas == 0, fT = in && s.t_meas == 0, fM = in && s.meas == 1;
    const uint64_t bR = __ballot(fR), bT = __ballot(fT), bM = __ballot(fM);
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // kept power and max |dir|^2 (k_count's per-ray order: reflected, then refracted)
    double pk = 0.0;
    float dm = 0.0f;
    if (fR) {
        pk += (double)s.r_pow;
        dm = fmaxf(dm, s.r_dir.x * s.r_dir.x + s.r_dir.y * s.r_dir.y + s.r_dir.z * s.r_dir.z);
    }
    if (fT) {
        pk += (double)s.t_pow;
        dm = fmaxf(dm, s.t_dir.x * s.t_dir.x + s.t_dir.y * s.t_dir.y + s.t_dir.z * s.t_dir.z);
    }
    pk = wave_sum(pk);
    dm = wave_max(dm);
    if (A.tbox) {       // the kept children's origins (= dest): the next population's key box
        const bool kb = (fR || fT) && isfinite(dest.x) && isfinite(dest.y) && isfinite(dest.z);
        const float v[3] = {dest.x, dest.y, dest.z};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float lo = wave_red(kb ? v[k] : INFINITY, 0), hi = wave_red(kb ? v[k] : -INFINITY, 1);
            if (lane == 0) { s_bx[wv][k] = ord_f32(lo); s_bx[wv][3 + k] = ord_f32(hi); }
        }
    }
    // measured power per measure mesh (fixed order: waves, then tiles in k_stage_move)
    for (int m = 0; m < A.nmp; ++m) {
        const double v = wave_sum((fM && po.hit_mesh == A.mpm[m]) ? (double)s.pow : 0.0);
        if (lane == 0) s_mp[m][wv] = v;
    }
    if (lane == 0) {
        s_w[0][wv] = __popcll(bR); s_w[1][wv] = __popcll(bT); s_w[2][wv] = __popcll(bM);
        s_pow[wv] = pk; s_dm[wv] = dm;
    }
    __syncthreads();
    int32_t wo[3] = {0, 0, 0};
    for (int w = 0; w < wv; ++w)
        for (int f = 0; f < 3; ++f) wo[f] += s_w[f][w];
    if (threadIdx.x < A.nmp) {
        double v = 0.0;
        for (int k = 0; k < LPC_ST_TILE / 64; ++k) v += s_mp[threadIdx.x][k];
        A.tmp[tile * LPC_MP_MAX + threadIdx.x] = v;
    }
    const int64_t c = A.cst, t0 = tile * LPC_ST_TILE;
    auto put = [&](float *b, int64_t q, f3 d, float pw) {
        b[q] = dest.x; b[c + q] = dest.y; b[2 * c + q] = dest.z;
        b[3 * c + q] = d.x; b[4 * c + q] = d.y; b[5 * c + q] = d.z;
        b[6 * c + q] = pw; ((int32_t *)b)[7 * c + q] = po.hit_mesh;
    };
    if (fR) put(A.stR, t0 + wo[0] + __popcll(bR & below), s.r_dir, s.r_pow);
    if (fT) put(A.stT, t0 + wo[1] + __popcll(bT & below), s.t_dir, s.t_pow);
    if (fM) {
        const int64_t q = t0 + wo[2] + __popcll(bM & below);
        A.stM[q] = dest.x; A.stM[c + q] = dest.y; A.stM[2 * c + q] = dest.z; A.stM[3 * c + q] = s.pow;
        ((int32_t *)A.stM)[4 * c + q] = po.hit_mesh;
    }
    if (threadIdx.x == 0) {
        uint32_t cR = 0, cT = 0, cM = 0;
        double tp = 0.0;                      // fixed order over the tile's waves
        float td = 0.0f;
        for (int k = 0; k < LPC_ST_TILE / 64; ++k) {
            cR += s_w[0][k]; cT += s_w[1][k]; cM += s_w[2][k];
            tp += s_pow[k]; td = fmaxf(td, s_dm[k]);
        }
        A.tcnt[tile] = cR | (cT << 9) | (cM << 18);
        A.tpow[tile] = tp;
        A.tdm[tile] = __float_as_uint(td);
        if (A.tbox) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                uint32_t lo = s_bx[0][k], hi = s_bx[0][3 + k];
                for (int w = 1; w < LPC_ST_TILE / 64; ++w) {
                    lo = min(lo, s_bx[w][k]);
                    hi = max(hi, s_bx[w][3 + k]);
                }
                A.tbox[tile * 6 + k] = lo;
                A.tbox[tile * 6 + 3 + k] = hi;
            }
        }
        if (cR | cT | cM) atomicAdd(&A.gsum[tile / LPC_ST_GROUP], gsum_pack(cR, cT, cM));
    }
    };
    if constexpr (!DS) {
        tile_body(blockIdx.x);                    // one tile per block
    } else {                                      // device-sized: grid-stride over the tiles
        const int64_t ntiles = (S.n + LPC_ST_TILE - 1) / LPC_ST_TILE;
        for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
            tile_body(tile);
            __syncthreads();                      // the shared sums are reused by the next tile
        }
    }
}

template <bool DS>
static __device__ __forceinline__ void stage_move(MoveArgs A)
{
    __shared__ long long s_red[LPC_ST_TILE / 64][6];
    __shared__ long long s_pre[3], s_tot[3];
    __shared__ double s_p[LPC_ST_TILE];
    __shared__ float s_d[LPC_ST_TILE];
    __shared__ double s_m[LPC_MP_MAX][LPC_ST_TILE];
    __shared__ uint32_t s_b[6][LPC_ST_TILE / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    // device-sized launch (DS): the population size and measured-record length
    // the previous iteration left in A.ctl; grid-stride over the tiles (tile 0's
    // block also publishes an empty iteration's counters)
    int64_t ntiles = A.ntiles, ngroups = A.ngroups;
    unsigned long long m_base = A.m_base;
    // chunked iteration: this chunk's rows go after the earlier chunks'
    const bool chunked = !DS && A.popT != nullptr;
    unsigned long long r_base = 0, t_base = 0;
    if (chunked && !A.first) { r_base = A.cbase_in[0]; t_base = A.cbase_in[1]; m_base = A.cbase_in[2]; }
    if constexpr (DS) {
        const long long n = A.ctl->n[A.par];
        ntiles = (n + LPC_ST_TILE - 1) / LPC_ST_TILE;
        ngroups = (ntiles + LPC_ST_GROUP - 1) / LPC_ST_GROUP;
        m_base = A.ctl->m[A.par];
    }
    auto tile_body = [&](const int64_t tile) {
    // this tile's prefix and the totals: the group counts (the groups before this
    // tile's, all groups), then this group's tiles before it
    long long pre[3] = {0, 0, 0}, tot[3] = {0, 0, 0};
    const int64_t g = tile / LPC_ST_GROUP;
    const unsigned long long m21 = (1ull << 21) - 1ull;
    for (int64_t k = t; k < ngroups; k += LPC_ST_TILE) {
        const unsigned long long v = A.gsum[k];
        const long long c[3] = {(long long)(v & m21), (long long)((v >> 21) & m21), (long long)((v >> 42) & m21)};
        for (int f = 0; f < 3; ++f) {
            tot[f] += c[f];
            if (k < g) pre[f] += c[f];
        }
    }
    for (int64_t j = g * LPC_ST_GROUP + t; j < tile; j += LPC_ST_TILE) {
        const uint32_t v = A.tcnt[j];
        pre[0] += v & 511u; pre[1] += (v >> 9) & 511u; pre[2] += (v >> 18) & 511u;
    }
    for (int f = 0; f < 3; ++f) {
        long long a = pre[f], b = tot[f];
        for (int o = 32; o >= 1; o >>= 1) { a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64); }
        pre[f] = a; tot[f] = b;
    }
    if (lane == 0)
        for (int f = 0; f < 3; ++f) { s_red[wv][f] = pre[f]; s_red[wv][3 + f] = tot[f]; }
    __syncthreads();
    if (t < 6) {
        long long v = 0;
        for (int k = 0; k < LPC_ST_TILE / 64; ++k) v += s_red[k][t];
        if (t < 3) s_pre[t] = v; else s_tot[t - 3] = v;
    }
    __syncthreads();
    if (tile == 0) {
        // iteration counters: fixed-order power sum, max |dir|^2
        double lp = 0.0, lm[LPC_MP_MAX] = {0.0, 0.0, 0.0, 0.0};
        float ld = 0.0f;
        // eight of this thread's tiles per round, loaded before they are added
        // (one load latency per round instead of one per tile; same order of adds).
        // The first measure mesh's sums ride with the power sums; further measure
        // meshes take rounds of their own, so the round's registers stay few (this
        // path sets the VGPR count, i.e. the occupancy, of every block's row moves)
        constexpr int UB = 8;
        for (int64_t j0 = t; j0 < ntiles; j0 += (int64_t)UB * LPC_ST_TILE) {
            double vp[UB], v0[UB];
            uint32_t vd[UB];
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                const int64_t j = j0 + (int64_t)u * LPC_ST_TILE;
                const bool ok = j < ntiles;
                vp[u] = ok ? A.tpow[j] : 0.0;
                vd[u] = ok ? A.tdm[j] : 0u;
                v0[u] = (ok && A.nmp > 0) ? A.tmp[j * LPC_MP_MAX] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                if (j0 + (int64_t)u * LPC_ST_TILE >= ntiles) break;
                lp += vp[u];
                ld = fmaxf(ld, __uint_as_float(vd[u]));
                if (A.nmp > 0) lm[0] += v0[u];
            }
        }
#pragma unroll
        for (int m = 1; m < LPC_MP_MAX; ++m) {
            if (m >= A.nmp) break;
            double a = 0.0;
            for (int64_t j0 = t; j0 < ntiles; j0 += (int64_t)UB * LPC_ST_TILE) {
                double vm[UB];
#pragma unroll
                for (int u = 0; u < UB; ++u) {
                    const int64_t j = j0 + (int64_t)u * LPC_ST_TILE;
                    vm[u] = j < ntiles ? A.tmp[j * LPC_MP_MAX + m] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < UB; ++u) {
                    if (j0 + (int64_t)u * LPC_ST_TILE >= ntiles) break;
                    a += vm[u];
                }
            }
            lm[m] = a;
        }
        s_p[t] = lp;
        s_d[t] = ld;
        for (int m = 0; m < LPC_MP_MAX; ++m) s_m[m][t] = lm[m];
        for (int off = LPC_ST_TILE / 2; off >= 1; off >>= 1) {
            __syncthreads();
            if (t < off) {
                s_p[t] += s_p[t + off];
                s_d[t] = fmaxf(s_d[t], s_d[t + off]);
                for (int m = 0; m < LPC_MP_MAX; ++m) s_m[m][t] += s_m[m][t + off];
            }
        }
        __syncthreads();
        if (A.tbox && A.pbox) {     // the next population's origin box over the tiles (order-free)
            uint32_t b[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
            for (int64_t j = t; j < ntiles; j += LPC_ST_TILE)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    b[k] = min(b[k], A.tbox[j * 6 + k]);
                    b[3 + k] = max(b[3 + k], A.tbox[j * 6 + 3 + k]);
                }
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                uint32_t v = b[k];
                for (int o = 32; o >= 1; o >>= 1) {
                    const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
                    v = k < 3 ? min(v, u) : max(v, u);
                }
                if (lane == 0) s_b[k][wv] = v;
            }
            __syncthreads();
            if (t < 6) {
                uint32_t v = s_b[t][0];
                for (int w = 1; w < LPC_ST_TILE / 64; ++w) v = t < 3 ? min(v, s_b[t][w]) : max(v, s_b[t][w]);
                if (chunked && !A.first) v = t < 3 ? min(v, A.pbox[t]) : max(v, A.pbox[t]);
                A.pbox[t] = v;
            }
        }
        if (t == 0) {
            // the counters in registers (a DevAcc local indexed by m would live in
            // scratch, on the iteration's critical path)
            DevAcc a;
            double mp[LPC_MP_MAX];
#pragma unroll
            for (int m = 0; m < LPC_MP_MAX; ++m) {    // the trace's running sums, in iteration order
                mp[m] = 0.0;
                if (m < A.nmp) {
                    mp[m] = (m_base == 0 ? 0.0 : A.mrun[m]) + s_m[m][0];
                    A.mrun[m] = mp[m];
                }
            }
            a.nR = (unsigned long long)s_tot[0]; a.nT = (unsigned long long)s_tot[1];
            a.m_total = m_base + (unsigned long long)s_tot[2];
            a.nM_iter = (unsigned long long)s_tot[2];
            a.pow_next = s_p[0];
            a.dmax2_bits = __float_as_uint(s_d[0]);
            a.qerr = A.acc->qerr;
            if (chunked) {
                // the next chunk's bases, and this chunk's counters added to the
                // iteration's (the earlier chunks' in acc; chunk order, so the
                // float64 power sum is deterministic)
                A.cbase_out[0] = r_base + a.nR;
                A.cbase_out[1] = t_base + a.nT;
                A.cbase_out[2] = a.m_total;
                if (!A.first) {
                    const DevAcc &p = *A.acc;
                    a.nR += p.nR; a.nT += p.nT; a.nM_iter += p.nM_iter;
                    a.pow_next = p.pow_next + a.pow_next;
                    a.dmax2_bits = __float_as_uint(fmaxf(__uint_as_float(p.dmax2_bits), s_d[0]));
                }
            }
            {
                DevAcc *d = A.acc;
                d->nR = a.nR; d->nT = a.nT; d->m_total = a.m_total; d->nM_iter = a.nM_iter;
                d->pow_next = a.pow_next; d->dmax2_bits = a.dmax2_bits; d->qerr = a.qerr;
                d->seq = 0u; d->pneg = 0u;
#pragma unroll
                for (int m = 0; m < LPC_MP_MAX; ++m) d->mpow[m] = mp[m];
            }
            if (A.ctl) {
                // the next iteration's size for device-sized launches: 0 once the
                // trace ends (trace_run's rules, iterative_tracer.py:383-391) or a
                // kept direction exceeds the filter records' Dcap (the host rebuilds)
                const unsigned long long kept = a.nR + a.nT;
                // the whole iteration's max |D|^2 (a chunked iteration: every
                // chunk's, combined above; the last chunk publishes)
                const bool dc = !((double)__uint_as_float(a.dmax2_bits) <= A.dcap2);
                const bool stop = a.pow_next < A.thr || kept == 0 || dc || (long long)kept > A.nmax;
                A.ctl->n[A.par ^ 1] = stop ? 0 : (long long)kept;
                A.ctl->m[A.par ^ 1] = a.m_total;
                A.ctl->dm2[A.par ^ 1] = a.dmax2_bits;
                if (dc && kept) A.ctl->dcap_hit = 1u;
            }
            if (A.host_acc) {
                // publish to the mapped host copy, the sequence number last: the
                // host launches the next iteration while the rows still move
                DevAcc *o = A.host_acc;
                __hip_atomic_store(&o->nR, a.nR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&o->nT, a.nT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&o->m_total, a.m_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&o->nM_iter, a.nM_iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store((unsigned long long *)&o->pow_next, __double_as_longlong(a.pow_next),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&o->dmax2_bits, a.dmax2_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&o->qerr, a.qerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
                for (int m = 0; m < LPC_MP_MAX; ++m)
                    if (m < A.nmp)
                        __hip_atomic_store((unsigned long long *)&o->mpow[m], __double_as_longlong(mp[m]),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&o->seq, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        // the next launch's words (k_slot_init's misc reset) and group counts
        if (A.misc)
            for (int i = t; i < LPC_MISC_WORDS; i += LPC_ST_TILE) A.misc[i] = i < 3 ? 0xffffffffu : 0u;
        for (int64_t k = t; k < A.gdirty_next; k += LPC_ST_TILE) A.gsum_next[k] = 0ull;
    }
    // this tile's staged rows into place: kept children (two per thread at most,
    // loads of both issued before the stores), then measured rays
    const uint32_t v = tile < ntiles ? A.tcnt[tile] : 0u;
    const int cR = (int)(v & 511u), cT = (int)((v >> 9) & 511u), cM = (int)((v >> 18) & 511u);
    const int64_t c = A.cst, cb = A.capR, cm = A.capM, s0 = tile * LPC_ST_TILE;
    float row[2][8];
    int64_t dst[2] = {-1, -1};
    bool toT[2] = {false, false};             // chunked: a refracted row into the staging population
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int i = t + h * LPC_ST_TILE;
        if (i < cR + cT) {
            const bool isR = i < cR;
            toT[h] = chunked && !isR;
            const float *src = isR ? A.stR : A.stT;
            const int64_t q = s0 + (isR ? i : i - cR);
            dst[h] = isR ? (int64_t)r_base + s_pre[0] + i
                         : chunked ? (int64_t)t_base + s_pre[1] + (i - cR) : s_tot[0] + s_pre[1] + (i - cR);
#pragma unroll
            for (int a = 0; a < 8; ++a) row[h][a] = src[a * c + q];
        }
    }
    float mrow[5];
    const bool hasM = t < cM;
    if (hasM)
#pragma unroll
        for (int a = 0; a < 5; ++a) mrow[a] = A.stM[a * c + s0 + t];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (dst[h] < 0) continue;
        float *P = toT[h] ? A.popT : A.popR;
        const int64_t pc = toT[h] ? A.capT : cb;
#pragma unroll
        for (int a = 0; a < 8; ++a) P[a * pc + dst[h]] = row[h][a];
    }
    if (hasM) {
        const int64_t d = (int64_t)m_base + s_pre[2] + t;
#pragma unroll
        for (int a = 0; a < 5; ++a) A.mrec[a * cm + d] = mrow[a];
    }
    };
    if constexpr (!DS) {
        tile_body(blockIdx.x);                    // one tile per block
    } else {
        for (int64_t tile = blockIdx.x; tile < max(ntiles, (int64_t)1); tile += gridDim.x) {
            tile_body(tile);
            __syncthreads();                      // s_red / s_pre / s_tot reused by the next tile
        }
    }
}

// The one-tile-per-block form at 8 waves per SIMD (64 VGPRs, no scratch): its
// blocks are row moves, more of them in flight hide the loads' latency; the
// grid-stride device-sized form keeps more live across its tile loop and would
// spill at that bound.
#ifndef LPC_MOVE_OCC
#define LPC_MOVE_OCC 1
#endif
#if LPC_MOVE_OCC
#define LPC_MOVE_ATTR __attribute__((amdgpu_waves_per_eu(8)))
#else
#define LPC_MOVE_ATTR
#endif
template <bool DS>
__global__ __launch_bounds__(LPC_ST_TILE) void k_stage_move(MoveArgs A);
template <>
__global__ __launch_bounds__(LPC_ST_TILE) LPC_MOVE_ATTR void k_stage_move<false>(MoveArgs A)
{
    stage_move<false>(A);
}
template <>
__global__ __launch_bounds__(LPC_ST_TILE) void k_stage_move<true>(MoveArgs A)
{
    stage_move<true>(A);
}

// Append the refracted block after the reflected one (next population).
__global__ __launch_bounds__(256) void k_append(RaysOut dst, RaysIn src, const DevAcc *acc, int64_t cap_dst,
                                                int64_t cap_src)
{
    const int64_t nR = (int64_t)acc->nR, nT = (int64_t)acc->nT;
    if (nR < 0 || nT < 0 || nT > cap_src || nR + nT > cap_dst) return;   // broken counts (reported by the host)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nT;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = nR + i;
        dst.ox[q] = src.ox[i]; dst.oy[q] = src.oy[i]; dst.oz[q] = src.oz[i];
        dst.dx[q] = src.dx[i]; dst.dy[q] = src.dy[i]; dst.dz[q] = src.dz[i];
        dst.pw[q] = src.pw[i]; dst.pmid[q] = src.pmid[i];
    }
}

// Population copy (trace reset: emitted rays -> current population), one launch.
__global__ __launch_bounds__(256) void k_copy_pop(RaysOut dst, RaysIn src, int64_t n)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        dst.ox[i] = src.ox[i]; dst.oy[i] = src.oy[i]; dst.oz[i] = src.oz[i];
        dst.dx[i] = src.dx[i]; dst.dy[i] = src.dy[i]; dst.dz[i] = src.dz[i];
        dst.pw[i] = src.pw[i]; dst.pmid[i] = src.pmid[i];
    }
}

// Iteration counters start: kept children 0, measured record length m_total
// (in-stream, no host round trip).
__global__ void k_acc_init(DevAcc *acc, unsigned long long m_total)
{
    if (threadIdx.x == 0) {
        DevAcc z;
        memset(&z, 0, sizeof(z));
        z.m_total = m_total;
        *acc = z;
    }
}

// SoA xyz -> (n,4) rows with w = 0
// Scene upload: the hit triangles' vertices (9 floats each, the shading's
// normal) and the exact records in leaf order (xorder: triangle per record),
// from the (M,4) rows on the device.
__global__ __launch_bounds__(256) void k_vertex_rows(int64_t M, const float4 *__restrict__ v0,
                                                     const float4 *__restrict__ v1, const float4 *__restrict__ v2,
                                                     float *__restrict__ verts)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const float4 a = v0[i], b = v1[i], c = v2[i];
    float *o = verts + 9 * i;
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = b.x; o[4] = b.y; o[5] = b.z; o[6] = c.x; o[7] = c.y; o[8] = c.z;
}

__global__ __launch_bounds__(256) void k_exact_records(int64_t nx, const int32_t *__restrict__ xorder,
                                                       const float4 *__restrict__ v0, const float4 *__restrict__ v1,
                                                       const float4 *__restrict__ v2, ExactRec *__restrict__ xrec)
{
    LPC_EXACT
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nx) return;
    const int32_t i = xorder[p];
    const float4 a = v0[i], b = v1[i], c = v2[i];
    ExactRec x;
    x.v0x = a.x; x.v0y = a.y; x.v0z = a.z;
    x.e1x = b.x - a.x; x.e1y = b.y - a.y; x.e1z = b.z - a.z;       // E1 = V1 - V0, E2 = V2 - V0 (float, .cl:72-73)
    x.e2x = c.x - a.x; x.e2y = c.y - a.y; x.e2z = c.z - a.z;
    x.idx = i;
    x.pad1 = x.pad2 = 0.0f;
    xrec[p] = x;
}

__global__ __launch_bounds__(256) void k_pack4(int64_t n, const float *__restrict__ x,
                                               const float *__restrict__ y,
                                               const float *__restrict__ z, float4 *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_float4(x[i], y[i], z[i], 0.0f);
}

// Results export (iterative_tracer.py:335-355): one chunk's part of the
// iteration's results tuple in its host layout, so one DMA moves it:
// [origin (n,4) if org][dest (n,4)][pow (n)][meas (n)], w = 0.  Each thread
// writes whole 16-byte rows (coalesced); the copy to the caller's pinned block
// runs on the export stream while the next kernels run.
__global__ __launch_bounds__(256) void k_export(int64_t n, RaysIn in, ShadeOutPtrs o, int org,
                                                float4 *__restrict__ xo, float4 *__restrict__ xd,
                                                float *__restrict__ xp, int32_t *__restrict__ xm)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (org) xo[i] = make_float4(in.ox[i], in.oy[i], in.oz[i], 0.0f);
    xd[i] = make_float4(o.destx[i], o.desty[i], o.destz[i], 0.0f);
    xp[i] = o.pw[i];
    xm[i] = o.meas[i];
}

// (n,4) rows -> SoA xyz
// Results export into a mapped host block (the drop-in's results mode): a
// grid-stride copy with 16-byte vector stores (a 4-byte tail) written over PCIe
// from the export stream, instead of a DMA copy.
typedef uint32_t lpc_u4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy_host(const lpc_u4 *__restrict__ src, lpc_u4 *__restrict__ dst,
                                                   int64_t n16, int64_t bytes)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        __builtin_nontemporal_store(src[i], &dst[i]);
    const int64_t t0 = n16 * 16, nt = (bytes - t0) / 4;
    if (blockIdx.x == 0 && (int64_t)threadIdx.x < nt)
        ((uint32_t *)((char *)dst + t0))[threadIdx.x] = ((const uint32_t *)((const char *)src + t0))[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_unpack4(int64_t n, const float4 *__restrict__ in,
                                                 float *__restrict__ x, float *__restrict__ y,
                                                 float *__restrict__ z)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { const float4 v = in[i]; x[i] = v.x; y[i] = v.y; z[i] = v.z; }
}

// ---------------------------------------------------------------------------
// Drop-in kernels on the reference's (n,4) / [ray][mesh] device buffers.
__global__ __launch_bounds__(256) void k_postproc_aos(PostprocAosArgs A)
{
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= A.n) return;
    const int32_t K = A.K;
    auto slot = [&](int32_t j, float &t, int32_t &c, int32_t &i) {
        const int64_t a = r * K + j;
        t = A.tmin[a]; c = A.cnt[a]; i = A.itmp[a];
    };
    const PostOut po = postproc(K, A.prev_mid[r], A.mat_type, A.max_ray_len, slot);
    const float4 o4 = A.origin[r], d4 = A.dir[r];
    const f3 dest = ray_dest(mk3(o4.x, o4.y, o4.z), mk3(d4.x, d4.y, d4.z), po.t_min);
    if (po.hit_mesh >= 0) A.entering[r] = po.entering;
    A.n1[r] = po.n1; A.n2[r] = po.n2;
    A.dest[r] = make_float4(dest.x, dest.y, dest.z, 0.0f);
    A.imid[r] = po.hit_mesh; A.iidx[r] = po.hit_idx;
}

__global__ __launch_bounds__(256) void k_fresnel_aos(FresnelAosArgs A)
{
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= A.n) return;
    const float4 o4 = A.origin[r], d4 = A.dir[r], e4 = A.dest[r];
    const f3 dest = mk3(e4.x, e4.y, e4.z);
    auto tri = [&](int32_t idx, f3 &v0, f3 &v1, f3 &v2) {
        const float *v = A.verts + (int64_t)idx * 9;
        v0 = mk3(v[0], v[1], v[2]); v1 = mk3(v[3], v[4], v[5]); v2 = mk3(v[6], v[7], v[8]);
    };
    const float pw_in = A.pow[r];
    const ShadeOut s = shade(mk3(o4.x, o4.y, o4.z), mk3(d4.x, d4.y, d4.z), dest, pw_in, A.meas[r],
                             A.imid[r], A.iidx[r], A.n1[r], A.n2[r], A.mat_type, A.ior, A.refl,
                             A.diss, A.ior_env, tri);
    if (s.pow != pw_in) A.pow[r] = s.pow;
    A.meas[r] = s.meas;
    const float4 e0 = make_float4(dest.x, dest.y, dest.z, 0.0f);
    A.r_origin[r] = e0; A.t_origin[r] = e0;
    A.r_dir[r] = make_float4(s.r_dir.x, s.r_dir.y, s.r_dir.z, 0.0f);
    A.t_dir[r] = make_float4(s.t_dir.x, s.t_dir.y, s.t_dir.z, 0.0f);
    A.r_pow[r] = s.r_pow; A.r_meas[r] = s.r_meas;
    A.t_pow[r] = s.t_pow; A.t_meas[r] = s.t_meas;
}

// ---------------------------------------------------------------------------
// Projection + binning.  Bin index = searchsorted(edges, v, 'right') - 1 with
// the value equal to the last edge counted in the last bin (numpy histogramdd).
static __device__ __forceinline__ int bin_of(double v, const double *__restrict__ e, int nbins)
{
    if (!(v >= e[0]) || !(v <= e[nbins])) return -1;   // outside (or NaN)
    if (v == e[nbins]) return nbins - 1;
    int lo = 0, hi = nbins;                              // e[lo] <= v < e[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (e[mid] <= v) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_project_hist(ProjArgs A)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n) return;
    f3 p;
    if (A.pos4) { const float4 v = A.pos4[i]; p = mk3(v.x, v.y, v.z); }
    else p = mk3(A.px[i], A.py[i], A.pz[i]);
    const f3 piv = mk3(A.piv[0], A.piv[1], A.piv[2]);
    const f3 R0 = mk3(A.rot[0], A.rot[1], A.rot[2]);
    const f3 R1 = mk3(A.rot[4], A.rot[5], A.rot[6]);
    const f3 R2 = mk3(A.rot[8], A.rot[9], A.rot[10]);
    float x, y, pc;
    if (A.mode == 0) angular_project(p, piv, R0, R1, R2, A.pwr[i], x, y, pc);
    else stereograph_project(p, piv, R0, R1, R2, A.pwr[i], x, y, pc);
    if (A.x) { A.x[i] = x; A.y[i] = y; A.pc[i] = pc; }
    const int bx = bin_of((double)x, A.xe, A.nx), by = bin_of((double)y, A.ye, A.ny);
    if (bx >= 0 && by >= 0) atomicAdd(&A.H[(int64_t)bx * A.ny + by], (double)pc / A.div);
}

// Per-measure-mesh power of the measured record, one block per 64K records,
// fixed-order sums (the host adds the block partials in order).
// Deterministic float64 per-mesh power: fixed tiles, fixed reduction tree.
#define LPC_MSUM_TILE 2048
__global__ __launch_bounds__(256) void k_mesh_sum(int64_t n, const float *__restrict__ mp,
                                                  const int32_t *__restrict__ mm, int32_t mesh,
                                                  double *__restrict__ out)
{
    __shared__ double s[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t lo = (int64_t)blockIdx.x * LPC_MSUM_TILE;
    const int64_t hi = lo + LPC_MSUM_TILE < n ? lo + LPC_MSUM_TILE : n;
    double acc = 0.0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256)
        if (mm[i] == mesh) acc += (double)mp[i];
    acc = wave_sum(acc);
    if (lane == 0) s[wv] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = ((s[0] + s[1]) + s[2]) + s[3];
}

}  // namespace lpck
