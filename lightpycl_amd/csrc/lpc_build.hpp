// lpc_build.hpp -- host build of the scene's filter records (plain C++, no HIP):
// per mesh run, the W-wide sphere hierarchy (NodeW<8> records, each node's test
// over ALL triangles below it) and the sliver / thin-triangle line-filter
// records.  lpc_scene_upload (lpc_runtime.hip) uploads what this builds;
// tools/scene_build_bench.cpp times it on the CPU.
//
// The runs are independent, so they are built on a pool of host threads and
// concatenated in run order afterwards (node ids offset by the nodes of the
// earlier runs): the records are the same bytes whatever the thread count.
// Per node, the bounding box and the Moller-Trumbore error factor kappa of the
// triangles below (node_record's max / min over them) combine from the
// children's, which were computed over the same triangles; only the radius
// about the node's own centre needs the vertices again.
#pragma once
#include "lpc_math.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

namespace lpc {

struct SceneBuildIn {
    const float *v0, *v1, *v2;          // (M, 4) rows, w ignored
    const int32_t *run_lo, *run_hi;     // runs of equal mesh id: triangles [lo, hi)
    size_t nr;
    double dcap;                        // largest |D| the filter records cover
    double scene_scale;                 // half diagonal of the scene box
    double thin_k;                      // thin-triangle rule factor (thin_axis)
    int stack_max;                      // the walk's node-stack depth
};

struct SceneBuildOut {
    std::vector<Node8> nodes;
    std::vector<SliverRec> slivers;
    std::vector<std::vector<int32_t>> run_levels;   // per run: (first node, count) per level, top down
    std::vector<FiltRec> node_self;                 // per node: its own test (node_record of all below)
    std::vector<int32_t> run_slo, run_shi;          // per run: its slivers [slo, shi)
    std::vector<int32_t> xorder;                    // per hierarchy position: the triangle (exact records
                                                    //   in leaf order; a leaf child's ref is ~position)
    std::vector<float> sliver_dmin;                 // per sliver record
    int64_t n_slivers = 0, n_thin = 0;
};

// Top-down partition of e[0, n) for a subtree of capacity cap (leaf * W^k):
// split at min(n, cap / 2) along the longest axis of the centroids' bbox
// (nth_element, ties by entry id), recurse on both halves with cap / 2, down to
// groups of `leaf`.  The centroids travel with their ids (contiguous, no gather).
struct CenEnt {
    double c[3];
    int64_t id;
};
static inline void split_order(CenEnt *e, int64_t n, int64_t cap, int64_t leaf)
{
    if (cap <= leaf || n <= 1) return;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            const double c = e[i].c[k];
            if (std::isfinite(c)) { lo[k] = std::min(lo[k], c); hi[k] = std::max(hi[k], c); }
        }
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (hi[k] - lo[k] > hi[ax] - lo[ax]) ax = k;
    const int64_t half = std::min(n, cap / 2);
    if (half < n)
        std::nth_element(e, e + half, e + n, [ax](const CenEnt &a, const CenEnt &b) {
            return a.c[ax] < b.c[ax] || (a.c[ax] == b.c[ax] && a.id < b.id);
        });
    split_order(e, half, cap / 2, leaf);
    split_order(e + half, n - half, cap / 2, leaf);
}

static inline FiltRec build_test_rec(float cx, float cy, float cz, float negB, float negA)
{
    FiltRec r;
    r.cx = cx; r.cy = cy; r.cz = cz; r.negB = negB; r.negA = negA; r.idx = -1; r.pad0 = r.pad1 = 0;
    return r;
}

namespace detail {

struct RunOut {
    std::vector<Node8> nodes;           // node refs local to the run (offset at the merge)
    std::vector<FiltRec> self;
    std::vector<SliverRec> sl;
    std::vector<std::pair<int32_t, int32_t>> levels;   // (first local node, count), bottom up
    std::vector<int32_t> order;         // the run's hierarchy triangles in leaf order (local positions)
    int64_t n_thin = 0;
    bool too_deep = false;
};

// Aggregates of a hierarchy entry (a triangle or a node) over its triangles.
struct Agg {
    double lo[3], hi[3], kappa;
};

static inline void build_run(const SceneBuildIn &in, size_t r, RunOut &out)
{
    const int W = 8;
    const FiltRec never = build_test_rec(0.0f, 0.0f, 0.0f, 0.0f, INFINITY);
    auto vptr = [&](int32_t t, int v) -> const float * {
        return (v == 0 ? in.v0 : v == 1 ? in.v1 : in.v2) + 4 * (size_t)t;
    };
    const int32_t lo = in.run_lo[r], cnt_all = in.run_hi[r] - lo;
    std::vector<FiltRec> fr;                         // hierarchy triangles
    std::vector<double> cen;
    std::vector<int32_t> sl;
    std::vector<int> sl_ax;                          // the sliver record's filter edge (thin_axis result)
    for (int32_t i = 0; i < cnt_all; ++i) {
        const int32_t t = lo + i;
        const float *V0 = vptr(t, 0), *V1 = vptr(t, 1), *V2 = vptr(t, 2);
        const FiltRec f = filter_record(V0, V1, V2, t, in.dcap, in.scene_scale);
        if (f.negA == INFINITY) continue;                           // never a candidate
        if (f.negB < -1e29f) { sl.push_back(t); sl_ax.push_back(1); continue; }
        // thin: the line filter about its longer edge (k_slivers) bounds it better
        const int ax = thin_axis(V0, V1, V2, f.cx, f.cy, f.cz, in.scene_scale, in.thin_k);
        if (ax) {
            sl.push_back(t);
            sl_ax.push_back(ax);
            ++out.n_thin;
            continue;
        }
        fr.push_back(f);
        for (int k = 0; k < 3; ++k) cen.push_back(((double)V0[k] + V1[k] + V2[k]) / 3.0);
    }
    // slivers ordered by dmin, so a 64-sliver piece holds similar ones
    {
        std::vector<std::pair<float, size_t>> sld;
        for (size_t q = 0; q < sl.size(); ++q) sld.push_back({sliver_dmin(vptr(sl[q], 0), vptr(sl[q], 1), vptr(sl[q], 2)), q});
        std::stable_sort(sld.begin(), sld.end(), [](const std::pair<float, size_t> &x, const std::pair<float, size_t> &y) {
            return x.first < y.first;
        });
        for (const auto &e : sld) {
            const int32_t t32 = sl[e.second];
            const float *V0 = vptr(t32, 0), *V1 = vptr(t32, 1), *V2 = vptr(t32, 2);
            SliverRec S;
            memset(&S, 0, sizeof(S));
            S.v0x = V0[0]; S.v0y = V0[1]; S.v0z = V0[2];
            // a thin triangle whose longer edge is E1 filters about E1 (e2 holds it)
            S.ax1 = sl_ax[e.second] == 2 ? 1 : 0;
            const float e1[3] = {V1[0] - V0[0], V1[1] - V0[1], V1[2] - V0[2]};
            const float e2[3] = {V2[0] - V0[0], V2[1] - V0[1], V2[2] - V0[2]};
            const float *ea = S.ax1 ? e1 : e2, *eb = S.ax1 ? e2 : e1;
            S.e2x = ea[0]; S.e2y = ea[1]; S.e2z = ea[2];
            S.e1x = eb[0]; S.e1y = eb[1]; S.e1z = eb[2];
            sliver_params_axis(V0, V1, V2, S.ax1, &S.a, &S.b);
            S.idx = t32;
            S.dmin = e.first;
            out.sl.push_back(S);
        }
    }
    const int32_t cnt = (int32_t)fr.size();
    if (cnt == 0) return;
    // top-down order: every aligned group of W^k entries is one median-split
    // cluster, so the bottom-up W-wide grouping below reproduces that tree
    std::vector<int32_t> perm((size_t)cnt);
    {
        std::vector<CenEnt> ce((size_t)cnt);
        for (int32_t i = 0; i < cnt; ++i) {
            for (int k = 0; k < 3; ++k) ce[(size_t)i].c[k] = cen[3 * (size_t)i + k];
            ce[(size_t)i].id = i;
        }
        int64_t cap = W;
        while (cap < cnt) cap *= W;
        split_order(ce.data(), cnt, cap, W);
        for (int32_t i = 0; i < cnt; ++i) perm[(size_t)i] = (int32_t)ce[(size_t)i].id;
    }
    // the ordered triangles' vertex pointers and aggregates
    std::vector<const float *> tv((size_t)cnt * 3);
    std::vector<Agg> tagg((size_t)cnt);
    for (int32_t a = 0; a < cnt; ++a) {
        const int32_t t = fr[(size_t)perm[(size_t)a]].idx;
        Agg &g = tagg[(size_t)a];
        for (int k = 0; k < 3; ++k) { g.lo[k] = INFINITY; g.hi[k] = -INFINITY; }
        for (int v = 0; v < 3; ++v) {
            const float *P = vptr(t, v);
            tv[3 * (size_t)a + v] = P;
            for (int k = 0; k < 3; ++k) { g.lo[k] = fmin(g.lo[k], (double)P[k]); g.hi[k] = fmax(g.hi[k], (double)P[k]); }
        }
        g.kappa = fmax(0.0, tri_kappa(tv[3 * (size_t)a], tv[3 * (size_t)a + 1], tv[3 * (size_t)a + 2]));
    }
    // node_record over the ordered triangles [a, b) with the aggregates g
    auto range_test = [&](int32_t a, int32_t b, const Agg &g) {
        FiltRec t = never;
        if (!(g.kappa < 0.1)) { t.negB = -1e30f; t.negA = 0.0f; return t; }      // always
        const float C[3] = {(float)(0.5 * (g.lo[0] + g.hi[0])), (float)(0.5 * (g.lo[1] + g.hi[1])),
                            (float)(0.5 * (g.lo[2] + g.hi[2]))};
        double R2 = 0.0;
        for (size_t i = 3 * (size_t)a; i < 3 * (size_t)b; ++i) {
            const float *P = tv[i];
            double d2 = 0.0;
            for (int k = 0; k < 3; ++k) { const double q = (double)P[k] - C[k]; d2 += q * q; }
            R2 = fmax(R2, d2);
        }
        t.cx = C[0]; t.cy = C[1]; t.cz = C[2];
        const double ra = sqrt(R2 * (1.0 + 1e-6)) * (1.0 + g.kappa);
        const double h = ra > 0.0 ? fmin(1.0, fmax(1e-3, g.kappa * in.scene_scale / ra)) : 1.0;
        store_test((1.0 + h) * ra * ra, (1.0 + 1.0 / h) * g.kappa * g.kappa, &t.negB, &t.negA);
        return t;
    };
    struct Ent { FiltRec t; int32_t ref, a, b; Agg g; };
    std::vector<Ent> ent((size_t)cnt);
    out.order.resize((size_t)cnt);
    for (int32_t a = 0; a < cnt; ++a) {
        const FiltRec &f = fr[(size_t)perm[(size_t)a]];
        ent[(size_t)a] = {f, ~a, a, a + 1, tagg[(size_t)a]};      // a leaf child: ~ its (local) position
        out.order[(size_t)a] = f.idx;
    }
    do {
        std::vector<Ent> up;
        const int32_t first = (int32_t)out.nodes.size();
        for (size_t i = 0; i < ent.size(); i += (size_t)W) {
            Node8 N;
            memset(&N, 0, sizeof(N));
            Agg g;
            for (int k = 0; k < 3; ++k) { g.lo[k] = INFINITY; g.hi[k] = -INFINITY; }
            g.kappa = 0.0;
            for (int k = 0; k < W; ++k) {
                const bool use = i + k < ent.size();
                const FiltRec &m = use ? ent[i + k].t : never;
                N.cx[k] = m.cx; N.cy[k] = m.cy; N.cz[k] = m.cz; N.negB[k] = m.negB; N.negA[k] = m.negA;
                N.ref[k] = use ? ent[i + k].ref : ~0;
                if (use) {
                    const Agg &c = ent[i + k].g;
                    for (int q = 0; q < 3; ++q) { g.lo[q] = fmin(g.lo[q], c.lo[q]); g.hi[q] = fmax(g.hi[q], c.hi[q]); }
                    g.kappa = fmax(g.kappa, c.kappa);
                }
            }
            const int32_t a = ent[i].a, b = ent[std::min(i + (size_t)W - 1, ent.size() - 1)].b;
            const FiltRec self = range_test(a, b, g);
            up.push_back({self, (int32_t)out.nodes.size(), a, b, g});
            out.nodes.push_back(N);
            out.self.push_back(self);
        }
        out.levels.push_back({first, (int32_t)up.size()});
        ent.swap(up);
    } while (ent.size() > 1);
    // W-wide: at most W - 1 siblings wait per level on a wave's stack
    if ((W - 1) * (int)out.levels.size() + 1 > in.stack_max) out.too_deep = true;
}

}  // namespace detail

// parfor(n, fn): fn(0) .. fn(n - 1), in any order, on host threads (the
// runtime's persistent pool; tools/scene_build_probe.cpp spawns threads).
using ParFor = std::function<void(int, const std::function<void(int)> &)>;

// The scene's records, the runs built as parallel tasks.  Returns "" or an
// error message.
static inline std::string build_scene_records(const SceneBuildIn &in, SceneBuildOut &out, const ParFor &parfor)
{
    std::vector<detail::RunOut> runs(in.nr);
    // the larger runs first, so the pool's last thread does not start a big one late
    std::vector<size_t> order(in.nr);
    for (size_t r = 0; r < in.nr; ++r) order[r] = r;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return in.run_hi[a] - in.run_lo[a] > in.run_hi[b] - in.run_lo[b];
    });
    parfor((int)in.nr, [&](int q) { detail::build_run(in, order[(size_t)q], runs[order[(size_t)q]]); });
    // concatenation in run order: the records of a serial build
    out = SceneBuildOut();
    size_t total = 0;
    for (const auto &R : runs) total += R.nodes.size();
    out.nodes.reserve(total + 1);
    out.node_self.reserve(total);
    for (size_t r = 0; r < in.nr; ++r) {
        detail::RunOut &R = runs[r];
        if (R.too_deep) return "mesh hierarchy too deep";
        const int32_t base = (int32_t)out.nodes.size();
        const int32_t pbase = (int32_t)out.xorder.size();
        out.xorder.insert(out.xorder.end(), R.order.begin(), R.order.end());
        out.run_slo.push_back((int32_t)out.slivers.size());
        out.slivers.insert(out.slivers.end(), R.sl.begin(), R.sl.end());
        out.run_shi.push_back((int32_t)out.slivers.size());
        out.n_slivers += (int64_t)R.sl.size();
        out.n_thin += R.n_thin;
        for (Node8 &N : R.nodes)
            for (int k = 0; k < 8; ++k) {
                if (N.ref[k] >= 0) N.ref[k] += base;                          // child node
                else if (N.negA[k] != INFINITY) N.ref[k] = ~(~N.ref[k] + pbase);   // triangle (unused: never)
            }
        out.nodes.insert(out.nodes.end(), R.nodes.begin(), R.nodes.end());
        out.node_self.insert(out.node_self.end(), R.self.begin(), R.self.end());
        std::vector<int32_t> lv;
        for (auto it = R.levels.rbegin(); it != R.levels.rend(); ++it) {
            lv.push_back(it->first + base);
            lv.push_back(it->second);
        }
        out.run_levels.push_back(std::move(lv));
    }
    return "";
}

}  // namespace lpc
