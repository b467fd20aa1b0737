// scene_build_probe.cpp -- CPU timing and byte-equality check of the scene
// record build (lightpycl_amd/csrc/lpc_build.hpp), no GPU.
//
//   g++ -O3 -std=c++17 -fPIC -shared -pthread -I lightpycl_amd/csrc tools/scene_build_probe.cpp \
//       -o tools/_scene_build_probe.so
//
// sbp_build(v0, v1, v2, mesh_id, M, dcap, scene_scale, threads, reps, out_ms, out_digest)
// flattens the runs as lpc_scene_upload does, builds `reps` times with
// `threads` host threads, and returns the best time and a 64-bit FNV digest of
// every record (nodes, node tests, slivers, levels), so builds with different
// thread counts can be compared byte for byte.
#include "lpc_build.hpp"

#include <chrono>
#include <cstdint>

using namespace lpc;

static uint64_t fnv(uint64_t h, const void *p, size_t n)
{
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
    return h;
}

extern "C" int sbp_build(const float *v0, const float *v1, const float *v2, const int32_t *mesh_id, int32_t M,
                         double dcap, double scene_scale, int threads, int reps, double *out_ms,
                         uint64_t *out_digest, int64_t *out_nodes)
{
    std::vector<int32_t> lo, hi;
    for (int32_t i = 0; i < M; ++i) {
        if (i == 0 || mesh_id[i] != mesh_id[i - 1]) { lo.push_back(i); hi.push_back(i + 1); }
        else hi.back() = i + 1;
    }
    SceneBuildIn in;
    in.v0 = v0; in.v1 = v1; in.v2 = v2;
    in.run_lo = lo.data(); in.run_hi = hi.data(); in.nr = lo.size();
    in.dcap = dcap; in.scene_scale = scene_scale; in.thin_k = 1.0; in.stack_max = 64;
    double best = 1e30;
    SceneBuildOut out;
    // tasks taken in index order by `threads` spawned threads
    const ParFor parfor = [threads](int n, const std::function<void(int)> &fn) {
        std::atomic<int> next(0);
        auto w = [&]() { for (int i; (i = next.fetch_add(1)) < n;) fn(i); };
        std::vector<std::thread> th;
        for (int k = 1; k < threads; ++k) th.emplace_back(w);
        w();
        for (std::thread &x : th) x.join();
    };
    for (int r = 0; r < reps; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        const std::string err = build_scene_records(in, out, parfor);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (!err.empty()) return -1;
        best = ms < best ? ms : best;
    }
    // leaf refs back to triangle indices (the round-5 layout the serial build makes)
    for (Node8 &N : out.nodes)
        for (int k = 0; k < 8; ++k)
            if (N.ref[k] < 0 && N.negA[k] != INFINITY) N.ref[k] = ~out.xorder[(size_t)~N.ref[k]];
    uint64_t h = 1469598103934665603ull;
    h = fnv(h, out.nodes.data(), out.nodes.size() * sizeof(Node8));
    h = fnv(h, out.node_self.data(), out.node_self.size() * sizeof(FiltRec));
    h = fnv(h, out.slivers.data(), out.slivers.size() * sizeof(SliverRec));
    for (const auto &L : out.run_levels) h = fnv(h, L.data(), L.size() * 4);
    h = fnv(h, out.run_slo.data(), out.run_slo.size() * 4);
    h = fnv(h, out.run_shi.data(), out.run_shi.size() * 4);
    *out_ms = best;
    *out_digest = h;
    *out_nodes = (int64_t)out.nodes.size();
    return 0;
}

static void old_split_order(int32_t *idx, int64_t n, int64_t cap, const std::vector<double> &cen, int64_t leaf)
{
    if (cap <= leaf || n <= 1) return;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            const double c = cen[3 * (size_t)idx[i] + k];
            if (std::isfinite(c)) { lo[k] = std::min(lo[k], c); hi[k] = std::max(hi[k], c); }
        }
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (hi[k] - lo[k] > hi[ax] - lo[ax]) ax = k;
    const int64_t half = std::min(n, cap / 2);
    if (half < n)
        std::nth_element(idx, idx + half, idx + n, [&](int32_t a, int32_t b) {
            const double ca = cen[3 * (size_t)a + ax], cb = cen[3 * (size_t)b + ax];
            return ca < cb || (ca == cb && a < b);
        });
    old_split_order(idx, half, cap / 2, cen, leaf);
    old_split_order(idx + half, n - half, cap / 2, cen, leaf);
}

// The round-5 serial build (lpc_runtime.hip build_records before round 6),
// kept here only as the byte-equality reference of the threaded build.
extern "C" int sbp_build_old(const float *v0, const float *v1, const float *v2, const int32_t *mesh_id, int32_t M,
                             double dcap, double scene_scale, double *out_ms, uint64_t *out_digest)
{
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<int32_t> run_lo, run_hi;
    for (int32_t i = 0; i < M; ++i) {
        if (i == 0 || mesh_id[i] != mesh_id[i - 1]) { run_lo.push_back(i); run_hi.push_back(i + 1); }
        else run_hi.back() = i + 1;
    }
    const int W = 8;
    const size_t node_bytes = sizeof(Node8);
    std::vector<uint8_t> nodes;
    int32_t n_nodes = 0;
    std::vector<SliverRec> slivers;
    std::vector<std::vector<int32_t>> run_levels;
    std::vector<FiltRec> node_self;
    std::vector<int32_t> run_slo, run_shi;
    const FiltRec never = build_test_rec(0.0f, 0.0f, 0.0f, 0.0f, INFINITY);
    auto vptr = [&](int32_t t, int v) -> const float * {
        return (v == 0 ? v0 : v == 1 ? v1 : v2) + 4 * (size_t)t;
    };
    for (size_t r = 0; r < run_lo.size(); ++r) {
        const int32_t lo = run_lo[r], cnt_all = run_hi[r] - lo;
        std::vector<FiltRec> fr;
        std::vector<double> cen;
        std::vector<int32_t> sl;
        for (int32_t i = 0; i < cnt_all; ++i) {
            const int32_t t = lo + i;
            const float *V0 = vptr(t, 0), *V1 = vptr(t, 1), *V2 = vptr(t, 2);
            const FiltRec f = filter_record(V0, V1, V2, t, dcap, scene_scale);
            if (f.negA == INFINITY) continue;
            if (f.negB < -1e29f) { sl.push_back(t); continue; }
            if (thin_axis(V0, V1, V2, f.cx, f.cy, f.cz, scene_scale, 1.0)) { sl.push_back(t); continue; }
            fr.push_back(f);
            for (int k = 0; k < 3; ++k) cen.push_back(((double)V0[k] + V1[k] + V2[k]) / 3.0);
        }
        run_slo.push_back((int32_t)slivers.size());
        std::vector<std::pair<float, int32_t>> sld;
        for (int32_t t32 : sl) sld.push_back({sliver_dmin(vptr(t32, 0), vptr(t32, 1), vptr(t32, 2)), t32});
        std::stable_sort(sld.begin(), sld.end(), [](const std::pair<float, int32_t> &x, const std::pair<float, int32_t> &y) {
            return x.first < y.first;
        });
        for (size_t q = 0; q < sld.size(); ++q) sl[q] = sld[q].second;
        for (int32_t t32 : sl) {
            const float *V0 = vptr(t32, 0), *V1 = vptr(t32, 1), *V2 = vptr(t32, 2);
            SliverRec S;
            memset(&S, 0, sizeof(S));
            S.v0x = V0[0]; S.v0y = V0[1]; S.v0z = V0[2];
            const FiltRec f = filter_record(V0, V1, V2, t32, dcap, scene_scale);
            const int ax = f.negB < -1e29f ? 1 : thin_axis(V0, V1, V2, f.cx, f.cy, f.cz, scene_scale, 1.0);
            S.ax1 = ax == 2 ? 1 : 0;
            const float e1[3] = {V1[0] - V0[0], V1[1] - V0[1], V1[2] - V0[2]};
            const float e2[3] = {V2[0] - V0[0], V2[1] - V0[1], V2[2] - V0[2]};
            const float *ea = S.ax1 ? e1 : e2, *eb = S.ax1 ? e2 : e1;
            S.e2x = ea[0]; S.e2y = ea[1]; S.e2z = ea[2];
            S.e1x = eb[0]; S.e1y = eb[1]; S.e1z = eb[2];
            sliver_params_axis(V0, V1, V2, S.ax1, &S.a, &S.b);
            S.idx = t32;
            S.dmin = sliver_dmin(V0, V1, V2);
            slivers.push_back(S);
        }
        run_shi.push_back((int32_t)slivers.size());
        run_levels.push_back(std::vector<int32_t>());
        const int32_t cnt = (int32_t)fr.size();
        if (cnt == 0) continue;
        std::vector<int32_t> perm_t((size_t)cnt);
        for (int32_t i = 0; i < cnt; ++i) perm_t[(size_t)i] = i;
        int64_t cap = W;
        while (cap < cnt) cap *= W;
        old_split_order(perm_t.data(), cnt, cap, cen, W);
        std::vector<const float *> tv;
        std::vector<int32_t> eo((size_t)cnt + 1, 0);
        for (int32_t i = 0; i < cnt; ++i) {
            const int32_t t = fr[(size_t)perm_t[(size_t)i]].idx;
            for (int v = 0; v < 3; ++v) tv.push_back(vptr(t, v));
            eo[(size_t)i + 1] = (int32_t)(tv.size() / 3);
        }
        auto range_test = [&](int32_t a, int32_t b) {
            FiltRec t = never;
            node_record(&tv[3 * (size_t)eo[(size_t)a]], eo[(size_t)b] - eo[(size_t)a], scene_scale, &t.cx, &t.cy,
                        &t.cz, &t.negB, &t.negA);
            return t;
        };
        struct Ent { FiltRec t; int32_t ref, a, b; };
        std::vector<Ent> ent((size_t)cnt);
        for (int32_t a = 0; a < cnt; ++a) {
            const FiltRec &f = fr[(size_t)perm_t[(size_t)a]];
            ent[(size_t)a] = {f, ~f.idx, a, a + 1};
        }
        std::vector<std::pair<int32_t, int32_t>> levels;
        do {
            std::vector<Ent> up;
            const int32_t first = n_nodes;
            for (size_t i = 0; i < ent.size(); i += (size_t)W) {
                std::vector<uint32_t> N(node_bytes / 4, 0u);
                for (int k = 0; k < W; ++k) {
                    const bool use = i + k < ent.size();
                    const FiltRec &m = use ? ent[i + k].t : never;
                    const float f5[5] = {m.cx, m.cy, m.cz, m.negB, m.negA};
                    for (int q = 0; q < 5; ++q) memcpy(&N[(size_t)q * W + k], &f5[q], 4);
                    const int32_t ref = use ? ent[i + k].ref : ~0;
                    memcpy(&N[(size_t)5 * W + k], &ref, 4);
                }
                const int32_t a = ent[i].a, b = ent[std::min(i + (size_t)W - 1, ent.size() - 1)].b;
                const FiltRec self = range_test(a, b);
                up.push_back({self, n_nodes, a, b});
                nodes.insert(nodes.end(), (const uint8_t *)N.data(), (const uint8_t *)N.data() + node_bytes);
                ++n_nodes;
                node_self.push_back(self);
            }
            levels.push_back({first, (int32_t)up.size()});
            ent.swap(up);
        } while (ent.size() > 1);
        for (auto it = levels.rbegin(); it != levels.rend(); ++it) {
            run_levels.back().push_back(it->first);
            run_levels.back().push_back(it->second);
        }
    }
    *out_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    uint64_t h = 1469598103934665603ull;
    h = fnv(h, nodes.data(), nodes.size());
    h = fnv(h, node_self.data(), node_self.size() * sizeof(FiltRec));
    h = fnv(h, slivers.data(), slivers.size() * sizeof(SliverRec));
    for (const auto &L : run_levels) h = fnv(h, L.data(), L.size() * 4);
    h = fnv(h, run_slo.data(), run_slo.size() * 4);
    h = fnv(h, run_shi.data(), run_shi.size() * 4);
    *out_digest = h;
    return 0;
}
