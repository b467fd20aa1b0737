// CPU harness for lpc_math.hpp (the header the HIP kernels include): evaluates the
// bounding-sphere filter the way k_intersect does (fused multiply-adds in float)
// and the exact Moller-Trumbore acceptance, for property tests of the filter margin.
#include <cmath>
#include <cstring>
#include <algorithm>
#include <vector>
#include "lpc_math.hpp"

using namespace lpc;

extern "C" void filt_eval(int n, const float *O, const float *D, const float *V, float eps, double dcap,
                          float *d_out, int *hit_out, float *t_out)
{
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *dd = D + 3 * i, *v = V + 9 * i;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        FiltRec r = filter_record(v0, v1, v2, 0, dcap);
        // k_intersect: unit direction, w = c - O, ww, wd, tq = negA - wd^2, d = ww*onemB + tq
        float s = 1.0f / sqrtf(fmaf(dd[2], dd[2], fmaf(dd[1], dd[1], dd[0] * dd[0])));
        float nx = dd[0] * s, ny = dd[1] * s, nz = dd[2] * s;
        float wx = r.cx - o[0], wy = r.cy - o[1], wz = r.cz - o[2];
        float ww = fmaf(wz, wz, fmaf(wy, wy, wx * wx));
        float wd = fmaf(wz, nz, fmaf(wy, ny, wx * nx));
        float tq = fmaf(-wd, wd, r.negA);
        d_out[i] = fmaf(ww, r.onemB, tq);
        f3 V0 = mk3(v[0], v[1], v[2]);
        f3 E1 = mk3(v[3] - v[0], v[4] - v[1], v[5] - v[2]);
        f3 E2 = mk3(v[6] - v[0], v[7] - v[1], v[8] - v[2]);
        float t = 0.0f;
        int h = mt_exact(mk3(o[0], o[1], o[2]), mk3(dd[0], dd[1], dd[2]), V0, E1, E2, &t);
        hit_out[i] = h && t > eps;
        t_out[i] = t;
    }
}

// Cluster test vs member tests: rays (n) x one cluster of m triangles.  Writes
// each member's float test value (n*m) and the cluster's (n).
static inline float eval_test(const float *o, float nx, float ny, float nz, float cx, float cy, float cz,
                              float onemB, float negA)
{
    float wx = cx - o[0], wy = cy - o[1], wz = cz - o[2];
    float ww = fmaf(wz, wz, fmaf(wy, wy, wx * wx));
    float wd = fmaf(wz, nz, fmaf(wy, ny, wx * nx));
    float tq = fmaf(-wd, wd, negA);
    return fmaf(ww, onemB, tq);
}

extern "C" void cluster_eval(int n, const float *O, const float *D, int m, const float *V, double dcap,
                             float *d_tri, float *d_cl)
{
    FiltRec rec[64];
    for (int j = 0; j < m; ++j) {
        const float *v = V + 9 * j;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        rec[j] = filter_record(v0, v1, v2, j, dcap);
    }
    float cx, cy, cz, ob, na;
    cluster_record(rec, m, &cx, &cy, &cz, &ob, &na);
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *dd = D + 3 * i;
        float s = 1.0f / sqrtf(fmaf(dd[2], dd[2], fmaf(dd[1], dd[1], dd[0] * dd[0])));
        float nx = dd[0] * s, ny = dd[1] * s, nz = dd[2] * s;
        for (int j = 0; j < m; ++j)
            d_tri[(size_t)i * m + j] = eval_test(o, nx, ny, nz, rec[j].cx, rec[j].cy, rec[j].cz, rec[j].onemB, rec[j].negA);
        d_cl[i] = eval_test(o, nx, ny, nz, cx, cy, cz, ob, na);
    }
}

// Sliver line filter as k_intersect evaluates it (fused = 1: with FMA contraction,
// 0: without), plus the exact Moller-Trumbore acceptance of the same pairs.
extern "C" void sliver_eval(int n, const float *O, const float *D, const float *V, float eps, int fused,
                            float *d_out, int *hit_out, float *t_out)
{
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *dd = D + 3 * i, *v = V + 9 * i;
        float a, b;
        sliver_params(v, v + 3, v + 6, &a, &b);
        const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
        const float tx = o[0] - v[0], ty = o[1] - v[1], tz = o[2] - v[2];
        const float tm = fmaxf(fmaxf(fabsf(tx), fabsf(ty)), fabsf(tz));
        const float dl = sqrtf(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
        float d;
        if (fused) {
            const float cx = fmaf(e2y, tz, -(e2z * ty));
            const float cy = fmaf(e2z, tx, -(e2x * tz));
            const float cz = fmaf(e2x, ty, -(e2y * tx));
            const float x = fmaf(dd[2], cz, fmaf(dd[1], cy, dd[0] * cx));
            const float rhs = dl * fmaf(b, tm, a);
            d = fmaf(x, x, -(rhs * rhs));
        } else {
            const float cx = e2y * tz - e2z * ty;
            const float cy = e2z * tx - e2x * tz;
            const float cz = e2x * ty - e2y * tx;
            const float x = dd[0] * cx + dd[1] * cy + dd[2] * cz;
            const float rhs = dl * (a + b * tm);
            d = x * x - rhs * rhs;
        }
        d_out[i] = d;
        f3 V0 = mk3(v[0], v[1], v[2]);
        f3 E1 = mk3(v[3] - v[0], v[4] - v[1], v[5] - v[2]);
        f3 E2 = mk3(e2x, e2y, e2z);
        float t = 0.0f;
        int h = mt_exact(mk3(o[0], o[1], o[2]), mk3(dd[0], dd[1], dd[2]), V0, E1, E2, &t);
        hit_out[i] = h && t > eps;
        t_out[i] = t;
    }
}

// filter_record's classification: 0 sphere test, 1 never, 2 always (-> sliver list)
extern "C" void filt_class(int n, const float *V, double dcap, int *cls)
{
    for (int i = 0; i < n; ++i) {
        const float *v = V + 9 * i;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        FiltRec r = filter_record(v0, v1, v2, 0, dcap);
        cls[i] = r.negA == INFINITY ? 1 : (r.onemB < -1e29f ? 2 : 0);
    }
}

// Packet bound of rays [0, n) as k_packet builds it (sequential reductions).
static PacketRec packet_build(int n, const float *O, const float *D)
{
    PacketRec Q;
    memset(&Q, 0, sizeof(Q));
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool fin = true;
    float sx = 0, sy = 0, sz = 0;
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *d = D + 3 * i;
        for (int k = 0; k < 3; ++k) { mn[k] = fminf(mn[k], o[k]); mx[k] = fmaxf(mx[k], o[k]); }
        const float l = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        fin = fin && std::isfinite(l) && l > 0 && std::isfinite(o[0] + o[1] + o[2]);
        sx += d[0] / l; sy += d[1] / l; sz += d[2] / l;
    }
    packet_centre(mn, mx, Q);
    float r = 0;
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i;
        const float x = o[0] - Q.ox, y = o[1] - Q.oy, z = o[2] - Q.oz;
        r = fmaxf(r, sqrtf(x * x + y * y + z * z));
    }
    packet_finish(r, sx, sy, sz, Q);
    float ang = 0;
    for (int i = 0; i < n; ++i) {
        const float *d = D + 3 * i;
        const float l = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        ang = fmaxf(ang, packet_angle(d[0] / l, d[1] / l, d[2] / l, Q.ax, Q.ay, Q.az));
    }
    packet_angle_finish(ang, fin, Q);
    return Q;
}

// Soundness of the packet tests: rays in packets of `pk`, records = m triangles'
// sphere records (kind 0), their 64-triangle cluster records (kind 1), or their
// sliver line filters (kind 2).  out[0] = violations (a ray passes its per-ray
// test but the packet test fails), out[1] = (packet, record) pairs passing the
// packet test, out[2] = pairs with some ray passing, out[3] = incoherent packets.
extern "C" void packet_eval(int n, const float *O, const float *D, int pk, int m, const float *V, int kind,
                            double dcap, long long *out)
{
    std::vector<FiltRec> recs;
    std::vector<SliverRec> sl;
    for (int j = 0; j < m; ++j) {
        const float *v = V + 9 * j;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        if (kind == 2) {
            SliverRec S;
            memset(&S, 0, sizeof(S));
            S.v0x = v[0]; S.v0y = v[1]; S.v0z = v[2];
            S.e2x = v[6] - v[0]; S.e2y = v[7] - v[1]; S.e2z = v[8] - v[2];
            sliver_params(v0, v1, v2, &S.a, &S.b);
            sl.push_back(S);
        } else {
            recs.push_back(filter_record(v0, v1, v2, j, dcap));
        }
    }
    if (kind == 1) {
        std::vector<FiltRec> cl;
        for (size_t a = 0; a < recs.size(); a += 64) {
            FiltRec c;
            memset(&c, 0, sizeof(c));
            cluster_record(&recs[a], (int)std::min<size_t>(64, recs.size() - a), &c.cx, &c.cy, &c.cz, &c.onemB,
                           &c.negA);
            cl.push_back(c);
        }
        recs.swap(cl);
    }
    out[0] = out[1] = out[2] = out[3] = 0;
    for (int p0 = 0; p0 < n; p0 += pk) {
        const int np = std::min(pk, n - p0);
        const PacketRec Q = packet_build(np, O + 3 * p0, D + 3 * p0);
        out[3] += Q.all;
        const size_t nr = kind == 2 ? sl.size() : recs.size();
        for (size_t j = 0; j < nr; ++j) {
            bool any = false;
            for (int i = p0; i < p0 + np && !any; ++i) {
                const float *o = O + 3 * i, *dd = D + 3 * i;
                if (kind == 2) {
                    const SliverRec &S = sl[j];
                    const float tx = o[0] - S.v0x, ty = o[1] - S.v0y, tz = o[2] - S.v0z;
                    const float cx = fmaf(S.e2y, tz, -(S.e2z * ty)), cy = fmaf(S.e2z, tx, -(S.e2x * tz));
                    const float cz = fmaf(S.e2x, ty, -(S.e2y * tx));
                    const float x = fmaf(dd[2], cz, fmaf(dd[1], cy, dd[0] * cx));
                    const float tm = fmaxf(fmaxf(fabsf(tx), fabsf(ty)), fabsf(tz));
                    const float dl = sqrtf(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
                    const float rhs = dl * fmaf(S.b, tm, S.a);
                    any = fmaf(x, x, -(rhs * rhs)) <= 0.0f;
                } else {
                    const FiltRec &r = recs[j];
                    float s = 1.0f / sqrtf(fmaf(dd[2], dd[2], fmaf(dd[1], dd[1], dd[0] * dd[0])));
                    any = eval_test(o, dd[0] * s, dd[1] * s, dd[2] * s, r.cx, r.cy, r.cz, r.onemB, r.negA) <= 0.0f;
                }
            }
            const bool pass = kind == 2 ? packet_sliver_test(Q, sl[j])
                                        : packet_sphere_test(Q, recs[j].cx, recs[j].cy, recs[j].cz, recs[j].onemB,
                                                             recs[j].negA);
            out[1] += pass;
            out[2] += any;
            out[0] += (any && !pass);
        }
    }
}

// Per-ray filter candidate count over m triangles (kernel evaluation of the
// sphere test; "always" records are skipped, they go to the sliver list).
extern "C" void cand_count(int n, const float *O, const float *D, int m, const float *V, double dcap, int *cnt)
{
    std::vector<FiltRec> rec((size_t)m);
    for (int j = 0; j < m; ++j) {
        const float *v = V + 9 * j;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        rec[(size_t)j] = filter_record(v0, v1, v2, j, dcap);
    }
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *dd = D + 3 * i;
        float s = 1.0f / sqrtf(fmaf(dd[2], dd[2], fmaf(dd[1], dd[1], dd[0] * dd[0])));
        int c = 0;
        for (int j = 0; j < m; ++j) {
            const FiltRec &r = rec[(size_t)j];
            if (r.onemB < -1e29f) continue;
            c += eval_test(o, dd[0] * s, dd[1] * s, dd[2] * s, r.cx, r.cy, r.cz, r.onemB, r.negA) <= 0.0f;
        }
        cnt[i] = c;
    }
}
