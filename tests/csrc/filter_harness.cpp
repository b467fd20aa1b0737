// CPU harness for lpc_math.hpp (the header the HIP kernels include): evaluates the
// bounding-sphere filter the way k_intersect does (plain and FMA-contracted float)
// and the exact Moller-Trumbore acceptance, for property tests of the filter margin.
#include <cmath>
#include <cstring>
#include <algorithm>
#include <vector>
#include "lpc_math.hpp"

using namespace lpc;

// filter_test with explicit FMAs (what the device compiler may contract to)
static inline float filter_test_fma(float cx, float cy, float cz, float negB, float negA, const float *o, float nx,
                                    float ny, float nz)
{
    const float wx = cx - o[0], wy = cy - o[1], wz = cz - o[2];
    const float px = fmaf(wy, nz, -(wz * ny)), py = fmaf(wz, nx, -(wx * nz)), pz = fmaf(wx, ny, -(wy * nx));
    const float pp = fmaf(pz, pz, fmaf(py, py, px * px));
    const float ww = fmaf(wz, wz, fmaf(wy, wy, wx * wx));
    return pp + fmaf(negB, ww, negA);
}

// max of the plain and the fused evaluation: a pair is a sure candidate only if
// both pass
static inline float eval_test(const float *o, float nx, float ny, float nz, float cx, float cy, float cz,
                              float negB, float negA)
{
    const float a = filter_test(cx, cy, cz, negB, negA, o[0], o[1], o[2], nx, ny, nz);
    const float b = filter_test_fma(cx, cy, cz, negB, negA, o, nx, ny, nz);
    return a > b ? a : b;
}

static inline void unit_dir(const float *dd, float &nx, float &ny, float &nz)
{
    const float s = 1.0f / sqrtf(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
    nx = dd[0] * s; ny = dd[1] * s; nz = dd[2] * s;
}

extern "C" void filt_eval(int n, const float *O, const float *D, const float *V, float eps, double dcap, double S,
                          float *d_out, int *hit_out, float *t_out)
{
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *dd = D + 3 * i, *v = V + 9 * i;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        FiltRec r = filter_record(v0, v1, v2, 0, dcap, S);
        float nx, ny, nz;
        unit_dir(dd, nx, ny, nz);
        d_out[i] = r.negB < -1e29f ? -1.0f : eval_test(o, nx, ny, nz, r.cx, r.cy, r.cz, r.negB, r.negA);
        f3 V0 = mk3(v[0], v[1], v[2]);
        f3 E1 = mk3(v[3] - v[0], v[4] - v[1], v[5] - v[2]);
        f3 E2 = mk3(v[6] - v[0], v[7] - v[1], v[8] - v[2]);
        float t = 0.0f;
        int h = mt_exact(mk3(o[0], o[1], o[2]), mk3(dd[0], dd[1], dd[2]), V0, E1, E2, &t);
        hit_out[i] = h && t > eps;
        t_out[i] = t;
    }
}

// Node test vs its triangles: rays (n) x one node over m triangles.  Writes each
// triangle's exact Moller-Trumbore acceptance (n*m, t > eps) and the node's float
// test value (n, the max of the plain and the fused evaluation).
extern "C" void cluster_eval(int n, const float *O, const float *D, int m, const float *V, float eps, double S,
                             int *hit_tri, float *d_cl)
{
    std::vector<const float *> tv((size_t)m * 3);
    for (int j = 0; j < m; ++j)
        for (int v = 0; v < 3; ++v) tv[3 * (size_t)j + v] = V + 9 * j + 3 * v;
    float cx, cy, cz, nb, na;
    node_record(tv.data(), m, S, &cx, &cy, &cz, &nb, &na);
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *dd = D + 3 * i;
        float nx, ny, nz;
        unit_dir(dd, nx, ny, nz);
        for (int j = 0; j < m; ++j) {
            const float *v = V + 9 * j;
            float t = 0.0f;
            const int h = mt_exact(mk3(o[0], o[1], o[2]), mk3(dd[0], dd[1], dd[2]), mk3(v[0], v[1], v[2]),
                                   mk3(v[3] - v[0], v[4] - v[1], v[5] - v[2]), mk3(v[6] - v[0], v[7] - v[1], v[8] - v[2]),
                                   &t);
            hit_tri[(size_t)i * m + j] = h && t > eps;
        }
        d_cl[i] = nb < -1e29f ? -1.0f : eval_test(o, nx, ny, nz, cx, cy, cz, nb, na);
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

// The line filter about E2 (ax1 = 0) or E1 (ax1 = 1) as k_slivers evaluates a
// SliverRec (sliver_params_axis; the filter edge in e2, the exact test in the
// triangle's own E1/E2 order), plus the exact acceptance of the same pairs.
extern "C" void sliver_eval_axis(int n, const float *O, const float *D, const float *V, float eps, int fused,
                                 int ax1, float *d_out, int *hit_out)
{
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *dd = D + 3 * i, *v = V + 9 * i;
        float a, b;
        sliver_params_axis(v, v + 3, v + 6, ax1, &a, &b);
        const float *w = ax1 ? v + 3 : v + 6;
        const float ex = w[0] - v[0], ey = w[1] - v[1], ez = w[2] - v[2];
        const float tx = o[0] - v[0], ty = o[1] - v[1], tz = o[2] - v[2];
        const float tm = fmaxf(fmaxf(fabsf(tx), fabsf(ty)), fabsf(tz));
        const float dl = sqrtf(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
        float d;
        if (fused) {
            const float cx = fmaf(ey, tz, -(ez * ty)), cy = fmaf(ez, tx, -(ex * tz)), cz = fmaf(ex, ty, -(ey * tx));
            const float x = fmaf(dd[2], cz, fmaf(dd[1], cy, dd[0] * cx));
            const float rhs = dl * fmaf(b, tm, a);
            d = fmaf(x, x, -(rhs * rhs));
        } else {
            const float cx = ey * tz - ez * ty, cy = ez * tx - ex * tz, cz = ex * ty - ey * tx;
            const float x = dd[0] * cx + dd[1] * cy + dd[2] * cz;
            const float rhs = dl * (a + b * tm);
            d = x * x - rhs * rhs;
        }
        d_out[i] = d;
        float t = 0.0f;
        const int h = mt_exact(mk3(o[0], o[1], o[2]), mk3(dd[0], dd[1], dd[2]), mk3(v[0], v[1], v[2]),
                               mk3(v[3] - v[0], v[4] - v[1], v[5] - v[2]), mk3(v[6] - v[0], v[7] - v[1], v[8] - v[2]),
                               &t);
        hit_out[i] = h && t > eps;
    }
}

// The engine's thin-triangle rule (build_records: thin_axis on filter_record's
// sphere): 0 sphere test, 1 line filter about E2, 2 about E1; -1 never / sliver.
extern "C" void thin_class(int n, const float *V, double dcap, double S, double k, int *cls)
{
    for (int i = 0; i < n; ++i) {
        const float *v = V + 9 * i;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        FiltRec r = filter_record(v0, v1, v2, 0, dcap, S);
        if (r.negA == INFINITY || r.negB < -1e29f) { cls[i] = -1; continue; }
        cls[i] = thin_axis(v0, v1, v2, r.cx, r.cy, r.cz, S, k);
    }
}

// filter_record's classification: 0 sphere test, 1 never, 2 always (-> sliver list)
extern "C" void filt_class(int n, const float *V, double dcap, double S, int *cls)
{
    for (int i = 0; i < n; ++i) {
        const float *v = V + 9 * i;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        FiltRec r = filter_record(v0, v1, v2, 0, dcap, S);
        cls[i] = r.negA == INFINITY ? 1 : (r.negB < -1e29f ? 2 : 0);
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
                            double dcap, double S, long long *out)
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
            recs.push_back(filter_record(v0, v1, v2, j, dcap, S));
        }
    }
    if (kind == 1) {
        std::vector<FiltRec> cl;
        std::vector<const float *> tv((size_t)m * 3);
        for (int j = 0; j < m; ++j)
            for (int v = 0; v < 3; ++v) tv[3 * (size_t)j + v] = V + 9 * j + 3 * v;
        for (int a = 0; a < m; a += 64) {
            FiltRec c;
            memset(&c, 0, sizeof(c));
            node_record(&tv[3 * (size_t)a], std::min(64, m - a), S, &c.cx, &c.cy, &c.cz, &c.negB, &c.negA);
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
                    float nx, ny, nz;
                    unit_dir(dd, nx, ny, nz);
                    any = filter_test(r.cx, r.cy, r.cz, r.negB, r.negA, o[0], o[1], o[2], nx, ny, nz) <= 0.0f ||
                          filter_test_fma(r.cx, r.cy, r.cz, r.negB, r.negA, o, nx, ny, nz) <= 0.0f;
                }
            }
            const bool pass = kind == 2 ? packet_sliver_test(Q, sl[j])
                                        : packet_sphere_test(Q, recs[j].cx, recs[j].cy, recs[j].cz, recs[j].negB,
                                                             recs[j].negA);
            out[1] += pass;
            out[2] += any;
            out[0] += (any && !pass);
        }
    }
}

// Per-ray filter candidate count over m triangles (kernel evaluation of the
// sphere test; "always" records are skipped, they go to the sliver list).
extern "C" void cand_count(int n, const float *O, const float *D, int m, const float *V, double dcap, double S,
                           int *cnt)
{
    std::vector<FiltRec> rec((size_t)m);
    for (int j = 0; j < m; ++j) {
        const float *v = V + 9 * j;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        rec[(size_t)j] = filter_record(v0, v1, v2, j, dcap, S);
    }
    for (int i = 0; i < n; ++i) {
        const float *o = O + 3 * i, *dd = D + 3 * i;
        float nx, ny, nz;
        unit_dir(dd, nx, ny, nz);
        int c = 0;
        for (int j = 0; j < m; ++j) {
            const FiltRec &r = rec[(size_t)j];
            if (r.negB < -1e29f) continue;
            c += filter_test(r.cx, r.cy, r.cz, r.negB, r.negA, o[0], o[1], o[2], nx, ny, nz) <= 0.0f;
        }
        cnt[i] = c;
    }
}

// Filter records of m triangles: (cx, cy, cz, negB, negA) each.
extern "C" void filt_records(int m, const float *V, double dcap, double S, float *out)
{
    for (int j = 0; j < m; ++j) {
        const float *v = V + 9 * j;
        float v0[4] = {v[0], v[1], v[2], 0}, v1[4] = {v[3], v[4], v[5], 0}, v2[4] = {v[6], v[7], v[8], 0};
        const FiltRec r = filter_record(v0, v1, v2, j, dcap, S);
        out[5 * j] = r.cx; out[5 * j + 1] = r.cy; out[5 * j + 2] = r.cz; out[5 * j + 3] = r.negB; out[5 * j + 4] = r.negA;
    }
}

// sliver_dmin (SliverRec::dmin) and Moller-Trumbore's DEN (.cl:75-76) as float,
// plain and with FMA contraction, for rays D against triangles V.
extern "C" void sliver_den(int n, const float *D, const float *V, float *dmin_out, float *den_plain,
                           float *den_fma)
{
    for (int i = 0; i < n; ++i) {
        const float *d = D + 3 * i, *v = V + 9 * i;
        dmin_out[i] = sliver_dmin(v, v + 3, v + 6);
        const float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
        const float e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
        const float px = d[1] * e2[2] - d[2] * e2[1], py = d[2] * e2[0] - d[0] * e2[2], pz = d[0] * e2[1] - d[1] * e2[0];
        den_plain[i] = px * e1[0] + py * e1[1] + pz * e1[2];
        const float fx = fmaf(d[1], e2[2], -(d[2] * e2[1])), fy = fmaf(d[2], e2[0], -(d[0] * e2[2])),
                    fz = fmaf(d[0], e2[1], -(d[1] * e2[0]));
        den_fma[i] = fmaf(fz, e1[2], fmaf(fy, e1[1], fx * e1[0]));
    }
}

// node_record of m triangles as one record (cx, cy, cz, negB, negA): the test a
// hierarchy node / piece root carries (tests/test_gpu_filter.py evaluates it on
// the device).
extern "C" void node_rec(int m, const float *V, double S, float *out)
{
    std::vector<const float *> tv((size_t)m * 3);
    for (int j = 0; j < m; ++j)
        for (int v = 0; v < 3; ++v) tv[3 * (size_t)j + v] = V + 9 * j + 3 * v;
    node_record(tv.data(), m, S, &out[0], &out[1], &out[2], &out[3], &out[4]);
}
