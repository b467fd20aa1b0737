// CPU harness for lpc_math.hpp (the header the HIP kernels include): evaluates the
// bounding-sphere filter the way k_intersect does (fused multiply-adds in float)
// and the exact Moller-Trumbore acceptance, for property tests of the filter margin.
#include <cmath>
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
