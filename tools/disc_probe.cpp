// disc_probe: how many of the sphere filter's candidate (ray, triangle) pairs a
// per-triangle plane test would remove, and whether that test keeps every pair
// Moller-Trumbore accepts (the superset property the walk's results rest on).
// Host build of the kernel's own header (lpc_math.hpp):
//   g++ -O2 -fopenmp -std=c++17 -ffp-contract=off -fPIC -shared -Ilightpycl_amd/csrc tools/disc_probe.cpp -o tools/_disc_probe.so
//
// The plane test of a triangle with circumsphere centre c (the filter record's,
// in the triangle's plane), radius rho, unit normal N, for a ray (O, unit n),
// w = c - O, wn = w.N, dn = n.N, q = wn n - dn w (q / dn = the plane hit - c):
//   disc:   |q|^2 <= (rho |dn| + K (|w| + rho) + beta)^2
//   behind: wn dn < 0 and |wn| > K (|w| + rho) + beta and |dn| > K   (the plane
//           hit is behind the origin by more than Moller-Trumbore's rounding)
// K covers Moller-Trumbore's line distance (2 kappa, the filter's kappa) and the
// float evaluation, beta the float rounding of c.
#include <math.h>
#include <stdint.h>
#include <string.h>
#include "lpc_math.hpp"

using namespace lpc;

struct DiscRec { float nx, ny, nz, rho, K, beta; };

static DiscRec disc_record(const float *V0, const float *V1, const float *V2, float cx, float cy, float cz)
{
    const double eps = 1.0 / 16777216.0;
    double a[3], b[3];
    for (int k = 0; k < 3; ++k) { a[k] = (double)V1[k] - V0[k]; b[k] = (double)V2[k] - V0[k]; }
    const double n[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    const double nl = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    DiscRec r;
    r.nx = (float)(n[0] / nl); r.ny = (float)(n[1] / nl); r.nz = (float)(n[2] / nl);
    const float *Vs[3] = {V0, V1, V2};
    const double c[3] = {cx, cy, cz};
    double rho2 = 0.0;
    for (int v = 0; v < 3; ++v) {
        double d2 = 0.0;
        for (int k = 0; k < 3; ++k) { const double q = (double)Vs[v][k] - c[k]; d2 += q * q; }
        rho2 = fmax(rho2, d2);
    }
    const double rho = sqrt(rho2) * (1.0 + 1e-6);
    const double kap = tri_kappa(V0, V1, V2);
    const double cm = fmax(fabs(c[0]), fmax(fabs(c[1]), fabs(c[2])));
    r.rho = (float)rho;
    if ((double)r.rho < rho) r.rho = nextafterf(r.rho, INFINITY);
    r.K = (float)(2.0 * kap + 64.0 * eps);
    r.beta = (float)(16.0 * eps * (cm + rho));
    return r;
}

// 1: the pair may be accepted (keep it), 0: the plane test rejects it; *behind: it
// was the behind-origin rule
static inline int disc_test(const DiscRec &R, float cx, float cy, float cz, const float *o, float nx, float ny,
                            float nz, int *behind)
{
    const float wx = cx - o[0], wy = cy - o[1], wz = cz - o[2];
    const float wn = wx * R.nx + wy * R.ny + wz * R.nz;
    const float dn = nx * R.nx + ny * R.ny + nz * R.nz;
    const float qx = wn * nx - dn * wx, qy = wn * ny - dn * wy, qz = wn * nz - dn * wz;
    const float qq = qx * qx + qy * qy + qz * qz;
    const float T = sqrtf(wx * wx + wy * wy + wz * wz) + R.rho;
    const float sl = R.K * T + R.beta;
    const float rhs = (R.rho * fabsf(dn) + sl) * 1.0001f;
    *behind = 0;
    if (wn * dn < 0.0f && fabsf(wn) > sl * 1.0001f && fabsf(dn) > R.K * 1.0001f) { *behind = 1; return 0; }
    return qq <= rhs * rhs;
}

static inline void unit_dir_h(const float *dd, float &nx, float &ny, float &nz)
{
    const float u = 1.0f / sqrtf(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
    nx = dd[0] * u; ny = dd[1] * u; nz = dd[2] * u;
}

// out[0] sphere candidates, [1] ... that pass the plane test, [2] culled as behind,
// [3] culled by the disc, [4] accepted by Moller-Trumbore, [5] accepted but
// rejected by the sphere, [6] accepted but rejected by the plane test (must be 0)
extern "C" void disc_probe(int n, const float *O, const float *D, int m, const float *V, float eps, double dcap,
                           double S, long long *out, int *viol_idx)
{
    FiltRec *fr = new FiltRec[m];
    DiscRec *dr = new DiscRec[m];
    for (int i = 0; i < m; ++i) {
        const float *v0 = V + 9 * i, *v1 = v0 + 3, *v2 = v0 + 6;
        fr[i] = filter_record(v0, v1, v2, i, dcap, S);
        dr[i] = disc_record(v0, v1, v2, fr[i].cx, fr[i].cy, fr[i].cz);
    }
    long long c[7] = {0, 0, 0, 0, 0, 0, 0};
    int nviol = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : c[:7])
    for (int r = 0; r < n; ++r) {
        const float *o = O + 3 * r, *d = D + 3 * r;
        float nx, ny, nz;
        unit_dir_h(d, nx, ny, nz);
        const f3 Of = mk3(o[0], o[1], o[2]), Df = mk3(d[0], d[1], d[2]);
        for (int i = 0; i < m; ++i) {
            const FiltRec &f = fr[i];
            const bool sph = filter_test(f.cx, f.cy, f.cz, f.negB, f.negA, o[0], o[1], o[2], nx, ny, nz) <= 0.0f;
            // never / always (slivers: the sliver list's line filter, not the walk)
            if (!(f.negA < INFINITY) || f.negB <= -1e29f) continue;
            const bool special = false;
            int beh = 0;
            const bool pl = special ? true : disc_test(dr[i], f.cx, f.cy, f.cz, o, nx, ny, nz, &beh) != 0;
            const float *v0 = V + 9 * i;
            const f3 V0 = mk3(v0[0], v0[1], v0[2]);
            const f3 E1 = mk3(v0[3] - v0[0], v0[4] - v0[1], v0[5] - v0[2]);
            const f3 E2 = mk3(v0[6] - v0[0], v0[7] - v0[1], v0[8] - v0[2]);
            float t;
            const bool mt = mt_exact(Of, Df, V0, E1, E2, &t) && t > eps;
            if (sph) {
                ++c[0];
                if (pl) ++c[1];
                else if (beh) ++c[2];
                else ++c[3];
            }
            if (mt) {
                ++c[4];
                if (!sph && !special) ++c[5];
                if (!pl) {
                    ++c[6];
#pragma omp critical
                    if (nviol < 16) { viol_idx[2 * nviol] = r; viol_idx[2 * nviol + 1] = i; ++nviol; }
                }
            }
        }
    }
    for (int k = 0; k < 7; ++k) out[k] = c[k];
    delete[] fr;
    delete[] dr;
}
