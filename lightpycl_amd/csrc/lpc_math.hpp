// lpc_math.hpp -- per-ray arithmetic of the LightPyCL bounce, shared by the HIP
// kernels (lpc.hip) and the CPU-side property tests (tests/csrc/).
//
// Two kinds of code live here:
//  * EXACT functions: the reference's arithmetic (kernel_reflect_refract_intersect.cl)
//    operation for operation as ROCm's OpenCL compiler builds it for gfx950 with
//    IEEE division/sqrt and no FP contraction in the kernel's own expressions
//    (oracle/_ref/lpc_ref_ieee.co), single-precision constants, the OpenCL
//    library's dot/cross/length/normalize (below).  Decisions (hit/miss,
//    entering, n1/n2, TIR) and values (t, dest, children) are therefore
//    bit-identical to the reference's own kernels and to the CPU oracle.
//  * the CONSERVATIVE bounding-sphere filter used by the hot loop: a cheap test
//    that is a superset of the exact Moller-Trumbore acceptance (see
//    filter_record() for the margin derivation); only pairs that pass it are
//    re-tested exactly, so the fast path gives the exact result.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LPC_HD __host__ __device__ __forceinline__
#else
#define LPC_HD static inline
#endif

#if defined(__clang__)
#define LPC_EXACT _Pragma("clang fp contract(off)")
#else
#define LPC_EXACT
#endif

namespace lpc {

struct f3 { float x, y, z; };

LPC_HD f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
LPC_HD f3 add3(f3 a, f3 b) { LPC_EXACT return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
LPC_HD f3 sub3(f3 a, f3 b) { LPC_EXACT return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
LPC_HD f3 scl3(f3 a, float s) { LPC_EXACT return mk3(a.x * s, a.y * s, a.z * s); }
LPC_HD f3 neg3(f3 a) { return mk3(-a.x, -a.y, -a.z); }
// OpenCL's geometric builtins for float3 exactly as ROCm's OpenCL device library
// (the library the reference's kernels link when built for an AMD GPU,
// oracle/Makefile `ref`) evaluates them: dot = fma(z, z', fma(y, y', x x')),
// cross.x = fma(a.y, b.z, -(a.z b.y)) (and cyclic), length = the hardware square
// root of that dot, normalize = v times the hardware reciprocal square root,
// each with the library's rescaling outside the normal range.  fma is exactly
// rounded on every target, so the host build (gcc fmaf) computes the same bits.
LPC_HD float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
LPC_HD f3 cross3(f3 a, f3 b) {
    return mk3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
// gfx950 v_sqrt_f32 / v_rsq_f32 (ldexp-scaled for denormal inputs as the library
// does).  Host: correctly rounded, which tools/rsq_check.py measures the
// hardware to be on every float in [1, 4).
LPC_HD float hw_sqrt(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
LPC_HD float hw_rsq(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rsqf(x);
#else
    return (float)(1.0 / sqrt((double)x));
#endif
}
// length(v): __ocml_len3_f32
LPC_HD float len3(f3 a)
{
    LPC_EXACT
    const float s = dot3(a, a);
    if (s >= 1.17549435e-38f || s != s) {
        if (s != INFINITY) return hw_sqrt(s);
        const f3 b = mk3(a.x * 0x1p-66f, a.y * 0x1p-66f, a.z * 0x1p-66f);   // rescale (overflow)
        const float t = dot3(b, b);
        const bool sc = t < 1.17549435e-38f;
        const float q = hw_sqrt(sc ? ldexpf(t, 32) : t);
        return (sc ? ldexpf(q, -16) : q) * 0x1p66f;
    }
    const f3 b = mk3(a.x * 0x1p86f, a.y * 0x1p86f, a.z * 0x1p86f);          // rescale (underflow)
    const float t = dot3(b, b);
    const bool sc = t < 1.17549435e-38f;
    const float q = hw_sqrt(sc ? ldexpf(t, 32) : t);
    return (sc ? ldexpf(q, -16) : q) * 0x1p-86f;
}
// normalize(v): OpenCL library normalize for float3
LPC_HD f3 nrm3(f3 a)
{
    LPC_EXACT
    float s = dot3(a, a);
    if (s >= 1.17549435e-38f || s != s) {
        if (s == INFINITY) {
            a = mk3(a.x * 0x1p-66f, a.y * 0x1p-66f, a.z * 0x1p-66f);
            s = dot3(a, a);
            if (s == INFINITY) {          // infinite components -> +-1, the rest +-0
                a = mk3(copysignf(isinf(a.x) ? 1.0f : 0.0f, a.x), copysignf(isinf(a.y) ? 1.0f : 0.0f, a.y),
                        copysignf(isinf(a.z) ? 1.0f : 0.0f, a.z));
                s = dot3(a, a);
            }
        }
    } else {
        a = mk3(a.x * 0x1p86f, a.y * 0x1p86f, a.z * 0x1p86f);
        s = dot3(a, a);
    }
    const bool sc = s < 1.17549435e-38f;
    float r = hw_rsq(sc ? s * 0x1p24f : s);
    if (sc) r = r * 0x1p12f;
    return mk3(a.x * r, a.y * r, a.z * r);
}

// ---------------------------------------------------------------------------
// Moller-Trumbore exactly as intersect_triangle (.cl:50-101), with the two edge
// vectors precomputed (E1 = V1-V0, E2 = V2-V0 are the same single roundings the
// reference performs per call, .cl:72-73).  Returns 1 and t on a u/v hit.
LPC_HD int mt_exact(f3 O, f3 D, f3 V0, f3 E1, f3 E2, float *t)
{
    LPC_EXACT
    const float EPSILON_NUM = 0.000001f;
    f3 P = cross3(D, E2);
    float DEN = dot3(P, E1);
    if (DEN > -EPSILON_NUM && DEN < EPSILON_NUM) return 0;
    float iDEN = 1.0f / DEN;
    f3 T = sub3(O, V0);
    float u = dot3(P, T) * iDEN;
    if (u < 0.0f || u > 1.0f) return 0;
    f3 Q = cross3(T, E1);
    float v = dot3(Q, D) * iDEN;
    if (v < 0.0f || u + v > 1.0f) return 0;
    *t = dot3(Q, E2) * iDEN;
    return 1;
}

// Accumulator update of the intersect kernel's inner loop (.cl:277-283).
LPC_HD void mt_accumulate(f3 O, f3 D, f3 V0, f3 E1, f3 E2, int32_t idx, float eps,
                          float &tmin, int32_t &imin, int32_t &cnt)
{
    float t;
    if (mt_exact(O, D, V0, E1, E2, &t) && t > eps) {
        // first minimum in triangle-index order (the reference's strict `<` over
        // increasing i) == lowest index among equal t, whatever order we visit in
        if (t < tmin || (t == tmin && idx < imin)) { tmin = t; imin = idx; }
        cnt += 1;
    }
}

// ---------------------------------------------------------------------------
// intersect_postproc (.cl:105-240) given the per-mesh (slot) results of one ray.
// `slot(j, t, c)` must return slot j's min t and hit count.  KU > 0 (K <= KU)
// unrolls both mesh loops KU times, so a slot function over a register array
// indexes it with constants.
struct PostOut { int32_t hit_mesh, hit_idx, n1, n2, entering; float t_min; };

template <int KU = 0, class SlotFn>
LPC_HD PostOut postproc(int32_t K, int32_t prev, const int32_t *mat_type, float max_ray_len,
                        SlotFn slot)
{
    LPC_EXACT
    const float EPSILON = 0.000001f * max_ray_len;
    PostOut o;
    o.hit_mesh = -1; o.hit_idx = -1; o.n1 = -1; o.n2 = -1; o.entering = -1;
    float t_min = max_ray_len;
    int32_t hit_cnt = 0;
    constexpr int32_t KL = KU > 0 ? KU : 0x7fffffff;
    constexpr int32_t UF = KU > 0 ? KU : 1;                             // unroll factor (KU = 0: a loop)
#pragma unroll UF
    for (int32_t j = 0; j < KL; ++j) {                                  // .cl:127-135
        if (KU == 0 && j >= K) break;
        float tj; int32_t cj, ij;
        slot(j, tj, cj, ij);
        if (j < K && tj < t_min) { t_min = tj; o.hit_mesh = j; o.hit_idx = ij; hit_cnt = cj; }
    }
    if (o.hit_mesh >= 0) {
        int32_t entering = 1 - (hit_cnt % 2);                            // .cl:142
        o.entering = entering;
        if (prev == -2 || prev == -1) {                                  // .cl:145-166
            if (entering == 1) { o.n1 = -1; o.n2 = o.hit_mesh; }
            else { o.n1 = o.hit_mesh; o.n2 = -1; }
        } else {                                                         // .cl:167-177
            if (entering == 1) { o.n1 = prev; o.n2 = o.hit_mesh; }
            else { o.n1 = o.hit_mesh; o.n2 = -1; }
        }
        float t_minmin = t_min, t_maxmin = t_min, t_minmax = max_ray_len;
        int32_t maxmin_entering = 0, maxmin_idx = -1, minmax_idx = -1;
#pragma unroll UF
        for (int32_t j = 0; j < KL; ++j) {                              // .cl:193-214
            if (KU == 0 && j >= K) break;
            int32_t mt = j < K ? mat_type[j] : -1;
            if (mt == 0 || mt == 4) {
                float tj; int32_t cj, ij;
                slot(j, tj, cj, ij);
                int32_t ent = 1 - (cj % 2);
                if (tj <= t_minmin + EPSILON && tj >= t_maxmin) {
                    t_maxmin = tj; maxmin_idx = j; maxmin_entering = ent;
                }
                if (tj > t_minmin + EPSILON && ent == 0 && tj <= t_minmax) {
                    t_minmax = tj; minmax_idx = j;
                }
            }
        }
        if (maxmin_entering == 1) { t_min = t_maxmin; o.n2 = maxmin_idx; }   // .cl:216-229
        else {
            if (maxmin_idx >= 0) t_min = t_maxmin;
            if (minmax_idx >= 0) o.n2 = minmax_idx;
        }
    }
    o.t_min = t_min;
    return o;
}

// dest = o + d * t_min (.cl:237)
LPC_HD f3 ray_dest(f3 O, f3 D, float t) { LPC_EXACT return add3(O, scl3(D, t)); }

// ---------------------------------------------------------------------------
// reflect_refract_rays (.cl:346-474) for one ray, reflect_refract (.cl:293-343)
// inlined.  Inputs are the ray, its postproc result and the material tables;
// `tri(idx, v0, v1, v2)` gathers the hit triangle's vertices.
struct ShadeOut {
    float pow;                 // possibly dissipated input power (.cl:392)
    int32_t meas;              // in-ray measured state after the kernel
    f3 r_dir, t_dir;
    float r_pow, t_pow;
    int32_t r_meas, t_meas;
};

template <class TriFn>
LPC_HD ShadeOut shade(f3 O, f3 D, f3 dest, float pw, int32_t meas_in, int32_t rmid,
                      int32_t ridx, int32_t n1id, int32_t n2id, const int32_t *mat_type,
                      const float *ior, const float *refl, const float *diss, float ior_env,
                      TriFn tri)
{
    LPC_EXACT
    const float EPSILON_NUM = 0.000001f;
    ShadeOut s;
    int32_t mesh_mat = 2;
    float R_mesh = 0.0f;
    if (rmid >= 0) { mesh_mat = mat_type[rmid]; R_mesh = refl[rmid]; }
    float IOR_in = ior_env, IOR_n2 = ior_env;
    if (n1id >= 0) {                                                     // .cl:385-394
        IOR_in = ior[n1id];
        if (mat_type[n1id] == 0 && diss[n1id] > EPSILON_NUM) {
            float ray_len = len3(sub3(dest, O));
            pw = pw * expf(-diss[n1id] * ray_len);
        }
    }
    if (n2id >= 0) IOR_n2 = ior[n2id];
    s.pow = pw;
    s.meas = meas_in;
    const f3 zero = mk3(0.0f, 0.0f, 0.0f);
    // dead children by default (also what the NaN-TIR path leaves)
    s.r_dir = zero; s.t_dir = zero; s.r_pow = 0.0f; s.t_pow = 0.0f; s.r_meas = -1; s.t_meas = -1;
    if (meas_in == 0 && rmid >= 0 && (mesh_mat == 0 || mesh_mat == 1)) {   // .cl:408
        f3 v0, v1, v2;
        tri(ridx, v0, v1, v2);
        f3 nrm_in = nrm3(cross3(sub3(v1, v0), sub3(v2, v1)));           // .cl:413
        // reflect_refract (.cl:293-343)
        f3 nrm = nrm_in;
        float n1 = IOR_in, n2 = IOR_n2;
        float r = n1 / n2;
        float cosT1 = -dot3(nrm, D);
        if (cosT1 < 0.0f) { nrm = neg3(nrm_in); cosT1 = -dot3(nrm, D); }
        float TIR_check = 1.0f - (r * r) * (1.0f - (cosT1 * cosT1));
        f3 rdir = zero, tdir = zero;
        float rp = 0.0f, tp = 0.0f;
        int32_t rm = -1, tm = -1;
        if (TIR_check >= 0.0f) {
            float cosT2 = sqrtf(TIR_check);
            float a = fabsf((n1 * cosT1 - n2 * cosT2) / (n1 * cosT1 + n2 * cosT2));
            float b = fabsf((n1 * cosT2 - n2 * cosT1) / (n1 * cosT2 + n2 * cosT1));
            float Rs = a * a, Rp = b * b;
            float reflect_power = pw * (Rs + Rp) / 2.0f;
            rdir = add3(D, scl3(nrm, 2.0f * cosT1));
            rp = reflect_power; rm = 0;
            tdir = add3(scl3(D, r), scl3(nrm, r * cosT1 - cosT2));
            tp = pw - reflect_power; tm = 0;
        } else if (TIR_check < 0.0f) {
            rdir = add3(D, scl3(nrm, 2.0f * cosT1));
            rp = pw; rm = 0;
            tdir = zero; tp = 0.0f; tm = -1;
        }
        if (mesh_mat == 0) {                                             // .cl:429-439
            s.r_dir = rdir; s.r_pow = rp; s.r_meas = rm;
            s.t_dir = tdir; s.t_pow = tp; s.t_meas = tm;
        } else {                                                         // .cl:440-452 mirror
            s.r_dir = rdir; s.r_pow = pw * R_mesh; s.r_meas = rm;
            s.t_dir = zero; s.t_pow = 0.0f; s.t_meas = -1;
        }
    } else {                                                             // .cl:455-472
        if (mesh_mat == 2 || rmid < 0) s.meas = -1;
        if (mesh_mat == 3 && rmid >= 0) s.meas = 1;
    }
    return s;
}

// ---------------------------------------------------------------------------
// angular_project (.cl:509-538) and stereograph_project (.cl:488-506).
LPC_HD void angular_project(f3 p, f3 piv, f3 R0, f3 R1, f3 R2, float pwr, float &x, float &y,
                            float &pc)
{
    LPC_EXACT
    const float EPSILON = 0.000001f;
    f3 vec = sub3(p, piv);
    float u = dot3(vec, R0) + piv.x;
    float v = dot3(vec, R1) + piv.y;
    float w = dot3(vec, R2) + piv.z;
    float l = sqrtf(u * u + v * v + w * w);
    f3 vr = mk3(u / l, v / l, w / l);
    float cosT = dot3(mk3(0.0f, 0.0f, 1.0f), vr);
    float phi = atan2f(v, u);
    float r = acosf(cosT);
    float A = 1.0f;
    if (r > EPSILON) A = sinf(r) / r;
    x = r * cosf(phi);
    y = r * sinf(phi);
    pc = pwr / A;
}

LPC_HD void stereograph_project(f3 p, f3 piv, f3 R0, f3 R1, f3 R2, float pwr, float &x,
                                float &y, float &pc)
{
    LPC_EXACT
    f3 vec = sub3(p, piv);
    float u = dot3(vec, R0) + piv.x;
    float v = dot3(vec, R1) + piv.y;
    float w = dot3(vec, R2) + piv.z;
    float l = sqrtf(u * u + v * v + w * w);
    float xt = u / (l + w), yt = v / (l + w);
    float q = 1.0f + xt * xt + yt * yt;
    float A = 4.0f / (q * q);
    x = xt; y = yt; pc = pwr / A;
}

// ---------------------------------------------------------------------------
// Conservative bounding-sphere filter.
//
// Per (ray, record) the hot loop evaluates, in float (FMA contraction allowed),
//     w = c - O,  p = w x n,  d = p.p + (negA + negB w.w)        (n = D/|D|)
// and calls the pair a candidate when d <= 0, i.e. when dist(c, line)^2 <= A + B |w|^2
// (p.p is the squared distance from c to the ray's line, computed without the
// cancellation of |w|^2 - (w.n)^2).  For a triangle record A and B make the
// candidate set a superset of the pairs the exact Moller-Trumbore test accepts:
//  * an accepted pair's line passes within kappa |T| of the triangle, kappa =
//    kmt eps |E|^2 / |E1 x E2| (Moller-Trumbore's error for a nearly parallel ray,
//    kmt = 256 deliberately generous), |T| <= |w| + rho, so
//        dist(c, line) <= rho (1 + kappa) + kappa |w|;
//  * (a + b)^2 <= (1+h) a^2 + (1+1/h) b^2 for any h > 0 gives A + B |w|^2; h is
//    chosen per record for the scene's scale S (h = kappa S / a);
//  * store_test() adds the float evaluation of d: |p_f| <= dist (1 + 3 eps) + 7 eps |w|,
//    so exact dist^2 <= A + B ww  ==>  d_float <= 0 for the stored (negA, negB);
//    conversely d_float <= 0  ==>  exact dist^2 <= implied_test(negA, negB).
// tests/test_filter_superset.py measures the actual worst case on adversarial inputs.
// Triangles with an exactly-zero edge are never accepted by Moller-Trumbore
// (DEN == 0) and get A = +inf ("never", d = +inf).  Triangles with |E1||E2| below
// 1e-6/Dcap can never reach |DEN| >= 1e-6 for rays with |D| <= Dcap and are
// "never" too (the engine checks |D| <= Dcap at run time).  negB = -1e30 marks a
// record that always passes ("always"; triangles with kappa >= 0.1 are slivers).
struct FiltRec {
    float cx, cy, cz;   // sphere centre (float)
    float negB;         // -B
    float negA;         // -A
    int32_t idx;        // original triangle index
    int32_t pad0, pad1;
};

LPC_HD float filter_test(float cx, float cy, float cz, float negB, float negA, float ox, float oy, float oz,
                         float nx, float ny, float nz)
{
    const float wx = cx - ox, wy = cy - oy, wz = cz - oz;
    const float px = wy * nz - wz * ny, py = wz * nx - wx * nz, pz = wx * ny - wy * nx;
    const float pp = px * px + py * py + pz * pz;
    const float ww = wx * wx + wy * wy + wz * wz;
    return pp + (negA + negB * ww);
}

// filter_test for two records at once (packed FP32 on gfx950: v_pk_fma_f32 /
// v_pk_mul_f32 evaluate both halves with the same IEEE operations, so each half
// is one plain or FMA-contracted evaluation of filter_test, inside the slack).
typedef float lpc_f2 __attribute__((ext_vector_type(2)));
LPC_HD lpc_f2 filter_test2(lpc_f2 cx, lpc_f2 cy, lpc_f2 cz, lpc_f2 negB, lpc_f2 negA, float ox, float oy,
                           float oz, float nx, float ny, float nz)
{
    const lpc_f2 wx = cx - ox, wy = cy - oy, wz = cz - oz;
    const lpc_f2 px = wy * nz - wz * ny, py = wz * nx - wx * nz, pz = wx * ny - wy * nx;
    const lpc_f2 pp = px * px + py * py + pz * pz;
    const lpc_f2 ww = wx * wx + wy * wy + wz * wz;
    return pp + (negA + negB * ww);
}

// filter_test2 with the half-line cull (LPC_HALF): a record whose test sphere
// (radius^2 = A + B |w|^2) lies wholly behind the ray origin by a margin is
// failed (+1): wn = w.n < 0 and wn^2 > 2 (A + B ww) + LPC_HALF_MU2 ww.  Moller-
// Trumbore accepts such a triangle with t > eps only through rounding on rays
// nearly parallel to its plane (scope of the filter proof).
#define LPC_HALF_MU2 8e-4f
#if defined(__HIP__)          // lane access of the 2-vector (gcc builds of this header, tests/csrc, see one float)
LPC_HD lpc_f2 filter_test2h(lpc_f2 cx, lpc_f2 cy, lpc_f2 cz, lpc_f2 negB, lpc_f2 negA, float ox, float oy,
                            float oz, float nx, float ny, float nz)
{
    const lpc_f2 wx = cx - ox, wy = cy - oy, wz = cz - oz;
    const lpc_f2 px = wy * nz - wz * ny, py = wz * nx - wx * nz, pz = wx * ny - wy * nx;
    const lpc_f2 pp = px * px + py * py + pz * pz;
    const lpc_f2 ww = wx * wx + wy * wy + wz * wz;
    const lpc_f2 q = negA + negB * ww;                       // -(A + B ww)
    const lpc_f2 wn = wx * nx + wy * ny + wz * nz;
    const lpc_f2 b = wn * wn + (q + q) - LPC_HALF_MU2 * ww;  // > 0: sphere behind, clear of the origin
    lpc_f2 d = pp + q;
    if (wn.x < 0.0f && b.x > 0.0f) d.x = 1.0f;
    if (wn.y < 0.0f && b.y > 0.0f) d.y = 1.0f;
    return d;
}
#endif

// filter_test with the half-line cull (filter_test2h, one record)
LPC_HD float filter_testh(float cx, float cy, float cz, float negB, float negA, float ox, float oy, float oz,
                          float nx, float ny, float nz)
{
    const float wx = cx - ox, wy = cy - oy, wz = cz - oz;
    const float px = wy * nz - wz * ny, py = wz * nx - wx * nz, pz = wx * ny - wy * nx;
    const float pp = px * px + py * py + pz * pz;
    const float ww = wx * wx + wy * wy + wz * wz;
    const float q = negA + negB * ww;
    const float wn = wx * nx + wy * ny + wz * nz;
    const float d = pp + q;
    return ((wn < 0.0f) & (wn * wn + (q + q) - LPC_HALF_MU2 * ww > 0.0f)) ? 1.0f : d;   // a select, no branch
}

// Float-evaluation slack of filter_test, both ways (factor on A and B, and an
// absolute term on B = (1 + 1/h') 49 eps^2 with h' = 1e-3, rounded up).
#define LPC_FILT_REL 2e-3
#define LPC_FILT_ABS 2e-10

// One node of a mesh run's W-wide sphere hierarchy (W = 4 or 8), children in
// SoA form.  ref[k] >= 0: child node; ref[k] < 0: exact record ~ref[k] (records in
// leaf order, ExactRec::idx the triangle), whose test
// is the triangle's own filter record.  A node's test (in its parent) is
// node_record() of ALL triangles below it, so a ray whose line Moller-Trumbore
// accepts against some triangle passes every test on the way down.  Unused
// children: never.  128 B (W 4) / 256 B (W 8): whole scalar-load lines.
// ref >= 0: child node; ref < 0: exact record ~ref (leaf order).
template <int W>
struct NodeW {
    float cx[W], cy[W], cz[W], negB[W], negA[W];
    int32_t ref[W];
    int32_t pad[W == 4 ? 8 : 16];
};
typedef NodeW<4> Node4;
typedef NodeW<8> Node8;

// A "sliver": a triangle whose sphere test degenerates (B >= 0.5, e.g.
// revolve_curve's pole triangles with two vertices 1e-11 apart).  For it
// Moller-Trumbore is rounding noise that can accept rays anywhere along the line
// through V0 with direction E2, so it gets a line filter instead (sliver_params).
// Padding records have a = NaN (never pass).
// A "thin" triangle (round 4, LPC_THIN) gets the same kind of record: one whose
// bounding sphere is far wider than the triangle (the lens meshes' discs through
// the optical axis: 10 mm long, 0.4 mm wide, every axial ray passes all their
// spheres) is bounded better by the line filter about its longer edge.  The
// filter's edge ("axis") sits in e2; ax1 = 1 says it is E1 (the v-test's line,
// sliver_params_axis), and the exact test then takes E1 = e2, E2 = e1.
struct SliverRec {
    float v0x, v0y, v0z, e2x, e2y, e2z, a, b;
    int32_t idx;
    float e1x, e1y, e1z;    // with v0, e2: the exact record (Moller-Trumbore input)
    float dmin;             // |DEN| >= 1e-6 needs |D| >= dmin (sliver_dmin)
    int32_t ax1;            // 1: e2 holds E1 and e1 holds E2 (line filter about E1)
};

// Bound of one wave's packet of rays (k_packet): every origin lies within ro of
// (ox,oy,oz) and every direction within angle th of the unit axis a.  all = 1
// (incoherent packet, non-finite input) makes every packet test pass.
struct PacketRec {
    float ox, oy, oz, ro;
    float ax, ay, az;
    float th, sth, cth;
    int32_t all;
    int32_t pad[5];
};

// Packet test of a sphere record: false only if NO ray of the packet can pass the
// per-ray float test (filter_test).  A passing ray satisfies (exactly)
// dist(c, line)^2 <= A + B |w|^2 with (A, B) = implied_test, so the angle psi
// between w = c - O and its line obeys sin^2 psi <= B + A / |w|^2 =: sin^2 beta.
// With W = c - o_c, L = |W|, |w| >= L - ro, angle(W, w) <= gamma = asin(ro / L) and
// angle(line n, line a) <= th, the angle phi between W and the axis line obeys
//     phi <= th + gamma + beta =: Sigma,
// tested as |W x a| <= L sin(Sigma) (all angles in [0, pi/2]).  Float evaluation
// error is covered by 1e-3 relative + 1e-6 absolute on sin(Sigma) and by passing
// outright when a cosine would be computed with cancellation (sin > 0.99).
LPC_HD bool packet_sphere_test(const PacketRec &Q, float cx, float cy, float cz, float negB, float negA)
{
    if (Q.all) return true;
    if (!(negA < INFINITY)) return false;                  // never record
    const float A = -negA * (1.0f + 2.0f * (float)LPC_FILT_REL);
    const float B = -negB * (1.0f + 2.0f * (float)LPC_FILT_REL) + 2.0f * (float)LPC_FILT_ABS;
    const float wx = cx - Q.ox, wy = cy - Q.oy, wz = cz - Q.oz;
    const float L2 = wx * wx + wy * wy + wz * wz;
    const float L = sqrtf(L2);
    const float Lw = (L * 0.999999f - Q.ro * 1.000001f) * 0.999999f;   // <= |w| for every origin
    if (!(Lw > 0.0f)) return true;
    const float sg = (Q.ro / L) * 1.000002f;
    if (!(sg < 0.99f)) return true;
    const float s2 = B + A / (Lw * Lw);
    if (!(s2 < 0.98f)) return true;
    const float cg = sqrtf(1.0f - sg * sg), sb = sqrtf(s2), cb = sqrtf(1.0f - s2);
    const float s1 = Q.sth * cg + Q.cth * sg, c1 = Q.cth * cg - Q.sth * sg;   // th + gamma
    if (!(c1 > 0.15f)) return true;
    const float sS = s1 * cb + c1 * sb, cS = c1 * cb - s1 * sb;               // + beta
    if (!(cS > 0.15f)) return true;
    const float px = wy * Q.az - wz * Q.ay, py = wz * Q.ax - wx * Q.az, pz = wx * Q.ay - wy * Q.ax;
    const float cr2 = px * px + py * py + pz * pz;
    const float sm = sS * 1.001f + 1e-6f;
    return cr2 <= L2 * (sm * sm);
}

// Packet test of a sliver: a ray (origin O = o_c + delta, unit direction
// n = a + nu, |delta| <= ro, |nu| <= th) passing the line filter has
// |n.(E2 x T)| <= a_s + b_s |T| with T = O - V0 = Tc + delta, so
//     |a.(E2 x Tc)| <= a_s + b_s (|Tc| + ro) + |E2| (ro + th (|Tc| + ro)).
LPC_HD bool packet_sliver_test(const PacketRec &Q, const SliverRec &S)
{
    if (Q.all) return true;
    if (!(S.a == S.a)) return false;                       // padding
    const float tx = Q.ox - S.v0x, ty = Q.oy - S.v0y, tz = Q.oz - S.v0z;
    const float tn = sqrtf(tx * tx + ty * ty + tz * tz);
    const float e2n = sqrtf(S.e2x * S.e2x + S.e2y * S.e2y + S.e2z * S.e2z);
    const float cx = S.e2y * tz - S.e2z * ty, cy = S.e2z * tx - S.e2x * tz, cz = S.e2x * ty - S.e2y * tx;
    const float f = fabsf(Q.ax * cx + Q.ay * cy + Q.az * cz);
    const float tr = (tn + Q.ro) * 1.000001f;
    const float rhs = (S.a + S.b * tr) + e2n * (Q.ro + Q.th * tr);
    return f <= rhs * 1.001f + 1e-6f * e2n * tn;
}

// Packet bound from its reductions (shared by k_packet and the tests): centre =
// bbox centre of the origins; ro = max distance of an origin from it; axis =
// normalised sum of the unit directions; th = max angle of a direction from it.
LPC_HD void packet_centre(const float *mn, const float *mx, PacketRec &Q)
{
    Q.ox = 0.5f * (mn[0] + mx[0]);
    Q.oy = 0.5f * (mn[1] + mx[1]);
    Q.oz = 0.5f * (mn[2] + mx[2]);
}
LPC_HD float packet_angle(float nx, float ny, float nz, float ax, float ay, float az)
{
    const float px = ny * az - nz * ay, py = nz * ax - nx * az, pz = nx * ay - ny * ax;
    return atan2f(sqrtf(px * px + py * py + pz * pz), nx * ax + ny * ay + nz * az);
}
LPC_HD void packet_finish(float rmax, float sx, float sy, float sz, PacketRec &Q)
{
    Q.ro = rmax * 1.00001f;
    const float sl = sqrtf(sx * sx + sy * sy + sz * sz);
    Q.ax = sx / sl; Q.ay = sy / sl; Q.az = sz / sl;
}
LPC_HD void packet_angle_finish(float angmax, bool finite, PacketRec &Q)
{
    Q.th = angmax * 1.00001f + 1e-6f;
    Q.all = (!finite || !(Q.th < 1.2f) || !(Q.ro < INFINITY) || !(Q.ax == Q.ax)) ? 1 : 0;
    Q.sth = sinf(Q.th);
    Q.cth = cosf(Q.th);
}

struct ExactRec {       // V0, E1 = V1-V0, E2 = V2-V0 (float, exactly as the reference), the triangle index
    float v0x, v0y, v0z, e1x, e1y, e1z, e2x, e2y, e2z;
    int32_t idx;
    float pad1, pad2;
};

// Host: float record of the exact bound dist^2 <= A + B ww (A rounded up, B up).
static inline void store_test(double A, double B, float *negB, float *negA)
{
    const double As = A * (1.0 + LPC_FILT_REL), Bs = B * (1.0 + LPC_FILT_REL) + LPC_FILT_ABS;
    if (!(Bs < 1.0) || !(As < 1e30)) { *negB = -1e30f; *negA = 0.0f; return; }   // always
    float Af = (float)As, Bf = (float)Bs;
    if ((double)Af < As) Af = nextafterf(Af, INFINITY);
    if ((double)Bf < Bs) Bf = nextafterf(Bf, INFINITY);
    *negA = -Af;
    *negB = -Bf;
}

// Host: exact bound implied by a passing float test of the record (negB, negA).
static inline void implied_test(float negB, float negA, double &A, double &B)
{
    A = -(double)negA * (1.0 + LPC_FILT_REL);
    B = -(double)negB * (1.0 + LPC_FILT_REL) + LPC_FILT_ABS;
}

// Host: Moller-Trumbore's line-distance error factor of a triangle: an accepted
// pair's line passes within kappa |T| of the triangle, kappa = kmt eps |E|^2 / |E1 x E2|
// (kmt = 256, deliberately generous; inf for a degenerate triangle).
static inline double tri_kappa(const float *V0, const float *V1, const float *V2)
{
    const double eps = 1.0 / 16777216.0, kmt = 256.0;
    double a[3], b[3];
    for (int k = 0; k < 3; ++k) { a[k] = (double)V1[k] - (double)V0[k]; b[k] = (double)V2[k] - (double)V0[k]; }
    const double n[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    const double nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
    const double aa = a[0] * a[0] + a[1] * a[1] + a[2] * a[2], bb = b[0] * b[0] + b[1] * b[1] + b[2] * b[2];
    const double cc = (b[0] - a[0]) * (b[0] - a[0]) + (b[1] - a[1]) * (b[1] - a[1]) + (b[2] - a[2]) * (b[2] - a[2]);
    const double emax2 = fmax(aa, fmax(bb, cc));
    return nn > 0.0 ? kmt * eps * emax2 / sqrt(nn) : INFINITY;
}

// Host: build the filter record of triangle (V0,V1,V2) given as floats.
#if defined(__HIPCC__)
static inline __host__ FiltRec filter_record(
#else
static inline FiltRec filter_record(
#endif
                                    const float *V0, const float *V1, const float *V2,
                                    int32_t idx, double Dcap, double S)
{
    const double eps = 1.0 / 16777216.0;   // 2^-24
    FiltRec r;
    r.idx = idx; r.pad0 = 0; r.pad1 = 0;
    double a[3], b[3], p0[3];
    float e1f[3], e2f[3];
    for (int k = 0; k < 3; ++k) {
        p0[k] = V0[k];
        a[k] = (double)V1[k] - (double)V0[k];
        b[k] = (double)V2[k] - (double)V0[k];
        e1f[k] = V1[k] - V0[k];
        e2f[k] = V2[k] - V0[k];
    }
    double n[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    double nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
    double aa = a[0] * a[0] + a[1] * a[1] + a[2] * a[2];
    double bb = b[0] * b[0] + b[1] * b[1] + b[2] * b[2];
    double cm[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    double cc = cm[0] * cm[0] + cm[1] * cm[1] + cm[2] * cm[2];
    // minimal enclosing sphere of the triangle
    double ctr[3];
    bool obtuse = (aa + bb <= cc) || (aa + cc <= bb) || (bb + cc <= aa) || nn <= 0.0;
    if (obtuse) {
        const float *P = V1, *Q = V2;            // longest edge midpoint
        if (aa >= bb && aa >= cc) { P = V0; Q = V1; }
        else if (bb >= aa && bb >= cc) { P = V0; Q = V2; }
        for (int k = 0; k < 3; ++k) ctr[k] = 0.5 * ((double)P[k] + (double)Q[k]);
    } else {
        // circumcentre: V0 + ((|a|^2 b - |b|^2 a) x n) / (2 |n|^2)
        double m[3] = {aa * b[0] - bb * a[0], aa * b[1] - bb * a[1], aa * b[2] - bb * a[2]};
        double x[3] = {m[1] * n[2] - m[2] * n[1], m[2] * n[0] - m[0] * n[2], m[0] * n[1] - m[1] * n[0]};
        for (int k = 0; k < 3; ++k) ctr[k] = p0[k] + x[k] / (2.0 * nn);
    }
    r.cx = (float)ctr[0]; r.cy = (float)ctr[1]; r.cz = (float)ctr[2];
    double fc[3] = {r.cx, r.cy, r.cz};
    double rho2 = 0.0;
    const float *Vs[3] = {V0, V1, V2};
    for (int v = 0; v < 3; ++v) {
        double d2 = 0.0;
        for (int k = 0; k < 3; ++k) { double q = (double)Vs[v][k] - fc[k]; d2 += q * q; }
        if (d2 > rho2) rho2 = d2;
    }
    rho2 *= (1.0 + 1e-6);
    bool zero_edge = (e1f[0] == 0.0f && e1f[1] == 0.0f && e1f[2] == 0.0f) ||
                     (e2f[0] == 0.0f && e2f[1] == 0.0f && e2f[2] == 0.0f);
    double e1n = sqrt((double)e1f[0] * e1f[0] + (double)e1f[1] * e1f[1] + (double)e1f[2] * e1f[2]);
    double e2n = sqrt((double)e2f[0] * e2f[0] + (double)e2f[1] * e2f[1] + (double)e2f[2] * e2f[2]);
    bool tiny = e1n * e2n * Dcap * (1.0 + 1e-4) < 1e-6;
    if (zero_edge || tiny) {           // never a candidate: d = +inf
        r.negB = 0.0f; r.negA = INFINITY;
        return r;
    }
    const double kappa = tri_kappa(V0, V1, V2);
    if (!(kappa < 0.1)) { r.negB = -1e30f; r.negA = 0.0f; return r; }   // always (sliver)
    const double ra = sqrt(rho2) * (1.0 + kappa);
    const double h = ra > 0.0 ? fmin(1.0, fmax(1e-3, kappa * S / ra)) : 1.0;
    store_test((1.0 + h) * ra * ra, (1.0 + 1.0 / h) * kappa * kappa, &r.negB, &r.negA);
    return r;
}

// Host: line-filter constants of a sliver.  Moller-Trumbore accepts only if
// |u| <= 1, i.e. |fl(P.T)| <= |fl(DEN)| (1+2eps) with P = D x E2, DEN = P.E1.
// With |fl(P.T) - (D x E2).T| <= 10 eps |D||E2||T| and
// |fl(DEN)| <= |D||E2 x E1| + 10 eps |D||E2||E1|, acceptance implies
//     |D.(E2 x T)| <= |D| (|E2 x E1|(1+3eps) + 11 eps |E2||E1| + 10 eps |E2||T|).
// The kernel tests x^2 <= (|D|(a + b tmax))^2 with x = D.(E2 x T) in float and
// tmax = max|T_i| (|T| <= sqrt(3) tmax).  Its own float evaluation adds at most
// 10 eps |D||E2||T| to |x| and 5 eps relative to the right side, so
// a = |E1 x E2| (1 + 16 eps) + 32 eps |E1||E2| and b = 64 sqrt(3) eps |E2| (b tmax >=
// 64 eps |E2||T|) cover both.  (Round 3 doubled the |E1 x E2| term as well: harmless
// for slivers, where it is ~0, but twice the width for a thin triangle's line.)
// Smallest |D| for which Moller-Trumbore's DEN = E1 . (D x E2) (float, .cl:75-79)
// can reach the 1e-6 threshold.  Per component P_i = (D x E2)_i is a difference
// of two products: |P^_i - P_i| <= 2.01 u s_i with s_i = |d_j e2_k| + |d_k e2_j|
// (with or without FMA); the 3-term float dot adds <= 3.01 u sum |e1_i| |P^_i|.
// With E1 . (D x E2) = D . (E2 x E1):
//     |DEN^| <= |D| (|E1 x E2| + 5.03 u G),  G = sum_i |e1_i| (|e2_j| + |e2_k|),
// so |D| < 0.999e-6 / (|E1 x E2| + 5.1 u G) never passes the DEN test.  revolve_curve's
// pole triangles are collinear (E1 x E2 = 0 exactly): their dmin is ~1e-6 / (5 u |E1||E2|),
// far above unit directions unless |E1||E2| is large.  Rounded down to float.
static inline float sliver_dmin(const float *V0, const float *V1, const float *V2)
{
    const double u = 1.0 / 16777216.0;
    double e1[3], e2[3];
    for (int k = 0; k < 3; ++k) { e1[k] = (double)(V1[k] - V0[k]); e2[k] = (double)(V2[k] - V0[k]); }
    const double c[3] = {e2[1] * e1[2] - e2[2] * e1[1], e2[2] * e1[0] - e2[0] * e1[2],
                         e2[0] * e1[1] - e2[1] * e1[0]};
    const double nc = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    const double n2 = sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
    double G = 0.0;
    for (int i = 0; i < 3; ++i) G += fabs(e1[i]) * (fabs(e2[(i + 1) % 3]) + fabs(e2[(i + 2) % 3]));
    const double coef = nc * (1.0 + 1e-9) + 1e-15 * n1 * n2 + 5.1 * u * G;
    if (!(coef > 0.0)) return INFINITY;                     // zero edge: DEN == 0 exactly
    const double dmin = 0.999e-6 / coef;
    float f = (float)dmin;
    if ((double)f > dmin) f = nextafterf(f, 0.0f);
    return f;
}

// The same bound about E1 (the v-test): Moller-Trumbore accepts only if
// 0 <= v and fl(u + v) <= 1 with u >= 0, so |fl(Q.D)| <= |fl(DEN)| (1 + 3eps) with
// Q = T x E1, and |fl(Q.D) - D.(T x E1)| <= 10 eps |D||E1||T| as for P.T: acceptance
// implies |D.(E1 x T)| <= |D| (|E1 x E2|(1+3eps) + 11 eps |E1||E2| + 10 eps |E1||T|),
// i.e. sliver_params with the roles of |E1| and |E2| swapped in the |T| term.
static inline void sliver_params_axis(const float *V0, const float *V1, const float *V2, int ax1, float *a_out,
                                      float *b_out)
{
    const double eps = 1.0 / 16777216.0;
    double e1[3], e2[3];
    for (int k = 0; k < 3; ++k) { e1[k] = (double)(V1[k] - V0[k]); e2[k] = (double)(V2[k] - V0[k]); }
    const double c[3] = {e2[1] * e1[2] - e2[2] * e1[1], e2[2] * e1[0] - e2[0] * e1[2],
                         e2[0] * e1[1] - e2[1] * e1[0]};
    const double nc = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    const double n2 = sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
#ifdef LPC_LINE_A2                  // round 3's constant (A/B builds only)
    double a = 2.0 * (nc * (1.0 + 4.0 * eps) + 16.0 * eps * n2 * n1);
#else
    double a = nc * (1.0 + 16.0 * eps) + 32.0 * eps * n2 * n1;
#endif
    double b = 2.0 * sqrt(3.0) * 32.0 * eps * (ax1 ? n1 : n2);
    float af = (float)a, bf = (float)b;
    if ((double)af < a) af = nextafterf(af, INFINITY);
    if ((double)bf < b) bf = nextafterf(bf, INFINITY);
    *a_out = af; *b_out = bf;
}

// Thin-triangle rule (LPC_THIN = k percent): the line filter about the longer of
// E1, E2 passes rays within h = |E1 x E2| / max(|E1|, |E2|) of a line, about 2 h S of
// a scene-sized cross-section (S the scene's half diagonal, 4 h S), the sphere test
// those within its radius rho (pi rho^2): the line filter is taken when
// k/100 * 8 h S < pi rho^2.  Returns 0 (sphere), 1 (line about E2) or 2 (about E1).
static inline int thin_axis(const float *V0, const float *V1, const float *V2, float cx, float cy, float cz,
                            double S, double k)
{
    if (!(k > 0.0)) return 0;
    double e1[3], e2[3], r2 = 0.0;
    const float *Vs[3] = {V0, V1, V2};
    const double fc[3] = {cx, cy, cz};
    for (int v = 0; v < 3; ++v) {
        double d2 = 0.0;
        for (int q = 0; q < 3; ++q) { const double x = (double)Vs[v][q] - fc[q]; d2 += x * x; }
        r2 = fmax(r2, d2);
    }
    for (int q = 0; q < 3; ++q) { e1[q] = (double)(V1[q] - V0[q]); e2[q] = (double)(V2[q] - V0[q]); }
    const double c[3] = {e2[1] * e1[2] - e2[2] * e1[1], e2[2] * e1[0] - e2[0] * e1[2],
                         e2[0] * e1[1] - e2[1] * e1[0]};
    const double nc = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    const double n2 = sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
    const double el = fmax(n1, n2);
    if (!(el > 0.0)) return 0;
    const double hh = nc / el;
    if (!(k * 8.0 * hh * S < 3.141592653589793 * r2)) return 0;
    return n1 > n2 ? 2 : 1;
}

static inline void sliver_params(const float *V0, const float *V1, const float *V2, float *a_out,
                                 float *b_out)
{
    const double eps = 1.0 / 16777216.0;
    double e1[3], e2[3];
    for (int k = 0; k < 3; ++k) { e1[k] = (double)(V1[k] - V0[k]); e2[k] = (double)(V2[k] - V0[k]); }
    const double c[3] = {e2[1] * e1[2] - e2[2] * e1[1], e2[2] * e1[0] - e2[0] * e1[2],
                         e2[0] * e1[1] - e2[1] * e1[0]};
    const double nc = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    const double n2 = sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
#ifdef LPC_LINE_A2                  // round 3's constant (A/B builds only)
    double a = 2.0 * (nc * (1.0 + 4.0 * eps) + 16.0 * eps * n2 * n1);
#else
    double a = nc * (1.0 + 16.0 * eps) + 32.0 * eps * n2 * n1;
#endif
    double b = 2.0 * sqrt(3.0) * 32.0 * eps * n2;
    float af = (float)a, bf = (float)b;
    if ((double)af < a) af = nextafterf(af, INFINITY);
    if ((double)bf < b) bf = nextafterf(bf, INFINITY);
    *a_out = af; *b_out = bf;
}

// Host: test of a hierarchy node over `count` triangles (vertex pointers
// tri[3*i .. 3*i+2]).  It must pass for every ray whose line Moller-Trumbore
// accepts against SOME triangle below the node (the triangles' own filter tests
// then pick the candidates).  With C the centre and R the radius of a sphere
// containing all their vertices, an accepted triangle's closest point X to the
// line lies in that sphere, so dist(C, line) <= R + kappa |T| with
// |T| <= |w_C| + R:  dist <= R (1 + kappa) + kappa |w_C|, kappa = max over the
// triangles (tri_kappa) -- the same form as a triangle's own record.
static inline void node_record(const float *const *tri, int count, double S, float *cx, float *cy, float *cz,
                               float *negB, float *negA)
{
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double kappa = 0.0;
    for (int i = 0; i < count; ++i) {
        kappa = fmax(kappa, tri_kappa(tri[3 * i], tri[3 * i + 1], tri[3 * i + 2]));
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) {
                lo[k] = fmin(lo[k], (double)tri[3 * i + v][k]);
                hi[k] = fmax(hi[k], (double)tri[3 * i + v][k]);
            }
    }
    *cx = *cy = *cz = 0.0f;
    if (count == 0) { *negB = 0.0f; *negA = INFINITY; return; }                 // never
    if (!(kappa < 0.1)) { *negB = -1e30f; *negA = 0.0f; return; }             // always
    const float C[3] = {(float)(0.5 * (lo[0] + hi[0])), (float)(0.5 * (lo[1] + hi[1])),
                        (float)(0.5 * (lo[2] + hi[2]))};
    double R2 = 0.0;
    for (int i = 0; i < count; ++i)
        for (int v = 0; v < 3; ++v) {
            double d2 = 0.0;
            for (int k = 0; k < 3; ++k) { const double q = (double)tri[3 * i + v][k] - C[k]; d2 += q * q; }
            R2 = fmax(R2, d2);
        }
    *cx = C[0]; *cy = C[1]; *cz = C[2];
    const double ra = sqrt(R2 * (1.0 + 1e-6)) * (1.0 + kappa);
    const double h = ra > 0.0 ? fmin(1.0, fmax(1e-3, kappa * S / ra)) : 1.0;
    store_test((1.0 + h) * ra * ra, (1.0 + 1.0 / h) * kappa * kappa, negB, negA);
}

}  // namespace lpc
