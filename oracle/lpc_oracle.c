/*
 * lpc_oracle.c -- CPU ORACLE for the LightPyCL per-bounce hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in lightpycl_amd/ may link, load or call
 * this file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg use it, and only as the checker / the timed CPU baseline.
 *
 * What it is: a plain-C restatement of the four OpenCL kernels of the
 * reference (kernel_reflect_refract_intersect.cl) with the reference's
 * arithmetic order.  Every function cites the reference lines it follows.
 *
 * Numeric conventions: the reference's kernels as ROCm's OpenCL compiler
 * builds them for gfx950 with IEEE division/sqrt and no FP contraction in the
 * kernel's own expressions (oracle/_ref/lpc_ref_ieee.co):
 *   - single-precision constants everywhere (the .cl only compiles with
 *     -cl-single-precision-constant);
 *   - no FMA contraction in the kernel expressions (build with -ffp-contract=off);
 *   - the OpenCL library's builtins as ROCm's device library evaluates them:
 *     dot(a,b) = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x)), cross.x =
 *     fma(a.y,b.z, -(a.z*b.y)) (cyclic), length = sqrt of that dot,
 *     normalize = v * rsqrt(dot) (the hardware's sqrt / rsqrt, which
 *     tools/rsq_check.py measures as correctly rounded; computed here through
 *     double), pown(x,2) = x*x;  exp/acos/atan2/sin/cos are the C library's
 *     (1-2 ulp from the device library's).
 *
 * Parity status: pinned against the reference's own kernels compiled for
 * gfx950 (tests/test_ref_parity.py, on the GPU) and by the known-answer rows
 * recorded in SURVEY.md section 4 and the reference-scene counts
 * (tests/test_oracle_pins.py).
 *
 * Layouts follow the reference exactly: float3 buffers are (n,4) float32
 * arrays (16-byte stride, w ignored on read, written as 0), per-ray/per-mesh
 * scratch is [ray][mesh] (iterative_tracer.py:236-237,267).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

typedef struct { float x, y, z; } v3;

static inline v3 ld3(const float *p) { v3 r; r.x = p[0]; r.y = p[1]; r.z = p[2]; return r; }
static inline void st3(float *p, v3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; p[3] = 0.0f; }
static inline v3 mk3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline v3 add3(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 scl3(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
static inline v3 neg3(v3 a) { return mk3(-a.x, -a.y, -a.z); }
/* OpenCL dot / cross / length / normalize (ROCm device library forms) */
static inline float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 cross3(v3 a, v3 b) {
    return mk3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline float rsq(float x) { return (float)(1.0 / sqrt((double)x)); }
static inline float len3(v3 a)
{
    const float s = dot3(a, a);
    if (s >= 1.17549435e-38f || s != s) {
        if (s != INFINITY) return sqrtf(s);
        const v3 b = mk3(a.x * 0x1p-66f, a.y * 0x1p-66f, a.z * 0x1p-66f);
        const float t = dot3(b, b);
        const int sc = t < 1.17549435e-38f;
        const float q = sqrtf(sc ? ldexpf(t, 32) : t);
        return (sc ? ldexpf(q, -16) : q) * 0x1p66f;
    }
    const v3 b = mk3(a.x * 0x1p86f, a.y * 0x1p86f, a.z * 0x1p86f);
    const float t = dot3(b, b);
    const int sc = t < 1.17549435e-38f;
    const float q = sqrtf(sc ? ldexpf(t, 32) : t);
    return (sc ? ldexpf(q, -16) : q) * 0x1p-86f;
}
static inline v3 nrm3(v3 a)
{
    float s = dot3(a, a);
    if (s >= 1.17549435e-38f || s != s) {
        if (s == INFINITY) {
            a = mk3(a.x * 0x1p-66f, a.y * 0x1p-66f, a.z * 0x1p-66f);
            s = dot3(a, a);
            if (s == INFINITY) {
                a = mk3(copysignf(isinf(a.x) ? 1.0f : 0.0f, a.x), copysignf(isinf(a.y) ? 1.0f : 0.0f, a.y),
                        copysignf(isinf(a.z) ? 1.0f : 0.0f, a.z));
                s = dot3(a, a);
            }
        }
    } else {
        a = mk3(a.x * 0x1p86f, a.y * 0x1p86f, a.z * 0x1p86f);
        s = dot3(a, a);
    }
    const int sc = s < 1.17549435e-38f;
    float r = rsq(sc ? s * 0x1p24f : s);
    if (sc) r = r * 0x1p12f;
    return mk3(a.x * r, a.y * r, a.z * r);
}

/* Moller-Trumbore, kernel_reflect_refract_intersect.cl:50-101.  Returns 1 and
 * *t when u,v tests pass (t itself is not range-checked here, as in .cl:98). */
static int orc_intersect_triangle(v3 O, v3 D, v3 V0, v3 V1, v3 V2, float *t)
{
    const float EPSILON_NUM = 0.000001f;          /* .cl:56 */
    v3 E1 = sub3(V1, V0);                          /* .cl:72 */
    v3 E2 = sub3(V2, V0);                          /* .cl:73 */
    v3 P = cross3(D, E2);                          /* .cl:75 */
    float DEN = dot3(P, E1);                       /* .cl:76 */
    if (DEN > -EPSILON_NUM && DEN < EPSILON_NUM)   /* .cl:79 */
        return 0;
    float iDEN = 1.0f / DEN;                       /* .cl:82 */
    v3 T = sub3(O, V0);                            /* .cl:83 */
    float u = dot3(P, T) * iDEN;                   /* .cl:86 */
    if (u < 0.0f || u > 1.0f)                      /* .cl:87 */
        return 0;
    v3 Q = cross3(T, E1);                          /* .cl:90 */
    float v = dot3(Q, D) * iDEN;                   /* .cl:93 */
    if (v < 0.0f || u + v > 1.0f)                  /* .cl:94 */
        return 0;
    *t = dot3(Q, E2) * iDEN;                       /* .cl:98 */
    return 1;
}

/* __kernel intersect, .cl:243-289.  Brute force over all triangles (sorted by
 * mesh); per-mesh min t / argmin / hit count flushed to [rid][mesh] slots at
 * every mesh_id change (.cl:262-269, including the "previous mesh = current
 * mesh_id - 1" slot arithmetic) and after the loop (.cl:286-288). */
void orc_intersect(int64_t n, const float *rays_origin, const float *rays_dir,
                   const float *mesh_v0, const float *mesh_v1, const float *mesh_v2,
                   const int32_t *mesh_id, int32_t mesh_count, int32_t tri_count,
                   float max_ray_len, float *isect_min_ray_len, int32_t *isects_count,
                   int32_t *ray_isect_mesh_idx_tmp)
{
    const float EPSILON = 0.000001f * max_ray_len; /* .cl:245 */
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t rid = 0; rid < n; ++rid) {
        v3 O = ld3(rays_origin + 4 * rid), D = ld3(rays_dir + 4 * rid);
        int32_t cnt = 0, best_i = -1;
        float best_t = max_ray_len;
        int64_t slot = 0;
        float t = 0.0f;
        for (int32_t i = 0; i < tri_count; ++i) {
            slot = (int64_t)mesh_count * rid + mesh_id[i];                 /* .cl:260 */
            if (i > 0 && mesh_id[i - 1] != mesh_id[i]) {                   /* .cl:262 */
                isects_count[slot - 1] = cnt;
                isect_min_ray_len[slot - 1] = best_t;
                ray_isect_mesh_idx_tmp[slot - 1] = best_i;
                cnt = 0; best_t = max_ray_len; best_i = -1;
            }
            int hit = orc_intersect_triangle(O, D, ld3(mesh_v0 + 4 * (int64_t)i),
                                             ld3(mesh_v1 + 4 * (int64_t)i),
                                             ld3(mesh_v2 + 4 * (int64_t)i), &t);
            if (hit && t > EPSILON) {                                      /* .cl:277 */
                if (t < best_t) { best_t = t; best_i = i; }
                cnt += 1;
            }
        }
        isects_count[slot] = cnt;                                          /* .cl:286 */
        isect_min_ray_len[slot] = best_t;
        ray_isect_mesh_idx_tmp[slot] = best_i;
    }
}

/* __kernel intersect_postproc, .cl:105-240. */
void orc_intersect_postproc(int64_t n, const float *rays_origin, const float *rays_dir,
                            float *rays_dest, const int32_t *rays_prev_isect_mesh_id,
                            int32_t *rays_n1_mesh_id, int32_t *rays_n2_mesh_id,
                            int32_t *ray_entering, int32_t *ray_isect_mesh_id,
                            int32_t *ray_isect_mesh_idx, const int32_t *mesh_mat_type,
                            const float *isect_min_ray_len, const int32_t *isects_count,
                            const int32_t *ray_isect_mesh_idx_tmp, int32_t mesh_count,
                            float max_ray_len)
{
    const float EPSILON = 0.000001f * max_ray_len; /* .cl:112 */
#pragma omp parallel for schedule(static)
    for (int64_t rid = 0; rid < n; ++rid) {
        const int64_t b = (int64_t)mesh_count * rid;
        float t_tmp;
        int32_t hit_mesh = -1, hit_idx = -1;
        float t_min = max_ray_len;
        int32_t n1_id = -1, n2_id = -1;
        int32_t prev = rays_prev_isect_mesh_id[rid];
        for (int32_t j = 0; j < mesh_count; ++j) {                        /* .cl:127-135 */
            t_tmp = isect_min_ray_len[b + j];
            if (t_tmp < t_min) { t_min = t_tmp; hit_mesh = j; hit_idx = ray_isect_mesh_idx_tmp[b + j]; }
        }
        if (hit_mesh >= 0) {
            int32_t entering = 1 - (isects_count[b + hit_mesh] % 2);     /* .cl:142 */
            ray_entering[rid] = entering;
            if (prev == -2) {                                              /* .cl:145-155 */
                if (entering == 1) { n1_id = -1; n2_id = hit_mesh; }
                else { n1_id = hit_mesh; n2_id = -1; }
            } else if (prev == -1) {                                       /* .cl:156-166 */
                if (entering == 1) { n1_id = -1; n2_id = hit_mesh; }
                else { n1_id = hit_mesh; n2_id = -1; }
            } else {                                                       /* .cl:167-177 */
                if (entering == 1) { n1_id = prev; n2_id = hit_mesh; }
                else { n1_id = hit_mesh; n2_id = -1; }
            }
            float t_minmin = t_min, t_maxmin = t_min, t_minmax = max_ray_len; /* .cl:187-192 */
            int32_t maxmin_entering = 0, maxmin_idx = -1, minmax_idx = -1;
            for (int32_t j = 0; j < mesh_count; ++j) {                    /* .cl:193-214 */
                if (mesh_mat_type[j] == 0 || mesh_mat_type[j] == 4) {
                    t_tmp = isect_min_ray_len[b + j];
                    entering = 1 - (isects_count[b + j] % 2);
                    if (t_tmp <= t_minmin + EPSILON && t_tmp >= t_maxmin) {
                        t_maxmin = t_tmp; maxmin_idx = j; maxmin_entering = entering;
                    }
                    if (t_tmp > t_minmin + EPSILON && entering == 0 && t_tmp <= t_minmax) {
                        t_minmax = t_tmp; minmax_idx = j;
                    }
                }
            }
            if (maxmin_entering == 1) { t_min = t_maxmin; n2_id = maxmin_idx; }   /* .cl:216-219 */
            else {                                                                /* .cl:220-229 */
                if (maxmin_idx >= 0) t_min = t_maxmin;
                if (minmax_idx >= 0) n2_id = minmax_idx;
            }
        }
        rays_n1_mesh_id[rid] = n1_id;                                      /* .cl:235-239 */
        rays_n2_mesh_id[rid] = n2_id;
        st3(rays_dest + 4 * rid, add3(ld3(rays_origin + 4 * rid), scl3(ld3(rays_dir + 4 * rid), t_min)));
        ray_isect_mesh_id[rid] = hit_mesh;
        ray_isect_mesh_idx[rid] = hit_idx;
    }
}

/* reflect_refract, .cl:293-343 (unpolarised Fresnel + Snell).  Returns 1 and
 * leaves the outputs untouched when TIR_check is NaN (.cl:342). */
static int orc_reflect_refract(v3 dest, v3 dir, float pw, v3 *r_org, v3 *r_dir, float *r_pow,
                               int32_t *r_meas, v3 *t_org, v3 *t_dir, float *t_pow,
                               int32_t *t_meas, v3 nrm_in, float n1, float n2)
{
    v3 nrm = nrm_in;
    float r = n1 / n2;                                                     /* .cl:299 */
    float cosT1 = -dot3(nrm, dir);                                         /* .cl:303 */
    if (cosT1 < 0.0f) { nrm = neg3(nrm_in); cosT1 = -dot3(nrm, dir); }     /* .cl:304-307 */
    float TIR_check = 1.0f - (r * r) * (1.0f - (cosT1 * cosT1));          /* .cl:309 */
    if (TIR_check >= 0.0f) {                                               /* .cl:310-328 */
        float cosT2 = sqrtf(TIR_check);
        float a = fabsf((n1 * cosT1 - n2 * cosT2) / (n1 * cosT1 + n2 * cosT2));
        float b = fabsf((n1 * cosT2 - n2 * cosT1) / (n1 * cosT2 + n2 * cosT1));
        float Rs = a * a, Rp = b * b;
        float reflect_power = pw * (Rs + Rp) / 2.0f;
        *r_dir = add3(dir, scl3(nrm, 2.0f * cosT1));
        *r_org = dest; *r_pow = reflect_power; *r_meas = 0;
        *t_dir = add3(scl3(dir, r), scl3(nrm, r * cosT1 - cosT2));
        *t_org = dest; *t_pow = pw - reflect_power; *t_meas = 0;
        return 0;
    }
    if (TIR_check < 0.0f) {                                                /* .cl:329-341 */
        *r_dir = add3(dir, scl3(nrm, 2.0f * cosT1));
        *r_org = dest; *r_pow = pw; *r_meas = 0;
        *t_dir = mk3(0.0f, 0.0f, 0.0f);
        *t_org = dest; *t_pow = 0.0f; *t_meas = -1;
        return 0;
    }
    return 1;
}

/* __kernel reflect_refract_rays, .cl:346-474.  Children origins are written
 * as (n,4) arrays like the reference's rays_reflect_origin/rays_refract_origin.
 * Where the reference would store uninitialised locals (NaN TIR_check, .cl:342)
 * the children are written as terminated rays (documented deviation). */
void orc_reflect_refract_rays(int64_t n, const float *in_rays_origin, const float *in_rays_dest,
                              const float *in_rays_dir, float *in_rays_power,
                              int32_t *in_rays_measured, const int32_t *rays_n1_mesh_id,
                              const int32_t *rays_n2_mesh_id, float *rays_reflect_origin,
                              float *rays_reflect_dir, float *rays_reflect_power,
                              int32_t *rays_reflect_measured, float *rays_refract_origin,
                              float *rays_refract_dir, float *rays_refract_power,
                              int32_t *rays_refract_measured, const int32_t *ray_isect_mesh_id,
                              const int32_t *ray_isect_mesh_idx, const float *mesh_v0,
                              const float *mesh_v1, const float *mesh_v2,
                              const int32_t *mesh_mat_type, const float *mesh_ior,
                              const float *mesh_refl, const float *mesh_diss, float IOR_env)
{
    const float EPSILON_NUM = 0.000001f;                                   /* .cl:359 */
#pragma omp parallel for schedule(static)
    for (int64_t rid = 0; rid < n; ++rid) {
        int32_t rmid = ray_isect_mesh_id[rid];
        int32_t mesh_mat = 2;                                              /* .cl:364 */
        float R_mesh = 0.0f;
        if (rmid >= 0) { mesh_mat = mesh_mat_type[rmid]; R_mesh = mesh_refl[rmid]; }
        int32_t n1id = rays_n1_mesh_id[rid], n2id = rays_n2_mesh_id[rid];
        float IOR_in = IOR_env, IOR_n2 = IOR_env;                          /* .cl:380-381 */
        float pw = in_rays_power[rid];
        v3 dest = ld3(in_rays_dest + 4 * rid);
        if (n1id >= 0) {                                                   /* .cl:385-394 */
            IOR_in = mesh_ior[n1id];
            if (mesh_mat_type[n1id] == 0 && mesh_diss[n1id] > EPSILON_NUM) {
                float ray_len = len3(sub3(dest, ld3(in_rays_origin + 4 * rid)));
                pw = pw * expf(-mesh_diss[n1id] * ray_len);
                in_rays_power[rid] = pw;
            }
        }
        if (n2id >= 0) IOR_n2 = mesh_ior[n2id];                            /* .cl:401-403 */
        int32_t irm = in_rays_measured[rid];
        v3 zero = mk3(0.0f, 0.0f, 0.0f);
        if (irm == 0 && rmid >= 0 && (mesh_mat == 0 || mesh_mat == 1)) {   /* .cl:408 */
            int64_t m = ray_isect_mesh_idx[rid];
            v3 v0 = ld3(mesh_v0 + 4 * m), v1 = ld3(mesh_v1 + 4 * m), v2 = ld3(mesh_v2 + 4 * m);
            v3 nrm = nrm3(cross3(sub3(v1, v0), sub3(v2, v1)));           /* .cl:413 */
            v3 ro = dest, rd = zero, to = dest, td = zero;
            float rp = 0.0f, tp = 0.0f;
            int32_t rm = -1, tm = -1;
            orc_reflect_refract(dest, ld3(in_rays_dir + 4 * rid), pw, &ro, &rd, &rp, &rm,
                                &to, &td, &tp, &tm, nrm, IOR_in, IOR_n2);
            if (mesh_mat == 0) {                                           /* .cl:429-439 */
                st3(rays_reflect_origin + 4 * rid, ro); st3(rays_reflect_dir + 4 * rid, rd);
                rays_reflect_power[rid] = rp; rays_reflect_measured[rid] = rm;
                st3(rays_refract_origin + 4 * rid, to); st3(rays_refract_dir + 4 * rid, td);
                rays_refract_power[rid] = tp; rays_refract_measured[rid] = tm;
            } else {                                                       /* .cl:440-452 */
                st3(rays_reflect_origin + 4 * rid, ro); st3(rays_reflect_dir + 4 * rid, rd);
                rays_reflect_power[rid] = pw * R_mesh; rays_reflect_measured[rid] = rm;
                st3(rays_refract_origin + 4 * rid, to); st3(rays_refract_dir + 4 * rid, zero);
                rays_refract_power[rid] = 0.0f; rays_refract_measured[rid] = -1;
            }
        } else {                                                           /* .cl:455-472 */
            st3(rays_reflect_origin + 4 * rid, dest); st3(rays_reflect_dir + 4 * rid, zero);
            rays_reflect_power[rid] = 0.0f; rays_reflect_measured[rid] = -1;
            st3(rays_refract_origin + 4 * rid, dest); st3(rays_refract_dir + 4 * rid, zero);
            rays_refract_power[rid] = 0.0f; rays_refract_measured[rid] = -1;
            if (mesh_mat == 2 || rmid < 0) in_rays_measured[rid] = -1;
            if (mesh_mat == 3 && rmid >= 0) in_rays_measured[rid] = 1;
        }
    }
}

/* __kernel angular_project, .cl:509-538 (rot_mtx / pivot are float3 rows). */
void orc_angular_project(int64_t n, const float *vecs, const float *pwrs, const float *rot_mtx,
                         const float *pivot, float *x, float *y, float *pwrs_cor)
{
    const float EPSILON = 0.000001f;
#pragma omp parallel for schedule(static)
    for (int64_t gid = 0; gid < n; ++gid) {
        v3 piv = ld3(pivot);
        v3 vec = sub3(ld3(vecs + 4 * gid), piv);
        float pwr = pwrs[gid];
        float u = dot3(vec, ld3(rot_mtx + 0)) + piv.x;
        float v = dot3(vec, ld3(rot_mtx + 4)) + piv.y;
        float w = dot3(vec, ld3(rot_mtx + 8)) + piv.z;
        float l = sqrtf(u * u + v * v + w * w);
        v3 vecr = mk3(u / l, v / l, w / l);
        float cosT = dot3(mk3(0.0f, 0.0f, 1.0f), vecr);
        float phi = atan2f(v, u);
        float r = acosf(cosT);
        float A = 1.0f;
        if (r > EPSILON) A = sinf(r) / r;
        x[gid] = r * cosf(phi);
        y[gid] = r * sinf(phi);
        pwrs_cor[gid] = pwr / A;
    }
}

/* __kernel stereograph_project, .cl:488-506. */
void orc_stereograph_project(int64_t n, const float *vecs, const float *pwrs, const float *rot_mtx,
                             const float *pivot, float *x, float *y, float *pwrs_cor)
{
#pragma omp parallel for schedule(static)
    for (int64_t gid = 0; gid < n; ++gid) {
        v3 piv = ld3(pivot);
        v3 vec = sub3(ld3(vecs + 4 * gid), piv);
        float pwr = pwrs[gid];
        float u = dot3(vec, ld3(rot_mtx + 0)) + piv.x;
        float v = dot3(vec, ld3(rot_mtx + 4)) + piv.y;
        float w = dot3(vec, ld3(rot_mtx + 8)) + piv.z;
        float l = sqrtf(u * u + v * v + w * w);
        float xt = u / (l + w), yt = v / (l + w);
        float q = 1.0f + xt * xt + yt * yt;
        float A = 4.0f / (q * q);
        x[gid] = xt; y[gid] = yt; pwrs_cor[gid] = pwr / A;
    }
}

/* Build-identity helper for the ctypes loader. */
int orc_abi_version(void) { return 1; }

/* The OpenMP team of the calls above (the timed CPU baseline sets it to the
 * process's affinity mask explicitly instead of inheriting OMP_NUM_THREADS);
 * returns the team size in effect.  Not part of the reference. */
int32_t orc_set_threads(int32_t n)
{
    if (n > 0) omp_set_num_threads(n);
    return (int32_t)omp_get_max_threads();
}
