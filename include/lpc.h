/*
 * lpc.h -- C ABI of liblpc.so, the MI355X-native per-bounce engine of the
 * LightPyCL drop-in (package lightpycl_amd).
 *
 * The reference (ngchihuan/LightPyCL) drives its hot path through PyOpenCL:
 *   self.prg.intersect(queue, (n,), None, ...)            iterative_tracer.py:288
 *   self.prg.intersect_postproc(queue, (n,), None, ...)   iterative_tracer.py:303
 *   self.prg.reflect_refract_rays(queue, (n,), None, ...) iterative_tracer.py:318
 *   self.prg.angular_project(queue, (n,), None, ...)      iterative_tracer.py:546
 * around a host loop (iterative_tracer.py:241-391).  The entry points below
 * replace those launches and that loop.  Conventions:
 *   - every function returns 0 on success, a negative LPC_E* code on error;
 *     lpc_last_error() gives the message (the reference raises PyOpenCL
 *     exceptions; the Python layer turns a non-zero status into RuntimeError);
 *   - "host" arguments are caller-owned host buffers, copied in/out before
 *     the call returns; "dev" arguments are device pointers (hipMalloc'd or
 *     torch tensors' data_ptr) on the handle's device;
 *   - float3 data crosses the boundary in the reference's layout: (n,4)
 *     float32 rows, w ignored on input and written as 0 on output;
 *   - one handle per GPU; a handle is not thread-safe (the reference uses a
 *     single in-order queue per tracer, iterative_tracer.py:74).
 */
#ifndef LPC_H
#define LPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LPC_ABI_VERSION 4

enum {
    LPC_OK = 0,
    LPC_E_ARG = -1,      /* bad argument (null pointer, size, no scene, ...) */
    LPC_E_HIP = -2,      /* HIP runtime error (message has the hipError string) */
    LPC_E_STATE = -3,    /* call out of order (e.g. iterate before set_rays) */
    LPC_E_NOMEM = -4     /* device allocation failed */
};

typedef struct lpc_handle lpc_handle;

/* ---- library / device --------------------------------------------------- */
int lpc_abi_version(void);
/* Number of visible HIP devices (0 if none). */
int lpc_device_count(int *count);
/* Name, architecture (gcnArchName) and CU count of HIP device `device`
 * without opening a handle: the drop-in's device selection by name
 * (CL_Tracer(device_name=...), iterative_tracer.py:50-55). */
int lpc_device_query(int device, char *name, int name_len, char *arch, int arch_len, int *cu_count);
/* Open a handle on HIP device `device` (replaces CL_Tracer.__init__'s
 * platform/device/context/queue setup, iterative_tracer.py:36-74). */
int lpc_open(int device, lpc_handle **out);
int lpc_close(lpc_handle *h);
/* Last error message of `h` (or of the last failed lpc_open when h is NULL). */
const char *lpc_last_error(const lpc_handle *h);
/* Device name / CU count of the handle's GPU (diagnostics). */
int lpc_device_info(lpc_handle *h, char *name, int name_len, int *cu_count);

/* ---- scene (iterative_tracer.py:121-169) -------------------------------- */
/* Upload the flattened scene.  v0,v1,v2: host (tri_count,4) float32 rows;
 * mesh_id: host int32[tri_count], contiguous runs per mesh as the reference
 * builds them (:137-150); material tables host [mesh_count] (:122-135).
 * The reference's slot arithmetic for mesh_id changes (.cl:260-265) is
 * reproduced, so non-contiguous or empty meshes behave as in the reference. */
int lpc_scene_upload(lpc_handle *h, int32_t tri_count, const float *v0, const float *v1,
                     const float *v2, const int32_t *mesh_id, int32_t mesh_count,
                     const int32_t *mat_type, const float *ior, const float *refl,
                     const float *diss);

/* ---- one bounce on host arrays (iterative_tracer.py:280-348) ------------- */
/* Runs intersect + intersect_postproc + reflect_refract_rays (fused on the
 * device) for n rays.  pow and meas are read and written back (dissipation
 * .cl:392, measured state .cl:466-471).  prev_mid = rays_current_mid (-2 just
 * emitted, -1 outside, >=0 mesh).  Children origins equal dest (.cl:319,324,
 * 456,461), so only dest is returned.  Optional outputs may be NULL:
 * n1_mid, n2_mid, entering, isect_idx. */
int lpc_bounce_host(lpc_handle *h, int64_t n, const float *origin4, const float *dir4,
                    float *pow, int32_t *meas, const int32_t *prev_mid, float max_ray_len,
                    float ior_env, float *dest4, int32_t *isect_mid, float *r_dir4,
                    float *r_pow, int32_t *r_meas, float *t_dir4, float *t_pow,
                    int32_t *t_meas, int32_t *n1_mid, int32_t *n2_mid, int32_t *entering,
                    int32_t *isect_idx);

/* ---- reference-kernel drop-ins on device buffers ------------------------- */
/* Same argument meaning and (n,4)/[ray][mesh] layouts as the .cl kernels, for
 * a host that keeps its own device buffers and launch sequence.  The scene
 * (vertices, mesh ids, materials) is the one given to lpc_scene_upload; the
 * .cl kernels' mesh_v0/v1/v2/mesh_id/mesh_* arguments are therefore implicit.
 * Launches are stream-ordered on the handle's stream and synchronised before
 * return, as the reference's event.wait() does. */
/* __kernel intersect (.cl:243-289): per [ray][mesh] min t / argmin / count. */
int lpc_intersect(lpc_handle *h, int64_t n, const float *dev_origin4, const float *dev_dir4,
                  float max_ray_len, float *dev_isect_min_ray_len, int32_t *dev_isects_count,
                  int32_t *dev_isect_idx_tmp);
/* __kernel intersect_postproc (.cl:105-240). */
int lpc_intersect_postproc(lpc_handle *h, int64_t n, const float *dev_origin4,
                           const float *dev_dir4, float *dev_dest4,
                           const int32_t *dev_prev_mid, int32_t *dev_n1_mid,
                           int32_t *dev_n2_mid, int32_t *dev_entering,
                           int32_t *dev_isect_mid, int32_t *dev_isect_idx,
                           const float *dev_isect_min_ray_len,
                           const int32_t *dev_isects_count,
                           const int32_t *dev_isect_idx_tmp, float max_ray_len);
/* __kernel reflect_refract_rays (.cl:346-474); children origins written too. */
int lpc_reflect_refract_rays(lpc_handle *h, int64_t n, const float *dev_origin4,
                             const float *dev_dest4, const float *dev_dir4, float *dev_pow,
                             int32_t *dev_meas, const int32_t *dev_n1_mid,
                             const int32_t *dev_n2_mid, float *dev_r_origin4,
                             float *dev_r_dir4, float *dev_r_pow, int32_t *dev_r_meas,
                             float *dev_t_origin4, float *dev_t_dir4, float *dev_t_pow,
                             int32_t *dev_t_meas, const int32_t *dev_isect_mid,
                             const int32_t *dev_isect_idx, float ior_env);

/* ---- device-resident trace (iterative_tracer.py:241-391 on the GPU) ------- */
typedef struct {
    int64_t n_in;            /* rays traced this iteration                       */
    int64_t n_reflect;       /* kept reflected children (meas == 0)               */
    int64_t n_refract;       /* kept refracted children                           */
    int64_t n_measured;      /* rays that hit a measure surface this iteration    */
    double power_next;       /* sum of next-population power (float64)            */
    int64_t power_nonneg;    /* 1: every kept child's power is >= 0, 0: some is < 0
                                or NaN, -1: not tracked (traced iterations); the
                                host's bound on the reference's float32 sorted sum
                                (:372) needs 1                                      */
} lpc_iter_stats;

/* Load the initial population from host (n,4) rows and power[n]; prev_mid = -2,
 * meas = 0 (:117-118).  Also keeps a device copy for lpc_trace_reset. */
int lpc_trace_set_rays(lpc_handle *h, int64_t n, const float *origin4, const float *dir4,
                       const float *pow, float max_ray_len, float ior_env);
/* Restore the population given to lpc_trace_set_rays (device-to-device) and
 * zero the measured record / per-mesh power. */
int lpc_trace_reset(lpc_handle *h);
/* One iteration over the whole current population (processed in chunks of at
 * most lpc_set_chunk rays): bounce, on-device compaction into the next
 * population ([reflected kept ; refracted kept], :366-373), measured-ray record
 * and per-mesh measured power.  Optional host exports (NULL to skip), sized for
 * st->n_in = current population (known from the previous call / set_rays):
 *   out_origin4/out_dest4 (n_in,4), out_pow (n_in) post-dissipation,
 *   out_meas (n_in)                                    -> the results tuple :355
 *   out_next_pow (n_reflect + n_refract, capacity 2*n_in) -> termination sum :372
 * Without any export (and one chunk) the iteration runs in its coherence order:
 * the same per-ray results, but the next population and this iteration's part
 * of the measured record come in the parents' traced order instead of the
 * reference's (LPC_TRACED=0 keeps the reference order).  The call may return
 * while the iteration's last kernel still runs; the next call, lpc_trace_run
 * and every copy to the host wait for it. */
int lpc_trace_iterate(lpc_handle *h, float *out_origin4, float *out_dest4, float *out_pow,
                      int32_t *out_meas, float *out_next_pow, lpc_iter_stats *st);
/* lpc_trace_iterate with the results tuple (:335-355) exported asynchronously:
 * `host` is a block of the caller's (pinned: lpc_host_alloc, so the copy is a
 * DMA that overlaps the next kernels) laid out over the iteration's N = st->n_in
 * rays as [origin (N,4) if flags & 1][dest (N,4)][pow (N)][meas (N)] -- the
 * results tuple's arrays, reference ray order, w = 0.  The call returns once
 * the iteration's counters are read; the block is complete after lpc_sync (or
 * any call that copies device data to the host).  The host must not reuse or
 * free the block before then. */
int lpc_trace_iterate_export(lpc_handle *h, void *host, int32_t flags, lpc_iter_stats *st);
/* The current population's power (float32[n], n = lpc_trace_population): the
 * values the reference sums at :372 after compaction. */
int lpc_trace_population_power(lpc_handle *h, float *out);
/* Page-locked host memory for lpc_trace_iterate_export (hipHostMalloc). */
int lpc_host_alloc(size_t bytes, void **out);
int lpc_host_free(void *p);
/* The reference's input-power sum `sum(np.sort(rays_power))` (iterative_tracer.py
 * :115, :372) after the sort: a sequential float32 accumulation of x[0..n) left to
 * right, as Python's builtin sum over float32 scalars evaluates it (n = 0: 0).
 * Host code, no device; the drop-in runs it on a thread beside the upload. */
int lpc_host_seq_sum_f32(const float *x, int64_t n, float *out);
/* The reference's iteration loop on one device (iterative_tracer.py:241-391):
 * lpc_trace_iterate until the next population's power is below
 * power_threshold (= (1 - trace_until_dissipated) * input power, :383) or no
 * ray is kept (:389), at most max_iter iterations.  per_iter[max_iter]
 * receives each iteration's stats, *n_iter their number.  Same results as
 * calling lpc_trace_iterate from the host loop, without a host round trip
 * through the caller per iteration.  measured_count / mesh_power (may be NULL)
 * receive lpc_trace_measured's outputs at the end: mesh_power one double per
 * mesh of the current scene, into a buffer of mesh_power_cap doubles
 * (LPC_E_ARG, before anything runs, when the scene has more meshes; ABI 4). */
int lpc_trace_run(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                  int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap);
/* lpc_trace_run without waiting for the last iteration's kernels (the moves of
 * the next population's rows and of the measured record; the outputs above are
 * final when it returns): a caller that traces batch after batch lets the next
 * batch's launches queue behind them.  Every entry point that copies device data
 * to the host waits for them first; lpc_sync waits explicitly. */
int lpc_trace_run_async(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                        int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap);
/* lpc_trace_reset + lpc_trace_run_async in one call: the next batch of a caller
 * that re-traces the rays set with lpc_trace_set_rays (one host round trip less
 * between batches). */
int lpc_trace_rerun_async(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                          int32_t *n_iter, int64_t *measured_count, double *mesh_power, int32_t mesh_power_cap);
/* ---- streamed batches of new rays (round 6) ------------------------------- */
/* The reference uploads each partition's rays inside its loop
 * (iterative_tracer.py:280-284) and its examples trace batch after batch of new
 * sources.  lpc_trace_stage_rays queues the next batch (at most two staged): a
 * helper thread copies the caller's (n,4) rows and power to the device on a copy
 * stream (straight from the caller's memory; DESIGN.md section 7f measured the
 * pinned-staging variants slower) and runs the emitted rays' analysis there,
 * while the handle traces the batch before it.  The caller's arrays must stay
 * valid and unchanged until the lpc_trace_run_staged_async that traces the batch
 * returns.  lpc_trace_run_staged_async makes the oldest staged batch the emitted
 * rays (as lpc_trace_set_rays does, without the host copy inside the call) and
 * runs lpc_trace_run_async on it; its first kernels queue behind the previous
 * trace's last ones.  The pipelined caller stages batch k + 1, then traces batch
 * k.  Batches may be staged before a scene is uploaded (the drop-in stages its
 * rays before it builds the scene records) and survive a scene upload. */
int lpc_trace_stage_rays(lpc_handle *h, int64_t n, const float *origin4, const float *dir4, const float *pow,
                         float max_ray_len, float ior_env);
int lpc_trace_run_staged_async(lpc_handle *h, int32_t max_iter, double power_threshold, lpc_iter_stats *per_iter,
                               int32_t *n_iter, int64_t *measured_count, double *mesh_power,
                               int32_t mesh_power_cap);

/* ---- ray-sharded trace: one process per GPU ---------- */
/* All-reduce (sum, in place) of n doubles over the ranks of a sharded trace;
 * every rank must receive the identical bits.  Returns 0 on success. */
typedef int (*lpc_allreduce_fn)(void *ctx, double *vals, int32_t n);
/* Install (fn != NULL) or remove the all-reduce hook of h.  With a hook, the
 * loop of lpc_trace_run(_async) all-reduces each iteration's stats and takes
 * the reference's termination decisions (iterative_tracer.py:383-391) on the
 * sums over all ranks, so every rank takes the same decision; *measured_count
 * and mesh_power are then the sums over all ranks too.  per_iter keeps this
 * rank's own stats.  The power left is a rank-order float64 sum of per-rank
 * float64 sums: its rounding differs from a single device's tile-order sum
 * (and both from the reference's float32 sorted sum, :372), so a trace whose
 * power left lands within ~1e-12 relative of the threshold may stop one
 * iteration apart from a single-device trace.  Every exchange carries a
 * failure flag in slot 0 (0 from a healthy rank): a rank whose trace fails
 * locally still joins the exchange its peers wait in, with the flag set to 1;
 * a rank whose summed flag is not 0 fails with LPC_E_STATE ("a peer rank
 * failed").  The data slots may hold NaN (NaN powers are data: the trace goes
 * on, as the reference's `NaN < thr` is false). */
int lpc_set_allreduce(lpc_handle *h, lpc_allreduce_fn fn, void *ctx);
/* The all-reduced per-iteration stats of the last lpc_trace_run(_async) (this
 * rank's own without a hook).  *n_iter = iterations; at most cap are copied. */
int lpc_trace_global_stats(lpc_handle *h, lpc_iter_stats *per_iter, int32_t cap, int32_t *n_iter);
/* The library's all-reduce for the ranks of one node: POSIX shared memory
 * segment `name`, created by the rank passing create != 0 (the others wait for
 * it); rank-order sums, so identical bits on every rank.  lpc_shm_allreduce is
 * an lpc_allreduce_fn (ctx = the comm).  lpc_shm_comm_unlink removes the name
 * once every rank has opened it (the mapping stays); close unmaps.  A timed-out
 * exchange (300 s) or lpc_shm_comm_abort breaks the comm for good: every later
 * lpc_shm_allreduce on it fails, and so do the peers' current waits (they see
 * the rank's abort word), since the ranks no longer agree on which exchange is
 * which. */
typedef struct lpc_shm_comm lpc_shm_comm;
int lpc_shm_comm_open(const char *name, int32_t rank, int32_t world, int32_t create, lpc_shm_comm **out);
int lpc_shm_comm_unlink(lpc_shm_comm *comm);
int lpc_shm_allreduce(void *comm, double *vals, int32_t n);
int lpc_shm_comm_abort(lpc_shm_comm *comm);
int lpc_shm_comm_close(lpc_shm_comm *comm);

/* Wait until the handle's stream has finished every queued kernel. */
int lpc_sync(lpc_handle *h);
/* Current population size. */
int lpc_trace_population(lpc_handle *h, int64_t *n);
/* Measured record so far: count and per-mesh measured power (double[mesh_count]
 * into a buffer of mesh_power_cap doubles; LPC_E_ARG when it is smaller). */
int lpc_trace_measured(lpc_handle *h, int64_t *count, double *mesh_power, int32_t mesh_power_cap);
/* Copy the measured record to host: pos4 (count,4), pow (count), mesh (count);
 * any pointer may be NULL. */
int lpc_trace_fetch_measured(lpc_handle *h, float *pos4, float *pow, int32_t *mesh);
/* Rays per device chunk (0 = library default). */
int lpc_set_chunk(lpc_handle *h, int64_t rays_per_chunk);
/* Hierarchy-walk grid in single-wave blocks (64 .. 2^22; 0 = library default,
 * 65 536).  A launch policy with no reference counterpart, results unchanged:
 * handles that trace side by side on one GPU (lightpycl_amd.pool.TracePool,
 * bench.py's traces in flight) run faster with 16 384, one trace alone with the
 * default.  LPC_E_ARG out of range. */
int lpc_set_walk_grid(lpc_handle *h, int64_t blocks);

/* ---- trace-end projection + binning (iterative_tracer.py:503-562) -------- */
/* angular_project (.cl:509-538) / stereograph_project (.cl:488-506) of n host
 * points with rotation rows rot4 (4x4 float32 rows, reference R_dev) and
 * pivot4, followed by np.histogram2d-compatible binning into H[nx][ny]
 * (float64, += (double)pwr_cor / weight_div, iterative_tracer.py:556-560) over the given float64 bin edges
 * (nx+1, ny+1; value == last edge goes to the last bin, outside -> dropped).
 * mode 0 = angular, 1 = stereographic.  x/y/pwr_cor host outputs may be NULL.
 * If pos4 == NULL the trace's measured record (device-resident) is used. */
int lpc_project_hist(lpc_handle *h, int mode, int64_t n, const float *pos4, const float *pwr,
                     const float *rot4, const float *pivot4, const double *xedges, int nx,
                     const double *yedges, int ny, double weight_div, double *H,
                     float *x, float *y, float *pwr_cor);

/* ---- diagnostics ---------------------------------------------------------- */
/* The device's own conservative-filter code on n (ray, record) pairs, host
 * arrays: origin3/dir3 (n,3), rec5 (n,5) = centre xyz, negB, negA (filter_record /
 * node_record).  mode 0 filter_test, 1 filter_test2 (packed, record i with
 * record i^1), 2 filter_test2h (packed + half-line cull), 3 filter_testh (the
 * piece-root cull).  out_d[n]: the test value (pass = d <= 0).  Used by
 * tests/test_gpu_filter.py to check the superset property on the GPU's code. */
int lpc_filter_eval(lpc_handle *h, int64_t n, const float *origin3, const float *dir3, const float *rec5,
                    int mode, float *out_d);

/* ---- profiling ------------------------------------------------------------ */
typedef struct {
    double intersect_ms;     /* sum of k_intersect durations (HIP events)       */
    double shade_ms;         /* postproc+Fresnel+compaction kernels             */
    int64_t intersect_launches;
    int64_t pairs;           /* ray-triangle pairs of the brute-force algorithm */
    int64_t node_visits;     /* hierarchy nodes visited (per wave)              */
    int64_t group_tests;     /* 4-triangle filter groups tested (per wave)      */
    int64_t wave_traversals; /* (wave, piece) traversals                        */
    int64_t exact_tests;     /* exact Moller-Trumbore tests (per ray)           */
    int64_t wave_hist[24];   /* k_intersect wave durations: bin b counts waves that
                                ran [2^b, 2^(b+1)) wall-clock ticks (100 MHz)       */
    int64_t heavy_piece;     /* piece with the largest summed wave time (last launch) */
    int64_t heavy_piece_ticks;
    int64_t piece_ticks;     /* summed wave ticks over all pieces (last launch)  */
    int64_t tail_waves;      /* walk waves that ran >= 2^16 ticks (655 us)   */
    int64_t tail_nodes;      /* their node visits                               */
    int64_t tail_spread_urad;/* their summed direction spread (micro-radians)   */
    int64_t tail_exact;      /* their exact tests                               */
    double kernel_ms;        /* k_rootwalk launches alone (their own start/stop
                                timestamps; intersect_ms adds k_spill, k_packet, k_slivers) */
    double xchg_us;          /* host time spent in the all-reduce hook (lpc_set_allreduce) */
    int64_t xchg_calls;      /* its calls (per-iteration stats + trace-end aggregates)  */
    int64_t walk_cycles;     /* level 2: summed shader-clock cycles of the walk items (per wave) */
    int64_t drain_cycles;    /* ... of them inside the exact-test drains                         */
    int64_t fan_exact;       /* level 2: exact tests on fan triangles (a vertex shared by >= 32) */
    int64_t behind_exact;    /* ... on triangles wholly behind the ray origin                    */
    int64_t hit_exact;       /* ... accepted (t > eps)                                            */
} lpc_prof;
/* Enable per-launch HIP-event timing of the hot kernels (1), timing plus
 * traversal counters (2, diagnostic: adds atomics), only the walk kernel's
 * launches (4: kernel_ms, launches and pairs; the lightest, for timed runs;
 * 4 + 256 k: only every k-th walk launch, intersect_launches and pairs counting
 * those), or disable (0). */
int lpc_prof_enable(lpc_handle *h, int on);
int lpc_prof_read(lpc_handle *h, lpc_prof *out, int reset);

#ifdef __cplusplus
}
#endif
#endif /* LPC_H */
