#!/usr/bin/env python3
"""Benchmark: ray-bounces/s of the LightPyCL per-bounce path on the synthetic
1M-ray x 103,660-triangle scene (BASELINE.json metric), one process per GPU.

A "step" is one complete trace of the rank's 1M rays through the synthetic
scene (every iteration until the reference's termination rule), with the rays
resident in HBM when the timed region starts (lpc_trace_reset restores them
device-to-device).  value = ray-bounces of all ranks / max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rays R] [--no-cpu] [--no-configs]

Multi-GPU: run under torch.distributed.run (the driver's form), or directly with
--gpus N > 1, when the parent starts torch.distributed.run with N ranks as a child
process (before touching the GPU) and exits with its status; the rank count must
equal --gpus.  Rays shard by rank (independent
seeds, weak scaling), the scene is replicated.  Each iteration's termination
decision (iterative_tracer.py:383-391) is taken inside the library's trace loop
on the stats all-reduced over the ranks of the node through the library's
shared-memory hook (lpc_set_allreduce + lpc_shm_allreduce); the trace-end
histogram and the timing go over RCCL (torch.distributed "nccl").

The line also carries:
  strong        strong scaling: ONE fixed global set of --rays rays (seed 7, the
                N=1 headline's rays) split over the ranks with shard_bounds, traced
                to the global termination; per-rank ms, global counts;
  config5       BASELINE.json config 5: 100 M rays over the ranks (8 fixed blocks
                of 12.5 M rays, seeds 7..14, rank r of N takes blocks [8r/N, 8(r+1)/N));
  cold          N=1: a fresh CL_Tracer's first call (scene upload, new rays, no
                speculation prediction), and new rays on a warm engine;
  fresh_rays    N=1: a new 1 M-ray batch every step, the next batch's upload
                overlapped with the current trace (PCIe-inclusive);
  parity        the timed workload checked against the oracle: the first bounce
                of the rank's first --cpu-rays rays (the same oracle outputs the
                cpu_baseline leg times; decisions and destinations bit for bit,
                children within the oracle's stated tolerance), the trace's
                first-iteration counts against them, and every timed step's
                per-iteration counts and measured power identical;
  roofline      HBM roofline of k_rootwalk (algorithmic bytes / its own average
                launch time from HIP events; traffic from the committed rocprofv3
                --pmc summary);
  configs       BASELINE.json configs 2-4 at full size (N=1 only).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 vector peak
# VALU issue peak: MI355X_MICROARCH.md:54,473 -- a CU has 4 SIMD-32 units and a
# wave64 v_fma_f32 issues in 2 cycles when several waves share a SIMD (4 for one
# wave alone): 256 CUs x 4 SIMDs x 2.4 GHz / 2 = 1.229 T wave-instructions/s.
# Rounds 2-3 used 4 cycles (half this peak, so twice the fraction).  When the
# committed microbenchmark (tools/valu_issue.hip, profiles/r04_valu_issue.json)
# is present, its best measured chip rate replaces the guide's figure.
VALU_ISSUE_PEAK_GUIDE = 256 * 4 * 2.4e9 / 2
VALU_ISSUE_FILE = os.path.join(ROOT, "profiles", "r04_valu_issue.json")


def valu_issue_peak():
    """(peak wave-instructions/s, packed-FMA peak or None, source): the measured
    v_fma_f32 rate of the committed microbenchmark (best over 1-8 waves per SIMD)
    and its v_pk_fma_f32 rate (a packed FMA takes two issue slots), else the
    guide's figure."""
    try:
        with open(VALU_ISSUE_FILE) as f:
            rows = json.load(f)["rows"]
        best = max(r["wave_instr_per_s"] for r in rows if r["op"] == "v_fma_f32")
        pk = max(r["wave_instr_per_s"] for r in rows if r["op"] == "v_pk_fma_f32")
        return best, pk, ("measured: profiles/r04_valu_issue.json (tools/valu_issue.hip: v_fma_f32 best over "
                          "waves/SIMD; v_pk_fma_f32 issues at half that rate)")
    except (OSError, KeyError, ValueError):
        return VALU_ISSUE_PEAK_GUIDE, None, "MI355X_MICROARCH.md:54,473 (2 cycles per wave64 VALU instruction per SIMD)"
PROF_EVERY = int(os.environ.get("LPC_BENCH_PROF_EVERY", 1))   # timed walk launches with HIP events (all)
RAY_BYTES = 156                # algorithmic HBM bytes per ray-bounce
TRI_BYTES = 40                 # per triangle per bounce-iteration
MT_FLOPS = 46                  # Moller-Trumbore flops per ray-triangle test
WALK_KERNEL = "k_rootwalk"     # the hierarchy-walk kernel the HIP events time
# BASELINE.json configs 2-4: scene, rays, depth (full size, one GPU)
CONFIGS = [("parabolic", 1_000_000, 4), ("lens", 10_000_000, 8), ("eye", 10_000_000, 16),
           # beside the headline: the synthetic generator with ~79 % of the
           # rays entering a refractive sphere, so the secondaries are most of the work
           ("synthetic_dense", 1_000_000, 16)]
# the drop-in's default results mode end to end, as the reference's examples time
# it (example_directivity_parabolic_mirror.py:88-102: time() around
# CL_Tracer.iterative_tracer with per-iteration results tuples on the host)
RESULTS_CONFIG = ("parabolic", 1_000_000, 4)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=1_000_000, help="rays per GPU")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline / parity leg")
    ap.add_argument("--cpu-rays", type=int, default=1 << 20, help="CPU baseline sample (rays, one bounce)")
    ap.add_argument("--no-configs", action="store_true", help="skip BASELINE configs 2-4")
    ap.add_argument("--no-prof", action="store_true", help="no HIP events in the timed region (A/B of their cost)")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling and config-5 blocks")
    ap.add_argument("--strong-steps", type=int, default=100, help="timed steps of the strong-scaling block")
    ap.add_argument("--c5-steps", type=int, default=5, help="timed traces of the config-5 block")
    ap.add_argument("--c5-rays", type=int, default=100_000_000, help="config 5: global rays (8 blocks)")
    ap.add_argument("--inflight", type=int, default=int(os.environ.get("LPC_BENCH_INFLIGHT", 3)),
                    help="traces in flight per GPU: engines (handles, each its own stream) tracing the "
                         "workload's rays from their own host threads (1: one engine, traces back to back)")
    return ap.parse_args()


def src_sha16():
    h = hashlib.sha256()
    with open(os.path.join(ROOT, "lightpycl_amd", "csrc", "lpc_kernels.hip"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def load_pmc():
    """Per-launch PMC figures of the walk kernel from the committed rocprofv3 --pmc
    summary (profiles/pmc_intersect.json, tools/pmc_summary.py); marked stale when
    it was collected on another version of the kernels."""
    p = os.path.join(ROOT, "profiles", "pmc_intersect.json")
    try:
        with open(p) as f:
            pmc = json.load(f)
    except Exception:
        return {}
    pmc["stale"] = pmc.get("kernels_sha16") != src_sha16() or pmc.get("kernel") not in (None, WALK_KERNEL)
    if pmc["stale"]:
        print(f"bench: {p} was collected on other kernel sources or another kernel; PMC figures not used",
              file=sys.stderr)
    return pmc


def rays_of(sc):
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
    return o, d, p


def cpu_leg(sc, eng, o, d, p, nrays, first_stats, timed):
    """Oracle (C/OpenMP restatement of the reference kernels) on the first `nrays`
    rays of the workload, one bounce: timed as the CPU baseline (timed=True), and
    its outputs compared with liblpc's bounce of the same rays, and
    (when the sample is the whole population) with the timed trace's first
    iteration counts."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    n = min(nrays, len(p))
    o, d, p = o[:n], d[:n], p[:n]
    S = oracle.Scene(sc.meshes)
    z = np.zeros(n, np.int32)
    pm = np.full(n, -2, np.int32)
    model, affinity = cpu_info()
    # the CPU baseline is the FASTEST measured configuration of the oracle: its
    # OpenMP team at every core of the affinity mask (all host cores)
    # and at the container's cgroup CPU quota (on the GPU box 16 of 256: more
    # threads than the quota time-share it), each timed on a quarter of the sample;
    # the faster count then times the whole sample (the figure reported)
    probes = {}
    threads = oracle.set_threads(0)
    if timed:
        q = cgroup_cpu_max()
        cands = [affinity]
        if q and q.get("cpus") and int(q["cpus"]) < affinity:
            cands.append(max(int(q["cpus"]), 1))
        nq = min(n, 1 << 18)
        for c in cands:
            oracle.set_threads(c)
            tq = time.perf_counter()
            oracle.bounce(S, o[:nq], d[:nq], p[:nq], z[:nq], pm[:nq], sc.max_ray_len, sc.ior_env)
            tq = time.perf_counter() - tq
            probes[c] = {"value": nq / tq, "rays": nq, "seconds": tq}
        threads = oracle.set_threads(max(probes, key=lambda c: probes[c]["value"]))
    t = time.perf_counter()
    ref = oracle.bounce(S, o, d, p, z, pm, sc.max_ray_len, sc.ior_env)
    dt = time.perf_counter() - t
    g = eng.bounce(o, d, p, z, pm, sc.max_ray_len, sc.ior_env)
    # decisions, indices and destinations bit for bit; children directions and
    # powers within 4e-6 (the oracle computes gfx950's rsqrt / the device exp
    # correctly rounded / with libm: DESIGN.md section 2; liblpc is bit-exact with
    # the reference's own kernels, tests/test_ref_parity.py)
    disc = np.zeros(n, bool)
    for k in ("isect_mid", "isect_idx", "meas", "r_meas", "t_meas", "n1", "n2"):
        disc |= np.asarray(g[k]).reshape(-1) != np.asarray(ref[k]).reshape(-1)
    dest = np.any(g["dest"][:, :3] != ref["dest"][:, :3], axis=1)
    same = np.ones(n, bool)
    tol = np.zeros(n, bool)
    par = np.abs(np.asarray(ref["pow"], np.float64))
    for k in ("r_dir", "t_dir"):
        dd = np.abs(g[k][:, :3].astype(np.float64) - ref[k][:, :3])
        tol |= np.any(dd > 1e-5, axis=1)
        same &= np.all(dd == 0, axis=1)
    for k in ("pow", "r_pow", "t_pow"):
        dp = np.abs(np.asarray(g[k], np.float64) - ref[k])
        tol |= dp > 1e-5 * np.maximum(par, np.abs(np.asarray(ref[k], np.float64)))
        same &= dp == 0
    parity = {"rays": int(n), "mismatches": int((disc | dest).sum()),
              "beyond_tolerance": int((tol & ~(disc | dest)).sum()),
              "bitwise_identical_frac": float(np.mean(same & ~disc & ~dest)),
              "fields": "mismatches: hit mesh/triangle, n1, n2, meas flags or destination not bit-identical; "
                        "beyond_tolerance: children directions / powers beyond SURVEY 8c's 1e-5 (<= 0.1 % of rays "
                        "allowed: near total internal reflection the hardware rsqrt's last bit is amplified)",
              "checked_against": "oracle/lpc_oracle.c (C restatement of kernel_reflect_refract_intersect.cl; "
                                 "rsqrt/sqrt/exp correctly rounded / libm); liblpc vs the reference's own gfx950 "
                                 "kernels: bit-exact, tests/test_ref_parity.py"}
    # the reference's own kernels (the unmodified .cl compiled for gfx950 by ROCm's
    # OpenCL front end, IEEE division/sqrt, no contraction: oracle/_ref, DESIGN.md
    # section 3) on the same rays, every output field bit for bit
    co = os.path.join(ROOT, "oracle", "_ref", "lpc_ref_ieee.co")
    if os.path.exists(co):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import ref_gpu
        rk = ref_gpu.RefKernels("ieee")
        try:
            rr = rk.bounce(S, o, d, p, z, pm, sc.max_ray_len, sc.ior_env)
        finally:
            rk.close()
        bad = np.zeros(n, bool)
        per = {}
        names = ("dest", "pow", "meas", "isect_mid", "isect_idx", "n1", "n2", "entering", "r_dir", "r_pow",
                 "r_meas", "t_dir", "t_pow", "t_meas")
        for k in names:
            a = np.asarray(g[k]).reshape(n, -1)[:, :3]
            b = np.asarray(rr[k]).reshape(n, -1)[:, :3]
            diff = np.any((a != b) & ~(np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else a != b, axis=1)
            per[k] = int(diff.sum())
            bad |= diff
        parity["vs_reference_kernels"] = {
            "rays": int(n), "mismatched_rays": int(bad.sum()),
            "per_field": {k: v for k, v in per.items() if v},
            "fields": ", ".join(names) + " (values equal; NaN = NaN)",
            "build": "oracle/_ref/lpc_ref_ieee.co: /root/reference/kernel_reflect_refract_intersect.cl unmodified, "
                     "ROCm OpenCL C for gfx950, IEEE div/sqrt, -ffp-contract=off"}
    if n == len(first_stats["population"]):
        kr = int(np.sum(ref["r_meas"] == 0))
        kt = int(np.sum(ref["t_meas"] == 0))
        km = int(np.sum(ref["meas"] == 1))
        pw = float(np.sum(np.concatenate([ref["r_pow"][ref["r_meas"] == 0], ref["t_pow"][ref["t_meas"] == 0]]),
                          dtype=np.float64))
        st = first_stats["stats"]
        parity["trace_first_iteration"] = {
            "n_reflect": [int(st.n_reflect), kr], "n_refract": [int(st.n_refract), kt],
            "n_measured": [int(st.n_measured), km], "power_next": [float(st.power_next), pw],
            "match": bool(st.n_reflect == kr and st.n_refract == kt and st.n_measured == km
                          and abs(st.power_next - pw) <= 1e-6 * max(abs(pw), 1e-300))}
    base = None
    if timed:
        base = dict(value=n / dt, unit="ray-bounces/s", cores=threads, threads=threads, kind="port",
                    cpu_model=model, cores_in_affinity_mask=affinity, cgroup_cpu_max=cgroup_cpu_max(),
                    sample=f"first {n} rays of the workload, 1 bounce (intersect+postproc+Fresnel) over "
                           f"{S.tri_count} triangles, {dt:.2f} s, {threads} OpenMP threads",
                    ri_per_s=n * S.tri_count / dt,
                    thread_probes={str(c): v for c, v in probes.items()},
                    note=(f"value: the fastest of the probed OpenMP team sizes ({', '.join(map(str, probes))}: "
                          f"every core of the affinity mask and the cgroup's CPU quota), timed on the whole "
                          f"sample; thread_probes: each size on a quarter of it"))
    return parity, base


def run_configs(Engine, ShardedTrace, scenes):
    """BASELINE.json configs 2-4 at full size on this GPU: whole traces with the
    rays resident, the hierarchy walk's share of the step from HIP events."""
    out = {}
    for name, n, depth in CONFIGS:
        sc = scenes.BUILDERS[name](n=n, seed=7, iterations=depth)
        o, d, p = rays_of(sc)
        e = Engine(0)
        e.upload_meshes(sc.meshes)
        e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
        in_pow = float(np.sum(p, dtype=np.float64))
        run = ShardedTrace(e)
        steps = 1 if name == "eye" else 5
        for _ in range(1 if name == "eye" else 2):               # warm-up: allocations, then a trace with
            e.reset()                                            # the first's prediction (speculation)
            run.run(depth, sc.tau, in_pow, wait=False)
        e.sync()
        t = time.perf_counter()
        res = []
        for _ in range(steps):
            e.reset()
            res.append(run.run(depth, sc.tau, in_pow, wait=False))
        e.sync()
        dt = (time.perf_counter() - t) / steps
        # the walk kernel's share: one more trace with HIP events on its launches
        # (outside the timed traces: the events cost ~7 us per launch)
        e.prof_enable(True, light=True)
        e.prof_read(reset=True)
        t1 = time.perf_counter()
        e.reset()
        run.run(depth, sc.tau, in_pow, wait=False)
        e.sync()
        dt1 = time.perf_counter() - t1
        pr = e.prof_read(reset=True)
        e.prof_enable(False)
        r = res[-1]
        b = int(r["bounces"])
        out[name] = {"rays": n, "depth": depth, "triangles": int(e.tri_count), "iterations": int(r["iterations"]),
                     "ray_bounces": b, "ms_per_trace": dt * 1e3, "ray_bounces_per_s": b / dt,
                     "walk_kernel_share": pr["kernel_ms"] / (dt1 * 1e3) if dt1 > 0 else None,
                     "steps_identical": all(x["global_counts"] == r["global_counts"] for x in res),
                     "measured_power": float(np.sum(r["mesh_power"])), "input_power": in_pow}
        e.close()
    out["results_mode"] = run_results_mode()
    return out


def run_results_mode():
    """RESULTS_CONFIG through the drop-in exactly as a reference user calls it:
    CL_Tracer.iterative_tracer(keep_results=True) end to end (mesh flattening and
    upload, per-iteration results tuples exported to host numpy arrays, the
    reference's stop test), ray-bounces = sum of the results tuples' lengths."""
    from lightpycl_amd import scenes
    from lightpycl_amd.iterative_tracer import CL_Tracer
    name, n, depth = RESULTS_CONFIG
    sc = scenes.BUILDERS[name](n=n, seed=7, iterations=depth)
    import gc
    tr = CL_Tracer(device=0)
    kw = dict(trace_iterations=depth, trace_until_dissipated=sc.tau, max_ray_len=sc.max_ray_len, ior_env=sc.ior_env)
    gc.collect()            # the earlier legs' garbage, not this workload's (a collection inside a timed call)
    t_first = time.perf_counter()
    tr.iterative_tracer(sc.sources, sc.meshes, **kw)                 # warm-up (allocations, pinned blocks)
    t_first = time.perf_counter() - t_first
    times = []
    for _ in range(5):
        t = time.perf_counter()
        res = tr.iterative_tracer(sc.sources, sc.meshes, **kw)
        times.append(time.perf_counter() - t)
    b = sum(len(r[3]) for r in res)
    dt = sorted(times)[len(times) // 2]
    out = {"scene": name, "rays": n, "depth": depth, "iterations": len(res), "ray_bounces": b,
           "ms_per_trace_median": dt * 1e3, "ms_per_trace_all": [x * 1e3 for x in times],
           "first_call_ms": t_first * 1e3, "first_timed_over_median": times[0] / dt,
           "ray_bounces_per_s": b / dt, "exact_power_sums": int(getattr(tr, "exact_sums", 0)),
           "host_bytes_per_trace": int(sum(sum(a.nbytes for a in r) for r in res)),
           "note": "CL_Tracer(...).iterative_tracer(keep_results=True) end to end: the results tuples "
                   "(iterative_tracer.py:355) land in host numpy arrays; PCIe-inclusive, not the headline value"}
    tr.engine.close()
    return out


def cpu_info():
    """CPU model (/proc/cpuinfo) and the cores this process may run on (its
    affinity mask, not the machine's count: BASELINE.md asks for both)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    return model, affinity


def timed_block(eng, runner, comm, o, d, p, sc, steps, warmup, sync, dist, dev):
    """Trace fixed rays `steps` times (after `warmup` untimed traces) through the
    rank's engine and runner (global termination over the ranks), bracketed by
    barrier + sync.  Returns the rank-0 view: max-over-ranks time, all ranks'
    ray-bounces, per-rank ms, the global per-iteration counts, identical steps."""
    eng.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
    in_pow = float(np.sum(p, dtype=np.float64))
    in_all = float(comm.allreduce_sum([in_pow])[0]) if comm else in_pow

    def step():
        return runner.run(sc.iterations, sc.tau, in_pow, wait=False, input_power_global=in_all, reset=True)
    for _ in range(warmup):
        step()
    sync()
    t0 = time.perf_counter()
    res = [step() for _ in range(steps)]
    sync()
    dt = time.perf_counter() - t0
    bounces = float(sum(r["bounces"] for r in res))
    same = all(r["global_counts"] == res[0]["global_counts"] for r in res)
    rank_ms = [dt / steps * 1e3]
    rank_b = [bounces]
    if dist:
        import torch
        t = torch.tensor([dt, bounces, 0.0 if same else 1.0], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        per = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(dist.get_world_size())]
        dist.all_gather(per, torch.tensor([dt / steps * 1e3, bounces], dtype=torch.float64, device=dev))
        rank_ms = [float(x[0].item()) for x in per]
        rank_b = [float(x[1].item()) for x in per]
        dt, bounces, same = float(mx[0]), float(t[1]), float(mx[2]) == 0.0
    g = res[-1]["global_counts"]
    return {"ms_per_step": dt / steps * 1e3, "ray_bounces_per_s": bounces / dt, "steps": steps,
            "rank_ms_per_step": {"min": min(rank_ms), "max": max(rank_ms), "per_rank": rank_ms},
            "rank_ray_bounces_per_step": [b / steps for b in rank_b],
            "global_counts": [int(x) for x in g], "global_ray_bounces": int(sum(g)),
            "steps_identical": bool(same), "mesh_power": [float(x) for x in res[-1]["mesh_power"]]}


C5_BLOCKS = 8


def config5_rays(scenes, rank, world, total):
    """BASELINE config 5's fixed global ray set: 8 blocks of total/8 synthetic
    rays (seeds 7..14); rank r of `world` takes the contiguous blocks
    shard_bounds(8, r, world) (world <= 8; above, the block list is split by rays)."""
    from lightpycl_amd.distributed import shard_bounds
    per = total // C5_BLOCKS

    def block(b):
        ls = scenes.synthetic_rays(n=per, seed=7 + b)
        return (np.asarray(ls.rays_origin, np.float32), np.asarray(ls.rays_dir, np.float32),
                np.asarray(ls.rays_power, np.float32).reshape(-1))
    if world <= C5_BLOCKS:
        lo, hi = shard_bounds(C5_BLOCKS, rank, world)
        parts = [block(b) for b in range(lo, hi)]
        return tuple(np.concatenate([q[k] for q in parts]) for k in range(3))
    b = rank * C5_BLOCKS // world
    lo, hi = shard_bounds(per, rank - b * world // C5_BLOCKS, world // C5_BLOCKS)
    o, d, p = block(b)
    return o[lo:hi], d[lo:hi], p[lo:hi]


def cold_block(scenes, Engine, ShardedTrace, n):
    """The reference examples' measurement (example_directivity_parabolic_mirror.py:
    88-102: time() around one iterative_tracer call) on the headline scene: a
    fresh CL_Tracer's first call (mesh flatten, scene upload and record build,
    new rays, no speculation prediction), aggregate and results mode; then new
    rays on the warm engine (set_rays + one trace, a prediction from other rays)."""
    from lightpycl_amd.iterative_tracer import CL_Tracer
    out = {}
    sc = scenes.synthetic(n=64, seed=7)                  # the scene objects (meshes, trace parameters)
    for mode, keep, seed in (("aggregate", False, 1007), ("results", True, 1009)):
        src = [scenes.synthetic_rays(n=n, seed=seed)]
        t = time.perf_counter()
        tr = CL_Tracer(device=0)
        t_open = time.perf_counter() - t
        res = tr.iterative_tracer(src, sc.meshes, trace_iterations=sc.iterations, trace_until_dissipated=sc.tau,
                                  max_ray_len=sc.max_ray_len, ior_env=sc.ior_env, keep_results=keep)
        dt = time.perf_counter() - t
        b = tr.ray_bounces()
        out[f"fresh_tracer_{mode}"] = {"ms": dt * 1e3, "open_ms": t_open * 1e3, "ray_bounces": b,
                                       "ray_bounces_per_s": b / dt,
                                       "phases_ms": {k: (v * 1e3 if not isinstance(v, list) else sum(v) * 1e3)
                                                     for k, v in getattr(tr, "phase_s", {}).items()}}
        del res
        tr.engine.close()

    def arrays(ls):
        return (np.asarray(ls.rays_origin, np.float32), np.asarray(ls.rays_dir, np.float32),
                np.asarray(ls.rays_power, np.float32).reshape(-1))
    e = Engine(0)
    e.upload_meshes(sc.meshes)
    run = ShardedTrace(e)
    o, d, p = arrays(scenes.synthetic_rays(n=n, seed=7))
    e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
    for _ in range(3):                                  # warm: allocations, the prediction of these rays
        e.reset()
        run.run(sc.iterations, sc.tau, float(np.sum(p, dtype=np.float64)))
    e.sync()
    times = []
    for seed in (2001, 2002, 2003):
        o, d, p = arrays(scenes.synthetic_rays(n=n, seed=seed))
        t = time.perf_counter()
        e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
        r = run.run(sc.iterations, sc.tau, float(np.sum(p, dtype=np.float64)))
        times.append((time.perf_counter() - t, r["bounces"]))
    out["new_rays_warm_engine"] = {"ms": [x[0] * 1e3 for x in times],
                                   "ray_bounces_per_s": [x[1] / x[0] for x in times],
                                   "note": "set_rays (host->device rays, analysis) + one synchronous trace"}
    e.close()
    return out


def fresh_rays_block(scenes, Engine, n, steps=24, nbatch=8):
    """New rays every step, as a caller tracing batch after batch of sources does
    (the reference uploads each partition's rays inside its loop,
    iterative_tracer.py:280-284): `steps` traces of 1 M-ray batches (nbatch
    distinct seeded batches in turn, host numpy arrays), each staged -- copied to
    the device by the library's helper thread on a copy stream -- while the batch
    before it is traced (lpc_trace_stage_rays / lpc_trace_run_staged_async).  The
    timed region includes every host-to-device copy (PCIe-inclusive); beside it
    the same batches through set_rays + a synchronous trace each."""
    sc = scenes.synthetic(n=64, seed=7)
    batches = []
    for b in range(nbatch):
        ls = scenes.synthetic_rays(n=n, seed=3001 + b)
        batches.append((np.asarray(ls.rays_origin, np.float32), np.asarray(ls.rays_dir, np.float32),
                        np.asarray(ls.rays_power, np.float32).reshape(-1)))
    thr = [(1.0 - sc.tau) * float(np.sum(b[2], dtype=np.float64)) for b in batches]
    e = Engine(0)
    e.upload_meshes(sc.meshes)

    def pipelined(k0, K):
        bounces = 0
        e.stage_rays(*batches[k0 % nbatch], sc.max_ray_len, sc.ior_env)
        for k in range(K):
            if k + 1 < K:
                e.stage_rays(*batches[(k0 + k + 1) % nbatch], sc.max_ray_len, sc.ior_env)
            st, _ = e.run_staged(sc.iterations, thr[(k0 + k) % nbatch])
            bounces += sum(int(x.n_in) for x in st)
        e.sync()
        return bounces
    pipelined(0, 4)                                     # warm: allocations, pinned staging, predictions
    t = time.perf_counter()
    b = pipelined(4, steps)
    dt = time.perf_counter() - t
    seq = []
    for k in range(4):                                  # the same batches one at a time
        t1 = time.perf_counter()
        e.set_rays(*batches[k], sc.max_ray_len, sc.ior_env)
        st, _ = e.run_local(sc.iterations, thr[k])
        seq.append((time.perf_counter() - t1, sum(int(x.n_in) for x in st)))
    e.close()
    return {"ray_bounces_per_s": b / dt, "ms_per_step": dt / steps * 1e3, "steps": steps, "batches": nbatch,
            "rays_per_batch": n, "ray_bounces": b,
            "sequential_set_rays_ms": [x[0] * 1e3 for x in seq],
            "sequential_ray_bounces_per_s": sum(x[1] for x in seq) / sum(x[0] for x in seq),
            "note": "each step traces a different 1 M-ray batch from host numpy arrays; the next batch's "
                    "host-to-device copy runs on a copy stream during the current trace (PCIe-inclusive, "
                    "not the headline value)"}


def cgroup_cpu_max():
    """The container's CPU bandwidth limit (cgroup v2 cpu.max: "quota period" or
    "max period"), so a thread count above the quota reads as what it is."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        return {"raw": f"{q} {per}", "cpus": None if q == "max" else int(q) / int(per)}
    except (OSError, ValueError):
        return None


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a):
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start N ranks with
    torch.distributed.run as a child process and exit with its status.  Nothing
    here touches the GPU (device_count does not initialise it on this image), and
    the parent is never replaced (no exec)."""
    import subprocess
    rehearse = os.environ.get("LPC_BENCH_REHEARSE") == "1"
    if not rehearse:
        import torch
        have = torch.cuda.device_count()
        if have < a.gpus:
            print(f"bench: --gpus {a.gpus} but only {have} HIP devices are visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    dist = None
    # rehearsal of the multi-rank path on a one-GPU box (not a measurement):
    # LPC_BENCH_REHEARSE=1 puts every rank on GPU 0 and exchanges over gloo
    rehearse = os.environ.get("LPC_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("gloo" if rehearse else "nccl")
        dist = tdist

    from lightpycl_amd.build import build
    if rank == 0 or world == 1:
        build(verbose=False)
    if dist:
        dist.barrier()
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import Engine
    from lightpycl_amd.distributed import ShardedTrace, ShmComm, TorchComm

    sc = scenes.synthetic(n=a.rays, seed=7 + rank)
    E = max(1, int(a.inflight))
    o, d, p = rays_of(sc)
    comm = TorchComm(dist, local) if dist else None
    # E engines (traces in flight), each with the scene and the workload's rays,
    # its own stream and, over several ranks, its own per-iteration exchange: the
    # library's shared-memory hook on one node (one segment per engine),
    # torch.distributed through the hook when the ranks span nodes
    # (in flight: the walk grid TracePool uses for engines side by side)
    from lightpycl_amd.pool import INFLIGHT_WALK_GRID
    engines, shms, runners = [], [], []
    for _ in range(E):
        e = Engine(local)
        e.upload_meshes(sc.meshes)
        e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
        if E > 1:
            e.set_walk_grid(INFLIGHT_WALK_GRID)
        s_ = ShmComm.from_dist(dist, fallback=comm) if dist else None
        engines.append(e)
        shms.append(s_)
        runners.append(ShardedTrace(e, comm, iter_comm=s_))
    eng, shm, runner = engines[0], shms[0], runners[0]
    in_pow = float(np.sum(p, dtype=np.float64))
    in_pow_all = float(comm.allreduce_sum([in_pow])[0]) if comm else in_pow

    def step(j=0):
        # the trace returns once its outputs are final, so the engine's next step's
        # launches queue behind its last row moves (sync() waits for all)
        return runners[j].run(sc.iterations, sc.tau, in_pow, wait=False, input_power_global=in_pow_all,
                              reset=True)

    def sync():
        for e in engines:
            e.sync()
        if dist:
            import torch
            torch.cuda.synchronize(local)
            dist.barrier()

    def steps_inflight(n):
        """n steps over the E engines, each engine's share in order on a host
        thread of its own (ctypes releases the GIL inside the library calls), so
        up to E traces run on the GPU at once.  Returns every step's result."""
        share = [n // E + (1 if j < n % E else 0) for j in range(E)]
        out = [[] for _ in range(E)]
        errs = []

        def worker(j):
            try:
                for _ in range(share[j]):
                    out[j].append(step(j))
            except BaseException as ex:          # re-raised on the main thread
                errs.append(ex)
        if E == 1:
            worker(0)
        else:
            th = [threading.Thread(target=worker, args=(j,)) for j in range(E)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        if errs:
            raise errs[0]
        return [r for rs in out for r in rs]

    # the first iteration alone, for the parity leg (same stats the timed trace starts with)
    eng.reset()
    st0, _ = eng.iterate()
    first = {"stats": st0, "population": p}
    eng.sync()
    for j in range(E):
        for _ in range(a.warmup):
            step(j)
    if not a.no_prof:
        # HIP events around the walk kernel's launches only (created without the
        # system-scope fence, which cost ~7 us per launch; PROF_EVERY > 1 samples
        # every k-th launch), on every engine
        for e in engines:
            e.prof_enable(True, light=True, every=PROF_EVERY)
        # untimed: the same number of steps once with events, so the timed region
        # takes its events from the pools instead of creating them
        steps_inflight(a.steps)
    for e in engines:
        e.prof_read(reset=True)
    sync()
    t0 = time.perf_counter()
    res = steps_inflight(a.steps)
    sync()
    dt = time.perf_counter() - t0
    bounces = sum(r["bounces"] for r in res)
    iters = sum(r["iterations"] for r in res)
    results = [(r["global_counts"], [float(x) for x in r["mesh_power"]]) for r in res]
    profs = [e.prof_read(reset=True) for e in engines]
    prof = {k: sum(pr[k] for pr in profs) for k in ("kernel_ms", "intersect_launches", "xchg_us", "xchg_calls")}
    for e in engines:
        e.prof_enable(False)
    steps_identical = all(x == results[0] for x in results)
    # the same steps on one engine, back to back (the per-trace time without
    # overlap; beside the headline, not a separate workload)
    seq = None
    if E > 1:
        eng.set_walk_grid(0)                    # one trace alone: the library default
        for _ in range(3):
            step(0)
        sync()
        t1 = time.perf_counter()
        rs = [step(0) for _ in range(a.steps)]
        sync()
        dts = time.perf_counter() - t1
        if dist:
            import torch
            dv = "cpu" if rehearse else f"cuda:{local}"
            tt = torch.tensor([dts], dtype=torch.float64, device=dv)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dts = float(tt[0])
        bs = float(sum(r["bounces"] for r in rs))
        if dist:
            import torch
            tb = torch.tensor([bs], dtype=torch.float64, device=("cpu" if rehearse else f"cuda:{local}"))
            dist.all_reduce(tb, op=dist.ReduceOp.SUM)
            bs = float(tb[0])
        seq = {"ray_bounces_per_s": bs / dts, "ms_per_step": dts / a.steps * 1e3, "steps": a.steps,
               "identical_to_inflight": all((r["global_counts"], [float(x) for x in r["mesh_power"]]) == results[0]
                                            for r in rs)}
    # trace-end histogram over RCCL (the north star's all-reduce), outside the timed region
    eng.reset()
    hr = runner.run(sc.iterations, sc.tau, in_pow, hist=(sc.hist_limits, sc.hist_points),
                    input_power_global=in_pow_all)
    hist_total = float(np.sum(hr["hist"][0]) * ((sc.hist_limits[0][1] - sc.hist_limits[0][0]) / sc.hist_points) ** 2)
    dev = ("cpu" if rehearse else f"cuda:{local}") if dist else None
    blocks = {}
    if not a.no_strong:
        from lightpycl_amd.distributed import shard_bounds
        # strong scaling: the N=1 headline's global rays (seed 7), one shard per rank
        # (sc: the same scene and trace parameters as the weak block)
        g = scenes.synthetic_rays(n=a.rays, seed=7)
        go = np.asarray(g.rays_origin, np.float32)
        gd = np.asarray(g.rays_dir, np.float32)
        gp = np.asarray(g.rays_power, np.float32).reshape(-1)
        lo, hi = shard_bounds(a.rays, rank, world)
        blocks["strong"] = timed_block(eng, runner, comm, go[lo:hi], gd[lo:hi], gp[lo:hi], sc, a.strong_steps, 3,
                                       sync, dist, dev)
        blocks["strong"]["rays_global"] = a.rays
        del g, go, gd, gp
        # BASELINE config 5: 100 M rays over the ranks (8 fixed blocks)
        co, cd, cp = config5_rays(scenes, rank, world, a.c5_rays)
        blocks["config5"] = timed_block(eng, runner, comm, co, cd, cp, sc, a.c5_steps, 1, sync, dist, dev)
        blocks["config5"]["rays_global"] = a.c5_rays
        blocks["config5"]["rays_per_rank"] = int(len(cp))
        del co, cd, cp
    rank_ms = [dt / a.steps * 1e3]
    rank_b = [float(bounces)]
    if dist:
        import torch
        dev = "cpu" if rehearse else f"cuda:{local}"
        t = torch.tensor([dt, float(bounces), 0.0 if steps_identical else 1.0], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        # every rank's time and ray-bounces per step, so load imbalance between shards shows
        per = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(per, torch.tensor([dt / a.steps * 1e3, float(bounces)], dtype=torch.float64, device=dev))
        rank_ms = [float(x[0].item()) for x in per]
        rank_b = [float(x[1].item()) for x in per]
        dt, bounces_all = float(mx[0]), float(t[1])
        steps_identical = float(mx[2]) == 0.0
    else:
        bounces_all = float(bounces)
    def finish():
        for r_ in runners:
            r_.close()                          # the hook out of the engine before its comm closes
        for s_ in shms:
            if isinstance(s_, ShmComm):
                s_.close()
        if dist:
            dist.destroy_process_group()

    if rank != 0:
        finish()
        return

    M = eng.tri_count
    launches = max(prof["intersect_launches"], 1)       # the sampled walk launches
    avg_ms = prof["kernel_ms"] / launches               # the walk kernel's launches alone
    rays_per_launch = bounces / max(iters, 1)            # rank-0 launches: one walk per iteration
    alg_bytes = rays_per_launch * RAY_BYTES + M * TRI_BYTES
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    pairs_per_s = bounces_all * M / dt                   # reference-equivalent RI/s (sum N_iter * M / T)
    mt_tflops = pairs_per_s * MT_FLOPS / 1e12
    pmc = load_pmc()
    stale = pmc.get("stale", True)
    traffic = None if stale else pmc.get("hbm_bytes_per_launch")
    valu_per_launch = None if stale else pmc.get("sq_insts_valu_mean")
    valu_rate = valu_per_launch / (avg_ms * 1e-3) if valu_per_launch and avg_ms > 0 else None
    valu_peak, valu_peak_pk, valu_peak_src = valu_issue_peak()
    # the same HBM-traffic figure split by bounce: the primary launch (all rays) and the
    # secondary launches (the survivors), each against its own algorithmic bytes
    split = None
    ips = iters / max(a.steps, 1)
    if not stale and ips > 1:
        sec_rays = (bounces / max(a.steps, 1) - a.rays) / (ips - 1)
        split = {}
        for k, n in (("primary", a.rays), ("secondary", sec_rays)):
            hb = (pmc.get(k + "_launch") or {}).get("hbm_bytes")
            ab = n * RAY_BYTES + M * TRI_BYTES
            split[k] = {"rays_per_launch": n, "hbm_bytes": hb, "alg_bytes": ab,
                        "traffic_over_alg": hb / ab if hb else None}
    out = {
        "metric": "ray-bounces/sec @ 1M rays x 100k tris",
        "value": bounces_all / dt,
        "unit": "ray-bounces/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "inflight": {"traces_in_flight_per_gpu": E,
                     "note": "the timed steps run on E engines (liblpc handles, each its own HIP stream, scene "
                             "records and copy of the workload's rays) from E host threads, so up to E traces "
                             "of the same workload share the GPU; every step is a whole trace of the 1 M rays "
                             "(counts and per-mesh power identical in every step); ms_per_step = wall time / "
                             "steps; the engines' walk grid is walk_grid single-wave blocks (the sequential figure: one "
                             "engine, the library default)",
                     "walk_grid": INFLIGHT_WALK_GRID if E > 1 else None, "sequential": seq},
        "rank_ms_per_step": {"min": min(rank_ms), "max": max(rank_ms), "per_rank": rank_ms},
        "rank_ray_bounces_per_step": [b / a.steps for b in rank_b],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded rays, scene from the reference generator API)",
        "config": {"workload": f"synthetic compound scene: measure hemisphere + 9 refractive spheres, "
                               f"{M} triangles, {a.rays} rays per GPU, trace to termination",
                   "rays_per_gpu": a.rays, "triangles": int(M), "meshes": int(eng.mesh_count),
                   "parallelism": f"ray-sharded x{world}, {E} traces in flight per GPU",
                   "iterations_per_step": iters / a.steps},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": WALK_KERNEL, "avg_launch_ms": avg_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "launches_timed": int(prof["intersect_launches"]), "launches_all": int(iters),
                     "traffic_by_bounce": split,
                     "note": f"achieved = algorithmic bytes per launch (156 B x rays + 40 B x triangles) / "
                             f"{WALK_KERNEL}'s own average launch time (HIP events on its stream over the "
                             f"timed region, launches_timed of launches_all; with traces in flight the "
                             f"launches of different engines overlap, so this per-launch figure understates "
                             f"the chip's aggregate rate); traffic = "
                             f"2*FETCH_SIZE+WRITE_SIZE per {WALK_KERNEL} launch from profiles/pmc_intersect.json "
                             f"(null when that summary was collected on other kernel sources)"},
        # the bound that actually limits the walk kernel: executed VALU issue
        "roofline_valu": {"bound": "valu", "kernel": WALK_KERNEL,
                          "achieved": valu_rate, "peak": valu_peak, "peak_source": valu_peak_src,
                          "unit": "wave-instr/s", "frac": valu_rate / valu_peak if valu_rate else None,
                          "frac_if_all_packed": valu_rate / valu_peak_pk if valu_rate and valu_peak_pk else None,
                          "valu_insts_per_launch": valu_per_launch, "pmc_stale": stale,
                          "note": f"executed VALU wave-instructions per {WALK_KERNEL} launch (PMC SQ_INSTS_VALU, "
                                  "profiles/pmc_intersect.json) / its live average launch time / the chip's "
                                  "VALU issue peak (peak_source)"},
        # brute-force equivalent: what the reference's O(N*M) loop would have to sustain
        "ri_equivalent": {"ri_per_s": pairs_per_s, "mt_tflops_equiv": mt_tflops,
                          "fp32_peak_tflops": FP32_PEAK_TFLOPS,
                          "note": "reference-algorithm FLOPs (46 per ray-triangle test, every ray x every "
                                  "triangle) / whole-job time; above the FP32 peak because the hierarchy "
                                  "filter skips almost all tests: not a utilisation figure"},
        "ri_per_s": pairs_per_s,
        "exchange": {"per_iteration_us": prof["xchg_us"] / max(prof["xchg_calls"], 1),
                     "calls": prof["xchg_calls"], "transport": (("lpc_shm_allreduce" if isinstance(shm, ShmComm) else "torch.distributed via hook")
                                   if world > 1 else None),
                     "trace_end": (("gloo" if rehearse else "RCCL") + " all-reduce (histogram)") if world > 1 else None,
                     "rehearsal_one_gpu": rehearse or None},
        "hist_total_power": hist_total,
        "cpu_baseline": None,
    }
    par = {"steps_identical": bool(steps_identical)}
    if not a.no_cpu:
        # N=1: the timed CPU baseline and the bitwise check on the same oracle outputs;
        # N>1: rank 0 checks a 20k-ray sample of its shard (untimed)
        nr = a.cpu_rays if world == 1 else 20000
        pp, base = cpu_leg(sc, eng, o, d, p, nr, first, timed=(world == 1))
        par.update(pp)
        out["cpu_baseline"] = base
    out["parity"] = par
    if blocks:
        out["strong"] = dict(blocks["strong"], scaling="strong",
                             workload=f"one fixed set of {a.rays} rays (seed 7) split with shard_bounds over "
                                      f"{world} rank(s); value = global ray-bounces / max-over-ranks time")
        out["config5"] = dict(blocks["config5"], scaling="strong",
                              workload=f"BASELINE config 5: {a.c5_rays} synthetic rays as {C5_BLOCKS} blocks "
                                       f"(seeds 7..{6 + C5_BLOCKS}) over {world} rank(s)")
    out["weak_global_counts"] = [int(x) for x in hr["global_counts"]]
    if world == 1 and not a.no_configs:
        for r_ in runners:
            r_.close()
        for e in engines:
            e.close()
        out["configs"] = run_configs(Engine, ShardedTrace, scenes)
        out["cold"] = cold_block(scenes, Engine, ShardedTrace, a.rays)
        out["fresh_rays"] = fresh_rays_block(scenes, Engine, a.rays)
    print(json.dumps(out))
    if world > 1:
        finish()


if __name__ == "__main__":
    main()
