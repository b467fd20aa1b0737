#!/usr/bin/env python3
"""Benchmark: ray-bounces/s of the LightPyCL per-bounce path on the synthetic
1M-ray x 103,660-triangle scene (BASELINE.json metric), one process per GPU.

A "step" is one complete trace of the rank's 1M rays through the synthetic
scene (every iteration until the reference's termination rule), with the rays
resident in HBM when the timed region starts (lpc_trace_reset restores them
device-to-device).  value = ray-bounces of all ranks / max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rays R] [--no-cpu]

Multi-GPU: launched by torch.distributed.run; rays shard by rank (independent
seeds, weak scaling), the scene is replicated, and each iteration all-reduces
(power left, live rays) over RCCL so every rank takes the reference's global
termination decision; per-mesh measured power is all-reduced at trace end.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 vector peak
# MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, 2.4 GHz, a wave64 VALU instruction issues over
# 2 cycles -> chip-wide VALU issue peak in wave-instructions per second
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2
RAY_BYTES = 156                # algorithmic HBM bytes per ray-bounce
TRI_BYTES = 40                 # per triangle per bounce-iteration
MT_FLOPS = 46                  # Moller-Trumbore flops per ray-triangle test
# the hierarchy-traversal kernel timed for the roofline, by LPC_QUEUE launch policy
HIER_KERNEL = {"0": "k_intersect", "1": "k_trav", "2": "k_rootwalk"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rays", type=int, default=1_000_000, help="rays per GPU")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-rays", type=int, default=1 << 20, help="CPU baseline sample (rays, one bounce)")
    ap.add_argument("--no-prof", action="store_true", help="no HIP events in the timed region (A/B of their cost)")
    return ap.parse_args()


def load_pmc():
    """Per-launch PMC figures of the hierarchy kernel from the committed rocprofv3 --pmc
    summary (profiles/pmc_intersect.json, written by tools/pmc_summary.py), or {}."""
    p = os.path.join(ROOT, "profiles", "pmc_intersect.json")
    if os.path.exists(p):
        try:
            with open(p) as f:
                return json.load(f)
        except Exception:
            return {}
    return {}


def cpu_baseline(sc, nrays):
    """Oracle (C/OpenMP restatement of the reference kernels) on a bounded sample:
    the first `nrays` rays of the same workload, one bounce."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])[:nrays]
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])[:nrays]
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])[:nrays]
    S = oracle.Scene(sc.meshes)
    n = o.shape[0]
    t = time.perf_counter()
    oracle.bounce(S, o, d, p, np.zeros(n, np.int32), np.full(n, -2, np.int32), sc.max_ray_len, sc.ior_env)
    dt = time.perf_counter() - t
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return dict(value=n / dt, unit="ray-bounces/s", cores=cores, kind="port",
                sample=f"first {n} rays of the workload, 1 bounce (intersect+postproc+Fresnel) over "
                       f"{S.tri_count} triangles, {dt:.2f} s",
                ri_per_s=n * S.tri_count / dt)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")
        dist = tdist

    from lightpycl_amd.build import build
    if rank == 0 or world == 1:
        build(verbose=False)
    if dist:
        dist.barrier()
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import Engine
    from lightpycl_amd.distributed import ShardedTrace, TorchComm

    sc = scenes.synthetic(n=a.rays, seed=7 + rank)
    eng = Engine(local)
    eng.upload_meshes(sc.meshes)
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
    eng.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
    in_pow = float(np.sum(p, dtype=np.float64))
    comm = TorchComm(dist, local) if dist else None
    runner = ShardedTrace(eng, comm)

    def step():
        # one process: the trace returns once its outputs are final, so the next
        # step's launches queue behind its last row moves (sync() waits for all)
        eng.reset()
        return runner.run(sc.iterations, sc.tau, in_pow, wait=False)

    def sync():
        eng.sync()
        if dist:
            import torch
            torch.cuda.synchronize(local)
            dist.barrier()

    for _ in range(a.warmup):
        step()
    if not a.no_prof:
        eng.prof_enable(True, light=True)    # HIP events around the hierarchy kernel launches only
    eng.prof_read(reset=True)
    sync()
    t0 = time.perf_counter()
    bounces = 0
    iters = 0
    for _ in range(a.steps):
        r = step()
        bounces += r["bounces"]
        iters += r["iterations"]
    sync()
    dt = time.perf_counter() - t0
    prof = eng.prof_read(reset=True)
    if dist:
        import torch
        t = torch.tensor([dt, float(bounces)], dtype=torch.float64, device=f"cuda:{local}")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dt, bounces_all = float(mx[0]), float(t[1])
    else:
        bounces_all = float(bounces)
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    M = eng.tri_count
    launches = max(prof["intersect_launches"], 1)
    avg_ms = prof["kernel_ms"] / launches               # the hierarchy kernel's launches alone
    kernel = HIER_KERNEL.get(os.environ.get("LPC_QUEUE", "2"), "k_rootwalk")
    rays_per_launch = bounces / launches                 # rank-0 launches
    alg_bytes = rays_per_launch * RAY_BYTES + M * TRI_BYTES
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    pairs_per_s = bounces_all * M / dt                   # reference-equivalent RI/s (sum N_iter * M / T)
    mt_tflops = pairs_per_s * MT_FLOPS / 1e12
    pmc = load_pmc()
    traffic = pmc.get("hbm_bytes_per_launch")
    valu_per_launch = pmc.get("sq_insts_valu_mean")
    valu_rate = valu_per_launch / (avg_ms * 1e-3) if valu_per_launch and avg_ms > 0 else None
    out = {
        "metric": "ray-bounces/sec @ 1M rays x 100k tris",
        "value": bounces_all / dt,
        "unit": "ray-bounces/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded rays, scene from the reference generator API)",
        "config": {"workload": f"synthetic compound scene: measure hemisphere + 9 refractive spheres, "
                               f"{M} triangles, {a.rays} rays per GPU, trace to termination",
                   "rays_per_gpu": a.rays, "triangles": int(M), "meshes": int(eng.mesh_count),
                   "parallelism": f"ray-sharded x{world}", "iterations_per_step": iters / a.steps},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kernel, "avg_launch_ms": avg_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "note": f"achieved = algorithmic bytes per launch / {kernel}'s own average "
                             "launch time (HIP events on its stream); traffic = 2*FETCH_SIZE+WRITE_SIZE per "
                             f"{kernel} launch (profiles/pmc_intersect.json)"},
        # the bound that actually limits the hierarchy kernel: executed VALU issue
        "roofline_valu": {"bound": "valu", "kernel": kernel,
                          "achieved": valu_rate, "peak": VALU_ISSUE_PEAK, "unit": "wave-instr/s",
                          "frac": valu_rate / VALU_ISSUE_PEAK if valu_rate else None,
                          "valu_insts_per_launch": valu_per_launch,
                          "note": f"executed VALU wave-instructions per {kernel} launch (PMC SQ_INSTS_VALU, "
                                  "profiles/pmc_intersect.json) / its live average launch time / chip issue "
                                  "peak (256 CU x 4 SIMD x 2.4 GHz / 2 cycles)"},
        # brute-force equivalent: what the reference's O(N*M) loop would have to sustain
        "ri_equivalent": {"ri_per_s": pairs_per_s, "mt_tflops_equiv": mt_tflops,
                          "fp32_peak_tflops": FP32_PEAK_TFLOPS,
                          "note": "reference-algorithm FLOPs (46 per ray-triangle test, every ray x every "
                                  "triangle) / whole-job time; above the FP32 peak because the hierarchy "
                                  "filter skips almost all tests: not a utilisation figure"},
        "ri_per_s": pairs_per_s,
        "cpu_baseline": None,
    }
    if world == 1 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(sc, a.cpu_rays)
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
