"""bench.py's multi-rank path as the driver runs it: ``python bench.py --gpus N``
with no WORLD_SIZE starts N ranks itself (torch.distributed.run as a child
process).  On the one-GPU test box LPC_BENCH_REHEARSE=1 puts both ranks on GPU 0
(gloo for the trace-end exchange); the line must say n_gpus == 2, carry both
ranks' times, and every timed step must give identical counts -- the timed steps
run with three traces in flight per rank (three engines, three shared-memory
exchange segments), checked against the same steps on one engine.  The strong
block (one fixed global ray set split with shard_bounds) and the config-5 block
(fixed ray blocks split over the ranks) must give the global per-iteration
counts of the N = 1 trace of the same rays (the reference's global termination,
iterative_tracer.py:383-391, taken on the all-reduced sums)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


ARGS = ["--steps", "5", "--warmup", "1", "--no-cpu", "--no-configs", "--rays", "200000", "--strong-steps", "5",
        "--c5-rays", "1600000", "--c5-steps", "2"]


def _bench(gpus, args=ARGS):
    env = dict(os.environ, LPC_BENCH_REHEARSE="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus)] + args,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    out = _bench(2)
    assert out["n_gpus"] == 2
    assert out["parity"]["steps_identical"] is True
    assert len(out["rank_ms_per_step"]["per_rank"]) == 2
    assert out["rank_ms_per_step"]["max"] == pytest.approx(out["ms_per_step"], rel=1e-9)
    assert out["exchange"]["rehearsal_one_gpu"] is True
    assert out["value"] > 0
    # the timed steps ran with traces in flight (three engines per rank), and the
    # same steps back to back on one engine gave the same counts and power
    assert out["inflight"]["traces_in_flight_per_gpu"] == 3
    assert out["inflight"]["sequential"]["identical_to_inflight"] is True

    one = _bench(1)
    for blk in ("strong", "config5"):
        a, b = out[blk], one[blk]
        assert a["global_counts"] == b["global_counts"], (blk, a["global_counts"], b["global_counts"])
        assert a["steps_identical"] and b["steps_identical"]
        assert len(a["rank_ms_per_step"]["per_rank"]) == 2
        # per-mesh power: the ranks' float64 sums added in rank order vs one sum
        for x, y in zip(a["mesh_power"], b["mesh_power"]):
            assert x == pytest.approx(y, rel=1e-9, abs=1e-300)
    # at N = 1 the strong block traces the weak block's rays (seed 7)
    assert one["strong"]["global_counts"] == one["weak_global_counts"]


ARGS8 = ["--steps", "3", "--warmup", "1", "--no-cpu", "--no-configs", "--rays", "40000", "--strong-steps", "3",
         "--c5-rays", "320000", "--c5-steps", "1"]


def test_bench_gpus8_rehearsal():
    """The driver's N = 8 form rehearsed on the one GPU: eight ranks, the config-5
    split with one block per rank (world == 8), per-rank times and ray-bounces in
    the line, and the strong and config-5 blocks' global counts equal to N = 1."""
    out = _bench(8, ARGS8)
    assert out["n_gpus"] == 8 and out["parity"]["steps_identical"] is True
    assert out["inflight"]["sequential"]["identical_to_inflight"] is True
    assert len(out["rank_ms_per_step"]["per_rank"]) == 8
    assert len(out["rank_ray_bounces_per_step"]) == 8 and min(out["rank_ray_bounces_per_step"]) > 0
    assert out["config5"]["rays_per_rank"] == 320000 // 8
    one = _bench(1, ARGS8)
    for blk in ("strong", "config5"):
        a, b = out[blk], one[blk]
        assert a["global_counts"] == b["global_counts"], (blk, a["global_counts"], b["global_counts"])
        assert len(a["rank_ray_bounces_per_step"]) == 8
        assert sum(a["rank_ray_bounces_per_step"]) == pytest.approx(b["rank_ray_bounces_per_step"][0], rel=1e-12)
