"""bench.py's multi-rank path as the driver runs it: ``python bench.py --gpus N``
with no WORLD_SIZE starts N ranks itself (torch.distributed.run as a child
process).  On the one-GPU test box LPC_BENCH_REHEARSE=1 puts both ranks on GPU 0
(gloo for the trace-end exchange); the line must say n_gpus == 2, carry both
ranks' times, and every timed step must give identical counts."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_launches_two_ranks():
    env = dict(os.environ, LPC_BENCH_REHEARSE="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5",
                        "--warmup", "1", "--no-cpu", "--no-configs", "--rays", "200000"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["parity"]["steps_identical"] is True
    assert len(out["rank_ms_per_step"]["per_rank"]) == 2
    assert out["rank_ms_per_step"]["max"] == pytest.approx(out["ms_per_step"], rel=1e-9)
    assert out["exchange"]["rehearsal_one_gpu"] is True
    assert out["value"] > 0
