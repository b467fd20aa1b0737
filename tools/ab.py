"""A/B launch policies in separate processes (one bench.py process per run,
configurations alternated round-robin `reps` times): prints one JSON line per
run and a summary (median ms/step per configuration).

    python tools/ab.py reps 'NAME:VAR=V,VAR=V' 'NAME:...' ...   ('base:' = defaults;
    ARGS=... passes extra bench.py arguments, e.g. 'noprof:ARGS=--no-prof'; AB_STEPS, default 300)
"""
import json
import os
import statistics
import subprocess
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
reps = int(sys.argv[1])
cfgs = []
for a in sys.argv[2:]:
    name, _, rest = a.partition(":")
    env = dict(kv.split("=", 1) for kv in rest.split(",") if kv)
    cfgs.append((name, env))
res = {n: [] for n, _ in cfgs}
for r in range(reps):
    for name, env in cfgs:
        e = dict(os.environ, **{k: v for k, v in env.items() if k != "ARGS"})
        extra = env.get("ARGS", "").split()
        steps = os.environ.get("AB_STEPS", "300")
        out = subprocess.run([sys.executable, "bench.py", "--no-cpu", "--no-configs", "--no-strong", "--steps", steps, "--warmup", "5"]
                             + extra, cwd=root, env=e, capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if out.returncode != 0 or not line:
            print(json.dumps(dict(cfg=name, rc=out.returncode, err=out.stderr[-2000:])), flush=True)
            sys.exit(1)
        d = json.loads(line[-1])
        res[name].append(d["ms_per_step"])
        print(json.dumps(dict(cfg=name, rep=r, ms=d["ms_per_step"], walk_ms=d["roofline"]["avg_launch_ms"],
                              counts_ok=d["parity"]["steps_identical"])), flush=True)
print(json.dumps({n: dict(median=statistics.median(v), all=v) for n, v in res.items()}))
