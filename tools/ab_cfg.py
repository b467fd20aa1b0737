"""A/B launch policies on BASELINE config scenes, one process per run
(tools/cfg_trace.py), configurations alternated round-robin `reps` times:
one JSON line per run and a summary (median ms per trace per scene and policy).

    python tools/ab_cfg.py reps 'scene:rays:depth[:traces],...' 'NAME:VAR=V,VAR=V' 'NAME:...' ...
"""
import json
import os
import statistics
import subprocess
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
reps = int(sys.argv[1])
scenes = [s.split(":") for s in sys.argv[2].split(",")]
cfgs = []
for a in sys.argv[3:]:
    name, _, rest = a.partition(":")
    cfgs.append((name, dict(kv.split("=", 1) for kv in rest.split(",") if kv)))
res = {}
for r in range(reps):
    for sc in scenes:
        scene, rays, depth = sc[0], sc[1], sc[2]
        traces = sc[3] if len(sc) > 3 else "3"
        for name, env in cfgs:
            e = dict(os.environ, **env)
            out = subprocess.run([sys.executable, os.path.join(root, "tools", "cfg_trace.py"), scene, rays, depth,
                                  traces], cwd=root, env=e, capture_output=True, text=True, timeout=600)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
            if out.returncode != 0 or not line:
                print(json.dumps(dict(scene=scene, cfg=name, rc=out.returncode, err=out.stderr[-2000:])), flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            res.setdefault(f"{scene}/{name}", []).append(d["ms_per_trace"])
            print(json.dumps(dict(scene=scene, cfg=name, rep=r, ms=d["ms_per_trace"],
                                  populations=d["populations"])), flush=True)
print(json.dumps({k: dict(median=statistics.median(v), all=v) for k, v in res.items()}))
