"""Summarise a tools/gpu_round.sh profile/pmc run into profiles/ (committed evidence).

    python tools/pmc_summary.py gpurun_out/prof r01

writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats), profiles/<tag>_pmc.json
(per-kernel averages of every PMC pass) and profiles/pmc_intersect.json, which
bench.py reads for roofline.traffic: HBM bytes per launch of the hierarchy kernel (argv[3]) =
(2 * FETCH_SIZE + WRITE_SIZE) * 1024, the gfx950 correction of
MI355X_MICROARCH.md section HBM (FETCH_SIZE reads half of a wide streaming read).
"""
import collections
import csv
import hashlib
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
kname = sys.argv[3] if len(sys.argv) > 3 else "k_rootwalk"     # the bench roofline's kernel
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "profiles")
os.makedirs(out, exist_ok=True)
kst = os.path.join(src, "kt", "kt_kernel_stats.csv")
if os.path.exists(kst):                 # a kernel trace of the same run, when there is one
    shutil.copy(kst, os.path.join(out, f"{tag}_kernel_stats.csv"))
per = collections.defaultdict(lambda: collections.defaultdict(list))
if src.endswith(".json"):               # re-derive from a committed <tag>_pmc.json
    for k, cs in json.load(open(src)).items():
        for c, v in cs.items():
            per[k][c] = list(v["values"])
for d in ([] if src.endswith(".json") else sorted(os.listdir(src))):
    f = os.path.join(src, d, "pmc_counter_collection.csv")
    if d.startswith("pmc") and os.path.exists(f):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {k: {c: {"launches": len(v), "mean": sum(v) / len(v), "values": v} for c, v in cs.items()}
           for k, cs in per.items()}
if not src.endswith(".json"):
    json.dump(summary, open(os.path.join(out, f"{tag}_pmc.json"), "w"), indent=1)
ki = next((v for k, v in summary.items() if kname in k), {})
if "FETCH_SIZE" in ki and "WRITE_SIZE" in ki:
    fetch, write = ki["FETCH_SIZE"]["mean"], ki["WRITE_SIZE"]["mean"]
    rec = {"source": f"profiles/{tag}_pmc.json", "kernel": kname,
           "fetch_size_kb_mean": fetch, "write_size_kb_mean": write,
           "hbm_bytes_per_launch": (2.0 * fetch + write) * 1024.0,
           "kernels_sha16": hashlib.sha256(open(os.path.join(root, "lightpycl_amd", "csrc", "lpc_kernels.hip"),
                                                "rb").read()).hexdigest()[:16],
           "note": f"mean over the {kname} launches of one bench step (all iterations)"}
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES",
              "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"):
        if c in ki:
            rec[c.lower() + "_mean"] = ki[c]["mean"]
    # the primary (1 M-ray) launches alone: bench.py --steps 1 --warmup 0 runs the
    # first iteration by itself (launch 0), then traces of three iterations each
    # (pre-warm, timed, histogram): launches 1, 4, 7, ... are primaries
    # the other launches are the secondary bounces (iterations 2 and 3)
    prim, sec = {}, {}
    for c, v in ki.items():
        n = len(v["values"])
        idx = [0] + [i for i in range(1, n) if (i - 1) % 3 == 0]
        for want, dst in ((idx, prim), ([i for i in range(n) if i not in idx], sec)):
            vals = [v["values"][i] for i in want]
            if vals:
                dst[c] = sum(vals) / len(vals)
    for dst in (prim, sec):
        if "FETCH_SIZE" in dst and "WRITE_SIZE" in dst:
            dst["hbm_bytes"] = (2.0 * dst["FETCH_SIZE"] + dst["WRITE_SIZE"]) * 1024.0
    rec["primary_launch"] = prim
    rec["secondary_launch"] = sec
    json.dump(rec, open(os.path.join(out, "pmc_intersect.json"), "w"), indent=1)
    print(json.dumps(rec, indent=1))
