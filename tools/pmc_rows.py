"""Per-dispatch counter rows of the tools/gpu_round.sh pmc passes for kernels matching a
regex (the last bench step's dispatches: grid size tells the iteration)."""
import collections
import csv
import glob
import os
import re
import sys

root, pat = sys.argv[1], re.compile(sys.argv[2])
rows = collections.defaultdict(dict)          # (pass-local dispatch order, kernel) -> counters
for p in sorted(glob.glob(os.path.join(root, "p*"))):
    if not os.path.isdir(p):
        continue
    f = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    seq = collections.Counter()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0]
        if not pat.search(name):
            continue
        key = (int(r["Dispatch_Id"]), name)
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[key] = int(r.get("Grid_Size", 0) or 0)
    for k in sorted(per):
        idx = seq[k[1]]
        seq[k[1]] += 1
        rows[(k[1], idx)].update(per[k])
        rows[(k[1], idx)]["grid"] = meta[k]
for (name, idx), c in sorted(rows.items()):
    g = c.get("GRBM_GUI_ACTIVE", 0) or 1
    occ = c.get("SQ_WAVE_CYCLES", 0) / g
    print(f"{name[:24]:24s} #{idx:2d} grid {int(c.get('grid', 0)):9d} gui {g:10.0f} waves {c.get('SQ_WAVES', 0):8.0f} "
          f"wave_cyc/gui {occ:8.1f} " + " ".join(
              f"{k.replace('SQ_', '')}={v:.3g}" for k, v in sorted(c.items())
              if k not in ("grid", "GRBM_GUI_ACTIVE", "SQ_WAVES", "SQ_WAVE_CYCLES")))
