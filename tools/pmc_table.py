"""Per-launch table of the PMC passes written by tools/pmc_stalls.sh.

    python tools/pmc_table.py gpurun_out/stalls [kernel-substring]
"""
import collections
import csv
import os
import sys

src = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "k_intersect"
rows = collections.defaultdict(dict)
for d in sorted(os.listdir(src)):
    f = os.path.join(src, d, "pmc_counter_collection.csv")
    if not os.path.exists(f):
        continue
    seq = collections.Counter()
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        if want not in name:
            continue
        key = (r["Dispatch_Id"], r["Counter_Name"])
        rows[(d, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
# group by pass, print launches in order
passes = collections.defaultdict(list)
for (d, disp), cs in rows.items():
    passes[d].append((int(disp), cs))
for d in sorted(passes):
    print(f"== {d}")
    for disp, cs in sorted(passes[d]):
        print(f"  dispatch {disp:5d} " + "  ".join(f"{k}={v:.4g}" for k, v in sorted(cs.items())))
