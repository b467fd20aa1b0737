"""Summarise the eye's PMC passes of tools/gpu_final.sh (gpurun_out/eye/pmc_sq,
pmc_fetch) into profiles/<tag>_eye_pmc.json: per-kernel means over the
launches, and for k_rootwalk the fetch bytes (2 x FETCH_SIZE x 1024, the gfx950
correction) and the VALU issue fraction (SQ_INSTS_VALU over GRBM_GUI_ACTIVE / 8
XCDs x 256 wave-instructions per cycle: 256 CUs x 4 SIMDs, 4 cycles each).

    python tools/eye_pmc.py gpurun_out/eye r03
"""
import csv
import glob
import json
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
acc = {}
for f in glob.glob(os.path.join(src, "pmc_*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        c = r["Counter_Name"]
        acc.setdefault(k, {}).setdefault(c, {}).setdefault(int(r["Dispatch_Id"]), 0.0)
        acc[k][c][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
kernels = {}
for k, cs in acc.items():
    kernels[k] = {c: {"launches": len(v), "mean": sum(v.values()) / len(v), "total": sum(v.values())}
                  for c, v in sorted(cs.items())}
walk = next(k for k in kernels if "k_rootwalk" in k)
w = kernels[walk]
out = {
    "source": "tools/gpu_final.sh: rocprofv3 --pmc over tools/cfg_trace.py eye 300000 16 1 "
              "(a warm-up trace + one trace)",
    "note": "per-kernel means over the launches of both traces; k_rootwalk fetch bytes = 2 x FETCH_SIZE x 1024 "
            "(gfx950 correction)",
    "kernels": kernels,
    "k_rootwalk_fetch_bytes_per_launch": 2 * w["FETCH_SIZE"]["mean"] * 1024,
    "k_rootwalk_valu_per_launch": w["SQ_INSTS_VALU"]["mean"],
    "k_rootwalk_valu_issue_fraction_over_busy": w["SQ_INSTS_VALU"]["total"] / (w["GRBM_GUI_ACTIVE"]["total"] / 8 * 256),
}
json.dump(out, open(os.path.join(root, "profiles", f"{tag}_eye_pmc.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))
