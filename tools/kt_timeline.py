"""Print the dispatch timeline of the last bench step from a rocprofv3
kernel_trace.csv: kernel, grid, duration, gap before it."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
sel = rows[-n_last:]
prev = None
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
    print(f"{name:48s} grid {int(r.get('Grid_Size', 0) or 0):9d}  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}")
