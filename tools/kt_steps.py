"""Per-step and per-iteration spans from a rocprofv3 kernel trace of bench.py:
a step starts at k_raykey (the emitted rays' key), an iteration at k_roots_s.
Prints, per step: span, and per iteration: span, idle time before it, and the
summed kernel time of the main categories (walk, spill, slivers, shade, sort)."""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
      for r in rows]
steps = [i for i, e in enumerate(ev) if "k_raykey" in e[2] or "k_bkey" in e[2]]
for a, b in zip(steps, steps[1:] + [len(ev)]):
    seg = [e for e in ev[a:b] if "k_project_hist" not in e[2] and "copyBuffer" not in e[2]]
    t0, t1 = seg[0][0], max(e[1] for e in seg)
    # busy time: union of kernel intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sorted(seg):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    cat = collections.Counter()
    for s, e, n in seg:
        k = ("walk" if "rootwalk" in n else "spill" if "k_spill" in n else "slivers" if "sliver" in n or "k_packet" in n
             else "shade" if "shade" in n or "stage_move" in n else "roots" if "roots" in n
             else "sort" if ("rocprim" in n or "raykey" in n or "gather" in n or "fill" in n or "lpck::k_b" in n) else "other")
        cat[k] += e - s
    print(f"step span {(t1 - t0) / 1e3:7.1f} us  busy {busy / 1e3:7.1f} us  " +
          "  ".join(f"{k} {v / 1e3:.1f}" for k, v in sorted(cat.items())))
