"""GPU box: enqueue time of async device-to-host copies into reused pinned
blocks (hipHostMalloc via torch.pin_memory), in the results mode's pattern: two
sets of blocks used alternately, a block's second use coming two calls later.
Prints one JSON line per copy: which block, its use count, the enqueue time."""
import json
import time

import torch

dev = torch.device("cuda", 0)
n = 40_000_000 // 4
src = torch.ones(n, dtype=torch.float32, device=dev)
s = torch.cuda.Stream()
blocks = {k: torch.empty(n, dtype=torch.float32).pin_memory() for k in ("A", "B")}
uses = {k: 0 for k in blocks}
torch.cuda.synchronize()
for pattern in (["A", "B"] * 4, ["A", "A", "A"], ["B", "A", "B", "A"]):
    for k in pattern:
        with torch.cuda.stream(s):
            t = time.perf_counter()
            blocks[k].copy_(src, non_blocking=True)
            dt = time.perf_counter() - t
        s.synchronize()
        uses[k] += 1
        print(json.dumps(dict(block=k, use=uses[k], enqueue_us=round(dt * 1e6, 1))), flush=True)
        time.sleep(0.005)
