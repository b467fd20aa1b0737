#!/usr/bin/env python3
"""bench.py's fresh_rays and cold blocks alone (GPU): python tools/fresh_probe.py [rays]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.distributed import ShardedTrace  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
print(json.dumps({"fresh_rays": bench.fresh_rays_block(scenes, Engine, n)}), flush=True)
print(json.dumps({"cold": bench.cold_block(scenes, Engine, ShardedTrace, n)}), flush=True)
