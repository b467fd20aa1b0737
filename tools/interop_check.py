"""GPU box: liblpc and torch in one process, both import orders (subprocesses)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

A = """
import sys; sys.path.insert(0, %r)
from lightpycl_amd.engine import Engine
e = Engine(0); print('lpc', e.info())
import torch; x = torch.ones(4, device='cuda'); print('torch', float(x.sum()), torch.cuda.get_device_name(0))
"""
B = """
import sys; sys.path.insert(0, %r)
import torch; x = torch.ones(4, device='cuda'); print('torch', float(x.sum()))
from lightpycl_amd.engine import Engine
e = Engine(0); print('lpc', e.info())
"""
ok = True
for name, code in (("lpc-first", A % ROOT), ("torch-first", B % ROOT)):
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    print(name, "rc", r.returncode, r.stdout.strip().replace("\n", " | "), r.stderr.strip()[-300:])
    ok &= r.returncode == 0
sys.exit(0 if ok else 1)
