"""Build compile-time variants of liblpc.so in-tree for A/B runs (LPC_LIB_PATH):

    python tools/build_variant.py NAME -DMACRO=V ...   ->  lightpycl_amd/liblpc_NAME.so
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd.build import HERE, command  # noqa: E402

name, extra = sys.argv[1], sys.argv[2:]
out = os.path.join(HERE, f"liblpc_{name}.so")
subprocess.run(command(out=out, extra=extra), check=True)
print(out)
