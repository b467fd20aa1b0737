"""Build liblpc.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "lpc_runtime.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in ("lpc_runtime.hip", "lpc_kernels.hip", "lpc_math.hpp",
                                               "lpc_internal.hpp", "lpc_comm.hpp", "lpc_build.hpp")] + [os.path.join(ROOT, "include", "lpc.h")]
OUT = os.path.join(HERE, "liblpc.so")
ARCH = os.environ.get("LPC_ARCH", "gfx950")


def command(out=OUT, extra=()):
    return ["hipcc", f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17",
            "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(HERE, "csrc"),
            *extra, SRC, "-o", out]


def up_to_date(out=OUT):
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    cmd = command()
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
