import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU case")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def engine():
    """One liblpc handle for the whole GPU session (fails loudly without a GPU)."""
    from lightpycl_amd.build import build
    build(verbose=False)
    from lightpycl_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="session")
def exact_ref():
    """The exact checker of the GPU parity tests: the reference's own kernels
    (oracle/_ref/lpc_ref_ieee.co, tests/ref_gpu.py), with which liblpc is
    bit-identical.  None when the code object was not built (the tests then fall
    back to the CPU oracle and its 1-ulp tolerance on the hardware rsqrt)."""
    import ref_gpu
    if not ref_gpu.available("ieee"):
        yield None
        return
    r = ref_gpu.RefKernels("ieee")
    yield r
    r.close()


@pytest.fixture(scope="session")
def checker(exact_ref, oracle_mod):
    """(bounce_fn, exact): the reference kernels (exact) or the CPU oracle."""
    if exact_ref is not None:
        return exact_ref.bounce, True
    return oracle_mod.bounce, False
