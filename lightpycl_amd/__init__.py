"""lightpycl_amd -- MI355X-native drop-in for LightPyCL's per-bounce ray tracer.

Modules mirroring the reference API: ``light_source``, ``geo_optical_elements``,
``iterative_tracer`` (``CL_Tracer``).  The per-bounce hot path runs in
``liblpc.so`` (HIP for gfx950, C ABI in ``include/lpc.h``); ``engine`` is its
Python front, ``distributed`` the one-process-per-GPU sharded trace.
"""
from . import geo_optical_elements, light_source  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # the tracer loads liblpc.so on first use only
    if name in ("iterative_tracer", "engine", "scenes", "distributed"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    if name in ("CL_Tracer", "CLTracer"):
        from .iterative_tracer import CL_Tracer
        return CL_Tracer
    raise AttributeError(name)
