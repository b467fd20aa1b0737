"""Top-level ``iterative_tracer`` module for scripts written against LightPyCL.

Put ``lightpycl_amd.compat.PATH`` on ``sys.path`` (or ``PYTHONPATH``) and
``import iterative_tracer`` resolves to the MI355X-native drop-in."""
from lightpycl_amd.iterative_tracer import *  # noqa: F401,F403
from lightpycl_amd.iterative_tracer import CL_Tracer, CLTracer  # noqa: F401
