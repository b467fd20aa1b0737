"""Top-level ``light_source`` module for scripts written against LightPyCL.

Put ``lightpycl_amd.compat.PATH`` on ``sys.path`` (or ``PYTHONPATH``) and
``import light_source`` resolves to the MI355X-native drop-in."""
from lightpycl_amd.light_source import light_source  # noqa: F401
