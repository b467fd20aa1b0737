"""Top-level ``geo_optical_elements`` module for scripts written against LightPyCL.

Put ``lightpycl_amd.compat.PATH`` on ``sys.path`` (or ``PYTHONPATH``) and
``import geo_optical_elements`` resolves to the MI355X-native drop-in."""
from lightpycl_amd.geo_optical_elements import GeoObject, optical_elements  # noqa: F401
