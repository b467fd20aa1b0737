"""Directory of reference-named shim modules (light_source, geo_optical_elements,
iterative_tracer).  ``sys.path.insert(0, lightpycl_amd.compat.PATH)`` makes a
LightPyCL script's ``import iterative_tracer as it`` use this package."""
import os

PATH = os.path.dirname(os.path.abspath(__file__))
