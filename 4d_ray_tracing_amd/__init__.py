"""rt4 — MI355X-native 4D path tracer (drop-in for executable/shader.frag of BusyginIvan/4D_ray_tracing).

The package name starts with a digit, so import it with importlib:
    rt4 = importlib.import_module("4d_ray_tracing_amd")
Everything here is a thin binding of librt4.so (include/rt4.h); see rt4.py.
"""
from .rt4 import *  # noqa: F401,F403
from .rt4 import LIB_PATH, RT4Error, lib  # noqa: F401
