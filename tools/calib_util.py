"""Calibration load for the lane-utilisation counter formula: rt4_eval_kernel on acos (branch-free,
every lane active except the grid tail) and on w_by_volume (divergent Newton loop)."""
import importlib, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rt4 = importlib.import_module("4d_ray_tracing_amd")
t = rt4.Tracer(0)
x = np.linspace(-1, 1, 1 << 24, dtype=np.float32)
t.debug_eval(rt4.EVAL_ACOS, x)
t.debug_eval(rt4.EVAL_W_BY_VOLUME, (x + 1) / 2)
