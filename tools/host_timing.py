"""Host field / curve operation timings of libmsm's host tail code (tuning tool; runs anywhere).

    python tools/host_timing.py
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "webgpu-msm_amd"))
import msm_amd as M  # noqa: E402

L = M.load()
out = {}
for what, name, iters in ((0, "fq_mul", 200000), (1, "pt_dbl", 100000), (2, "pt_add", 50000), (3, "fq_inv", 2000)):
    ns = ctypes.c_double()
    best = None
    for _ in range(5):
        assert L.msm_test_host_timing(what, iters, ctypes.byref(ns)) == 0
        best = ns.value if best is None else min(best, ns.value)
    out[name + "_ns"] = round(best, 1)
try:
    out["cpu"] = next(ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name"))
except (OSError, StopIteration):
    pass
print(json.dumps(out))
