"""Write the bench's 2^k-point inputs as wire files for the Node tools (P_i = (i+1)G, scalar set 0):

    python tools/write_inputs.py <dir> [--n 1048576]   -> <dir>/p.bin, <dir>/s.bin
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "webgpu-msm_amd")]
os.environ.setdefault("MSM_AMD_NO_TORCH", "1")
import numpy as np  # noqa: E402

import msm_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--n", type=int, default=1 << 20)
a = ap.parse_args()
os.makedirs(a.dir, exist_ok=True)
M.gen_points(a.n).astype(np.uint32).tofile(os.path.join(a.dir, "p.bin"))
M.gen_scalars(a.n).astype(np.uint32).tofile(os.path.join(a.dir, "s.bin"))
