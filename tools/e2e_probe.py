"""msm_compute end to end from host arrays (upload + MSM + result), for timeline profiling:

    python tools/e2e_probe.py [--n 1048576] [--runs 6]
    rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/e2e -- python3 tools/e2e_probe.py

Prints one JSON line: per-run wall times (ms) and whether each result matched the closed form.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "webgpu-msm_amd")):
    sys.path.insert(0, p)

import msm_amd as M  # noqa: E402


def rehome(a, src):
    """A copy of `a` in the requested kind of host memory."""
    if src == "numpy":
        return a
    import mmap

    import numpy as np

    flags = mmap.MAP_SHARED if src == "shared" else mmap.MAP_PRIVATE
    m = mmap.mmap(-1, a.nbytes, flags=flags | mmap.MAP_ANONYMOUS)
    if src == "nohuge":
        m.madvise(mmap.MADV_NOHUGEPAGE)
    out = np.frombuffer(m, dtype=a.dtype).reshape(a.shape)
    out[...] = a
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--src", choices=("numpy", "nohuge", "shared"), default="numpy",
                    help="host memory the inputs live in: numpy's own (huge-page backed when large), an "
                         "anonymous private mapping with MADV_NOHUGEPAGE, or a MAP_SHARED mapping (as a "
                         "Node SharedArrayBuffer may be)")
    args = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "bench_expected.json")) as f:
        row = json.load(f)["rows"].get(f"{args.n}:0")
    exp = (int(row[0]), int(row[1])) if row else None
    pts = rehome(M.gen_points(args.n), args.src)
    sc = rehome(M.gen_scalars(args.n), args.src)
    times, ok = [], []
    for _ in range(args.runs):
        t0 = time.perf_counter()
        r = M.compute_msm_wire(pts, sc)
        times.append(round((time.perf_counter() - t0) * 1e3, 3))
        ok.append(exp is None or r == exp)
    print(json.dumps({"n": args.n, "src": args.src, "e2e_ms": times, "correct": all(ok) if exp else None,
                      "x_low64": hex(r[0] & (2**64 - 1))}))


if __name__ == "__main__":
    main()
