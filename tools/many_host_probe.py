"""msm_compute_many from host arrays (the batch API over host-resident inputs): wall time of one
call over `count` MSMs of n points each, median over runs after one warm-up, every result checked
against the closed form.

    python tools/many_host_probe.py [--n 262144] [--count 16] [--runs 5]

Prints one JSON line.  Used for the packed-upload A/B (MSM_HOST_PACK=1/0).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "webgpu-msm_amd"), os.path.join(ROOT, "tests")]
import msm_amd as M  # noqa: E402
from _closed_form import as_xy, closed_form  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--count", type=int, default=16)
    ap.add_argument("--runs", type=int, default=5)
    a = ap.parse_args()
    pts = [M.gen_points(a.n, k0=1 + b, step=3) for b in range(a.count)]
    scs = [M.gen_scalars(a.n, seed=900 + b) for b in range(a.count)]
    exp = [closed_form(1 + b, 3, scs[b]) for b in range(a.count)]
    ts, ok = [], True
    for r in range(a.runs + 1):
        t0 = time.perf_counter()
        res = M.compute_msm_many(pts, scs, a.n)
        t1 = time.perf_counter()
        if r:
            ts.append((t1 - t0) * 1e3)
        ok = ok and all(tuple(as_xy(res[b])) == tuple(exp[b]) for b in range(a.count))
    print(json.dumps({"n": a.n, "count": a.count, "ms_per_call": round(statistics.median(ts), 3),
                      "ms_per_msm": round(statistics.median(ts) / a.count, 4), "runs_ms": [round(t, 3) for t in ts],
                      "correct": ok, "pack": os.environ.get("MSM_HOST_PACK", "1")}))


if __name__ == "__main__":
    main()
