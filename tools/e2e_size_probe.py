"""Host-input msm_compute wall time over a list of sizes (looking for cliffs at the path and plan
thresholds: the host split from 2^18 points, pipelined_window's steps).

    python tools/e2e_size_probe.py --sizes 262143,262144,393216 [--runs 5] [--rounds 2]

One JSON line per (size, round): median / min ms over the runs after one warm-up, checked against
the closed form of P_i = (i + 1) G."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "webgpu-msm_amd"), os.path.join(ROOT, "tests")]
import msm_amd as M  # noqa: E402
from _closed_form import closed_form  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", required=True)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--windows", default="0", help="window widths to time each size at (0 = the library's choice)")
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    pts = M.gen_points(max(sizes))
    sc = M.gen_scalars(max(sizes), seed=3)
    for r in range(a.rounds):
        for n, w in ((n, int(w)) for n in sizes for w in a.windows.split(",")):
            p, s = pts[:n], sc[:n]
            ok = M.compute_msm_wire(p, s, window_size=w or None) == closed_form(1, 1, s)
            ts = []
            for _ in range(a.runs):
                t0 = time.perf_counter()
                M.compute_msm_wire(p, s, window_size=w or None)
                ts.append((time.perf_counter() - t0) * 1e3)
            print(json.dumps({"n": n, "window": w, "round": r + 1, "median_ms": round(statistics.median(ts), 3),
                              "min_ms": round(min(ts), 3), "ns_per_point": round(statistics.median(ts) * 1e6 / n, 2),
                              "correct": ok}), flush=True)


if __name__ == "__main__":
    main()
