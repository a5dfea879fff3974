"""Wall time of the CPU/GPU co-compute (msm_compute_cocompute, ?cpuWorkRatio of
submission.ts:94-154) from host arrays at 2^20 points, per ratio: the evidence behind DESIGN.md
§7's "any CPU share only delays the result".

    python tools/cocompute_probe.py [--n 1048576] [--ratios 0,0.0005,0.001,0.005,0.02] [--runs 5]

One JSON line per ratio: median / min wall ms over the runs (after one warm-up), the host share's
point count, whether the result equals the ratio-0 result, and the GPU share alone (msm_compute
on points [share, n): what the split costs without the host thread)."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "webgpu-msm_amd")]
import msm_amd as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--ratios", default="0,0.0005,0.001,0.005,0.02")
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16, help="host Pippenger threads (the box's CPU share)")
    a = ap.parse_args()
    pts = M.gen_points(a.n)
    sc = M.gen_scalars(a.n, seed=M.XORSHIFT_SEED)
    ref = M.compute_msm_wire(pts, sc)
    for r in (float(x) for x in a.ratios.split(",")):
        M.compute_msm_wire(pts, sc, cpu_work_ratio=r, cpu_threads=a.threads)  # warm-up
        ts, ok = [], True
        for _ in range(a.runs):
            t0 = time.perf_counter()
            res = M.compute_msm_wire(pts, sc, cpu_work_ratio=r, cpu_threads=a.threads)
            ts.append((time.perf_counter() - t0) * 1e3)
            ok = ok and res == ref
        share = int(r * a.n)
        gs = []
        for _ in range(a.runs if share else 0):
            t0 = time.perf_counter()
            M.compute_msm_wire(pts[share:], sc[share:])
            gs.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"n": a.n, "cpu_work_ratio": r, "cpu_points": share, "cpu_threads": a.threads,
                          "median_ms": round(statistics.median(ts), 3), "min_ms": round(min(ts), 3),
                          "gpu_share_alone_median_ms": round(statistics.median(gs), 3) if gs else None,
                          "correct": ok}), flush=True)


if __name__ == "__main__":
    main()
