"""Single-MSM latency (the reference's one awaited compute_msm, Benchmark.tsx:29-39) on
device-resident inputs: median / min / p90 of `runs` msm_compute_device calls after warm-up, plus
the host tail of the last profiled call.  Every result is checked against its closed form.

    python tools/latency_probe.py [--n 1048576] [--runs 40]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "webgpu-msm_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--runs", type=int, default=40)
    ap.add_argument("--run-length", type=int, default=0, help="entries per accumulation lane (0: the plan's)")
    ap.add_argument("--window", type=int, default=0)
    args = ap.parse_args()
    import torch

    import msm_amd as M
    from bench import load_expected

    exp = load_expected().get((args.n, 0))
    dev = torch.device("cuda", 0)
    dp = torch.from_numpy(M.gen_points(args.n).view(np.int32)).to(dev)
    ds = torch.from_numpy(M.gen_scalars(args.n).view(np.int32)).to(dev)
    torch.cuda.synchronize()
    kw = dict(run_length=args.run_length or None, window_size=args.window or None)
    for _ in range(5):
        M.compute_msm_device(dp, ds, args.n, **kw)
    lat, bad = [], 0
    for _ in range(args.runs):
        t0 = time.perf_counter()
        r = M.compute_msm_device(dp, ds, args.n, **kw)
        lat.append((time.perf_counter() - t0) * 1e3)
        bad += exp is not None and r != exp
    M.set_profiling(2)
    tails = []
    accs = []
    for _ in range(10):
        M.compute_msm_device(dp, ds, args.n, **kw)
        prof = M.last_profile()
        tails.append(prof["host_tail"])
        accs.append(prof["accumulate"])
    M.set_profiling(False)
    env = {k: v for k, v in os.environ.items() if k.startswith("MSM_")}
    print(json.dumps({"n": args.n, "runs": args.runs, "latency_ms_median": round(float(np.median(lat)), 4),
                      "latency_ms_min": round(float(np.min(lat)), 4),
                      "latency_ms_p90": round(float(np.percentile(lat, 90)), 4),
                      "host_tail_ms_median": round(float(np.median(tails)), 4),
                      "accumulate_ms_median": round(float(np.median(accs)), 4), "run_length": args.run_length,
                      "correct": (bad == 0) if exp is not None else None, "env": env}))


if __name__ == "__main__":
    main()
