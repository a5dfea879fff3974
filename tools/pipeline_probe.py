"""Timed pipelined calls (bench.py's point bench without the extras), printing the host's
CLOCK_MONOTONIC at each call's start and end so a rocprofv3 kernel trace of the same run shows
the pipeline's fill and drain:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pipe -- python3 tools/pipeline_probe.py
    python tools/timeline.py ... (or tools/pipeline_probe.py --analyse <kernel_trace.csv> <probe.json>)
"""
import argparse
import csv
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "webgpu-msm_amd")):
    sys.path.insert(0, p)


def run(args):
    import numpy as np
    import torch
    import msm_amd as M

    n = args.n
    d_pts = torch.from_numpy(M.gen_points(n).view(np.int32)).cuda()
    sets = [torch.from_numpy(M.gen_scalars(n, seed=M.XORSHIFT_SEED + j).view(np.int32)).cuda() for j in range(4)]
    torch.cuda.synchronize()
    calls = []
    for k in [args.warmup] + [args.steps] * args.calls:
        torch.cuda.synchronize()
        t0 = time.monotonic_ns()
        M.compute_msm_many_device([d_pts] * k, [sets[i % 4] for i in range(k)], n)
        torch.cuda.synchronize()
        t1 = time.monotonic_ns()
        calls.append({"k": k, "t0": t0, "t1": t1, "ms_per_msm": (t1 - t0) / 1e6 / k})
    print(json.dumps({"n": n, "calls": calls}))


def analyse(trace, probe):
    with open(probe) as f:
        calls = json.loads(f.read().strip().splitlines()[-1])["calls"]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(trace))]
    for c in calls[1:]:
        inside = sorted(k for k in ks if c["t0"] <= k[0] <= c["t1"])
        if not inside:
            continue
        busy, lo, hi = 0, inside[0][0], inside[0][1]
        for s, e, _ in inside:
            if s > hi:
                busy += hi - lo
                lo, hi = s, e
            else:
                hi = max(hi, e)
        busy += hi - lo
        acc = [(s, e) for s, e, nm in inside if "k_accumulate" in nm]
        print(json.dumps({"k": c["k"], "wall_ms": (c["t1"] - c["t0"]) / 1e6,
                          "first_kernel_after_ms": (inside[0][0] - c["t0"]) / 1e6,
                          "last_kernel_end_before_ms": (c["t1"] - max(e for _, e, _ in inside)) / 1e6,
                          "device_busy_ms": busy / 1e6,
                          "acc_first_start_ms": (acc[0][0] - c["t0"]) / 1e6 if acc else None,
                          "acc_last_end_ms": (acc[-1][1] - c["t0"]) / 1e6 if acc else None}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--analyse", nargs=2, metavar=("TRACE_CSV", "PROBE_JSON"))
    a = ap.parse_args()
    if a.analyse:
        analyse(*a.analyse)
    else:
        run(a)
