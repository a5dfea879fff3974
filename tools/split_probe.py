"""How to cut one 2^20-point MSM over D GPUs: the per-GPU work of every (points x windows) split,
measured on ONE GPU.

    python tools/split_probe.py [--n 1048576] [--gpus 8] [--steps 40] [--window 16]

A split P x Q (P * Q = D) gives GPU (p, q) the p-th contiguous 1/P of the points and the q-th of Q
window ranges (msm_opts MSM_FLAG_WINDOWS; contiguous ranges of the msm_window_count(c) windows,
balanced by main-window count, the overflow window with the top range; cut at half windows,
MSM_FLAG_HALF_WINDOWS, unless --whole-windows).  For each split this
runs every one of the D virtual GPUs' work in turn on the one GPU -- K pipelined MSMs of its shard
and range through msm_compute_many_device_partial, device-resident inputs, exactly what that GPU
would run -- times each (wall, K MSMs, after a warm-up), and joins all D x K partials on the host:
every step's joined result is checked against its closed form.  The split's per-GPU time is the
slowest virtual GPU's ms per MSM (the job waits for it).  P x 1 is today's point sharding.
Prints one JSON line per split and a summary line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "webgpu-msm_amd")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--window", type=int, default=0, help="window width for the window-split runs (0: 16)")
    ap.add_argument("--splits", default="", help="comma-separated PxQ (default: every factorisation of --gpus)")
    ap.add_argument("--run-length", type=int, default=0, help="accumulation run length K (0: the plan's)")
    ap.add_argument("--whole-windows", action="store_true",
                    help="cut the window ranges at whole windows (default: half windows, as split_part)")
    a = ap.parse_args()
    import torch

    import msm_amd as M
    from msm_amd.dist import SPLIT_HALF_WINDOWS, shard_range, window_ranges

    D, n, K = a.gpus, a.n, a.steps
    with open(os.path.join(ROOT, "tests", "golden", "bench_expected.json")) as f:
        rows = json.load(f)["rows"]
    sets = 4
    exp = [tuple(map(int, rows[f"{n}:{j}"])) if f"{n}:{j}" in rows else None for j in range(sets)]
    full = [M.gen_scalars(n, seed=M.XORSHIFT_SEED + j) for j in range(sets)]
    splits = ([tuple(map(int, s.split("x"))) for s in a.splits.split(",")] if a.splits else
              [(p, D // p) for p in range(D, 0, -1) if D % p == 0])
    dev = torch.device("cuda", 0)
    summary = {}
    for P, Q in splits:
        c = a.window or (16 if Q > 1 else 0)  # point shards alone keep the tuned (pipelined) width
        wm = M.window_count(c) if c else None
        ranges = window_ranges(wm, Q, SPLIT_HALF_WINDOWS and not a.whole_windows) if Q > 1 else [None]
        per_gpu, parts = [], []
        js = [s % sets for s in range(K)]
        for p in range(P):
            lo, hi = shard_range(n, p, P)
            d_pts = torch.from_numpy(M.gen_points(hi - lo, k0=lo + 1).view(np.int32)).to(dev)
            d_sc = [torch.from_numpy(np.ascontiguousarray(s[lo:hi]).view(np.int32)).to(dev) for s in full]
            torch.cuda.synchronize()
            for r in ranges:
                run = lambda k: M.compute_msm_many_device_partial(  # noqa: E731
                    [d_pts] * k, [d_sc[j] for j in js[:k]], hi - lo, window_size=c or None, windows=r,
                    run_length=a.run_length or None)
                run(a.warmup)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                out = run(K)
                dt = time.perf_counter() - t0
                per_gpu.append({"points": [lo, hi], "windows": list(r) if r else None,
                                "ms_per_msm": round(dt * 1e3 / K, 4)})
                parts.append(out)
            del d_pts, d_sc
        joined = M.combine_partials_many(np.stack(parts))
        ok = all(e is None or g == e for g, e in zip(joined, [exp[j] for j in js]))
        worst = max(g["ms_per_msm"] for g in per_gpu)
        line = {"split": f"{P}x{Q}", "gpus": D, "n": n, "window_bits": c or "auto", "steps": K,
                "run_length": a.run_length or "plan",
                "per_gpu_ms_per_msm_max": worst,
                "per_gpu_ms_per_msm_mean": round(float(np.mean([g["ms_per_msm"] for g in per_gpu])), 4),
                "correct": ok, "virtual_gpus": per_gpu}
        print(json.dumps(line), flush=True)
        summary[f"{P}x{Q}"] = worst
        if not ok:
            raise SystemExit(f"split {P}x{Q}: joined result mismatch")
    print(json.dumps({"summary_ms_per_msm_slowest_gpu": summary,
                      "best": min(summary, key=summary.get)}), flush=True)


if __name__ == "__main__":
    main()
