"""Phase timing of the sort kernels (tuning tool; needs a -DMSM_PHASE_PROBE=1 library variant).

Runs the pipelined two-MSM 2^20 launch a few times (one stream: run with MSM_SLOTS=1), dumps the
last launch's per-workgroup phase stamps (msm_test_probe_dump) and prints, per kernel, the
launch span, the workgroups' mean lifetime, how many were resident on average, and each phase's
median / p90 duration.

    MSM_SLOTS=1 MSM_AMD_LIB=.../libmsm_probe.so python tools/phase_probe.py [--n 1048576]
    (one 8-GPU share: --n 262144 --count 4 --window 15 --split-q 2 --wrange 0)
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "webgpu-msm_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

KERNELS = {0: ("k_recode_hist", {1: "zero", 2: "recode", 7: "flush"}),
           1: ("k_part_scatter", {1: "load", 2: "rank", 3: "reserve", 4: "scan", 5: "stage", 6: "store"}),
           2: ("k_fine_sort", {1: "head", 2: "load", 3: "rank", 4: "scan", 5: "bounds", 6: "stage", 7: "store"}),
           3: ("k_accumulate", {7: "all"})}
WG, SLOTS = 16384, 10


def analyse(raw):
    a = raw.reshape(4, WG, SLOTS).astype(np.int64)
    out = {}
    for k, (name, phases) in KERNELS.items():
        live = a[k][a[k][:, 8] != 0]
        if len(live) == 0:
            continue
        rt0, rt1 = live[:, 8], live[:, 9]
        span_us = (rt1.max() - rt0.min()) / 100.0
        life_us = (rt1 - rt0) / 100.0
        cyc = (live[:, 7] - live[:, 0]).astype(np.float64)
        ghz = float(np.median(cyc / np.maximum(life_us, 1e-3) / 1e3))
        rec = {"workgroups": int(len(live)), "span_us": round(float(span_us), 2),
               "life_us_mean": round(float(life_us.mean()), 3), "life_us_p90": round(float(np.percentile(life_us, 90)), 3),
               "life_us_pct": {str(q): round(float(np.percentile(life_us, q)), 2) for q in (1, 10, 50, 90, 99, 100)},
               "end_us_pct": {str(q): round(float(np.percentile((rt1 - rt0.min()) / 100.0, q)), 2)
                              for q in (1, 10, 50, 90, 99, 100)},
               "resident_mean": round(float(life_us.sum() / span_us), 1), "clock_ghz": round(ghz, 3), "phases": {}}
        prev = 0
        for s in sorted(phases):
            d = (live[:, s] - live[:, prev]) / (ghz * 1e3)
            ok = live[:, s] != 0
            rec["phases"][phases[s]] = {"median_us": round(float(np.median(d[ok])), 3),
                                        "p90_us": round(float(np.percentile(d[ok], 90)), 3),
                                        "mean_us": round(float(d[ok].mean()), 3)}
            prev = s
        # start times: how the launch fills (first / median / last start after the first)
        st = (rt0 - rt0.min()) / 100.0
        rec["start_us"] = {"p50": round(float(np.median(st)), 2), "p90": round(float(np.percentile(st, 90)), 2),
                           "max": round(float(st.max()), 2)}
        out[name] = rec
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--count", type=int, default=2)
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--out", default="gpurun_out/phase_probe.bin")
    ap.add_argument("--window", type=int, default=0, help="window width (0: the plan's)")
    ap.add_argument("--split-q", type=int, default=0,
                    help="run one share of a points x Q window split: Q window ranges at half windows")
    ap.add_argument("--wrange", type=int, default=0, help="which of the Q window ranges (with --split-q)")
    args = ap.parse_args()
    import torch

    import msm_amd as M

    L = M.load()
    L.msm_test_probe_dump.argtypes = [ctypes.c_char_p]
    dev = torch.device("cuda", 0)
    pts = [torch.from_numpy(M.gen_points(args.n).view(np.int32)).to(dev) for _ in range(1)] * args.count
    scs = [torch.from_numpy(M.gen_scalars(args.n, seed=17 + i).view(np.int32)).to(dev) for i in range(args.count)]
    torch.cuda.synchronize()
    if args.split_q:
        from msm_amd.dist import SPLIT_HALF_WINDOWS, window_ranges
        r = window_ranges(M.window_count(args.window), args.split_q, SPLIT_HALF_WINDOWS)[args.wrange]
        for _ in range(args.runs):
            M.compute_msm_many_device_partial(pts, scs, args.n, window_size=args.window or None, windows=r)
    else:
        for _ in range(args.runs):
            M.compute_msm_many_device(pts, scs, args.n, window_size=args.window or None)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    rc = L.msm_test_probe_dump(args.out.encode())
    assert rc == 0, rc
    raw = np.fromfile(args.out, dtype=np.uint64)
    res = analyse(raw)
    res["lib"] = os.path.basename(M.lib_path())
    res["n"] = args.n
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
