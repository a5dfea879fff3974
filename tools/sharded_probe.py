"""msm_compute's device-list path from host arrays, rehearsed on one GPU (the test hook
msm_test_sharded repeats device 0 D times: D shards, one host thread each, their contexts' pools
sized for a D-device call -- which on one device run one after another).  Median of `runs` calls
per D, each checked against its closed form, beside the pool sizes a D-device call uses.

    python tools/sharded_probe.py [--n 1048576] [--runs 7] [--shards 1,2,8]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "webgpu-msm_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--runs", type=int, default=7)
    ap.add_argument("--shards", default="1,2,8")
    args = ap.parse_args()
    import msm_amd as M
    from _closed_form import closed_form

    L = M.load()
    pts = M.gen_points(args.n, k0=1, step=1)
    sc = M.gen_scalars(args.n, seed=4242)
    exp = closed_form(1, 1, sc)
    out = {"n": args.n, "runs": args.runs, "shards": {}}
    for D in (int(x) for x in args.shards.split(",")):
        pools = (ctypes.c_int * 5)()
        L.msm_test_pools(D, 0, pools)
        M._test_sharded(0, pts, sc, args.n, [0] * D)  # warm-up (contexts, pools, graphs)
        ts, ok = [], True
        for _ in range(args.runs):
            t0 = time.perf_counter()
            r = M._test_sharded(0, pts, sc, args.n, [0] * D)
            ts.append((time.perf_counter() - t0) * 1e3)
            ok = ok and tuple(r) == tuple(exp)
        out["shards"][str(D)] = {"e2e_ms_median": round(float(np.median(ts)), 3), "e2e_ms_min": round(min(ts), 3),
                                 "correct": ok, "cpu_budget": pools[0], "pack_threads": pools[1],
                                 "tail_helpers": pools[2], "horner_threads": pools[3], "library_threads": pools[4]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
