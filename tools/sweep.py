"""Parameter / library-variant sweep on the GPU box (tuning tool, not part of the product).

    python tools/sweep.py [--libs libmsm.so,libmsm_b.so] [--windows 15,16,17] [--runs 16,32,64]
                          [--logn 20] [--steps 10]

Each library variant runs in its own process (MSM_AMD_LIB); inside, every (window, run length)
pair is timed over `steps` MSMs on device-resident inputs and checked against the closed form.
Prints one JSON line per configuration.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "webgpu-msm_amd", "msm_amd", "_lib")
for p in (ROOT, os.path.join(ROOT, "webgpu-msm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def ints(s):
    return [int(x) for x in s.split(",") if x]


def worker(args):
    import numpy as np
    import torch

    import msm_amd as M
    from bench import EXPECTED

    n = 1 << args.logn
    dev = torch.device("cuda", 0)
    pts = torch.from_numpy(M.gen_points(n).view(np.int32)).to(dev)
    sc = torch.from_numpy(M.gen_scalars(n).view(np.int32)).to(dev)
    torch.cuda.synchronize()
    lib = os.path.basename(M.lib_path())
    for c in args.windows:
        for k in args.runs:
            res = M.compute_msm_device(pts, sc, n, window_size=c, run_length=k)
            M.set_profiling(2)
            prof = []
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                res = M.compute_msm_device(pts, sc, n, window_size=c, run_length=k)
                prof.append(M.last_profile())
            dt = (time.perf_counter() - t0) / args.steps
            M.set_profiling(1)
            M.compute_msm_device(pts, sc, n, window_size=c, run_length=k)
            ph1 = M.last_profile()
            M.set_profiling(False)
            keys = [k2 for k2 in ph1 if isinstance(ph1[k2], float)]
            ph = {k2: round(float(ph1[k2]), 4) for k2 in keys}
            acc = round(float(np.mean([p["accumulate"] for p in prof])), 4)
            dev = round(float(np.mean([p["device_total"] for p in prof])), 4)
            print(json.dumps({"lib": lib, "n": n, "c": c, "K": k, "ms": round(dt * 1e3, 4), "acc_graph": acc,
                              "dev_graph": dev, "ok": res == EXPECTED.get(n, res), "phases": ph}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="libmsm.so")
    ap.add_argument("--windows", type=ints, default=[16])
    ap.add_argument("--runs", type=ints, default=[32])
    ap.add_argument("--logn", type=int, default=20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--worker", action="store_true")
    args = ap.parse_args()
    if args.worker:
        worker(args)
        return
    rc = 0
    for lib in args.libs.split(","):
        env = dict(os.environ, MSM_AMD_LIB=os.path.join(LIBDIR, lib))
        cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--windows",
               ",".join(map(str, args.windows)), "--runs", ",".join(map(str, args.runs)),
               "--logn", str(args.logn), "--steps", str(args.steps)]
        r = subprocess.run(cmd, env=env)
        if r.returncode != 0:
            print(f"variant {lib} failed rc={r.returncode}", file=sys.stderr)
            rc = r.returncode
            if rc < 0 or rc > 1:
                break
    sys.exit(rc)


if __name__ == "__main__":
    main()
