"""k_accumulate's own launch duration for library variants, results unchecked (for variants that
skip work on purpose: they bound what a change of that work could save).

    python tools/acc_probe.py [--libs libmsm.so,libmsm_x.so] [--rounds 3] [--n 1048576]

For each library (files under webgpu-msm_amd/msm_amd/_lib, one subprocess each, interleaved over
the rounds) it runs bench.py's serial pass: two-MSM pipelined-plan launches one at a time on one
stream for >= 1.5 s, each k_accumulate bracketed by the graph's event nodes (profiling mode 2), and
prints one JSON line per run: the mean bracket in ms (bench.py's roofline.kernel_ms).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "webgpu-msm_amd", "msm_amd", "_lib")

CHILD = r"""
import sys, time, json
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/webgpu-msm_amd"]
import numpy as np, torch
import msm_amd as M
n = int(sys.argv[2])
dev = torch.device("cuda", 0)
pts = torch.from_numpy(M.gen_points(n).view(np.int32)).to(dev)
sc = [torch.from_numpy(M.gen_scalars(n, seed=M.XORSHIFT_SEED + j).view(np.int32)).to(dev) for j in range(4)]
js = [j % 4 for j in range(8)]
M.compute_msm_many_device([pts] * 8, [sc[j] for j in js], n)  # warm-up
M.set_profiling(2)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.5:
    M.compute_msm_many_device([pts] * 8, [sc[j] for j in js], n, flags=M.MSM_FLAG_SERIAL)
p = M.last_profile()
M.set_profiling(False)
print(json.dumps({"kernel_ms": round(float(p["accumulate_sum"]) / max(1, int(p["profiled"])), 4),
                  "launches": int(p["profiled"])}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="libmsm.so")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 20)
    a = ap.parse_args()
    for r in range(a.rounds):
        for lib in a.libs.split(","):
            env = dict(os.environ, MSM_AMD_LIB=os.path.join(LIBDIR, lib))
            out = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(a.n)], env=env, capture_output=True, text=True,
                                 timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                raise SystemExit(f"{lib}: rc {out.returncode}")
            line = json.loads(out.stdout.strip().splitlines()[-1])
            print(json.dumps({"lib": lib, "round": r + 1, "n": a.n, **line}), flush=True)


if __name__ == "__main__":
    main()
