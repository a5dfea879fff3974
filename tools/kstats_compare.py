"""Side-by-side per-kernel mean durations (us) of rocprofv3 --stats runs (tuning tool).

    python tools/kstats_compare.py gpurun_out/<tag>_kstats1_<lib>_d ...
"""
import csv
import os
import sys

cols, names = [], []
for d in sys.argv[1:]:
    f = os.path.join(d, "run_kernel_stats.csv")
    m = {}
    for r in csv.DictReader(open(f)):
        k = r["Name"].replace("void msm::", "").split("(")[0]
        m[k] = float(r["AverageNs"]) / 1e3
    cols.append(m)
    n = os.path.basename(d.rstrip("/"))
    n = n.split("kstats1_")[-1].split("kstats_")[-1]
    names.append(n[:-2] if n.endswith("_d") else n)
keys = sorted({k for m in cols for k in m}, key=lambda k: -max(m.get(k, 0) for m in cols))
print("%-34s" % "kernel" + "".join("%14s" % n[-14:] for n in names))
for k in keys:
    if k.startswith("__amd"):
        continue
    print("%-34s" % k[:34] + "".join("%14.1f" % m[k] if k in m else "%14s" % "-" for m in cols))
print("%-34s" % "sum" + "".join("%14.1f" % sum(v for k, v in m.items() if not k.startswith("__amd")) for m in cols))
