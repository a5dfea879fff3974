"""Timeline analysis of a rocprofv3 kernel trace (tuning tool): per-queue kernel sequence of a
window of the run, and how much of the time each kernel overlaps others.

    python tools/timeline.py gpurun_out/kstats_X/run_kernel_trace.csv [--skip 200] [--count 60]
"""
import csv
import sys
import argparse

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--skip", type=int, default=300)
ap.add_argument("--count", type=int, default=70)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows = [r for r in rows if "fillBuffer" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = rows[a.skip:a.skip + a.count]
t0 = int(sel[0]["Start_Timestamp"])
short = lambda n: n.replace("void msm::", "").split("<")[0].split("(")[0][:18]
for r in sel:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"q{r['Queue_Id']:>2} {short(r['Kernel_Name']):18s} {s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:8.1f}")
# busy-time union vs sum
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
union, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
print(f"span {span/1e6:.3f} ms, busy union {union/1e6:.3f} ms, idle {(span-union)/1e6:.3f} ms")
