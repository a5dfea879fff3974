"""Copy/kernel timeline of host-array msm_compute calls from a rocprofv3 kernel + memory-copy trace
(tools/gpu_session.sh e2etrace):

    python tools/e2e_timeline.py gpurun_out/<tag>_e2etrace_d [--call 3]

Calls are separated by device-idle gaps (no copy or kernel running) > --gap us.  Per call: every copy
and kernel (start, end, duration, relative to the call's first copy), the upload span, the gaps
between consecutive copies, and what runs after the last copy.
"""
import argparse
import csv
import os

ap = argparse.ArgumentParser()
ap.add_argument("d")
ap.add_argument("--call", type=int, default=-2, help="which call (python index) to print in full")
ap.add_argument("--gap", type=float, default=150.0, help="device-idle gap (us) that separates calls")
a = ap.parse_args()
cp = list(csv.DictReader(open(os.path.join(a.d, "run_memory_copy_trace.csv"))))
kn = list(csv.DictReader(open(os.path.join(a.d, "run_kernel_trace.csv"))))
ev = [("copy:" + r["Direction"].replace("MEMORY_COPY_", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s" + r["Stream_Id"])
      for r in cp]
ev += [(r["Kernel_Name"].replace("void msm::", "").split("(")[0].split("<")[0][:22], int(r["Start_Timestamp"]),
        int(r["End_Timestamp"]), "q" + r["Queue_Id"]) for r in kn if "fillBuffer" not in r["Kernel_Name"]]
ev.sort(key=lambda e: e[1])
calls, cur, last = [], [], None
for e in ev:
    if last is not None and e[1] - last > a.gap * 1e3:
        calls.append(cur)
        cur = []
    cur.append(e)
    last = max(last or 0, e[2])
calls.append(cur)
print(f"{len(calls)} calls")
for ci, c in enumerate(calls):
    t0 = c[0][1]
    copies = [e for e in c if e[0].startswith("copy")]
    end = max(e[2] for e in c)
    if not copies:
        continue
    up = max(e[2] for e in copies)
    kbusy = sum(e[2] - e[1] for e in c if not e[0].startswith("copy"))
    cbusy = sum(e[2] - e[1] for e in copies)
    cs = sorted(copies, key=lambda e: e[1])
    gaps = [(cs[i + 1][1] - cs[i][2]) / 1e3 for i in range(len(cs) - 1)]
    print(f"call {ci}: span {(end - t0) / 1e3:8.1f} us, copies {len(copies)} busy {cbusy / 1e3:8.1f} us "
          f"(gaps {sum(gaps):6.1f} us: {' '.join(f'{g:.0f}' for g in gaps)}), upload ends {(up - t0) / 1e3:8.1f} us, "
          f"after upload {(end - up) / 1e3:7.1f} us, kernels busy {kbusy / 1e3:8.1f}")
c = calls[a.call]
t0 = c[0][1]
for name, s, e, q in c:
    print(f"{q:>4} {name:26s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}")
