"""Print a window of a rocprofv3 kernel trace, or the k_accumulate durations over a whole run.

    python tools/trace_window.py <run_kernel_trace.csv> --acc-index 23 --before-us 1500 --len-us 9000
    python tools/trace_window.py <run_kernel_trace.csv> --acc-series [--out f.json]

The first form lists every kernel that starts inside [t, t + len) with t the start of the
--acc-index-th k_accumulate of the largest grid minus --before-us: start, end and length (us,
relative to t), the kernel, and its hardware queue and HIP stream -- what showed a slot's
reduction and the next launch's sort starved beside the other slot's accumulation
(profiles/r5/pipeline_gap.txt).  The second prints each k_accumulate's start (ms from the first
kernel of the run) and duration, in groups of 8: the device speeding up over a run's first
~130 ms (profiles/r5/clock_ramp.json).
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--acc-index", type=int, default=20)
    ap.add_argument("--before-us", type=float, default=1500.0)
    ap.add_argument("--len-us", type=float, default=9000.0)
    ap.add_argument("--acc-series", action="store_true")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].replace("void msm::", "").split("(")[0], r["Queue_Id"], r["Stream_Id"],
                 int(r["Grid_Size_X"])) for r in rows)
    acc = [x for x in ev if x[2] == "k_accumulate"]
    if a.acc_series:
        t0 = ev[0][0]
        out = {"t0": "first kernel of the run", "groups": []}
        for i in range(0, len(acc), 8):
            seg = acc[i:i + 8]
            out["groups"].append({"first_index": i, "start_ms": round((seg[0][0] - t0) / 1e6, 1),
                                  "durations_us": [round((e - s) / 1e3) for s, e, *_ in seg],
                                  "grid": [g for *_, g in seg]})
        text = json.dumps(out, indent=1)
        print(text)
        if a.out:
            with open(a.out, "w") as f:
                f.write(text + "\n")
        return
    big = max(x[5] for x in acc)
    acc = [x for x in acc if x[5] == big]
    t0 = acc[a.acc_index][0] - int(a.before_us * 1e3)
    lines = [f"{'start':>8} {'end':>8} {'us':>7}  kernel             queue stream"]
    for s, e, k, q, st, _ in ev:
        if t0 <= s < t0 + a.len_us * 1e3:
            lines.append(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {k:18s} q{q:<4} s{st}")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
