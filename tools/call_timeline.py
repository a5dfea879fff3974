"""Fill and drain of one pipelined call in a rocprofv3 kernel trace (the bench's timed region).

    python tools/call_timeline.py <run_kernel_trace.csv> [--launches 10] [--gap-us 150] [--out f.json]

Takes the last `--launches` k_accumulate dispatches of the largest grid (the timed call of `bench.py
--no-extras`, which is the last pipelined call of the run), walks back from the first of them to the
first kernel after a device-idle gap longer than `--gap-us` (the host's work between calls), and
reports for that call window [t0, t1]: its span, the kernels' busy union, the idle time inside it,
the fill (t0 -> first accumulation start), the drain (last accumulation end -> t1) with the kernels
that ran in it, and the accumulation starts' periods.  The span divided by the MSMs of the call is
the device's ms per MSM for that call; the bench's wall-clock ms_per_step adds the host's part.
"""
import argparse
import collections
import csv
import json
import statistics


def short(name):
    return name.replace("void msm::", "").split("(")[0].split("<")[0]


def union(ivs):
    tot, cur = 0, None
    for s, e in sorted(ivs):
        if cur is None or s > cur:
            tot += e - s
            cur = e
        elif e > cur:
            tot += e - cur
            cur = e
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--gap-us", type=float, default=150.0)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Grid_Size_X"]))
                for r in rows)
    acc = [x for x in ev if x[2] == "k_accumulate"]
    big = max(x[3] for x in acc)
    acc = [x for x in acc if x[3] == big][-a.launches:]
    first = acc[0][0]
    # walk back from the first accumulation to the call's first kernel
    i0 = max(i for i, x in enumerate(ev) if x[0] <= first)
    reach = ev[i0][1]
    t0 = ev[i0][0]
    j = i0 - 1
    while j >= 0:
        s, e = ev[j][0], ev[j][1]
        if e < t0 - a.gap_us * 1e3 and e < reach - a.gap_us * 1e3:
            break
        t0 = min(t0, s)
        j -= 1
    call = [x for x in ev if x[0] >= t0]
    t1 = max(x[1] for x in call)
    span = t1 - t0
    busy = union([(s, e) for s, e, _, _ in call])
    last_acc_end = acc[-1][1]
    drain = collections.defaultdict(float)
    for s, e, k, _ in call:
        if e > last_acc_end:
            drain[k] += (e - max(s, last_acc_end)) / 1e3
    fill = collections.defaultdict(float)
    for s, e, k, _ in call:
        if s < first:
            fill[k] += (min(e, first) - s) / 1e3
    starts = [x[0] for x in acc]
    periods = [(b - a_) / 1e3 for a_, b in zip(starts, starts[1:])]
    kern = collections.defaultdict(float)
    for s, e, k, _ in call:
        kern[k] += (e - s) / 1e3
    out = {
        "launches": len(acc), "acc_grid_threads": big,
        "span_us": round(span / 1e3, 1), "busy_union_us": round(busy / 1e3, 1),
        "idle_us": round((span - busy) / 1e3, 1),
        "fill_us": round((first - t0) / 1e3, 1), "fill_kernels_us": {k: round(v, 1) for k, v in fill.items()},
        "drain_us": round((t1 - last_acc_end) / 1e3, 1),
        "drain_kernels_us": {k: round(v, 1) for k, v in drain.items()},
        "acc_period_median_us": round(statistics.median(periods), 1) if periods else None,
        "acc_periods_us": [round(p, 1) for p in periods],
        "acc_durations_us": [round((e - s) / 1e3, 1) for s, e, _, _ in acc],
        "kernel_sum_us": {k: round(v, 1) for k, v in sorted(kern.items(), key=lambda kv: -kv[1])},
    }
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
