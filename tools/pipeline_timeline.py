"""Steady-state shape of the pipelined launches in a rocprofv3 kernel trace of bench.py.

    python tools/pipeline_timeline.py <run_kernel_trace.csv> [--out f.json]

Takes the k_accumulate dispatches of the largest grid (the timed region's multi-MSM launches and
the serial pass's), keeps consecutive pairs less than 5 ms apart, and for each period between two
accumulation starts reports: the period, the accumulation's own span, the gap from one
accumulation's end to the next one's start, the time no kernel ran, and how long each other
kernel ran inside the period and how much of that beside an accumulation.  Medians over the
periods; the period is the device's time per launch (ms per MSM = period / MSMs per launch).
"""
import argparse
import collections
import csv
import json
import statistics


def short(name):
    return name.replace("void msm::", "").split("(")[0].split("<")[0]


def covered(ivs, lo, hi):
    """Length of [lo, hi) covered by the union of the intervals."""
    tot, cur = 0, lo
    for s, e in sorted(ivs):
        s, e = max(s, cur), min(e, hi)
        if e > s:
            tot += e - s
            cur = e
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Grid_Size_X"]))
                for r in rows)
    acc = [x for x in ev if x[2] == "k_accumulate"]
    big = max(x[3] for x in acc)
    acc = [x for x in acc if x[3] == big]
    per = collections.defaultdict(list)
    for (s0, e0, _, _), (s1, _, _, _) in zip(acc, acc[1:]):
        if s1 - s0 > 5_000_000:
            continue
        inside = [(max(s, s0), min(e, s1), k) for s, e, k, _ in ev if e > s0 and s < s1]
        per["period_us"].append((s1 - s0) / 1e3)
        per["acc_us"].append((e0 - s0) / 1e3)
        per["acc_end_to_next_start_us"].append((s1 - e0) / 1e3)
        per["idle_us"].append((s1 - s0 - covered([(s, e) for s, e, _ in inside], s0, s1)) / 1e3)
        by = collections.defaultdict(list)
        for s, e, k in inside:
            by[k].append((s, e))
        acc_iv = [(s, e) for s, e, k in inside if k == "k_accumulate"]
        for k, ivs in by.items():
            if k == "k_accumulate":
                continue
            per[k + "_us"].append(covered(ivs, s0, s1) / 1e3)
            per[k + "_beside_acc_us"].append(sum(covered(acc_iv, s, e) for s, e in ivs) / 1e3)
    n = len(per["period_us"])
    out = {"periods": n, "acc_grid_threads": big}
    for k, v in per.items():
        v = v + [0.0] * (n - len(v))  # a kernel missing from some periods ran 0 us there
        out[k] = round(statistics.median(v), 1)
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
