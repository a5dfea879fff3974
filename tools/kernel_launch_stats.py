"""Per-launch-shape duration summary of one kernel in a rocprofv3 kernel trace.

    python tools/kernel_launch_stats.py <run_kernel_trace.csv> [--kernel k_accumulate] [--out f.json]

rocprofv3 --stats averages a kernel over every dispatch of the run, and bench.py dispatches
k_accumulate with several grid sizes (two-MSM launches of the timed region and of the serial
pass, single-MSM launches of the latency pass, the 2^17-point slices of the host-input pass).
This groups the dispatches by grid size and, within a grid size, by whether another kernel
overlapped them on the device (a timed-region launch shares the GPU with the other slot's
kernels; a serial-pass launch runs alone), so a figure can be compared with the bench line's
roofline.kernel_ms (the serial pass's two-MSM launches).
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_accumulate")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in rows)
    mine = [(s, e, r) for s, e, r in iv if r["Kernel_Name"].split("(")[0] == a.kernel]
    groups = collections.defaultdict(list)
    for s, e, r in mine:
        # overlapped if any other dispatch on another queue runs for > 5% of this one's span
        ov = 0
        for s2, e2, r2 in iv:
            if s2 >= e:
                break
            if r2 is r or r2["Queue_Id"] == r["Queue_Id"] or e2 <= s:
                continue
            ov += min(e, e2) - max(s, s2)
        alone = ov < 0.05 * (e - s)
        groups[(int(r["Grid_Size_X"]), alone)].append((e - s) / 1e3)
    out = []
    for (grid, alone), d in sorted(groups.items(), key=lambda kv: (-kv[0][0], not kv[0][1])):
        d.sort()
        out.append({"kernel": a.kernel, "grid_threads": grid, "workgroups": grid // int(mine[0][2]["Workgroup_Size_X"]),
                    "alone": alone, "launches": len(d), "mean_us": round(sum(d) / len(d), 1),
                    "median_us": round(d[len(d) // 2], 1), "min_us": round(d[0], 1), "max_us": round(d[-1], 1)})
    for o in out:
        print(json.dumps(o))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
