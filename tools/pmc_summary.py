"""Summarise tools/profile_pmc.sh output: per-kernel mean of every collected counter, derived
clock / VALU-busy / HBM bytes.  Usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [n_points]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.split("(")[0]
    return name.replace("void msm::", "").replace("msm::", "")


def load(d):
    vals = defaultdict(lambda: defaultdict(list))
    grids = defaultdict(dict)  # kernel -> counter -> [(dispatch grid size, summed value)]
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", row.get("Kernel-Name", "?")))
                c = row.get("Counter_Name", row.get("Counter-Name"))
                v = float(row.get("Counter_Value", row.get("Counter-Value", "nan")))
                disp = row.get("Dispatch_Id", row.get("Dispatch-Id"))
                vals[k][c].append((disp, v))
                grids[k][(c, disp)] = float(row.get("Grid_Size", "nan"))
    out = {}
    for k, cs in vals.items():
        out[k] = {}
        for c, lst in cs.items():
            per = defaultdict(float)
            for disp, v in lst:  # counters may be reported per XCD / instance: sum per dispatch
                per[disp] += v
            xs = list(per.values())
            out[k][c] = sum(xs) / len(xs)
            # per unit of the smallest launch (one MSM): launches carrying a batch of MSMs have
            # proportionally larger grids
            g = {disp: grids[k][(c, disp)] for disp in per}
            gmin = min(g.values())
            units = sum(gv / gmin for gv in g.values())
            out[k][c + "_per_unit"] = sum(xs) / units if units else float("nan")
    return out


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else None
    s = load(d)
    rows = []
    for k, cs in sorted(s.items()):
        r = {"kernel": k, **{c: round(v, 1) for c, v in cs.items()}}
        if "FETCH_SIZE" in cs:
            r["fetch_bytes"] = cs["FETCH_SIZE"] * 1024
            r["fetch_bytes_x2_gfx950"] = cs["FETCH_SIZE"] * 2048
        if "WRITE_SIZE" in cs:
            r["write_bytes"] = cs["WRITE_SIZE"] * 1024
        if "SQ_ACTIVE_INST_VALU" in cs and "SQ_WAVE_CYCLES" in cs and cs["SQ_WAVE_CYCLES"]:
            r["valu_active_frac_of_wave_cycles"] = round(cs["SQ_ACTIVE_INST_VALU"] / cs["SQ_WAVE_CYCLES"], 3)
        if "SQ_WAIT_ANY" in cs and "SQ_WAVE_CYCLES" in cs and cs["SQ_WAVE_CYCLES"]:
            r["wait_any_frac"] = round(cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"], 3)
            r["wait_inst_frac"] = round(cs.get("SQ_WAIT_INST_ANY", 0) / cs["SQ_WAVE_CYCLES"], 3)
        rows.append(r)
    acc = s.get("k_accumulate")
    tr = None
    if acc and n:
        fetch = acc.get("FETCH_SIZE_per_unit", 0) * 1024
        write = acc.get("WRITE_SIZE_per_unit", 0) * 1024
        tr = {"n": n, "kernel": "k_accumulate", "source": os.path.basename(os.path.normpath(d)),
              "accumulate_fetch_size_bytes_per_msm": fetch,
              "accumulate_write_bytes_per_msm": write,
              "accumulate_hbm_bytes_per_msm": 2 * fetch + write,
              "note": "2 x FETCH_SIZE + WRITE_SIZE of k_accumulate per MSM (separate rocprofv3 --pmc passes; "
                      "a launch carrying a batch of MSMs is counted per MSM by its grid size). FETCH_SIZE is "
                      "doubled as MI355X_MICROARCH.md prescribes for 16-B/lane reads on gfx950 (the kernel "
                      "gathers 108 B of each 128-B point record, mostly with 16-B/lane loads). Counted at the L2's fabric side: "
                      "includes Infinity-Cache hits (the 128 MiB point table stays resident in the 256 MiB "
                      "Infinity Cache), so it is an upper bound on HBM bytes."}
    print(json.dumps({"kernels": rows, "traffic": tr}, indent=1))
    if tr and len(sys.argv) > 3:  # traffic file read by bench.py
        with open(sys.argv[3], "w") as f:
            json.dump(tr, f)


if __name__ == "__main__":
    main()
