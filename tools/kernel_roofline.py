"""Per-kernel roofline table of one launch shape: mean duration (rocprofv3 --stats of a run whose
launches all have that shape, e.g. MSM_SLOTS=1 bench.py --no-extras) against the PMC bytes of the
same plan (tools/profile_pmc.sh + tools/pmc_summary.py).

    python tools/kernel_roofline.py <run_kernel_stats.csv> <pmc summary.json> [--out f.json]

HBM bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE counts half
the bytes of 16-B/lane reads on gfx950), counted at the L2's fabric side (Infinity-Cache hits
included, so an upper bound on DRAM bytes); peak 8 TB/s.
"""
import argparse
import csv
import json

PEAK_GBS = 8000.0


def short(name):
    return name.replace("void msm::", "").replace("msm::", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("pmc")
    ap.add_argument("--out")
    a = ap.parse_args()
    dur = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(a.stats))}
    pmc = {r["kernel"]: r for r in json.load(open(a.pmc))["kernels"]}
    rows = []
    for k, ns in sorted(dur.items(), key=lambda kv: -kv[1]):
        p = pmc.get(k)
        if not p or "fillBuffer" in k:
            continue
        fetch = p.get("fetch_bytes", 0.0)
        write = p.get("write_bytes", 0.0)
        hbm = 2 * fetch + write
        gbs = hbm / ns  # bytes per ns = GB/s
        row = {"kernel": k, "us": round(ns / 1e3, 1), "hbm_MB": round(hbm / 1e6, 1), "GBps": round(gbs, 1),
               "frac_hbm": round(gbs / PEAK_GBS, 3)}
        if "valu_active_frac_of_wave_cycles" in p:
            row["valu_active_per_wave"] = p["valu_active_frac_of_wave_cycles"]
        if p.get("SQ_INSTS_LDS"):
            row["lds_bank_conflicts_per_lds_inst"] = round(p.get("SQ_LDS_BANK_CONFLICT", 0) / p["SQ_INSTS_LDS"], 2)
        rows.append(row)
    for r in rows:
        print(json.dumps(r))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
