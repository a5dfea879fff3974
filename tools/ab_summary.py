"""Condense gpu_session.sh A/B outputs into JSON lines (tuning tool): one line per run with the
figures DESIGN.md quotes.  Bench runs (a JSON line from bench.py) give value / kernel_ms /
latency / frac_isa_measured; latency-probe runs give the lone-MSM latency figures.

    python tools/ab_summary.py gpurun_out/r3a_ab_*.txt > profiles/r3/ab_wide_digits.jsonl
"""
import json
import os
import re
import sys


def last_json(path):
    line = None
    with open(path, errors="replace") as f:
        for ln in f:
            if ln.startswith("{"):
                line = ln
    return json.loads(line) if line else None


def main():
    for path in sys.argv[1:]:
        d = last_json(path)
        name = os.path.basename(path)
        m = re.match(r"(r\d+\w?)_(.*?)(?:_(\d+))?\.txt$", name)
        row = {"session": m.group(1) if m else None, "run": m.group(2) if m else name,
               "round": int(m.group(3)) if m and m.group(3) else None}
        if d is None:
            row["error"] = "no result line"
        elif "latency_ms_median" in d:
            for k in ("latency_ms_median", "latency_ms_min", "latency_ms_p90", "host_tail_ms_median",
                      "accumulate_ms_median", "run_length", "correct"):
                row[k] = d.get(k)
        else:
            r = d.get("roofline", {})
            c = r.get("compute_roofline") or d.get("compute_roofline") or {}
            row.update(value=d.get("value"), kernel_ms=r.get("kernel_ms"), latency_ms=d.get("latency_ms"),
                       frac_isa_measured=c.get("frac_isa_measured"),
                       instructions=c.get("isa_instructions_per_entry_wave"))
        print(json.dumps(row))


if __name__ == "__main__":
    main()
