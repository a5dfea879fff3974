#!/bin/bash
# Per-kernel durations (rocprofv3 kernel trace, one stream) for each library variant.
#   bash tools/kprof_ab.sh libmsm_a.so,libmsm_b.so [logn]
# Writes gpurun_out/kp_<lib>/run_kernel_stats.csv and prints a compact table.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
logn=${2:-20}
for lib in ${1//,/ }; do
  tag=${lib%.so}
  echo "== $tag" >&2
  MSM_SLOTS=1 MSM_AMD_LIB=$PWD/webgpu-msm_amd/msm_amd/_lib/$lib timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/kp_$tag" -o run -- \
    python tools/sweep.py --worker --windows 16 --runs 0 --logn "$logn" --steps 10 > "gpurun_out/kp_$tag.txt" 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "ABORT $tag rc=$rc" >&2; tail -5 "gpurun_out/kp_$tag.txt" >&2; exit $rc; }
  python3 - "gpurun_out/kp_$tag/run_kernel_stats.csv" <<'EOF' >&2
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].replace("void msm::", "").split("(")[0].split("<")[0]
    print(f"  {name:24s} {float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']}")
EOF
done
