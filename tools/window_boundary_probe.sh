# Pipelined device-resident ms per MSM just below the window thresholds of pipelined_window (msm_host.hip),
# each with the two candidate widths.  Run on the GPU box: bash tools/window_boundary_probe.sh
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
for spec in ${SPECS:-393216:15 393216:16 524287:15 524287:16 98304:14 98304:15 131071:14 131071:15}; do
  n=${spec%%:*}; c=${spec#*:}
  v=$(timeout -k 10 120 python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline --n $n --window $c | grep '^{"metric"' | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')
  echo "{\"n\": $n, \"window\": $c, \"round\": $r, \"ms_per_msm\": $v}" | tee -a gpurun_out/${TAG:-winb}.jsonl
done
done
