#!/bin/bash
# Round-2 GPU session 10: host-split geometry A/B (slice size x MSMs per launch) for msm_compute e2e.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2l}
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 1 "gpurun_out/${TAG}_$name.txt" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for rep in 1 2; do
  run p17_auto_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_HOST_NM=1 run p17_nm1_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_HOST_PIECE_LOG=16 run p16_auto_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_HOST_PIECE_LOG=16 MSM_HOST_NM=1 run p16_nm1_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_HOST_SPLIT=0 run nosplit_$rep 120 python tools/e2e_probe.py --runs 8
done
