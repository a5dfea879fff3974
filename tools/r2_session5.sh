#!/bin/bash
# Round-2 GPU session 5: persistent-accumulate / part_scatter-LDS A/B (pipelined 2^20 and 2^17),
# correctness of the persistent kernel on the skew tests, the new bench line.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2g}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 1 "gpurun_out/${TAG}_$name.txt" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
run t_wpc3 300 env MSM_ACC_WPC=3 python -u -m pytest tests/test_gpu_msm.py -m gpu -q -x --timeout 120 --timeout-method thread -k "giant or skew or few or run_lengths or survey or sparse or pipelined"
for rep in 1 2; do
  run base_$rep 120 $B
  run wpc3_$rep 120 env MSM_ACC_WPC=3 $B
  run wpc2_$rep 120 env MSM_ACC_WPC=2 $B
  run ps512_$rep 120 env MSM_AMD_LIB=$L/libmsm_ps512.so $B
  run ps512_wpc3_$rep 120 env MSM_AMD_LIB=$L/libmsm_ps512.so MSM_ACC_WPC=3 $B
done
run base17 120 $B --n 131072
run wpc3_17 120 env MSM_ACC_WPC=3 $B --n 131072
run ps512_wpc3_17 120 env MSM_AMD_LIB=$L/libmsm_ps512.so MSM_ACC_WPC=3 $B --n 131072
run bench 300 python bench.py
