#!/bin/bash
# Round-2 GPU session 27: k_bucket_reduce_1 software-pipelined running sums (two independent adds
# per step) vs sequential; with and without amdgpu_waves_per_eu(1, 1).
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ae}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|passed.*\|failed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 600 python -u -m pytest tests/test_gpu_msm.py -m gpu -x -q --timeout 300 --timeout-method thread
for lib in libmsm libmsm_ilp1w1 libmsm_ilp0; do
  for lg in 17 20; do
    MSM_AMD_LIB=$L/$lib.so MSM_SLOTS=1 run ks_${lib}_$lg 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ks_${lib}_$lg -o run -- python3 bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 4 --serial-min-s 0 --n $((1 << lg))
  done
done
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  for lib in libmsm libmsm_ilp0; do
    for lg in 17 20; do MSM_AMD_LIB=$L/$lib.so run ${lib}_${lg}_$rep 120 $B --n $((1 << lg)); done
  done
done
