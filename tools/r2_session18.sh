#!/bin/bash
# Round-2 GPU session 18: host path with three slots, rocprofv3 summary of the default bench
# command, and a two-rank rehearsal of the sharded bench (gloo, both ranks on the one GPU).
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2u}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"e2e_ms": \[[^]]*\|passed.*\|failed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 600 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread
run e2e_1 120 python tools/e2e_probe.py --runs 8
run e2e_2 120 python tools/e2e_probe.py --runs 8
run kstats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kstats -o run -- python3 bench.py
MSM_DIST_BACKEND=gloo run dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --no-cpu-baseline
MSM_DIST_BACKEND=gloo run dist2b 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --batch 16 --points 262144
