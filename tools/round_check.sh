#!/bin/bash
# GPU tests, default bench, prover-batch bench, and a 2-rank gloo rehearsal of the sharded bench.
set -u
mkdir -p gpurun_out
run() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 3 "gpurun_out/$name.txt" | cut -c1-600 >&2
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
}
run pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
run bench 300 python bench.py
run bench_batch 300 python bench.py --batch 64 --n 262144 --steps 5 --warmup 1
MSM_DIST_BACKEND=gloo run bench_gloo2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
