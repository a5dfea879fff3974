set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for k in 0 128; do
    timeout -k 10 180 python bench.py --steps 40 --warmup 10 --no-extras --no-cpu-baseline --run-length $k > gpurun_out/u06_k${k}_$r.txt 2>&1 || { echo "FAIL k=$k r=$r"; tail -5 gpurun_out/u06_k${k}_$r.txt; exit 1; }
    echo "k=$k r=$r $(grep -o '"value": [0-9.]*' gpurun_out/u06_k${k}_$r.txt | head -1)"
  done
done
