set -e
mkdir -p gpurun_out
nproc > gpurun_out/r2a_nproc.txt; python -c "import os;print(len(os.sched_getaffinity(0)))" >> gpurun_out/r2a_nproc.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r2a_nproc.txt 2>/dev/null || true
for i in 1 2; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2a_b20_$i.json 2>gpurun_out/r2a_b20_$i.err; done
timeout -k 10 120 python bench.py --steps 50 --warmup 20 --no-cpu-baseline > gpurun_out/r2a_b50.json 2>gpurun_out/r2a_b50.err
MSM_SLOTS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2a_b20_s1.json 2>gpurun_out/r2a_b20_s1.err
