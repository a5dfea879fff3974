set -e
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/isa_rates > gpurun_out/r2_isa_rates.txt 2>&1
timeout -k 10 120 tools/ubench/fmul_bench > gpurun_out/r2_fmul_bench.txt 2>&1
timeout -k 10 300 tools/ubench/h2d_bench 160 > gpurun_out/r2_h2d.jsonl 2>&1
lscpu > gpurun_out/r2_lscpu.txt 2>&1 || true
