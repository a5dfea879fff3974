#!/bin/bash
# One parametrised GPU session (replaces the round-2 one-off session scripts).  Run on the GPU box:
#
#   bash tools/gpu_session.sh <tag> <step> [<step> ...]
#
# Every step runs under its own time limit; its output goes to gpurun_out/<tag>_<step>.txt (or a
# directory of that name for profiles), and the session stops at the first step that crashes,
# times out or fails (no GPU step after a fault).  Steps:
#   tests        the -m gpu parity suites (libmsm.so)
#   tests_alt    the same with eager launches, then with one slot and one MSM per launch
#   testslib:LIBS  the parity suites (random sweep aside) against in-tree library variants
#   bench        python bench.py (the driver's command)
#   bench50      50 timed steps, no extras
#   sizes        pipelined ms per MSM at 2^16..2^19 (20 and 50 steps)
#   size:LG:LIBS pipelined ms per MSM at 2^LG points for each listed library variant
#   steps:K1,K2[:R]  the 2^20 bench over timed step counts
#   win:LG:C1,C2[:R]  pipelined ms per MSM at 2^LG points over window widths
#   batch64      the 64 x 2^18 prover batch (BASELINE configs[4])
#   gloo8        the sharded bench with 8 gloo ranks on the one GPU (configs[3]'s shard shape)
#   multidev     bench.py --multi-device: msm_compute over every visible device in one process
#   sharded      tools/sharded_probe.py: msm_compute's device-list path from host arrays, 1/2/8 shards
#   rocprof20    rocprofv3 --kernel-trace --stats of bench.py --steps 20 --warmup 5 (exit status 0)
#   splitrl:K1,K2[:R]  the 4 x 2 shares over accumulation run lengths (0 = the plan's)
#   splitlib:LIBS[:R]  the 4 x 2 shares for each in-tree library variant
#   splitk       one-stream kernel trace of the 4 x 2 (c = 15) shares of an 8-GPU split
#   split        per-GPU work of every points x windows split of a 2^20 MSM over 8 GPUs, on this one
#   kstats       rocprofv3 --kernel-trace --stats of the default bench command
#   ktrace:VAR=A,B  kernel trace of the pipelined bench per value of one knob (tools/pipeline_timeline.py)
#   kstats1      the same on one stream, kernels in order (MSM_SLOTS=1 MSM_FORK_PREP=0), two-MSM 2^20
#                launches only (the serial pass warms the GPU first, so the trace averages the
#                launches kernel_ms measures)
#   kstats1lib:LIBS  kstats1 for each in-tree library variant (names suffixed with $KS if set)
#   latprof      rocprofv3 kernel trace of single-MSM latency runs (tools/timeline.py reads it)
#   e2etrace     rocprofv3 kernel + memory-copy trace of msm_compute from host arrays (tools/e2e_probe.py)
#   e2e          msm_compute from host arrays, wall times only
#   e2esrc       the same with the inputs in numpy / no-huge-page / MAP_SHARED host memory
#   h2d          the host->device upload microbenchmark (tools/ubench/h2d_bench)
#   e2erocm      msm_compute from host arrays on /opt/rocm's HIP runtime (no torch loaded)
#   e2eenv:VAR=A,B[:R]  msm_compute from host arrays over values of one knob (interleaved)
#   node         the Node flat-buffer compute_msm (tools/node_flat.mjs), shared and plain buffers
#   nodetrace    rocprofv3 kernel + memory-copy trace of the Node shared-buffer path
#   pmc          the PMC passes of tools/profile_pmc.sh (one counter group per rocprofv3 run)
#   ab:LIBS[:R]  interleaved bench A/B of in-tree library variants (comma-separated file names
#                under webgpu-msm_amd/msm_amd/_lib), R rounds (default 3); $BENCH_X adds bench.py
#                arguments and $KS suffixes the output names
#   env:VAR=A,B[:R]  the same A/B over values of one environment knob (e.g. env:MSM_FORK_PREP=0,1)
#   envsize:LG:VAR=A,B[:R]  the same at 2^LG points (no extras)
#   lat:VAR=A,B[:R]  single-MSM latency (tools/latency_probe.py) over values of one knob
#   latlib:LIBS[:R]  single-MSM latency over in-tree library variants
#   latk:K1,K2[:R]   single-MSM latency over accumulation run lengths
#   set:VAR=VAL / unset:VAR  environment for the steps that follow (e.g. set:MSM_RED_L=8 kstats1;
#                set:KS=_x suffixes the output names of the steps after it, so repeated steps do not collide)
#   ubench       the field-multiply and ISA-rate microbenchmarks (tools/ubench)
#   ldshist      the sort's LDS counting atomics under random, bank-spread and equal keys
set -u
[ $# -ge 2 ] || { awk 'NR > 1 && /^#/ { print; next } NR > 1 { exit }' "$0"; exit 2; }
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBDIR=$PWD/webgpu-msm_amd/msm_amd/_lib
BENCH_Q=(--no-cpu-baseline)

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  local out=gpurun_out/${TAG}_$name.txt
  echo "== $name: $*" >&2
  timeout -k 10 "$to" "$@" > "$out" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -ao '"value": [0-9.]*\|[0-9]* passed[^=]*\|[0-9]* failed' "$out" | head -2 | tr '\n' ' ')" >&2
  if [ $rc -ne 0 ]; then
    tail -n 20 "$out" >&2
    echo "ABORT after $name (rc=$rc)" >&2
    exit $rc
  fi
}

PYTEST=(python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread)

for step in "$@"; do
  case $step in
    tests) run "tests${KS:-}" 900 "${PYTEST[@]}" ;;
    tests_alt)
      MSM_NO_GRAPH=1 run tests_eager 900 "${PYTEST[@]}" -k "not random_sweep"
      MSM_SLOTS=1 MSM_BATCH=1 run tests_1slot 900 "${PYTEST[@]}" -k "not random_sweep" ;;
    testk:*)  # testk:EXPR -- the GPU tests selected by pytest -k EXPR
      run testk 900 "${PYTEST[@]}" -k "${step#testk:}" ;;
    testslib:*)
      IFS=: read -r _ libs <<< "$step"
      for lib in ${libs//,/ }; do
        MSM_AMD_LIB=$LIBDIR/$lib run "tests_${lib%.so}" 900 "${PYTEST[@]}" -k "not random_sweep"
      done ;;
    bench) run bench 300 python bench.py ;;
    bench50) run bench50 300 python bench.py --steps 50 --warmup 20 --no-extras "${BENCH_Q[@]}" ;;
    steps:*)  # steps:K1,K2[:R] -- 2^20 bench over timed step counts (pipeline fill / drain share)
      IFS=: read -r _ ks rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for k in ${ks//,/ }; do
          run "steps${k}_$r" 300 python bench.py --steps "$k" --warmup 10 --no-extras "${BENCH_Q[@]}"
        done
      done ;;
    size:*)  # size:LOG2N[:LIBS] -- pipelined ms per MSM at one size for library variants (default libmsm.so)
      IFS=: read -r _ lg libs <<< "$step"
      libs=${libs:-libmsm.so}
      for lib in ${libs//,/ }; do
        MSM_AMD_LIB=$LIBDIR/$lib run "size${lg}_${lib%.so}${KS:-}" 120 python bench.py --steps 50 --warmup 20 --no-extras \
          "${BENCH_Q[@]}" --n $((1 << lg))
      done ;;
    win:*)  # win:LG:C1,C2[:R] -- pipelined ms per MSM at 2^LG points over window widths
      IFS=: read -r _ lg cs rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for cw in ${cs//,/ }; do
          run "win${lg}_c${cw}_$r" 120 python bench.py --steps 50 --warmup 20 --no-extras "${BENCH_Q[@]}" \
            --n $((1 << lg)) --window "$cw"
        done
      done ;;
    sizes)
      for lg in 16 17 18 19; do
        run size$lg 120 python bench.py --steps 50 --warmup 20 --no-extras "${BENCH_Q[@]}" --n $((1 << lg))
        run size${lg}_k20 120 python bench.py --no-extras "${BENCH_Q[@]}" --n $((1 << lg))
      done ;;
    batch64) run "batch64${KS:-}" 300 python bench.py --batch 64 --n 262144 ;;
    batch64d) run "batch64d${KS:-}" 300 python bench.py --batch 64 --n 262144 --distinct ;;  # distinct base vectors
    gloo8)
      MSM_DIST_BACKEND=gloo OMP_NUM_THREADS=2 run gloo8 400 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 10 --warmup 2 \
        --no-extras "${BENCH_Q[@]}" ;;
    multidev) run multidev 300 python bench.py --multi-device --no-extras "${BENCH_Q[@]}" ;;
    sharded) run sharded 300 python tools/sharded_probe.py ;;  # the device-list host path, D repeated shards
    rocprof20)  # the driver-shape bench (20 steps, 5 warm-up) under a kernel trace: must exit 0
      run rocprof20 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_rocprof20_d" -o run \
        -- python3 bench.py --steps 20 --warmup 5 ;;
    split) run split 600 python tools/split_probe.py --gpus 8 ;;
    splitrl:*)  # splitrl:K1,K2[:R] -- the 4 x 2 (c = 15) shares of an 8-GPU split over accumulation run lengths
      IFS=: read -r _ ks rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for k in ${ks//,/ }; do
          run "splitrl_k${k}_$r" 300 python tools/split_probe.py --gpus 8 --splits 4x2 --window 15 --run-length "$k"
        done
      done ;;
    split:*)  # split:D:SPLITS:C -- tools/split_probe.py over D GPUs for the listed PxQ splits at window width C
      IFS=: read -r _ ng sp cw <<< "$step"
      run "split${ng}_${sp//,/_}_c${cw}${KS:-}" 600 python tools/split_probe.py --gpus "$ng" --splits "$sp" --window "$cw" ;;
    splitlib:*)  # splitlib:LIBS[:R] -- the 4 x 2 (c = 15) shares of an 8-GPU split for each in-tree library variant
      IFS=: read -r _ libs rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for lib in ${libs//,/ }; do
          MSM_AMD_LIB=$LIBDIR/$lib run "splitlib_${lib%.so}_$r" 300 python tools/split_probe.py --gpus 8 --splits 4x2 --window 15
        done
      done ;;
    splitk)  # one-stream kernel trace of the 8-GPU 4 x 2 (c = 15) shares, each virtual GPU in turn
      MSM_SLOTS=1 MSM_FORK_PREP=0 run "splitk${KS:-}" 300 rocprofv3 --kernel-trace --output-format csv \
        -d "gpurun_out/${TAG}_splitk${KS:-}_d" -o run -- python3 tools/split_probe.py --gpus 8 --splits 4x2 --window 15 ;;
    kstats)
      run kstats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kstats_d -o run \
        -- python3 bench.py ;;
    ktrace:*)  # ktrace:VAR=A,B -- rocprofv3 kernel trace of the pipelined bench for each value of one knob
      IFS=: read -r _ spec <<< "$step"
      var=${spec%%=*}; vals=${spec#*=}
      for v in ${vals//,/ }; do
        export "$var=$v"
        run "ktrace_${var}_$v" 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "gpurun_out/${TAG}_ktrace_${var}_${v}_d" -o run -- python3 bench.py --no-extras "${BENCH_Q[@]}" --steps 40 --warmup 10
        unset "$var"
      done ;;
    kstats1)
      # shellcheck disable=SC2086
      MSM_SLOTS=1 MSM_FORK_PREP=0 run "kstats1${KS:-}" 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "gpurun_out/${TAG}_kstats1${KS:-}_d" -o run -- python3 bench.py --no-extras "${BENCH_Q[@]}" --steps 40 \
        --warmup 10 ${BENCH_X:-} ;;
    kstats1lib:*)
      IFS=: read -r _ libs <<< "$step"
      for lib in ${libs//,/ }; do
        # shellcheck disable=SC2086
        MSM_SLOTS=1 MSM_FORK_PREP=0 MSM_AMD_LIB=$LIBDIR/$lib run "kstats1_${lib%.so}${KS:-}" 300 rocprofv3 --kernel-trace \
          --stats --output-format csv -d "gpurun_out/${TAG}_kstats1_${lib%.so}${KS:-}_d" -o run -- python3 bench.py --no-extras \
          "${BENCH_Q[@]}" --steps 40 --warmup 10 ${BENCH_X:-}
      done ;;
    latprof)
      run latprof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_latprof_d -o run \
        -- python3 tools/latency_probe.py --runs 12 ;;
    e2etrace)  # kernels + host->device copies of msm_compute from host arrays (2^20)
      run e2etrace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
        -d gpurun_out/${TAG}_e2etrace_d -o run -- python3 tools/e2e_probe.py --runs 8 ;;
    e2e) run e2e 120 python tools/e2e_probe.py --runs 12 ;;
    manyhost:*)  # manyhost:NAME -- msm_compute_many from host arrays (16 x 2^18), under the current set: knobs
      run "manyhost_${step#manyhost:}" 300 python tools/many_host_probe.py ;;
    e2esz:*)  # e2esz:NAME:SIZES -- tools/e2e_size_probe.py over the listed sizes (under the current set: knobs)
      IFS=: read -r _ nm sz <<< "$step"
      run "e2esz_$nm" 300 python tools/e2e_size_probe.py --sizes "$sz" --runs 7 --rounds 1 ;;
    e2esrc)  # msm_compute from host arrays in numpy / no-huge-page / MAP_SHARED memory
      for src in numpy nohuge shared; do run "e2e_$src" 120 python tools/e2e_probe.py --runs 10 --src "$src"; done ;;
    h2d) run h2d 120 tools/ubench/h2d_bench ;;
    e2eenv:*)  # e2eenv:VAR=A,B[:R] -- msm_compute from host arrays over values of one knob, interleaved
      IFS=: read -r _ spec rounds <<< "$step"
      var=${spec%%=*}; vals=${spec#*=}
      for r in $(seq 1 "${rounds:-2}"); do
        for v in ${vals//,/ }; do
          export "$var=$v"
          run "e2eenv_${var}_${v}${KS:-}_$r" 120 python tools/e2e_probe.py --runs 12
          unset "$var"
        done
      done ;;
    e2erocm)  # msm_compute on /opt/rocm's HIP runtime (no torch in the process), as Node and C callers run
      MSM_AMD_NO_TORCH=1 run e2e_rocm 120 python tools/e2e_probe.py --runs 10 ;;
    node)  # the Node flat-buffer compute_msm (SharedArrayBuffer, then plain ArrayBuffer)
      run node_inputs 120 python tools/write_inputs.py /tmp/msm_in
      run node_shared 120 node tools/node_flat.mjs /tmp/msm_in/p.bin /tmp/msm_in/s.bin 1048576 8 shared
      run node_plain 120 node tools/node_flat.mjs /tmp/msm_in/p.bin /tmp/msm_in/s.bin 1048576 8 plain ;;
    nodetrace)
      run node_inputs 120 python tools/write_inputs.py /tmp/msm_in
      run nodetrace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_nodetrace_d \
        -o run -- node tools/node_flat.mjs /tmp/msm_in/p.bin /tmp/msm_in/s.bin 1048576 6 shared ;;
    pmc) run pmc 900 bash tools/profile_pmc.sh "$TAG" ;;
    ab:*)
      IFS=: read -r _ libs rounds <<< "$step"
      for r in $(seq 1 "${rounds:-3}"); do
        for lib in ${libs//,/ }; do
          # shellcheck disable=SC2086  # BENCH_X: extra bench.py arguments (set:BENCH_X=...), word-split on purpose
          MSM_AMD_LIB=$LIBDIR/$lib run "ab_${lib%.so}${KS:-}_$r" 180 python bench.py --steps 40 --warmup 10 "${BENCH_Q[@]}" ${BENCH_X:-}
        done
      done ;;
    env:*)
      IFS=: read -r _ spec rounds <<< "$step"
      var=${spec%%=*}; vals=${spec#*=}
      for r in $(seq 1 "${rounds:-3}"); do
        for v in ${vals//,/ }; do
          export "$var=$v"
          run "env_${var}_${v}${KS:-}_$r" 180 python bench.py --steps 40 --warmup 10 "${BENCH_Q[@]}"
          unset "$var"
        done
      done ;;
    envk:*)  # envk:K:VAR=A,B[:R] -- the 2^20 bench at K timed steps (warm-up 5: the driver's shape) over one knob
      IFS=: read -r _ k spec rounds <<< "$step"
      var=${spec%%=*}; vals=${spec#*=}
      for r in $(seq 1 "${rounds:-3}"); do
        for v in ${vals//,/ }; do
          export "$var=$v"
          run "envk${k}_${var}_${v}${KS:-}_$r" 180 python bench.py --steps "$k" --warmup 5 --no-extras "${BENCH_Q[@]}"
          unset "$var"
        done
      done ;;
    envsize:*)  # envsize:LG:VAR=A,B[:R] -- env:VAR=A,B at 2^LG points
      IFS=: read -r _ lg spec rounds <<< "$step"
      var=${spec%%=*}; vals=${spec#*=}
      for r in $(seq 1 "${rounds:-2}"); do
        for v in ${vals//,/ }; do
          export "$var=$v"
          run "envsize${lg}_${var}_${v}${KS:-}_$r" 180 python bench.py --steps 40 --warmup 10 --no-extras "${BENCH_Q[@]}" \
            --n $((1 << lg))
          unset "$var"
        done
      done ;;
    lat:*)
      IFS=: read -r _ spec rounds <<< "$step"
      var=${spec%%=*}; vals=${spec#*=}
      for r in $(seq 1 "${rounds:-3}"); do
        for v in ${vals//,/ }; do
          export "$var=$v"
          run "lat_${var}_${v}_$r" 120 python tools/latency_probe.py
          unset "$var"
        done
      done ;;
    latlib:*)
      IFS=: read -r _ libs rounds <<< "$step"
      for r in $(seq 1 "${rounds:-3}"); do
        for lib in ${libs//,/ }; do
          MSM_AMD_LIB=$LIBDIR/$lib run "latlib_${lib%.so}_$r" 120 python tools/latency_probe.py
        done
      done ;;
    latk:*)
      IFS=: read -r _ ks rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for k in ${ks//,/ }; do
          run "latk_${k}_$r" 120 python tools/latency_probe.py --run-length "$k"
        done
      done ;;
    calltrace:*)  # calltrace:K -- kernel trace of the 2^20 bench at K timed steps; fill / drain of the timed call
      IFS=: read -r _ k <<< "$step"
      # shellcheck disable=SC2086
      run "calltrace${k}${KS:-}" 300 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/${TAG}_calltrace${k}${KS:-}_d" \
        -o run -- python3 bench.py --steps "$k" --warmup 5 --no-extras "${BENCH_Q[@]}" ${BENCH_X:-}
      tr=$(find "gpurun_out/${TAG}_calltrace${k}${KS:-}_d" -name '*kernel_trace.csv' | head -1)
      run "calltrace${k}${KS:-}_tl" 60 python tools/call_timeline.py "$tr" --launches $(( (k + 1) / 2 )) ;;
    rl:*)  # rl:N:K1,K2[:R] -- pipelined ms per MSM at N points over accumulation run lengths (0 = the plan's)
      IFS=: read -r _ nn ks rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for k in ${ks//,/ }; do
          run "rl${nn}_k${k}_$r" 120 python bench.py --steps 20 --warmup 5 --no-extras "${BENCH_Q[@]}" --n "$nn" \
            --run-length "$k"
        done
      done ;;
    warm:*)  # warm:K:W1,W2[:R] -- the 2^20 bench at K timed steps over --warm-s values (clock ramp)
      IFS=: read -r _ k ws rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for w in ${ws//,/ }; do
          run "warm${k}_w${w}_$r" 120 python bench.py --steps "$k" --warmup 5 --no-extras "${BENCH_Q[@]}" --warm-s "$w"
        done
      done ;;
    batch64rl:*)  # batch64rl:K1,K2[:R] -- the 64 x 2^18 prover batch over run lengths (0 = the plan's)
      IFS=: read -r _ ks rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for k in ${ks//,/ }; do
          run "batch64_k${k}_$r" 180 python bench.py --batch 64 --n 262144 --steps 10 --warmup 3 --run-length "$k"
        done
      done ;;
    latn:*)  # latn:N:K1,K2[:R] -- single-MSM latency at N points over run lengths (0 = the plan's)
      IFS=: read -r _ nn ks rounds <<< "$step"
      for r in $(seq 1 "${rounds:-2}"); do
        for k in ${ks//,/ }; do
          run "latn${nn}_k${k}_$r" 120 python tools/latency_probe.py --n "$nn" --run-length "$k"
        done
      done ;;
    set:*) export "${step#set:}" ;;
    unset:*) unset "${step#unset:}" ;;
    ubench)
      run ubench_fmul 120 tools/ubench/fmul_bench
      run ubench_isa 120 tools/ubench/isa_rates ;;
    ldshist) run ldshist 120 tools/ubench/lds_hist ;;  # LDS counting atomics: random / spread / same keys
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "== session $TAG done" >&2
