#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 invocation per counter group: gfx950 cannot
# collect FETCH_SIZE and WRITE_SIZE in one pass).  Usage (on the GPU box):
#   bash tools/profile_pmc.sh <tag> [bench args...]
# Writes gpurun_out/pmc_<tag>/<pass>/... ; summarise with tools/pmc_summary.py.
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$tag
mkdir -p "$out"
pass() {
  local name=$1; shift
  echo "== pass $name: $*" >&2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extras --serial-msms 4 --serial-min-s 0 \
    "${BENCH_ARGS[@]}" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== pass $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -5 "$out/$name.log" >&2; fi
  return $rc
}
BENCH_ARGS=("$@")
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE && \
pass lds SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE && \
pass l2 TCC_HIT_sum TCC_MISS_sum
