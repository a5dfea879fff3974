#!/bin/bash
# Summary of one gpu_session.sh tag's records in gpurun_out/ (tuning aid): test tail, single-stream
# per-kernel means per library, phase-probe digest, interleaved bench A/B lines.
#   bash tools/session_summary.sh <tag>
T=$1
cd "$(dirname "$0")/.." || exit 2
[ -f gpurun_out/${T}_tests.txt ] && tail -1 gpurun_out/${T}_tests.txt
ks=$(ls -d gpurun_out/${T}_kstats1*_d 2>/dev/null)
[ -n "$ks" ] && python3 tools/kstats_compare.py $ks
for f in gpurun_out/${T}_probe*.json; do
  [ -f "$f" ] || continue
  echo "$f"
  grep -v '^/opt' "$f" | python3 -c "
import json,sys;d=json.load(sys.stdin)
for k,v in d.items():
  if isinstance(v,dict): print(' ',k, 'span',v['span_us'], 'life',v['life_us_mean'], 'resident',v['resident_mean'], {p:x['median_us'] for p,x in v['phases'].items()})
"
done
for f in gpurun_out/${T}_ab_*.txt gpurun_out/${T}_env*.txt; do
  [ -f "$f" ] || continue
  echo "$(basename $f .txt) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"kernel_ms": [0-9.]*' $f | head -1) $(grep -o '"device_ms_per_launch": [0-9.]*' $f)"
done
