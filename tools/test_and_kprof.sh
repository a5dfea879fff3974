set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.txt >&2
[ $rc -eq 0 ] || exit $rc
bash tools/kprof_ab.sh libmsm_head.so,libmsm.so
