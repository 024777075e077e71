set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused.log 2>&1; rc=$?
tail -5 gpurun_out/fused.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?
tail -1 gpurun_out/bench.log | grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}'
[ $rc -ne 0 ] && exit $rc
bash tools/_fused_ab.sh
