#!/bin/bash
# experiment: parity + in-process A/B of ablibs/ builds on both path kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_sgm_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/ab.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/ab.log)"; [ $rc -ne 0 ] && { grep -m3 Error gpurun_out/ab.log; exit $rc; }
for e in fused paths sgm; do
  timeout -k 10 300 python3 tools/ab_paths.py ${LIBS} --entry $e --iters 20 ${ABARGS:-}
done
