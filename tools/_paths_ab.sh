#!/bin/bash
# experiment: in-process A/B of the cost-volume path kernel across builds in ablibs/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sgm_gpu.py -q -x --timeout 120 --timeout-method thread -k "paths or pipeline" > gpurun_out/pa.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/pa.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/ab_paths.py ${LIBS} --entry paths --iters 30
