#!/bin/bash
# experiment: parity + in-process A/B of fused path-kernel builds in ablibs/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/fab3.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/fab3.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/ab_paths.py ${LIBS} --entry fused --iters 20
timeout -k 10 300 python3 tools/ab_paths.py ${LIBS} --entry fused --iters 6 --W 3840 --H 2160 --D 256
