#!/bin/bash
# experiment: in-process A/B of fused path-kernel builds in ablibs/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused.log 2>&1; rc=$?
tail -2 gpurun_out/fused.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/ab_paths.py ${LIBS:-ablibs/libsva_base.so ablibs/libsva_swp.so ablibs/libsva_base.so ablibs/libsva_swp.so} --entry fused --iters 20
