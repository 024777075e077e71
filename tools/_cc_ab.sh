#!/bin/bash
# census+cost kernel: GPU parity tests, then in-process A/B of full frames
# (ablibs/libsva_split.so = separate census + cost launches) over D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_census_cost_gpu.py tests/test_api_gpu.py -x -q > gpurun_out/cc_tests.log 2>&1; rc=$?
tail -3 gpurun_out/cc_tests.log; [ $rc -eq 0 ] || exit $rc
L="ablibs/libsva_split.so ablibs/libsva_cc.so"
for D in 64 128 192; do
  timeout -k 10 300 python3 tools/ab_paths.py $L $L --entry sgm --iters 30 --D $D || exit $?
done
timeout -k 10 300 python3 tools/ab_paths.py ablibs/libsva_cc.so --entry census_cost --iters 30 --D 128 || exit $?
timeout -k 10 300 python3 tools/ab_paths.py $L --entry sgm --iters 10 --W 3840 --H 2160 --D 256 || exit $?
