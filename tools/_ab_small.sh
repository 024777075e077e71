#!/bin/bash
# A/B of the census / cost kernel variants (env switches), interleaved.
# Needs the ablation build: make -C stereovisionarray_amd/csrc EXTRA=-DSVA_PATHS_ABLATION
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_sgm_gpu.py tests/test_array_gpu.py -q -m gpu -x > gpurun_out/ab_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/ab_tests.log
[ $rc -eq 0 ] || exit $rc
for combo in "0 0" "1 1" "0 0" "1 1" "0 1" "1 0"; do
  set -- $combo
  SVA_CENSUS_VARIANT=$1 SVA_COST_VARIANT=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  echo "census=$1 cost=$2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab.log) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/ab.log)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ab.log; exit $rc; }
done
