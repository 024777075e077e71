#!/bin/bash
# experiment: sgm_paths ablation variants (SVA_PATHS_VARIANT, D=128 only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in ${VARIANTS:-0 2 3 4 0}; do
  SVA_PATHS_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/var_$v.log 2>&1; rc=$?
  echo "variant $v rc=$rc $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/var_$v.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/var_$v.log; exit $rc; fi
done
