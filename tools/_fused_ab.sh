#!/bin/bash
# experiment: path kernels by line kind (ablation build): SVA_FUSED_KIND 1 = horizontal
# lines only, 2 = vertical + diagonal only; cost-volume kernel: SVA_PATHS_VARIANT 7 / 8 (D=128)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
cp stereovisionarray_amd/libsva.so gpurun_out/libsva_prod.so
cp stereovisionarray_amd/libsva_ab.so stereovisionarray_amd/libsva.so
for combo in ${COMBOS:-"fused 0 0" "fused 1 0" "fused 2 0"}; do
  set -- $combo
  SVA_FUSED_KIND=$2 SVA_PATHS_VARIANT=$3 timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --path-kernel $1 ${ARGS:-} > gpurun_out/fab.log 2>&1; rc=$?
  echo "$combo rc=$rc $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/fab.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/fab.log; break; fi
done
cp gpurun_out/libsva_prod.so stereovisionarray_amd/libsva.so
