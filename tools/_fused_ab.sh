#!/bin/bash
# experiment: fused vs cost-volume path kernel, by line kind (ablation build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
cp stereovisionarray_amd/libsva.so gpurun_out/libsva_prod.so
cp stereovisionarray_amd/libsva_ab.so stereovisionarray_amd/libsva.so
for combo in "1 0 0" "1 1 0" "1 2 0" "0 0 0" "0 0 7" "0 0 8" "1 0 0"; do
  set -- $combo
  SVA_FUSED=$1 SVA_FUSED_KIND=$2 SVA_PATHS_VARIANT=$3 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fab.log 2>&1; rc=$?
  echo "fused=$1 kind=$2 var=$3 rc=$rc $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/fab.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/fab.log; break; fi
done
cp gpurun_out/libsva_prod.so stereovisionarray_amd/libsva.so
