#!/bin/bash
# experiment: which SGM directions compute costs in registers (SVA_FUSED_MASK,
# bit r = direction r of DESIGN.md §2.3) vs read the cost volume (ablation build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
cp stereovisionarray_amd/libsva.so gpurun_out/libsva_prod.so
cp stereovisionarray_amd/libsva_ab.so stereovisionarray_amd/libsva.so
for m in ${MASKS:-0xff 0x00 0xfc 0x0c 0xf0 0x3c 0xcc 0x30 0xff 0x00}; do
  SVA_FUSED_MASK=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fab.log 2>&1; rc=$?
  echo "mask=$m rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/fab.log) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/fab.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/fab.log; break; fi
done
cp gpurun_out/libsva_prod.so stereovisionarray_amd/libsva.so
