#!/bin/bash
# experiment: frame overlap on 1/2/3 contexts, fused (0xff) vs cost-volume (0x00) path kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
cp stereovisionarray_amd/libsva.so gpurun_out/libsva_prod.so
cp stereovisionarray_amd/libsva_ab.so stereovisionarray_amd/libsva.so
for m in 0xff 0x00 0xff 0x00; do
  echo "mask $m: $(SVA_FUSED_MASK=$m timeout -k 10 200 python3 tools/overlap_test.py 2>&1 | tail -2 | tr '\n' ' ')"
done
cp gpurun_out/libsva_prod.so stereovisionarray_amd/libsva.so
