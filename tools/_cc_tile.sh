#!/bin/bash
# census+cost kernel tiling sweep (PXB pixels x rows per workgroup), in-process A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
L="ablibs/libsva_cc.so ablibs/libsva_cc128_2.so ablibs/libsva_cc128_4.so ablibs/libsva_cc128_16.so ablibs/libsva_cc64_4.so ablibs/libsva_cc64_8.so ablibs/libsva_cc256_4.so"
for D in 128 64 192; do
  timeout -k 10 300 python3 tools/ab_paths.py $L --entry census_cost --iters 20 --D $D || exit $?
done
timeout -k 10 300 python3 tools/ab_paths.py ablibs/libsva_split.so ablibs/libsva_split.so --entry cost --iters 20 --D 128 || exit $?
timeout -k 10 300 python3 tools/ab_paths.py ablibs/libsva_split.so ablibs/libsva_split.so --entry census --iters 20 --D 128 || exit $?
