#!/bin/bash
# experiment: cost kernel rows per workgroup over D (in-process A/B, ablibs/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
L="ablibs/libsva_c1.so ablibs/libsva_c2.so ablibs/libsva_c4.so ablibs/libsva_c16.so"
for D in 64 128 192 256; do
  timeout -k 10 300 python3 tools/ab_paths.py $L $L --entry cost --iters 30 --D $D
done
timeout -k 10 300 python3 tools/ab_paths.py $L --entry cost --iters 10 --W 3840 --H 2160 --D 256
