#!/bin/bash
# confirmation: block order o0 (horizontal, vertical, diagonal) vs o1 (diagonals first, down last)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
L="ablibs/libsva_o0.so ablibs/libsva_o1.so"
for D in 128 192 64; do timeout -k 10 300 python3 tools/ab_paths.py $L $L --entry sgm --iters 30 --D $D || exit $?; done
timeout -k 10 300 python3 tools/ab_paths.py $L --entry paths --iters 10 --W 3840 --H 2160 --D 256 || exit $?
