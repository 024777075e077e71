#!/bin/bash
# experiment: sgm_paths block order (diagonals first) and priority, in-process A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
L="ablibs/libsva_o0.so ablibs/libsva_o1.so ablibs/libsva_o2.so ablibs/libsva_o3.so"
timeout -k 10 300 python3 tools/ab_paths.py $L $L --entry paths --iters 20 --D 128 || exit $?
timeout -k 10 300 python3 tools/ab_paths.py $L --entry sgm --iters 20 --D 128 || exit $?
for D in 64 192; do timeout -k 10 300 python3 tools/ab_paths.py $L --entry paths --iters 20 --D $D || exit $?; done
SVA_LIB_PATH=ablibs/libsva_trace_o1.so timeout -k 10 120 python3 tools/paths_trace.py > gpurun_out/trace_o1.json || exit $?
