#!/bin/bash
# experiment: in-process A/B of fused path-kernel builds (ablibs/, ablation builds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_paths.py ablibs/libsva_pf8.so ablibs/libsva_pf6.so ablibs/libsva_pf4.so ablibs/libsva_lb4.so ablibs/libsva_pf8.so --entry fused --iters 20
SVA_FUSED_MASK=0 timeout -k 10 300 python3 tools/ab_paths.py ablibs/libsva_cv.so ablibs/libsva_lb4.so --entry sgm --iters 20
SVA_FUSED_MASK=0xff timeout -k 10 300 python3 tools/ab_paths.py ablibs/libsva_cv.so ablibs/libsva_lb4.so ablibs/libsva_pf8.so --entry sgm --iters 20
