#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
S=stereovisionarray_amd
timeout -k 10 300 python tools/ab_paths.py $S/libsva_pf_base.so $S/libsva_pf_d64_40_12.so $S/libsva_pf_d64_48_12.so $S/libsva_pf_d64_48_8.so $S/libsva_pf_d64_56_12.so --W 1920 --H 1080 --D 64 --iters 20 || exit 1
timeout -k 10 300 python tools/ab_paths.py $S/libsva_pf_d64_48_12.so $S/libsva_pf_base.so --W 640 --H 480 --D 64 --iters 20 || exit 1
timeout -k 10 300 python tools/ab_paths.py $S/libsva_pf_base.so $S/libsva_pf_d192_24_8.so $S/libsva_pf_d192_28_8.so $S/libsva_pf_d192_32_8.so $S/libsva_pf_d192_24_12.so --W 1920 --H 1080 --D 192 --iters 20 || exit 1
