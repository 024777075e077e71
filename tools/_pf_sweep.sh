#!/bin/bash
# sgm_paths prefetch-depth sweep: libsva_pf_<H>_<V>.so builds, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for v in ${PF_VARIANTS:-8_8 16_8 24_8 32_8 24_12 16_16 8_8 24_8 32_8}; do
  SVA_LIB_PATH=$PWD/stereovisionarray_amd/libsva_pf_$v.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pf.log 2>&1; rc=$?
  echo "pf=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/pf.log) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/pf.log)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pf.log; exit $rc; }
done
