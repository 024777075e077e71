#!/bin/bash
# experiment: fused parity per variant library (SVA_LIB_PATH), then an in-process A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
ok=""
for l in ${LIBS}; do
  SVA_LIB_PATH=$PWD/$l timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/fv.log 2>&1; rc=$?
  echo "$l rc=$rc $(tail -1 gpurun_out/fv.log)"; grep -m3 "AssertionError: direction" gpurun_out/fv.log
  [ $rc -eq 0 ] && ok="$ok $l $l"
done
[ -n "$ok" ] && timeout -k 10 300 python3 tools/ab_paths.py $ok --entry fused --iters 20
exit 0
