#!/bin/bash
# experiment: L2 behaviour of the fused vs cost-volume path kernel at 1080p D=128
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for pk in fused cost_volume; do
  i=0
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE"; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/l2_${pk}_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --path-kernel $pk > gpurun_out/l2.log 2>&1; rc=$?
    echo "$pk group $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/l2.log; exit $rc; }
    i=$((i+1))
  done
  mkdir -p gpurun_out/l2s_$pk; for d in gpurun_out/l2_${pk}_*; do mv $d gpurun_out/l2s_$pk/pmcK_${d##*_}; done
  echo "== $pk"; python3 tools/pmc_summary.py gpurun_out/l2s_$pk | grep -A 5 "sgm_"
done
