#!/bin/bash
# experiment: bench workloads under --streams / --path-kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
run() {
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/sm.log 2>&1; rc=$?
  echo "$* rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/sm.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sm.log) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/sm.log)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/sm.log; exit $rc; }
}
for pk in cost_volume fused; do
  for st in 1 2 3; do
    run --workload batch256_d192 --steps 2 --warmup 1 --path-kernel $pk --streams $st
  done
done
for pk in cost_volume fused; do
  for st in 1 2; do
    run --workload 1080p_d128 --pairs-per-rank 8 --steps 10 --warmup 3 --path-kernel $pk --streams $st
    run --workload 4k_d256 --pairs-per-rank 2 --steps 4 --warmup 2 --path-kernel $pk --streams $st
  done
done
