#!/bin/bash
# experiment: single-stream path-kernel selection sweep over D (bench.py --path-kernel)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for w in vga_d64 1080p_d64 1080p_d128 1080p_d192 1080p_d256 4k_d256; do
  for pk in cost_volume fused cost_volume fused; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload $w --path-kernel $pk --streams 1 > gpurun_out/pk.log 2>&1; rc=$?
    echo "$w $pk rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/pk.log) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/pk.log)"
    [ $rc -eq 0 ] || { tail -3 gpurun_out/pk.log; exit $rc; }
  done
done
