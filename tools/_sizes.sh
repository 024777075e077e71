set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for w in vga_d64 1080half_d128 1080p_d128 1080p_d192 4k_d256; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload $w > gpurun_out/sz.log 2>&1; rc=$?
  echo "$w rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/sz.log) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/sz.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sz.log; exit $rc; fi
done
