set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for combo in "0 1" "9 1" "0 0" "9 0" "0 1" "9 1" "0 0" "9 0"; do
  set -- $combo
  SVA_PATHS_VARIANT=$1 SVA_WTA_NT=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  echo "paths=$1 wta_nt=$2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab.log) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/ab.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab.log; exit $rc; fi
done
