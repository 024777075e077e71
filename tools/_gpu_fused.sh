set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_all.log
[ $rc -ne 0 ] && exit $rc
for args in "" "--workload 4k_d256 --steps 5 --warmup 2 --no-cpu-baseline" "--workload batch256_d192 --steps 2 --warmup 1 --no-cpu-baseline"; do
  timeout -k 10 300 python bench.py $args > gpurun_out/bench.log 2>&1; rc=$?
  echo "[$args] rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-900
  [ $rc -ne 0 ] && exit $rc
done
exit 0
