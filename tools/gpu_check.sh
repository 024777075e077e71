#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; stop at the
# first step that faults / aborts / times out (exit codes other than 0 and 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case "$step" in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 1200 python -u -m pytest tests -q -m "gpu and not slow" -x --timeout 120 --timeout-method thread ;;
    pytest_all) run pytest_gpu_all 1500 python -u -m pytest tests -q -m gpu -rf --timeout 300 --timeout-method thread ;;
    pytest_slow) run pytest_gpu_slow 900 python -u -m pytest tests -v -m "gpu and slow" -rf --timeout 300 --timeout-method thread ;;
    bench) run bench 600 python bench.py ;;
    pytest_array) run pytest_array 900 python -m pytest tests/test_array_gpu.py -q -m gpu ;;
    array) run center8 600 python bench.py --workload center8 --steps 5 --warmup 2 --no-cpu-baseline
           run grid8_all 600 python bench.py --workload grid8_all --steps 5 --warmup 2 --no-cpu-baseline ;;
    batch) run batch256 900 python bench.py --workload batch256_d192 --steps 2 --warmup 1 --no-cpu-baseline ;;
    gloo2) run bench_gloo2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo ;;
    batch_gloo2) run batch_gloo2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --workload batch256_d192 --steps 1 --warmup 1 --dist-backend gloo ;;
    array_gloo2) run center8_gloo2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --workload center8 --steps 3 --warmup 1 --dist-backend gloo ;;
    rccl1) run bench_rccl1 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --rehearse-rccl ;;
    engine) run bench_engine_n1 600 python bench.py --engine multi --steps 10 --warmup 3 --no-cpu-baseline
            run bench_engine_batch256 900 python bench.py --engine multi --workload batch256_d192 --steps 2 --warmup 1 --no-cpu-baseline ;;
    bench_test) run bench_test 600 python -u -m pytest tests/test_bench_gpu.py -q -m gpu --timeout 300 --timeout-method thread ;;
    bench4k) run bench4k 600 python bench.py --workload 4k_d256 --no-cpu-baseline ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    refine_bench) run refine_bench 600 python tools/bench_refine.py ;;
    prof4k) run prof4k 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4k -o run --output-format csv -- python3 bench.py --workload 4k_d256 --steps 5 --warmup 2 --no-cpu-baseline ;;
    pmc4k) run pmc4k_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc4k_fetch -o run --output-format csv -- python3 bench.py --workload 4k_d256 --steps 2 --warmup 1 --no-cpu-baseline
           run pmc4k_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc4k_write -o run --output-format csv -- python3 bench.py --workload 4k_d256 --steps 2 --warmup 1 --no-cpu-baseline
           run pmc4k_json 120 python3 tools/pmc_traffic.py gpurun_out/pmc4k_fetch gpurun_out/pmc4k_write 3840 2160 256 gpurun_out/pmc_4k_d256.json ;;
    prof_refpath) run prof_refpath 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_refpath -o run --output-format csv -- python3 tools/bench_refpath.py --reps 3 --cpu-rows 2 ;;
    prof_refine) run prof_refine 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_refine -o run --output-format csv -- python3 tools/bench_refine.py ;;
    pmcjson) run pmcjson 120 python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write 1920 1080 128 gpurun_out/pmc_1080p_d128.json ;;
    prof_center8) run prof_center8 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_center8 -o run --output-format csv -- python3 bench.py --workload center8 --steps 5 --warmup 2 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
