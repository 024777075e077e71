#!/bin/bash
# Round-6 final measurements at HEAD (after the placement check), part A: GPU suite, smoke, the driver's
# bench command (+ rocprof stats), default bench, 4K.  Each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6final3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -q -m gpu -rf --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1; rc=$?
tail -2 $O/pytest_gpu_all.log
[ $rc -eq 0 ] || { grep -B2 -A30 "^____" $O/pytest_gpu_all.log | head -80; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
show() { grep '^{' "$1" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), d['kernels_ms'])"; }
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }; }
run bench_w5_s20 400 python3 bench.py --gpus 1 --steps 20 --warmup 5; show $O/bench_w5_s20.log driver
run prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --pmc committed
run bench_default 400 python3 bench.py; show $O/bench_default.log default
run 4k_d256 500 python3 bench.py --workload 4k_d256 --steps 20 --warmup 10; show $O/4k_d256.log 4k_d256
SVA_LIB_PATH=ab_run/libsva_strip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tile_stages_gpu.py tests/test_sgm_gpu.py tests/test_any_d_gpu.py > $O/pytest_strip_split.log 2>&1 || { tail -30 $O/pytest_strip_split.log; exit 1; }
tail -1 $O/pytest_strip_split.log
echo final-a-done
