#!/bin/bash
# Round-5 final measurements at HEAD (Mode R every tile split + ranged walk): suite, smoke, benches, rocprof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5final5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -rf --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1; rc=$?
tail -2 $O/pytest_gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_w5_s20.log 2>&1 || exit $?
grep '^{' $O/bench_w5_s20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver', d['value'], d['ms_per_step'], d['roofline']['frac'], d['aggregation_roofline']['frac'], d['kernels_ms'], d['mode_r'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --pmc committed > $O/prof.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py > $O/bench_default.log 2>&1 || exit $?
grep '^{' $O/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['aggregation_roofline']['frac'], d['kernels_ms'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_modeR -o run --output-format csv -- python3 tools/bench_refpath.py --sizes 960x540,1920x1080 --pairs 12-11,12-7,12-6,12-18 --reps 10 --cpu-rows 8 > $O/mode_r_bench_refpath.log 2>&1 || exit $?
grep '^{' $O/mode_r_bench_refpath.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['size'], d['pair'], d.get('ref_match_ms'), d.get('gpu_ms'))"
show() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['kernels_ms'], (d.get('mode_r') or {}).get('roofline', {}).get('frac'))"; }
run() { local name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$name.log 2>&1 || exit $?; show $O/$name.log $name; }
run 4k_d256 --workload 4k_d256 --steps 20 --warmup 10
run vga_d64 --workload vga_d64 --steps 100 --warmup 50 --no-cpu-baseline
run center8 --workload center8 --steps 40 --warmup 20 --no-cpu-baseline
run batch256_d192 --workload batch256_d192 --no-cpu-baseline
