#!/bin/bash
# Round-6 final measurements, part B: the other BASELINE workloads, Mode R per pair, host boundary, rehearsals
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6final3b
mkdir -p $O
export TMPDIR=/tmp
show() { grep '^{' "$1" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), d['kernels_ms'])"; }
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }; }
run 4k_d256 500 python3 bench.py --workload 4k_d256 --steps 20 --warmup 10; show $O/4k_d256.log 4k_d256
run vga_d64 300 python3 bench.py --workload vga_d64 --steps 100 --warmup 50 --no-cpu-baseline; show $O/vga_d64.log vga_d64
run center8 400 python3 bench.py --workload center8 --steps 40 --warmup 20 --no-cpu-baseline; show $O/center8.log center8
run center8_half_d64 300 python3 bench.py --workload center8_half_d64 --steps 100 --warmup 30 --no-cpu-baseline; show $O/center8_half_d64.log center8_half_d64
run center8_half_d64_batch 300 python3 bench.py --workload center8_half_d64 --steps 100 --warmup 30 --no-cpu-baseline --batch; show $O/center8_half_d64_batch.log center8_half_d64_batch
run center8_half_d64_s3 300 python3 bench.py --workload center8_half_d64 --steps 100 --warmup 30 --no-cpu-baseline; show $O/center8_half_d64_s3.log center8_half_d64_again
run center8_half_d64_batch2 300 python3 bench.py --workload center8_half_d64 --steps 100 --warmup 30 --no-cpu-baseline --batch; show $O/center8_half_d64_batch2.log center8_half_d64_batch_again
run grid8_all 400 python3 bench.py --workload grid8_all --steps 10 --warmup 5 --no-cpu-baseline; show $O/grid8_all.log grid8_all
run batch256_d192 600 python3 bench.py --workload batch256_d192 --no-cpu-baseline; show $O/batch256_d192.log batch256_d192
run mode_r_bench_refpath 400 rocprofv3 --kernel-trace --stats -d $O/prof_modeR -o run --output-format csv -- python3 tools/bench_refpath.py --sizes 960x540,1920x1080,3840x2160 --pairs 12-11,12-7,12-6,12-18 --reps 10 --cpu-rows 8
run bench_host 300 python3 tools/bench_host.py
run rehearsal_bench_rccl1 400 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --rehearse-rccl
run rehearsal_bench_engine_n1 400 python3 bench.py --engine multi --steps 10 --warmup 3 --no-cpu-baseline
run rehearsal_bench_gloo2 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo
echo final-done
