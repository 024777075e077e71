set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1; rc=$?; echo "bench n1 rc=$rc"; tail -1 gpurun_out/bench_n1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > gpurun_out/bench_n2_gloo.log 2>&1; rc=$?; echo "bench n2 gloo rc=$rc"; grep '^{' gpurun_out/bench_n2_gloo.log | tail -1; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_n2_gloo.log
