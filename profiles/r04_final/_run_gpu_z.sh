#!/bin/bash
# A-B-A: the MFMA census_cost vs the round-1 VALU kernel under 2-stream batches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4z
mkdir -p $O
cp stereovisionarray_amd/libsva.so $O/libsva_mfma.so
show() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['kernels_ms'], d.get('frame_overlap',{}).get('2_streams'))"; }
for v in mfma valu mfma valu; do
  if [ $v = valu ]; then cp ab_libs/libsva_ccvalu.so stereovisionarray_amd/libsva.so; else cp $O/libsva_mfma.so stereovisionarray_amd/libsva.so; fi
  timeout -k 10 300 python3 bench.py --workload batch256_d192 --steps 4 --warmup 1 --no-cpu-baseline --pmc committed > $O/b256_$v.log 2>&1 || exit $?
  show $O/b256_$v.log "b256 $v"
  timeout -k 10 300 python3 bench.py --steps 100 --warmup 50 --no-cpu-baseline --pmc committed > $O/f1080_$v.log 2>&1 || exit $?
  show $O/f1080_$v.log "1080p $v"
done
cp $O/libsva_mfma.so stereovisionarray_amd/libsva.so
