#!/bin/bash
# Per-kernel SQ counter passes (one rocprofv3 --pmc pass per group, no trace
# domains) over a short bench run.  Output: gpurun_out/pmcK_<n>/.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           ${EXTRA_GROUPS:-}; do
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmcK_$i -o run --output-format csv -- ${PMC_CMD:-python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}} > gpurun_out/pmcK_$i.log 2>&1; rc=$?
  echo "group $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcK_$i.log; exit $rc; }
  i=$((i+1))
done
