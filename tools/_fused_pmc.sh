#!/bin/bash
# experiment: SQ stall breakdown of the path kernel, fused (0xff) vs cost-volume (0x00) directions
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
cp stereovisionarray_amd/libsva.so gpurun_out/libsva_prod.so
cp stereovisionarray_amd/libsva_ab.so stereovisionarray_amd/libsva.so
for m in 0xff 0x00; do
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU" \
             "SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SMEM"; do
    SVA_FUSED_MASK=$m timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmcK_${m}_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcK.log 2>&1; rc=$?
    echo "mask $m group $i rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcK.log; break 2; }
    i=$((i+1))
  done
done
cp gpurun_out/libsva_prod.so stereovisionarray_amd/libsva.so
for m in 0xff 0x00; do mkdir -p gpurun_out/s_$m; cp -r gpurun_out/pmcK_${m}_* gpurun_out/s_$m/ 2>/dev/null; echo "== mask $m"; python3 tools/pmc_summary.py gpurun_out/s_$m | grep -A 20 "sgm_" | head -24; done
