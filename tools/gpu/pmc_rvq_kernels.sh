#!/bin/bash
# SQ counters per RVQ kernel (project / chain / expand), two passes each, kernel-trace only.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/pmcr
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for K in ${KERNELS:-project chain expand}; do
  j=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    j=$((j+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "rvq_${K}" -d gpurun_out/pmcr/${K}p$j -o run --output-format csv -- python tools/rvq_bench.py --iters 8 > gpurun_out/pmcr/${K}p$j.log 2>&1
    rc=$?; echo "$K p$j rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
