#!/bin/bash
# PMC passes over single conv layers: usage pmc_conv2.sh "<layer args>" ...
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/pmc2/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc $(grep -v amdgpu.ids gpurun_out/pmc2/$name.log | grep median | tail -1)"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -5 gpurun_out/pmc2/$name.log; exit $rc; fi; return 0; }
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_IFETCH SQ_INSTS_SMEM GRBM_COUNT"
i=0
for L in "$@"; do
  i=$((i+1))
  run l${i}_bench 60 python tools/conv_bench.py $L
  j=0
  for P in "$P1" "$P2" "$P3"; do
    j=$((j+1))
    run l${i}p${j} 90 rocprofv3 --pmc $P --kernel-include-regex "conv_mfma.*" -d gpurun_out/pmc2/l${i}p${j} -o run --output-format csv -- python tools/conv_bench.py $L --iters 3
  done
done
exit 0
