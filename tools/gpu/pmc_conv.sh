#!/bin/bash
# PMC passes over single conv layers (tools/conv_bench.py), one counter set per run.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/pmc/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/pmc/$name.log" | grep -v "^[WE]2026" | tail -2
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
L1="--cin 384 --cout 384 --t 5568 --k 7 --dil 3"
L2="--cin 192 --cout 192 --t 22272 --k 7 --dil 3"
L3="--cin 192 --cout 192 --t 22272 --k 1 --res"
L4="--cin 768 --cout 384 --t 696 --convt 8"
for L in "$L1" "$L2" "$L3" "$L4"; do run bench 60 python tools/conv_bench.py $L; done
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for L in "$L1" "$L2" "$L3" "$L4"; do
  i=$((i+1)); j=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    j=$((j+1))
    run l${i}p${j} 90 rocprofv3 --pmc $P --kernel-include-regex "conv_mfma.*" -d gpurun_out/pmc/l${i}p${j} -o run --output-format csv -- python tools/conv_bench.py $L --iters 3
  done
done
exit 0
