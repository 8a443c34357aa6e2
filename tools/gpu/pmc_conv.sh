#!/bin/bash
# SQ counters of the largest conv layers of the configs[1] step (B=32, x3 path), one rocprofv3
# --pmc pass per counter set (kernel-trace only), plus the HIP-event time of each layer.
# LAYERS selects a subset (default: all); summaries: python tools/pmc_summary.py $OUT l<i>.
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/${TAG:-pmc_conv}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | grep -v "^[WE]20" | tail -1
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
declare -A L
L[1]="--x3 --ru --cin 192 --t 22272 --dil 3"
L[2]="--x3 --ru --cin 96 --t 44544 --dil 3"
L[3]="--x3 --ru --cin 128 --t 22272 --dil 3"
L[4]="--x3 --ru --cin 64 --t 44544 --dil 3"
L[5]="--x3 --cin 384 --cout 384 --t 5568 --k 7 --dil 3"
L[6]="--x3 --cin 768 --cout 768 --t 696 --k 7 --dil 3"
L[7]="--x3 --cin 384 --cout 384 --t 5568 --k 1 --res"
L[8]="--x3 --cin 256 --cout 256 --t 5568 --k 1 --res"
L[9]="--x3 --cin 512 --cout 1024 --t 696 --k 16 --stride 8"
L[10]="--x3 --cin 192 --cout 96 --t 22272 --convt 2"
L[11]="--x3 --cin 192 --cout 192 --t 22272 --k 1 --res"
L[12]="--x3 --cin 768 --cout 768 --t 696 --k 1 --res"
L[13]="--x3 --cin 192 --cout 192 --t 22272 --k 7 --dil 3"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
for i in ${LAYERS:-1 2 3 4 5 6 7 8 9 10}; do
  run l${i}_time 60 python tools/conv_bench.py ${L[$i]}
  j=0
  for P in "$P1" "$P2"; do
    j=$((j+1))
    run l${i}p${j} 90 rocprofv3 --pmc $P --kernel-include-regex "conv_|ru_" -d $OUT/l${i}p${j} -o run --output-format csv -- python tools/conv_bench.py ${L[$i]} --iters 3
  done
done
exit 0
