#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; cat "gpurun_out/$name.log" | grep -v amdgpu.ids | grep -v "^W2026\|^E2026" | tail -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run cb384 120 python tools/conv_bench.py --cin 384 --cout 384 --t 5568 --k 7 --dil 3
run cb96 120 python tools/conv_bench.py --cin 96 --cout 96 --t 44544 --k 7 --dil 3
run cb192k1 120 python tools/conv_bench.py --cin 192 --cout 192 --t 22272 --k 1 --res
run pmc1 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "conv_mfma.*" -d gpurun_out/pmc_conv1 -o run --output-format csv -- python tools/conv_bench.py --cin 384 --cout 384 --t 5568 --k 7 --dil 3 --iters 3
run pmc2 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --kernel-include-regex "conv_mfma.*" -d gpurun_out/pmc_conv2 -o run --output-format csv -- python tools/conv_bench.py --cin 384 --cout 384 --t 5568 --k 7 --dil 3 --iters 3
