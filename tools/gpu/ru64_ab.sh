#!/bin/bash
# A/B: the C = 64 ResidualUnits as two launches with the k7 on the 64 x 256 pair tile
# (VRVQ_CONV_PAIR_M64=1, VRVQ_RU_FUSED without 64) against the fused unit.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-ru64}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | grep -o '"value": [0-9.]*\|median.*\|[0-9]* passed.*' | head -1
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run ru64 60 python tools/conv_bench.py --x3 --ru --cin 64 --t 44544 --dil 3
run k7_64 60 env VRVQ_CONV_PAIR_M64=1 python tools/conv_bench.py --x3 --cin 64 --cout 64 --t 44544 --k 7 --dil 3
run k7_64_def 60 python tools/conv_bench.py --x3 --cin 64 --cout 64 --t 44544 --k 7 --dil 3
run k1_64 60 python tools/conv_bench.py --x3 --cin 64 --cout 64 --t 44544 --k 1 --res
run tests_B 300 env VRVQ_CONV_PAIR_M64=1 VRVQ_RU_FUSED=96,128,256 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "x3 or conv1d or fixture or residual"
for rep in 1 2; do
  run default_$rep 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  run split64_$rep 300 env VRVQ_CONV_PAIR_M64=1 VRVQ_RU_FUSED=96,128,256 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
exit 0
