#!/bin/bash
# ConvTranspose 192 -> 96 s2 tile A/B (VRVQ_CONV_CONVT96 = 1: 96 x 128 pair | 0: 192 x 128
# two-stage | 2: 192 x 64 single-stage), with its parity tests under each.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06t}
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
for v in 2 0; do
  VRVQ_CONV_CONVT96=$v timeout -k 10 300 $PT tests/test_gpu_parity.py -k "transpose" > gpurun_out/${TAG}_tests$v.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests$v.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests$v.log
done
timeout -k 10 300 $PT tests/test_gpu_parity.py -k "conv1d or golden or batch_invariance" > gpurun_out/${TAG}_small_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_small_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_small_tests.log
OUT=gpurun_out/${TAG}_layers.txt
: > $OUT
for rep in 1 2; do
  for v in 1 0 2; do
    r=$(VRVQ_CONV_CONVT96=$v timeout -k 10 60 python tools/conv_bench.py --x3 --convt 2 --cin 192 --cout 96 --t 22272 2>&1 | grep median) || { echo FAIL; exit 1; }
    echo "convt96=$v 192->96 s2: ${r##*:}" | tee -a $OUT
  done
done
for L in "--cin 32 --cout 8 --t 87 --k 3" "--cin 8 --cout 1 --t 87 --k 3" "--cin 128 --cout 32 --t 87 --k 3"; do
  r=$(timeout -k 10 60 python tools/conv_bench.py --x3 $L 2>&1 | grep median) || { echo FAIL; exit 1; }
  echo "$L: ${r##*:}" | tee -a $OUT
done
exit 0
