#!/bin/bash
# x-window prefetch on the 64 x 256 pair k7 tiles (VRVQ_CONV_XPF): x3 conv tests, per-layer
# times with / without, bench A/B.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06x}
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_parity.py -k "x3 or residual or conv1d or golden or batch_invariance" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
OUT=gpurun_out/${TAG}_layers.txt
: > $OUT
for rep in 1 2; do
for L in "--cin 192 --cout 192 --t 22272 --dil 3" "--cin 384 --cout 384 --t 5568 --dil 9" \
         "--cin 768 --cout 768 --t 696 --dil 1" "--cin 256 --cout 256 --t 5568 --dil 1" \
         "--cin 512 --cout 512 --t 696 --dil 3"; do
  for v in 0 1; do
    r=$(VRVQ_CONV_XPF=$v timeout -k 10 60 python tools/conv_bench.py --x3 --k 7 $L 2>&1 | grep median) || { echo FAIL; exit 1; }
    echo "xpf=$v $L: ${r##*:}" | tee -a $OUT
  done
done
done
NOTEST=1 TAG=${TAG} COMBOS="VRVQ_CONV_XPF=1 VRVQ_CONV_XPF=0" timeout -k 10 500 bash tools/gpu/r06_env_ab.sh || exit 1
exit 0
