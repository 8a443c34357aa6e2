#!/bin/bash
# Split-K of the 256 -> 512 s8 conv at T = 696 on 128 x 128 tiles (VRVQ_CONV_SPLITK_WIDE=S):
# strided tests with it on, the layer per S, bench A/B.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06w}
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
VRVQ_CONV_SPLITK_WIDE=2 timeout -k 10 600 $PT tests/test_gpu_parity.py -k "strided or golden or batch_invariance" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
OUT=gpurun_out/${TAG}_layers.txt
: > $OUT
for rep in 1 2; do
  for w in 0 2 3 4; do
    r=$(VRVQ_CONV_SPLITK_WIDE=$w timeout -k 10 60 python tools/conv_bench.py --x3 --cin 256 --cout 512 --t 5568 --k 16 --stride 8 2>&1 | grep median) || { echo FAIL; exit 1; }
    echo "wide=$w 256->512 s8 T696: ${r##*:}" | tee -a $OUT
  done
done
NOTEST=1 TAG=${TAG} COMBOS="VRVQ_CONV_SPLITK_WIDE=2 VRVQ_CONV_SPLITK_WIDE=0" timeout -k 10 500 bash tools/gpu/r06_env_ab.sh || exit 1
exit 0
