#!/bin/bash
# x prefetch in the fused ResidualUnits' phase 1 (VRVQ_RU_XPF): unit tests, per-unit times with /
# without, bench A/B.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06u}
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_parity.py -k "residual or golden or batch_invariance or x3" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
OUT=gpurun_out/${TAG}_layers.txt
: > $OUT
for rep in 1 2; do
for L in "--cin 64 --t 44544 --dil 3" "--cin 96 --t 44544 --dil 3" "--cin 128 --t 22272 --dil 3"; do
  for v in 0 1; do
    r=$(VRVQ_RU_XPF=$v timeout -k 10 60 python tools/conv_bench.py --x3 --ru $L 2>&1 | grep median) || { echo FAIL; exit 1; }
    echo "ru_xpf=$v $L: ${r##*:}" | tee -a $OUT
  done
done
done
NOTEST=1 TAG=${TAG} COMBOS="VRVQ_RU_XPF=1 VRVQ_RU_XPF=0" timeout -k 10 500 bash tools/gpu/r06_env_ab.sh || exit 1
exit 0
