#!/bin/bash
# Split-K T <= 96 layers: parity tests, per-layer time with / without the split, bench A/B.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06k}
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_parity.py -k "splitk or batch_invariance or golden or strided or x3 or model_forward" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
OUT=gpurun_out/${TAG}_layers.txt
: > $OUT
for L in "--cin 512 --cout 1024 --t 696 --k 16 --stride 8" "--cin 1024 --cout 1024 --t 87 --k 3" \
         "--cin 1024 --cout 512 --t 87 --k 3" "--cin 512 --cout 128 --t 87 --k 3" \
         "--cin 1024 --cout 1536 --t 87 --k 7"; do
  for sk in 0 -1; do
    r=$(VRVQ_CONV_SPLITK=$sk timeout -k 10 60 python tools/conv_bench.py --x3 $L 2>&1 | grep median) || { echo FAIL; exit 1; }
    echo "splitk=$sk $L: ${r##*:}" | tee -a $OUT
  done
done
NOTEST=1 TAG=${TAG} COMBOS="VRVQ_CONV_SPLITK=-1 VRVQ_CONV_SPLITK=0" timeout -k 10 500 bash tools/gpu/r06_env_ab.sh || exit 1
exit 0
