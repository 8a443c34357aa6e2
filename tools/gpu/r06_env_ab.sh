#!/bin/bash
# Correctness of the pt path, then the RVQ kernel in isolation and inside the bench step under
# each environment setting in COMBOS (space separated; each VAR=value[,VAR=value]), alternating
# on one box.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06e}
COMBOS=${COMBOS:-"VRVQ_RVQ_PAIR=1 VRVQ_RVQ_PAIR=0"}
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 $PT tests/test_gpu_rvq_part.py > gpurun_out/${TAG}_pt_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_pt_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pt_tests.log
fi
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
for rep in 1 2; do
  for c in $COMBOS; do
    envs=(${c//,/ })
    r=$(env "${envs[@]}" timeout -k 10 120 python tools/rvq_bench.py --paths pt --iters 50 ${RVQ_ARGS} 2>&1 | grep "^path") || { echo "FAIL"; exit 1; }
    echo "rep $rep $c iso: $r" | tee -a $OUT
    if [ -z "$NOSTEP" ]; then
      r=$(env "${envs[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} 2>&1 | tail -1) || { echo "FAIL"; exit 1; }
      echo "rep $rep $c step: $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel_us"], r["frac"])')" | tee -a $OUT
    fi
  done
done
if [ -n "$STAMP" ]; then
  envs=(${STAMP//,/ })
  env "${envs[@]}" timeout -k 10 120 python tools/rvq_fused_stamps.py --pt > gpurun_out/${TAG}_stamps.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/${TAG}_stamps.log | grep -E "end|start|done|stored"
fi
exit 0
