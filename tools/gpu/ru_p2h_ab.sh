#!/bin/bash
# C = 128 ResidualUnit: phase 2 on the split MFMA in two K-halves (VRVQ_RU_P2H=1, default) vs
# the fp32 phase 2 (0): RU / conv / fixture GPU tests, alternating bench A/B, per-layer trace.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-p2h}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[EW]20" | grep -o '"value": [0-9.]*\|passed.*\|failed.*' | tail -2
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -20 "gpurun_out/${TAG}_$name.log"; exit $rc; fi; return 0; }
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
run tests 600 $PT tests/test_gpu_parity.py -k "residual or x3 or model_forward or config2 or batch_invariance or golden"
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
run b1 300 env VRVQ_RU_P2H=1 $B
run b0 300 env VRVQ_RU_P2H=0 $B
run b1b 300 env VRVQ_RU_P2H=1 $B
run b0b 300 env VRVQ_RU_P2H=0 $B
run prof1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
