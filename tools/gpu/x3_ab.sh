#!/bin/bash
# A/B of the conv paths: x3 dispatch rule, block order, fp32 baseline; per-layer kernel traces.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[WE]2026" | grep -o '"value": [0-9.]*\|passed.*\|failed.*\|Error.*' | tail -3
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
run tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "x3 or forward_vs_reference or residual_unit" --timeout 120 --timeout-method thread
run default 300 $B
run fp32 300 env VRVQ_CONV_X3=0 $B
run allx3 300 env VRVQ_CONV_X3_RULE=0 VRVQ_RU_X3=2 $B
run prof_allx3 300 env VRVQ_CONV_X3_RULE=0 VRVQ_RU_X3=2 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_allx3 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline
run prof_default 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_default -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline
exit 0
