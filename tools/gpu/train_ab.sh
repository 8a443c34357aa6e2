#!/bin/bash
# Training step: GPU training tests, bench --train with the weight gradients on the fp32 MFMA
# (VRVQ_WGRAD_X3=0) and on the x3 kernel, and a rocprofv3 kernel trace of the x3 step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-trainab}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | tail -${TAIL:-3} | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run tests 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread
VRVQ_WGRAD_X3=0 run bench_fp32 400 python bench.py --train --steps 3 --warmup 2
run bench_x3 400 python bench.py --train --steps 3 --warmup 2
run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python bench.py --train --steps 3 --warmup 2
exit 0
