#!/bin/bash
# Round profile: bench line (with CPU baseline), rocprofv3 kernel stats of the bench and of the
# training step (--train), RVQ micro-bench.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[WE]2026" | tail -${TAIL:-2}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run bench 400 python -u bench.py --steps 10 --warmup 3
run prof_bench 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run prof_train 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_train -o run --output-format csv -- python bench.py --train --steps 2 --warmup 1
run rvq_b32 120 python tools/rvq_bench.py --batch 32 --nq 8
exit 0
