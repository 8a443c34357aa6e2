#!/bin/bash
# Phase-split view as a compile-time flag (stride-1 x3 kernels without its addressing): smoke, GPU suite, bench, A/B, trace.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*\|\[smoke\].*' "gpurun_out/${TAG}_$name.log" | tail -2
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; grep -E "Error|assert|FAILED" "gpurun_out/${TAG}_$name.log" | head -20; exit $rc; fi; return 0; }
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
run bench 400 python bench.py --steps 20 --warmup 3
run bench_nostrided 300 env VRVQ_CONV_X3_STRIDED=0 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
