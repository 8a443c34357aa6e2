#!/bin/bash
# Round-state check: smoke, GPU suite, bench with CPU baseline, rocprof traces (bench and the
# RVQ micro-bench), FETCH / WRITE PMC passes of the RVQ kernels, training bench.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*\|\[smoke\].*\|rvq_encode median.*' "gpurun_out/${TAG}_$name.log" | tail -3
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; grep -E "Error|assert|FAILED" "gpurun_out/${TAG}_$name.log" | head -20; exit $rc; fi; return 0; }
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
run bench 400 python bench.py --steps 20 --warmup 3
run rvq_b32 120 python tools/rvq_bench.py
run rvq_b64 120 python tools/rvq_bench.py --batch 64 --nq 32
run rvq_prof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rvqprof_$TAG -o run --output-format csv -- python tools/rvq_bench.py --iters 20
TAG=${TAG} bash tools/gpu/pmc_rvq.sh || exit 1
run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run train 400 python bench.py --train --steps 3 --warmup 2
exit 0
