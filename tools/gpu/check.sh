#!/bin/bash
# Round check on the GPU box: smoke, GPU suite, bench (+ CPU baseline), optional rocprof
# traces / RVQ PMC passes / training bench. Every step under its own time limit; the first
# failure ends the script. STEPS selects steps (default: smoke tests bench).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
STEPS=${STEPS:-"smoke tests bench"}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | tail -${TAIL:-4}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; grep -E "Error|assert|FAILED" "gpurun_out/${TAG}_$name.log" | head -20; exit $rc; fi; return 0; }
has() { [[ " $STEPS " == *" $1 "* ]]; }
has smoke && run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
has tests && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS}
has bench && run bench 500 python bench.py --steps 20 --warmup 3
has benchq && run benchq 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has cfg3 && run cfg3 300 python bench.py --batch 64 --n-codebooks 32 --steps 10 --warmup 3 --no-cpu-baseline
has sweep && run sweep 300 python bench.py --sweep --steps 10 --warmup 3
has rvq && run rvq_b32 120 python tools/rvq_bench.py && run rvq_b64 120 python tools/rvq_bench.py --batch 64 --nq 32
has rvqprof && run rvq_prof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rvqprof_$TAG -o run --output-format csv -- python tools/rvq_bench.py --iters 20
has rvqpmc && { TAG=${TAG} bash tools/gpu/pmc_rvq.sh || exit 1; }
has prof && run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
has train && run train 400 python bench.py --train --steps 3 --warmup 2
exit 0
