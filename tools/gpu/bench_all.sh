#!/bin/bash
# Bench lines for configs[1] (default, with CPU baseline), configs[2] shape (B=64, 32 cb) and the
# configs[4] level sweep, plus the RVQ PMC traffic and rocprof kernel stats of configs[1].
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-bench}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[EW]2026" | tail -${TAIL:-3}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run bench 400 python bench.py --steps 20 --warmup 3
run bench_cfg3 300 python bench.py --steps 10 --warmup 2 --batch 64 --n-codebooks 32 --no-cpu-baseline
run bench_sweep 300 python bench.py --steps 10 --warmup 2 --sweep
TAG=${TAG}pmc run pmc 300 bash tools/gpu/pmc_rvq.sh
run rvqprof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python tools/rvq_bench.py --batch 32 --nq 8 --iters 20
run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_step -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
