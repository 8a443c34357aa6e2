#!/bin/bash
# configs[2] shape (B=64, 32 codebooks): bench line, rocprofv3 kernel trace of the bench, RVQ
# kernel split and PMC traffic of the RVQ path at that shape.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-cfg3}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | tail -${TAIL:-1} | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run bench 300 python bench.py --batch 64 --n-codebooks 32 --steps 10 --warmup 3 --no-cpu-baseline
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python bench.py --batch 64 --n-codebooks 32 --steps 3 --warmup 2 --no-cpu-baseline
run rvqprof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rvqprof_$T -o run --output-format csv -- python tools/rvq_bench.py --batch 64 --nq 32 --iters 20 --paths 2 --variants 3
TAG=${T} PER_CALL=2 RVQ_ARGS="--batch 64 --nq 32 --paths 2 --variants 3" bash tools/gpu/pmc_rvq.sh || exit 1
exit 0
