#!/bin/bash
# Round-6 RVQ records of the pt launch: PMC traffic (FETCH / WRITE passes) and rocprofv3 kernel
# stats at the configs[1] (B=32, Nq=8) and configs[2] (B=64, Nq=32) shapes.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06r}
TAG=${TAG} RVQ_ARGS="--paths pt" bash tools/gpu/pmc_rvq.sh || exit 1
TAG=${TAG}_cfg3 RVQ_ARGS="--paths pt --batch 64 --nq 32" PER_CALL=2 bash tools/gpu/pmc_rvq.sh || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_rvq -o run --output-format csv -- python tools/rvq_bench.py --batch 32 --nq 8 --iters 20 --paths pt > gpurun_out/${TAG}_rvqprof.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_cfg3_rvq -o run --output-format csv -- python tools/rvq_bench.py --batch 64 --nq 32 --iters 20 --paths pt > gpurun_out/${TAG}_cfg3_rvqprof.log 2>&1 || exit 1
grep "^path" gpurun_out/${TAG}_rvqprof.log gpurun_out/${TAG}_cfg3_rvqprof.log
exit 0
