#!/bin/bash
# First run of the channel-split RVQ kernel: micro-bench + comparison, then its parity tests.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-8}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run split_bench 90 python -u tools/rvq_bench.py --iters 20
run split_tests 300 python -u -m pytest tests/test_gpu_parity.py -k "rvq_paths or big_batch" -x -q -rf --timeout 120 --timeout-method thread
run split_bench_nq32 90 python -u tools/rvq_bench.py --iters 20 --batch 64 --nq 32
VRVQ_SPLIT_GMAX=64 run split_bench_g64 90 python -u tools/rvq_bench.py --iters 20 --only split
exit 0
