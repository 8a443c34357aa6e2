#!/bin/bash
# First run of the single-launch RVQ kernel: its parity tests, micro-bench, then the full GPU
# suite and the bench. Stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-6}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run fused_tests 300 python -u -m pytest tests/test_gpu_parity.py -k "rvq_paths or big_batch" -x -q -rf --timeout 120 --timeout-method thread
run rvq_bench 120 python tools/rvq_bench.py --iters 30
run rvq_bench_nq32 120 python tools/rvq_bench.py --iters 30 --batch 64 --nq 32
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
run bench 400 python bench.py --steps 20 --warmup 3
exit 0
