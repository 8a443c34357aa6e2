#!/bin/bash
# Fused ResidualUnit: its parity tests first, then the full GPU suite, the bench and a rocprof
# kernel-trace of a short bench run. Stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ru}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-4}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run ru_tests 300 python -u -m pytest tests/test_gpu_parity.py -k "residual_unit" -x -q -rf --timeout 120 --timeout-method thread
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
run bench 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
