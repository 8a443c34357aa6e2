#!/bin/bash
# smoke() + the GPU parity suite (+ optional bench), each step under its own time limit.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | tail -${TAIL:-6}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS}
if [ -n "$BENCH" ]; then run bench 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline; fi
exit 0
