#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; cat "gpurun_out/$name.log" | grep -v amdgpu.ids | tail -4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf -x
run bench 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
