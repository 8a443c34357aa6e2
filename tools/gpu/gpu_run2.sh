#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf -x
run bench 600 python bench.py --steps 10 --warmup 3 --cpu-clips 16
run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
find gpurun_out/prof -name "*stats*" | head
