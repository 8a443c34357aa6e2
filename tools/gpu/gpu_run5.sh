#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; cat "gpurun_out/$name.log" | grep -v amdgpu.ids | tail -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run stamps_fg3 300 python tools/rvq_stamps.py
VRVQ_RVQ_FG=1 run stamps_fg1 300 python tools/rvq_stamps.py
