#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 90 python -u tools/split_debug.py > gpurun_out/split_dbg.log 2>&1 || { tail -20 gpurun_out/split_dbg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/split_dbg.log
VRVQ_SPLIT_SYS=1 timeout -k 10 90 python -u tools/split_debug.py > gpurun_out/split_dbg_sys.log 2>&1 || { tail -20 gpurun_out/split_dbg_sys.log; exit 1; }
echo "=== SYS"; grep -v amdgpu.ids gpurun_out/split_dbg_sys.log
