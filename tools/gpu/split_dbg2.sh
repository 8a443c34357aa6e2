#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
for m in 1 2; do
  echo "=== DBG $m"
  VRVQ_SPLIT_DBG=$m timeout -k 10 60 python -u tools/split_debug2.py 2>&1 | grep -v amdgpu.ids || exit 1
done
