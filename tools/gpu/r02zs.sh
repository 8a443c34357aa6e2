#!/bin/bash
# configs[2] shape (B=64, 32 codebooks) and configs[4] sweep on the round-state code.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/${TAG}_$name.log" | head -1
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -5 "gpurun_out/${TAG}_$name.log"; exit $rc; fi; return 0; }
run cfg3 300 python bench.py --batch 64 --n-codebooks 32 --steps 10 --warmup 3 --no-cpu-baseline
run sweep 300 python bench.py --sweep --steps 10 --warmup 3
exit 0
