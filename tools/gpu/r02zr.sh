#!/bin/bash
# Tile-dispatch knobs re-checked on the current x3 kernels (bench.py, 10 steps each, one box).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/${TAG}_$name.log" | head -1
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -5 "gpurun_out/${TAG}_$name.log"; exit $rc; fi; return 0; }
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
run default 200 $B
run k7_192_0 200 env VRVQ_CONV_K7_192=0 $B
run k7_192_2 200 env VRVQ_CONV_K7_192=2 $B
run mtslow 200 env VRVQ_CONV_MTSLOW=1 $B
run bnrule1 200 env VRVQ_CONV_BN_RULE=1 $B
run k1_192 200 env VRVQ_CONV_K1_192=0 $B
run default2 200 $B
exit 0
