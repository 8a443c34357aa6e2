#!/bin/bash
# Tile-choice knobs under the x3 path (bench A/B, B=32).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-knob}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/${TAG}_$name.log" | tail -1
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -5 "gpurun_out/${TAG}_$name.log"; exit $rc; fi; return 0; }
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
run default 300 $B
run k1_128 300 env VRVQ_CONV_K1_192=0 $B
run convt_128 300 env VRVQ_CONVT_192=0 $B
run k7_128 300 env VRVQ_CONV_K7_192=0 $B
run all128 300 env VRVQ_CONV_K1_192=0 VRVQ_CONVT_192=0 VRVQ_CONV_K7_192=0 $B
run mtslow 300 env VRVQ_CONV_MTSLOW=1 $B
exit 0
