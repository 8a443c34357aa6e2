#!/bin/bash
# T = 87 tile widths: the phase-split s8 conv at 96 (VRVQ_CONV_PH_T87=96) and the k3 / k7 layers
# at 96 (VRVQ_CONV_BN96_MIN=0), per-layer kernel traces + bench values.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-t87}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*\|passed.*\|failed.*' "gpurun_out/${TAG}_$name.log" | tail -2
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -20 "gpurun_out/${TAG}_$name.log"; exit $rc; fi; return 0; }
P="rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG}"
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline"
run def 300 $P/def -o run --output-format csv -- $B
run ph96 300 env VRVQ_CONV_PH_T87=96 $P/ph96 -o run --output-format csv -- $B
run bn96 300 env VRVQ_CONV_BN96_MIN=0 $P/bn96 -o run --output-format csv -- $B
run both 300 env VRVQ_CONV_PH_T87=96 VRVQ_CONV_BN96_MIN=0 $P/both -o run --output-format csv -- $B
exit 0
