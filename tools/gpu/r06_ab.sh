#!/bin/bash
# A/B of rvq_pt_kernel knobs (VRVQ_RVQ_WARM, VRVQ_RVQ_XF) on one box: the RVQ micro-bench's
# kernel time per combination, alternating, then the stamped timeline of one combination.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06ab}
COMBOS=${COMBOS:-"1:0 0:0 0:1 0:2 0:3 1:2"}
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
for rep in 1 2; do
  for c in $COMBOS; do
    w=${c%%:*}; x=${c##*:}
    r=$(VRVQ_RVQ_WARM=$w VRVQ_RVQ_XF=$x timeout -k 10 120 python tools/rvq_bench.py --batch ${B:-32} --nq ${NQ:-8} --paths pt --iters 50 2>&1 | grep "^path") || { echo "FAIL warm=$w xf=$x"; exit 1; }
    echo "rep $rep warm=$w xf=$x: $r" | tee -a $OUT
  done
done
if [ -n "$STAMP" ]; then
  w=${STAMP%%:*}; x=${STAMP##*:}
  VRVQ_RVQ_WARM=$w VRVQ_RVQ_XF=$x timeout -k 10 120 python tools/rvq_fused_stamps.py --pt > gpurun_out/${TAG}_stamps.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/${TAG}_stamps.log | tail -45
fi
exit 0
