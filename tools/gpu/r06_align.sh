#!/bin/bash
# RVQ pt launch at T = 87 / 96 / 88 / 80 frames (B = 32, Nq = 8): does the z_q_is rows' 128-B
# alignment (T a multiple of 32) change the expansion's store rate?
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06a}_align.txt
: > $OUT
for rep in 1 2; do
  for T in 87 96 88 80; do
    r=$(timeout -k 10 120 python tools/rvq_bench.py --paths pt --frames $T --iters 50 2>&1 | grep "^path") || { echo FAIL; exit 1; }
    echo "rep $rep T=$T: $r" | tee -a $OUT
  done
done
exit 0
