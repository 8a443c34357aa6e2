#!/bin/bash
# Stamped timelines of the pt launch: as built, without the chain's per-stage codebook stream
# (flags 2), without the expansion's MFMAs (flags 1); timing-only flags.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06d}_diag.txt
: > $OUT
for rep in 1 2; do
for f in 0 2 1 3; do
  echo "=== rep $rep flags $f" >> $OUT
  timeout -k 10 120 python tools/rvq_fused_stamps.py --pt --flags $f 2>&1 | grep -v amdgpu.ids | grep -E "stage 7 end|epilogue|stages done|z_q stored|last workgroup|flags" >> $OUT || exit 1
done
done
cat $OUT
exit 0
