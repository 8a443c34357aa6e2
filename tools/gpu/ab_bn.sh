#!/bin/bash
# A/B of the conv tile-width rule (VRVQ_CONV_BN_RULE) on the bench + per-layer trace.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 0 1; do
  echo "=== rule $r"
  VRVQ_CONV_BN_RULE=$r timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bn$r.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bn$r.log
done
VRVQ_CONV_BN_RULE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bn1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bn1.log 2>&1 || exit 1
exit 0
