#!/bin/bash
# Fused-ResidualUnit channel set A/B (VRVQ_RU_FUSED): bench + kernel trace per setting, after the
# GPU suite. RU_SETS: space-separated comma lists.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-ruab}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | tail -${TAIL:-1} | cut -c1-200
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
[ -n "$TESTS" ] && run tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
i=0
for S in ${RU_SETS:-64,96,128,192,256 64,96,128,256}; do
  i=$((i+1))
  VRVQ_RU_FUSED=$S run bench_s$i 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  VRVQ_RU_FUSED=$S run prof_s$i 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_s$i -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline
done
exit 0
