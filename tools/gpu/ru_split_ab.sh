#!/bin/bash
# End-to-end A/B of which ResidualUnit channel counts run fused (VRVQ_RU_FUSED) on one box.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-rusplit}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | grep -o '"value": [0-9.]*\|median.*\|[0-9]* passed.*' | head -1
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
for rep in 1 2; do
  for v in "f64_96_128_256" "f64_96_256" "f64_128_256" "f64_256" "f96_128_256"; do
    run ${v}_$rep 300 env VRVQ_RU_FUSED=$(echo ${v#f} | tr _ ,) python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  done
done
exit 0
