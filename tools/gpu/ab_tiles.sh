#!/bin/bash
# A/B of the x3 tile families (VRVQ_X3_TILE 0 / 1 / 2): conv parity tests under each, the bench,
# and a rocprofv3 kernel trace per mode for tools/layer_table.py.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-tiles}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | tail -${TAIL:-1} | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
for m in ${MODES:-1 2}; do
  VRVQ_X3_TILE=$m run tests_m$m 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "conv or model_forward or encoder or config2"
done
for m in ${MODES:-1 2} 0; do
  VRVQ_X3_TILE=$m run bench_m$m 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  VRVQ_X3_TILE=$m run prof_m$m 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_m$m -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline
done
exit 0
