#!/bin/bash
# x3 tile knobs A/B (KNOB, default VRVQ_CONV_X3_WIDE; WIDE_SETS values): conv tests, bench and kernel trace per setting.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-x3w}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | tail -${TAIL:-1} | cut -c1-200
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
for V in ${WIDE_SETS:-0 1 2}; do
  export ${KNOB:-VRVQ_CONV_X3_WIDE}=$V
  run tests_w$V 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "x3 or config2_full_batch"
  run bench_w$V 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  run prof_w$V 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_w$V -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline
done
exit 0
