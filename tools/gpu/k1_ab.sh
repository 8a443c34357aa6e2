#!/bin/bash
# A/B of the 192-row k = 1 conv tiles (VRVQ_CONV_K1_192): conv parity with the knob on, the
# k = 1 + skip layers of the 384 / 768 / 512-channel units, and the full bench, both ways.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-3}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
VRVQ_CONV_K1_192=1 run conv_tests_k1 300 python -u -m pytest tests/test_gpu_parity.py -k "conv1d" -x -q -rf --timeout 120 --timeout-method thread
for v in 0 1; do
  export VRVQ_CONV_K1_192=$v
  run k1_384_$v 60 python tools/conv_bench.py --cin 384 --cout 384 --t 5568 --k 1 --res
  run k1_768_$v 60 python tools/conv_bench.py --cin 768 --cout 768 --t 696 --k 1 --res
  run bench_k1_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
exit 0
