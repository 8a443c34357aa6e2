#!/bin/bash
# VRVQ_CONV_K7_192 = 1 (192-row k7 tiles at BN 64) vs 2 (also at BN 128: the 384-channel units).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-3}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
VRVQ_CONV_K7_192=2 run conv_tests_k7b 300 python -u -m pytest tests/test_gpu_parity.py -k "conv1d or forward_vs_reference" -x -q -rf --timeout 120 --timeout-method thread
for v in 1 2; do
  export VRVQ_CONV_K7_192=$v
  run k7_384_$v 60 python tools/conv_bench.py --cin 384 --cout 384 --t 5568 --k 7 --dil 3
done
for v in 1 2 1 2; do
  export VRVQ_CONV_K7_192=$v
  run bench_k7b_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
exit 0
