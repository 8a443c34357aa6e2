#!/bin/bash
# A/B of 192-row k7 conv tiles at BN 64 (VRVQ_CONV_K7_192) on the 768-channel units (T = 696).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-3}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
VRVQ_CONV_K7_192=1 run conv_tests_k7 300 python -u -m pytest tests/test_gpu_parity.py -k "conv1d or forward_vs_reference" -x -q -rf --timeout 120 --timeout-method thread
for v in 0 1; do
  export VRVQ_CONV_K7_192=$v
  run k7_768_$v 60 python tools/conv_bench.py --cin 768 --cout 768 --t 696 --k 7 --dil 3
  run k7_768d9_$v 60 python tools/conv_bench.py --cin 768 --cout 768 --t 696 --k 7 --dil 9
done
for v in 0 1 0 1; do
  export VRVQ_CONV_K7_192=$v
  run bench_k7_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
exit 0
