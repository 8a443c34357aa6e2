#!/bin/bash
# k = 1 conv tile A/B, second pass: VRVQ_CONV_K1_192 = 0 | 1 (192-row) | 2 (256-row where M % 256 == 0).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-3}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
for v in 1 2; do
  VRVQ_CONV_K1_192=$v run conv_tests_k1_$v 300 python -u -m pytest tests/test_gpu_parity.py -k "conv1d" -x -q -rf --timeout 120 --timeout-method thread
done
for v in 0 1 2; do
  export VRVQ_CONV_K1_192=$v
  run k1_512_$v 60 python tools/conv_bench.py --cin 512 --cout 512 --t 696 --k 1 --res
  run k1_768_$v 60 python tools/conv_bench.py --cin 768 --cout 768 --t 696 --k 1 --res
done
for v in 1 2; do
  export VRVQ_CONV_K1_192=$v
  run bench_k1_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
exit 0
