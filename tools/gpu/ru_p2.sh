#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-rup2}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*' "gpurun_out/${TAG}_$name.log" | tail -2
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; grep -E "Error|assert|FAILED" "gpurun_out/${TAG}_$name.log" | head -20; exit $rc; fi; return 0; }
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
run ru_tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "residual_unit or x3 or forward_vs_reference" --timeout 120 --timeout-method thread
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
run default 300 $B
run k1_128 300 env VRVQ_CONV_K1_192=0 $B
run convt_128 300 env VRVQ_CONVT_192=0 $B
run k7_128 300 env VRVQ_CONV_K7_192=0 $B
run all128 300 env VRVQ_CONV_K1_192=0 VRVQ_CONVT_192=0 VRVQ_CONV_K7_192=0 $B
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline
exit 0
