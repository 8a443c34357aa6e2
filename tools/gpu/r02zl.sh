#!/bin/bash
# T = 87 tile width A/B (VRVQ_CONV_BN96_MIN) per layer and end to end, training tests + bench with
# the strided x3 convs, then the SQ counters of the x3 kernels (tools/gpu/pmc_x3.sh).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*\|median.*' "gpurun_out/${TAG}_$name.log" | tail -2
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; grep -E "Error|assert|FAILED" "gpurun_out/${TAG}_$name.log" | head -20; exit $rc; fi; return 0; }
for V in 384 256 0; do
  run l_s8_$V 60 env VRVQ_CONV_BN96_MIN=$V python tools/conv_bench.py --x3 --cin 512 --cout 1024 --t 696 --k 16 --stride 8
  run l_k3_$V 60 env VRVQ_CONV_BN96_MIN=$V python tools/conv_bench.py --x3 --cin 1024 --cout 1024 --t 87 --k 3
  run l_k3b_$V 60 env VRVQ_CONV_BN96_MIN=$V python tools/conv_bench.py --x3 --cin 1024 --cout 512 --t 87 --k 3
  run bench_$V 300 env VRVQ_CONV_BN96_MIN=$V python bench.py --steps 10 --warmup 3 --no-cpu-baseline
done
run pytest_train 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -rf --timeout 120 --timeout-method thread
run train 400 python bench.py --train --steps 3 --warmup 2
bash tools/gpu/pmc_x3.sh
