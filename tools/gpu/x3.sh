#!/bin/bash
# bf16x3 conv path: kernel parity first, then the full GPU suite, bench A/B (x3 on / off) and
# a rocprofv3 kernel trace of the x3 bench.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-x3}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[WE]2026" | tail -${TAIL:-4}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run x3_tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "x3" --timeout 120 --timeout-method thread
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
run bench_x3 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run bench_fp32 300 env VRVQ_CONV_X3=0 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
