#!/bin/bash
# RVQ projection A/B: bit-identity + RVQ parity tests, micro-bench of both projection kernels
# (configs 2 and 3), rocprofv3 kernel trace of the default.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-rvqp}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | tail -${TAIL:-6} | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rvq or from_latents or from_codes or golden or config"
run bench_b32 120 python tools/rvq_bench.py --variants 1,2,1,2
run bench_b64 120 python tools/rvq_bench.py --batch 64 --nq 32 --variants 1,2
run prof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python tools/rvq_bench.py --iters 20
exit 0
