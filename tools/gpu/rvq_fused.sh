#!/bin/bash
# Fused RVQ launch: bit-identity / graph / uneven-load tests, the RVQ + fixture GPU tests, the
# micro-bench of both launch structures, rocprofv3 kernel stats of the fused launch.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-fused}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[EW]20" | tail -${TAIL:-6}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run fused_tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 120 --timeout-method thread -k "rvq_fused"
run bench_b32 120 python tools/rvq_bench.py --batch 32 --nq 8
run bench_b64 120 python tools/rvq_bench.py --batch 64 --nq 32
[ -n "$MORE" ] && run rvq_tests 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "rvq or golden or model_forward or from_codes or from_latents or config or sweep or smoke or graph or batch"
[ -n "$PROF" ] && run prof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python tools/rvq_bench.py --batch 32 --nq 8 --iters 20 --paths 2
exit 0
