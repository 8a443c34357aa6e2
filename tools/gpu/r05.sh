#!/bin/bash
# Round-5 GPU steps (STEPS selects; every step under its own time limit, the first failure ends
# the script): frame-major RVQ tests, the RVQ / fixture tests, RVQ micro-bench, bench line,
# rocprofv3 kernel stats, the whole GPU suite, smoke.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
STEPS=${STEPS:-"fm rvqtests rvqb bench"}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[EW]20" | tail -${TAIL:-6}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
has() { [[ " $STEPS " == *" $1 "* ]]; }
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
has smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has fm && run fm_tests 500 $PT tests/test_gpu_rvq_fm.py
has planes && run planes_tests 500 $PT tests/test_gpu_planes.py
has convtests && run conv_tests 600 $PT tests/test_gpu_parity.py -k "conv or strided or transpose or residual or model_forward or x3"
has rvqtests && run rvq_tests 700 $PT tests/test_gpu_parity.py -k "rvq or golden or model_forward or config or sweep or batch or ragged or deterministic or cbr"
has rvqb && run rvq_b32 180 python tools/rvq_bench.py --batch 32 --nq 8 --variants 3
has rvqb && run rvq_b64 180 python tools/rvq_bench.py --batch 64 --nq 32 --variants 3 --paths fm,2
has stamps && TAIL=45 run stamps 120 python tools/rvq_fused_stamps.py --fm
has bench && run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has benchab && run bench_noplanes 300 env VRVQ_CONV_PLANES=0 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has benchfull && run benchfull 500 python bench.py
has cfg3 && run cfg3 300 python bench.py --batch 64 --n-codebooks 32 --steps 10 --warmup 2 --no-cpu-baseline
has sweep && run sweep 300 python bench.py --sweep --steps 10 --warmup 2 --no-cpu-baseline
has rvqprof && run rvqprof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_rvq -o run --output-format csv -- python tools/rvq_bench.py --batch 32 --nq 8 --iters 20 --paths fm
has prof && run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
has profnp && run profnp 300 env VRVQ_CONV_PLANES=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_np -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
has long && run long_tests 500 $PT tests/test_gpu_long_clip.py
has bench10 && run bench10 400 python bench.py --clip-seconds 10 --batch 1 --sweep --steps 5 --warmup 2 --no-cpu-baseline
has all && run gpu_tests 1000 $PT tests -m gpu
exit 0
