#!/bin/bash
# Round-6 GPU steps (STEPS selects; every step under its own time limit, the first failure ends
# the script): the projection-epilogue RVQ path's tests, RVQ micro-bench and timeline, bench line,
# rocprofv3 kernel stats, fixture / parity tests, the whole GPU suite, smoke.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06}
STEPS=${STEPS:-"pt rvqb stamps bench"}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[EW]20" | tail -${TAIL:-6}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
has() { [[ " $STEPS " == *" $1 "* ]]; }
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
has smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has pt && run pt_tests 600 $PT tests/test_gpu_rvq_part.py

has rvqtests && run rvq_tests 700 $PT tests/test_gpu_parity.py -k "rvq or golden or model_forward or config or sweep or batch or ragged or deterministic or cbr"
has convtests && run conv_tests 600 $PT tests/test_gpu_parity.py -k "conv or strided or transpose or residual or model_forward or x3"
has long && run long_tests 500 $PT tests/test_gpu_long_clip.py
has rvqb && run rvq_b32 180 python tools/rvq_bench.py --batch 32 --nq 8 --variants 3 --paths pt,2,1
has rvqb && run rvq_b64 180 python tools/rvq_bench.py --batch 64 --nq 32 --variants 3 --paths pt,2
has rvqb10 && run rvq_b1x10 180 python tools/rvq_bench.py --batch 1 --frames 862 --nq 8 --variants 3 --paths pt,2
has stamps && TAIL=50 run stamps 120 python tools/rvq_fused_stamps.py --pt

has bench && run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has benchz && run benchz 300 env VRVQ_RVQ_PROJ=0 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has benchfull && run benchfull 500 python bench.py
has cfg3 && run cfg3 300 python bench.py --batch 64 --n-codebooks 32 --steps 10 --warmup 2 --no-cpu-baseline
has sweep && run sweep 300 python bench.py --sweep --steps 10 --warmup 2 --no-cpu-baseline
has bench10 && run bench10 400 python bench.py --clip-seconds 10 --batch 1 --sweep --steps 5 --warmup 2 --no-cpu-baseline
has train && run train 400 python bench.py --train --steps 3 --warmup 2
has rvqprof && run rvqprof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_rvq -o run --output-format csv -- python tools/rvq_bench.py --batch 32 --nq 8 --iters 20 --paths pt
has rvqprof3 && run rvqprof3 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_cfg3_rvq -o run --output-format csv -- python tools/rvq_bench.py --batch 64 --nq 32 --iters 20 --paths pt
has prof && run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
has all && run gpu_tests 1100 $PT tests -m gpu
exit 0
