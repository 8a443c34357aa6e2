#!/bin/bash
# Round-4 check: fused RVQ tests + micro-bench + timeline, conv parity tests, bench line, kernel
# stats. STEPS selects steps (default all but the full GPU suite).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
STEPS=${STEPS:-"fused rvqb stamps conv train bench knob rvqprof prof"}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[EW]20" | tail -${TAIL:-5}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
has() { [[ " $STEPS " == *" $1 "* ]]; }
PT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
has smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has fused && run fused_tests 300 $PT tests/test_gpu_parity.py -k "rvq_fused"
has rvqb && run rvq_b32 120 python tools/rvq_bench.py --batch 32 --nq 8
has rvqb && run rvq_b64 120 python tools/rvq_bench.py --batch 64 --nq 32
has stamps && TAIL=40 run stamps 120 python tools/rvq_fused_stamps.py
has nozqis && TAIL=40 run stamps_nozqis 120 python tools/rvq_fused_stamps.py --no-zqis
has nomfma && TAIL=40 run stamps_nomfma 120 python tools/rvq_fused_stamps.py --no-expand-mfma
has conv && run conv_tests 400 $PT tests/test_gpu_parity.py -k "conv or strided or transpose"
has benchfull && run benchfull 400 python bench.py
has bench && run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has sweep && run sweep 300 python bench.py --sweep --steps 10 --warmup 2 --no-cpu-baseline
has cfg3 && run cfg3 300 python bench.py --batch 64 --n-codebooks 32 --steps 10 --warmup 2 --no-cpu-baseline
has trainb && run trainb 400 python bench.py --train --steps 10 --warmup 3 --no-cpu-baseline
has knob && run bench_bn96 300 env VRVQ_CONV_BN96_MIN=200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has knob && run bench_ph1 300 env VRVQ_CONV_PH128=1 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has knob && run bench_ph2 300 env VRVQ_CONV_PH128=2 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
has knobprof && run prof_ph 300 env VRVQ_CONV_PH128=2 VRVQ_CONV_BN96_MIN=200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_ph -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
has rvqprof && run rvqprof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_rvq -o run --output-format csv -- python tools/rvq_bench.py --batch 32 --nq 8 --iters 20 --paths 2 --variants 3
has pmcrvq && run pmcrvq 300 env TAG=${TAG} RVQ_ARGS="--batch 32 --nq 8 --paths 2 --variants 3" bash tools/gpu/pmc_rvq.sh
has prof && run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
has train && run train_tests 400 $PT tests/test_gpu_train.py -k "wgrad or snake_conv_grads or golden"
has all && run gpu_tests 900 $PT tests -m gpu
exit 0
