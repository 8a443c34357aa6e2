#!/bin/bash
# The four decoder ConvTranspose1d layers at B=32 (conv_bench, HIP events) + parity tests.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ct}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/${TAG}_$name.log" | tail -${TAILN:-2}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run convt_tests 300 python -u -m pytest tests/test_gpu_parity.py -k "transpose or forward_vs_reference or encoder_and_decoder" -x -q -rf --timeout 120 --timeout-method thread
run ct1536 60 python tools/conv_bench.py --cin 1536 --cout 768 --t 87 --convt 8
run ct768 60 python tools/conv_bench.py --cin 768 --cout 384 --t 696 --convt 8
run ct384 60 python tools/conv_bench.py --cin 384 --cout 192 --t 5568 --convt 4
run ct192 60 python tools/conv_bench.py --cin 192 --cout 96 --t 22272 --convt 2
if [ -n "$AB" ]; then  # the same layers on a baseline build (VRVQ_TORCH_LIB / VRVQ_LIB in $AB/)
  export VRVQ_TORCH_LIB=$AB/libvrvq_torch.so VRVQ_LIB=$AB/libvrvq_hip.so
  run ab_ct1536 60 python tools/conv_bench.py --cin 1536 --cout 768 --t 87 --convt 8
  run ab_ct768 60 python tools/conv_bench.py --cin 768 --cout 384 --t 696 --convt 8
  run ab_ct384 60 python tools/conv_bench.py --cin 384 --cout 192 --t 5568 --convt 4
  run ab_ct192 60 python tools/conv_bench.py --cin 192 --cout 96 --t 22272 --convt 2
  unset VRVQ_TORCH_LIB VRVQ_LIB
fi
[ -n "$BENCH" ] && run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
exit 0
