#!/bin/bash
# Cout = 1 output conv (96 -> 1 k7 + Tanh at T = 44544, B = 32) + its parity tests.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-c1}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/${TAG}_$name.log" | tail -${TAILN:-2}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run tests 300 python -u -m pytest tests/test_gpu_parity.py -k "conv1d_vs_torch or cout1 or forward_vs_reference or encoder_and_decoder" -x -q -rf --timeout 120 --timeout-method thread
run c1 60 python tools/conv_bench.py --cin 96 --cout 1 --t 44544 --k 7 --no-snake-out
if [ -n "$AB" ]; then
  export VRVQ_TORCH_LIB=$AB/libvrvq_torch.so VRVQ_LIB=$AB/libvrvq_hip.so
  run ab_c1 60 python tools/conv_bench.py --cin 96 --cout 1 --t 44544 --k 7 --no-snake-out
  unset VRVQ_TORCH_LIB VRVQ_LIB
fi
exit 0
