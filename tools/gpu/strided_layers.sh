#!/bin/bash
# The four strided encoder convs at B=32 (conv_bench, HIP events, raw + Snake outputs as in the
# model) + parity tests; AB=<dir> repeats the layers on a baseline build.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-st}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/${TAG}_$name.log" | tail -${TAILN:-2}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
layers() {
  run ${1}s2 60 python tools/conv_bench.py --cin 64 --cout 128 --t 44544 --k 4 --stride 2 --raw
  run ${1}s4 60 python tools/conv_bench.py --cin 128 --cout 256 --t 22272 --k 8 --stride 4 --raw
  run ${1}s8a 60 python tools/conv_bench.py --cin 256 --cout 512 --t 5568 --k 16 --stride 8 --raw
  run ${1}s8b 60 python tools/conv_bench.py --cin 512 --cout 1024 --t 696 --k 16 --stride 8 --no-snake-out
}
run tests 300 python -u -m pytest tests/test_gpu_parity.py -k "strided or forward_vs_reference or encoder_and_decoder or conv" -x -q -rf --timeout 120 --timeout-method thread
layers new_
if [ -n "$AB" ]; then
  export VRVQ_TORCH_LIB=$AB/libvrvq_torch.so VRVQ_LIB=$AB/libvrvq_hip.so
  layers ab_
  unset VRVQ_TORCH_LIB VRVQ_LIB
fi
[ -n "$BENCH" ] && run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
exit 0
