#!/bin/bash
# VRVQ_CONVT_192 = 0 | 1: 192-row tiles for the polyphase ConvTranspose1d layers.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-3}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
VRVQ_CONVT_192=1 run convt_tests 300 python -u -m pytest tests/test_gpu_parity.py -k "transpose or forward_vs_reference or encoder_and_decoder" -x -q -rf --timeout 120 --timeout-method thread
for v in 0 1; do
  export VRVQ_CONVT_192=$v
  run ct_768_$v 60 python tools/conv_bench.py --cin 768 --cout 384 --t 696 --convt 8
  run ct_384_$v 60 python tools/conv_bench.py --cin 384 --cout 192 --t 5568 --convt 4
  run ct_1536_$v 60 python tools/conv_bench.py --cin 1536 --cout 768 --t 87 --convt 8
done
for v in 0 1 0 1; do
  export VRVQ_CONVT_192=$v
  run bench_ct_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
exit 0
