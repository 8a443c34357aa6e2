#!/bin/bash
# A/B of the fused RVQ kernel's z_q_is store flavour (VRVQ_RVQ_NT=0 plain | 1 non-temporal):
# RVQ parity tests with the non-temporal stores, the RVQ micro-bench and the full bench for both.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids\|^W2026\|^E2026" "gpurun_out/$name.log" | tail -${TAILN:-4}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
export VRVQ_RVQ_NT=1
run rvq_tests_nt 300 python -u -m pytest tests/test_gpu_parity.py -k "rvq or model" -x -q -rf --timeout 120 --timeout-method thread
for v in 0 1 0 1; do
  export VRVQ_RVQ_NT=$v
  run rvq_fused_nt$v 120 python tools/rvq_bench.py --iters 50 --only fused
done
for v in 0 1; do
  export VRVQ_RVQ_NT=$v
  run rvq_fused_nq32_nt$v 120 python tools/rvq_bench.py --iters 30 --batch 64 --nq 32 --only fused
  run bench_nt$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
exit 0
