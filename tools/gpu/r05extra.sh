#!/bin/bash
# Round-5 final-state secondary records: configs[2] shape (bench, fm RVQ kernel stats + PMC),
# the configs[4] sweep, the reference driver's 10-s x 12-level shape, the training step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zh}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' '; echo
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -20 "gpurun_out/${T}_$name.log"; exit $rc; fi; return 0; }
run cfg3 300 python bench.py --batch 64 --n-codebooks 32 --steps 10 --warmup 3 --no-cpu-baseline
run sweep 300 python bench.py --sweep --steps 10 --warmup 2 --no-cpu-baseline
run bench10 400 python bench.py --clip-seconds 10 --batch 1 --sweep --steps 5 --warmup 2 --no-cpu-baseline
run train 600 python bench.py --train --steps 5 --warmup 2 --no-cpu-baseline
run rvqprof_cfg3 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_cfg3_rvq -o run --output-format csv -- python tools/rvq_bench.py --batch 64 --nq 32 --iters 20 --paths fm
TAG=${T}_cfg3 RVQ_ARGS="--batch 64 --nq 32 --paths fm" bash tools/gpu/pmc_rvq.sh > /dev/null || exit 1
echo "pmc cfg3 done"
for fl in 0 2 1 3; do
  timeout -k 10 120 python tools/rvq_fused_stamps.py --fm --flags $fl > gpurun_out/${T}_stamps_f$fl.log 2>&1 || exit 1
  echo "stamps flags $fl: $(grep 'last workgroup' gpurun_out/${T}_stamps_f$fl.log)"
done
exit 0
