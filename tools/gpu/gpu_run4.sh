#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf -x
for fg in 1 2 3; do VRVQ_RVQ_FG=$fg run rvqbench_fg$fg 300 python tools/rvq_bench.py; done
for fg in 2 3; do VRVQ_RVQ_FG=$fg run rvqbench32_fg$fg 300 python tools/rvq_bench.py --batch 64 --nq 32; done
run bench 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
