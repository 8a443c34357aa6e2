#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf -x
run rvqbench 300 python tools/rvq_bench.py
run rvqbench32 300 python tools/rvq_bench.py --batch 64 --nq 32
run pmc_rvq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS --kernel-include-regex "rvq_.*" -d gpurun_out/pmc_rvq -o run --output-format csv -- python tools/rvq_bench.py --iters 10
run bench 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
