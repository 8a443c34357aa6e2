#!/bin/bash
# Round-6 validation of the tree: smoke, the whole GPU suite, bench line (with CPU baseline),
# rocprofv3 kernel stats of the bench step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06z}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | grep -v "^[EW]20" | tail -${TAIL:-3}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
has() { [[ " ${STEPS:-smoke all bench prof} " == *" $1 "* ]]; }
has smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has all && run gpu_tests 900 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests -m gpu
has bench && run bench 400 python bench.py --steps 20 --warmup 5
has prof && run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
has cfg3 && run cfg3 300 python bench.py --batch 64 --n-codebooks 32 --steps 10 --warmup 2 --no-cpu-baseline
has sweep && run sweep 300 python bench.py --sweep --steps 10 --warmup 2 --no-cpu-baseline
has train && run train 400 python bench.py --train --steps 3 --warmup 2
has bench10 && run bench10 400 python bench.py --clip-seconds 10 --batch 1 --sweep --steps 5 --warmup 2 --no-cpu-baseline
exit 0
