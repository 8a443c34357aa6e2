#!/bin/bash
# Training step under MIOpen's find modes (the discriminator's 2-D convolutions): bench --train.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-miopen}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' '; echo
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
run default 300 python bench.py --train --steps 5 --warmup 3 --no-cpu-baseline
run fast 300 env MIOPEN_FIND_MODE=2 python bench.py --train --steps 5 --warmup 3 --no-cpu-baseline
run hybrid 300 env MIOPEN_FIND_MODE=3 python bench.py --train --steps 5 --warmup 3 --no-cpu-baseline
run normal 400 env MIOPEN_FIND_MODE=1 python bench.py --train --steps 5 --warmup 3 --no-cpu-baseline
exit 0
