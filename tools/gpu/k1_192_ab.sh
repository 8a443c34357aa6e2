#!/bin/bash
# A/B of the x3 k1 + skip GEMMs on 192 x 64 tiles (VRVQ_CONV_K1X3_192=1) against the default.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-k1192}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | grep -o 'median.*\|"value": [0-9.]*\|[0-9]* passed.*' | head -1
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
for c in "384 5568" "768 696"; do set -- $c
  for v in A B A2 B2; do
    case $v in A*) E="";; B*) E="VRVQ_CONV_K1X3_192=1";; esac
    run k1_$1_$v 60 env $E python tools/conv_bench.py --x3 --cin $1 --cout $1 --t $2 --k 1 --res
  done
done
run tests_B 300 env VRVQ_CONV_K1X3_192=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "x3 or conv1d or fixture"
run bench_A 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run bench_B 300 env VRVQ_CONV_K1X3_192=1 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
exit 0
