#!/bin/bash
# A/B of two builds of the library on one box: the in-tree vrvq_amd/ build (A) and the build in
# abtest/ (B, a copy of libvrvq_hip.so + libvrvq_torch.so built with other -D flags; loaded
# through VRVQ_LIB / VRVQ_TORCH_LIB). CASES: conv_bench.py argument sets; BENCH=1 adds bench.py.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-ab}
B_ENV="VRVQ_LIB=$PWD/abtest/libvrvq_hip.so VRVQ_TORCH_LIB=$PWD/abtest/libvrvq_torch.so"
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | tail -1 | cut -c1-260
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
i=0
while IFS= read -r c; do
  [ -z "$c" ] && continue
  i=$((i+1))
  for rep in 1 2; do
    run c${i}_A_$rep 60 python tools/conv_bench.py $c
    run c${i}_B_$rep 60 env $B_ENV python tools/conv_bench.py $c
  done
done <<< "$CASES"
if [ "${BENCH:-0}" = 1 ]; then
  run bench_A 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  run bench_B 300 env $B_ENV python bench.py --steps 20 --warmup 3 --no-cpu-baseline
fi
exit 0
