#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
LAYERS=("--cin 384 --cout 384 --t 5568 --k 7 --dil 3" "--cin 192 --cout 192 --t 22272 --k 7 --dil 3"
        "--cin 96 --cout 96 --t 44544 --k 7 --dil 3" "--cin 128 --cout 128 --t 22272 --k 7 --dil 3"
        "--cin 64 --cout 64 --t 44544 --k 7 --dil 3" "--cin 192 --cout 192 --t 22272 --k 1 --res"
        "--cin 384 --cout 192 --t 5568 --convt 4" "--cin 192 --cout 96 --t 22272 --convt 2")
for v in 0 1; do
  for L in "${LAYERS[@]}"; do
    VRVQ_CONV_VARIANT=$v timeout -k 5 60 python tools/conv_bench.py $L 2>&1 | grep median | sed "s/^/v$v /" || exit 1
  done
done
VRVQ_CONV_VARIANT=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>&1 | grep metric
