#!/bin/bash
# Per-layer time of the split-K T <= 96 layers against the forced part count S.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ks}_sweep.txt
: > $OUT
for L in "--cin 512 --cout 1024 --t 696 --k 16 --stride 8" "--cin 1024 --cout 1024 --t 87 --k 3" \
         "--cin 1024 --cout 512 --t 87 --k 3" "--cin 512 --cout 128 --t 87 --k 3" \
         "--cin 1024 --cout 1536 --t 87 --k 7"; do
  for sk in ${SWEEP:-0 2 3 4 6 8}; do
    r=$(VRVQ_CONV_SPLITK=$sk timeout -k 10 60 python tools/conv_bench.py --x3 $L 2>&1 | grep median) || { echo FAIL; exit 1; }
    echo "S=$sk $L: ${r##*:}" | tee -a $OUT
  done
done
exit 0
