#!/bin/bash
# A/B of conv tile knobs on single layers (tools/conv_bench.py, HIP events, B=32).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/ab
run() { local name=$1; shift
  timeout -k 10 60 "$@" > "gpurun_out/ab/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $(grep -o 'median.*' gpurun_out/ab/$name.log)"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi; }
i=0
for L in "--cin 256 --cout 512 --t 5568 --k 16 --stride 8" \
         "--cin 128 --cout 256 --t 22272 --k 8 --stride 4" \
         "--cin 64 --cout 128 --t 44544 --k 4 --stride 2" \
         "--cin 512 --cout 1024 --t 696 --k 16 --stride 8" \
         "--cin 1536 --cout 768 --t 87 --convt 8" \
         "--cin 768 --cout 384 --t 696 --convt 8" \
         "--cin 384 --cout 192 --t 5568 --convt 4" \
         "--cin 192 --cout 96 --t 22272 --convt 2" \
         "--cin 1024 --cout 1536 --t 87 --k 7 --dil 1" \
         "--cin 1024 --cout 1024 --t 87 --k 3 --dil 1"; do
  i=$((i+1))
  for v in "VRVQ_CONV_BN_RULE=0" "VRVQ_CONV_BN_RULE=1" "VRVQ_CONV_VARIANT=1"; do
    run "l${i}_${v}" env $v python tools/conv_bench.py $L
  done
done
exit 0
