#!/bin/bash
# A/B of the ResidualUnit tiles: VRVQ_RU_BN64 (64-wide C = 64 / 128 units) and the
# single-buffered operand build in abtest/ (-DVRVQ_X3_SB_RU -DVRVQ_X3_SB_CONV), per unit and end to end.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04q
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/${T}_$name.log" | tail -1 | cut -c1-200
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; return 0; }
for c in "64 44544" "128 22272"; do set -- $c
  for d in 1 3 9; do
    run ru$1_d${d}_A 60 python tools/conv_bench.py --x3 --ru --cin $1 --t $2 --dil $d
    run ru$1_d${d}_B 60 env VRVQ_RU_BN64=1 python tools/conv_bench.py --x3 --ru --cin $1 --t $2 --dil $d
  done
done
B_ENV="VRVQ_LIB=$PWD/abtest/libvrvq_hip.so VRVQ_TORCH_LIB=$PWD/abtest/libvrvq_torch.so"
for c in "96 44544" "192 22272" "128 22272"; do set -- $c
  for d in 1 9; do
    run ru$1_d${d}_A2 60 python tools/conv_bench.py --x3 --ru --cin $1 --t $2 --dil $d
    run ru$1_d${d}_SB 60 env $B_ENV python tools/conv_bench.py --x3 --ru --cin $1 --t $2 --dil $d
  done
done
for c in "384 384 5568" "256 256 5568" "768 768 696" "512 512 696"; do set -- $c
  run k1_$1_A 60 python tools/conv_bench.py --x3 --cin $1 --cout $2 --t $3 --k 1 --res
  run k1_$1_SB 60 env $B_ENV python tools/conv_bench.py --x3 --cin $1 --cout $2 --t $3 --k 1 --res
done
run st_128_A 60 python tools/conv_bench.py --x3 --cin 128 --cout 256 --t 5568 --k 8 --stride 4
run st_128_SB 60 env $B_ENV python tools/conv_bench.py --x3 --cin 128 --cout 256 --t 5568 --k 8 --stride 4
run bench_SB 300 env $B_ENV python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run test_B 300 env VRVQ_RU_BN64=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "residual_unit or fixture or golden"
run bench_A 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run bench_B 300 env VRVQ_RU_BN64=1 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
exit 0
