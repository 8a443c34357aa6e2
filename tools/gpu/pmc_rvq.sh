#!/bin/bash
# HBM traffic of the RVQ kernels from PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# passes (MI355X_MICROARCH.md, HBM / rocprofv3 PMC slots), kernel-trace only, no sys-trace.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
for c in FETCH_SIZE WRITE_SIZE; do
  echo "=== $c"
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "rvq_" -d gpurun_out/${TAG}_$c -o run --output-format csv -- python tools/rvq_bench.py --iters 10 ${RVQ_ARGS} > gpurun_out/${TAG}_$c.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python tools/pmc_traffic.py gpurun_out/${TAG} gpurun_out/${TAG}_rvq_pmc.json ${PER_CALL:-1}
exit 0
