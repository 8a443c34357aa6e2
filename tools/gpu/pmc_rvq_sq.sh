#!/bin/bash
# SQ / GRBM counters of the RVQ kernels (one rocprofv3 --pmc pass each, kernel-trace only).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmcsq}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1
grep -o "SQ_[A-Z_0-9]*\|GRBM_[A-Z_0-9]*" gpurun_out/${TAG}_counters.txt | sort -u > gpurun_out/${TAG}_names.txt
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SMEM" ; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "rvq_" -d gpurun_out/${TAG}_p$i -o run --output-format csv -- python tools/rvq_bench.py --iters 10 ${BENCH_ARGS} > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "rc=$rc"; tail -2 gpurun_out/${TAG}_p$i.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
