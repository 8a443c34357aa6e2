#!/bin/bash
# SQ counters of the pt launch (chain and expansion waves together), one pass, kernel-trace only.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06y}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-include-regex "rvq_pt" -d gpurun_out/${TAG}_p1 -o run --output-format csv -- python tools/rvq_bench.py --paths pt --iters 5 > gpurun_out/${TAG}_p1.log 2>&1 || { tail -5 gpurun_out/${TAG}_p1.log; exit 1; }
python tools/pmc_summary.py gpurun_out ${TAG}_ || true
exit 0
