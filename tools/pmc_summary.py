#!/usr/bin/env python
"""Average PMC counters per dispatch from rocprofv3 counter_collection CSVs under a dir.

    python tools/pmc_summary.py gpurun_out/pmc2 l1
"""
import collections
import csv
import glob
import sys

root, pref = sys.argv[1], sys.argv[2]
agg = collections.OrderedDict()
for f in sorted(glob.glob(f"{root}/{pref}p*/**/*counter_collection.csv", recursive=True)):
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        disp[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    ds = list(disp.values())
    for k in ds[0]:
        agg[k] = sum(d[k] for d in ds) / len(ds)
for k, v in agg.items():
    print(f"  {k:28s} {v:14.4g}")
if "SQ_INSTS_MFMA" in agg and "GRBM_GUI_ACTIVE" in agg:
    cyc = agg["GRBM_GUI_ACTIVE"] / 8
    print(f"  MFMA busy / SIMD-cycles      {agg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * cyc):.3f}")
    print(f"  non-MFMA VALU per MFMA       {(agg['SQ_INSTS_VALU'] - agg['SQ_INSTS_MFMA']) / agg['SQ_INSTS_MFMA']:.2f}")
    print(f"  LDS instr per MFMA           {agg['SQ_INSTS_LDS'] / agg['SQ_INSTS_MFMA']:.2f}")
    w = agg["SQ_WAVE_CYCLES"]
    print(f"  wave-cycle split: wait_any {agg['SQ_WAIT_ANY']/w:.2f} wait_inst {agg['SQ_WAIT_INST_ANY']/w:.2f} active {agg['SQ_ACTIVE_INST_ANY']/w:.2f}")
