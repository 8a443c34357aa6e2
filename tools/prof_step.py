#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace database: per-kernel stats and the kernel sequence of
the last bench step (the dispatches after the last rvq_codes kernel's predecessor boundary)."""
import glob
import re
import sqlite3
import sys


def short(name):
    m = re.search(r"conv_mfma_kernel<([^>]*)>", name)
    if m:
        return "conv<" + m.group(1) + ">"
    m = re.search(r"::(\w+_kernel)", name)
    return m.group(1) if m else name[:40]


def main(path):
    db = glob.glob(path + "/**/*.db", recursive=True)[0] if not path.endswith(".db") else path
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, duration, grid_x, workgroup_x, vgpr_count, lds_size from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if "rvq_codes_kernel" in r[0]]
    print(f"{len(rows)} dispatches, {len(idx)} rvq_codes launches")
    # one step = from the first encoder conv after the previous step's decoder to the final conv
    if len(idx) >= 2:
        a, b = idx[-2], idx[-1]
        step = rows[a:b]
        # rotate: step starts at first conv after previous rvq (encoder of next step begins after decoder)
        tot = sum(r[1] for r in step) / 1e3
        print(f"one step (rvq_codes -> next rvq_codes): {len(step)} kernels, {tot:.3f} ms busy")
        for r in step:
            print(f"  {short(r[0]):28s} {r[1]/1e3:9.3f} us  grid={r[2]//max(r[3],1):7d} vgpr={r[4]} lds={r[5]}")
    print("\nper-kernel totals (all dispatches):")
    agg = {}
    for r in rows:
        k = short(r[0])
        n, t = agg.get(k, (0, 0))
        agg[k] = (n + 1, t + r[1])
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:28s} calls={n:5d} total={t/1e6:9.3f} ms avg={t/n/1e3:9.2f} us")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
