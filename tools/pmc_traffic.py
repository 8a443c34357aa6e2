#!/usr/bin/env python
"""HBM bytes per launch of the RVQ kernels from the FETCH_SIZE / WRITE_SIZE rocprofv3 passes
(tools/gpu/pmc_rvq.sh) -> profiles/<tag>_rvq_pmc.json (read by bench.py as roofline.traffic).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 derived counters). Per
MI355X_MICROARCH.md (HBM / rocprofv3), gfx950's FETCH_SIZE reports exactly half of the bytes of
a wide coalesced streaming read, so the fetch bytes are doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores (the expansion's z_q_is / z_q stores are 16 B per lane).

    python tools/pmc_traffic.py gpurun_out/<tag> profiles/<tag>_rvq_pmc.json [launches per call]

The path is rvq_pt_kernel (the launch from the conv's partials), rvq_fm_kernel (r05's frame-major launch) or rvq_fused_kernel where a fused launch ran (one dispatch per <= 32 clips: the
third argument, default 1, scales a dispatch to one rvq_encode call), else the three kernels.
"""
import collections
import csv
import glob
import json
import sys


def per_kernel(root, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{root}_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
                name = name.split("(")[0].split("<")[0].strip()
                vals[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    root, out = sys.argv[1], sys.argv[2]
    per_call = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    fetch = per_kernel(root, "FETCH_SIZE")
    write = per_kernel(root, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f_kib, w_kib = fetch.get(k, 0.0), write.get(k, 0.0)
        kernels[k] = {"fetch_size_kib": f_kib, "write_size_kib": w_kib,
                      "fetch_bytes_corrected": 2 * f_kib * 1024, "write_bytes": w_kib * 1024,
                      "total": 2 * f_kib * 1024 + w_kib * 1024}
    if "rvq_pt_kernel" in kernels:  # the eval encode's launch from the conv's partials (r06)
        path = ["rvq_pt_kernel"]
    elif "rvq_fm_kernel" in kernels:
        path = ["rvq_fm_kernel"]
    elif "rvq_fused_kernel" in kernels:
        path = ["rvq_fused_kernel"]
    else:
        path = [k for k in kernels
                if any(s in k for s in ("rvq_project", "rvq_chain", "rvq_expand"))]
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
                     "python tools/rvq_bench.py, kernel-trace only",
           "fetch_correction": "x2 (MI355X_MICROARCH.md: gfx950 FETCH_SIZE = half the bytes "
                               "of wide coalesced reads)",
           "kernels": kernels,
           "path": path,
           "launches_per_call": per_call,
           "path_total_bytes": per_call * sum(kernels[k]["total"] for k in path),
           "path_total_bytes_uncorrected": per_call * sum(
               1024 * (kernels[k]["fetch_size_kib"] + kernels[k]["write_size_kib"])
               for k in path)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
