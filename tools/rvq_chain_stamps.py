#!/usr/bin/env python
"""Per-stage timeline of rvq_chain_kernel from in-kernel s_memtime stamps (diagnostic build
vrvq_amd/libvrvq_hip_stamps.so, built with `python -m vrvq_amd.build --stamps`). Stamps are
taken by lane 0 of waves 0 and 7 of every workgroup at 8 points per stage:
  0 S1 start | 1 after deferred U updates | 2 after prefetch issue | 3 after scan |
  4 after barrier 1 | 5 after S2 argmin/codeword | 6 after next z_e | 7 after barrier 2
Prints the median (over workgroups) cycles between consecutive points, per stage."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vrvq_amd  # noqa: E402
from vrvq_amd.recipe import load_recipe  # noqa: E402

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--nq", type=int, default=8)
    ap.add_argument("--frames", type=int, default=87)
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "vrvq_amd", "libvrvq_hip_stamps.so"))
    dev = torch.device("cuda:0")
    model = vrvq_amd.DAC_VRVQ(n_codebooks=args.nq)
    load_recipe(model, 0)
    q = model.quantizer.to(dev).eval()
    st = q.stacked()
    B, T, nq = args.batch, args.frames, args.nq
    g = torch.Generator(device="cpu").manual_seed(1)
    z = (torch.randn(B, 1024, T, generator=g) * 0.3).to(dev)
    imp = torch.rand(B, T, generator=g).to(dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    NF = B * T
    part = torch.empty(8 * NF * nq * 8, device=dev)
    codes = torch.empty(B, nq, T, dtype=torch.int64, device=dev)
    lat = torch.empty(B, nq * 8, T, device=dev)
    loss = torch.empty(B, nq, T, device=dev)
    zst = torch.empty(B, nq, T, 8, device=dev)
    mask = torch.empty(B, nq, T, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    stamps = torch.zeros(8192 * (nq + 1) * 2 * 8, dtype=torch.int64, device=dev)
    F = min(16, max(1, -(-NF // 256)))
    grid = -(-NF // F)

    def run(with_stamps):
        lib.vrvq_debug_set_stamps(P(stamps) if with_stamps else None)
        rc = lib.vrvq_rvq_project(P(z), B, 1024, T, nq, 8, P(st.w_in_t), P(part), stream)
        assert rc == 0, rc
        rc = lib.vrvq_rvq_chain(P(part), B, T, nq, 1024, 8, P(st.b_in), P(st.qb), P(st.mcol),
                                P(st.cb), P(st.cbf), P(st.c2), P(imp), ctypes.c_float(1.0),
                                P(codes), P(lat), P(loss), P(zst), P(mask), stream)
        assert rc == 0, rc

    for _ in range(5):
        run(False)
    run(True)
    torch.cuda.synchronize()
    ref = vrvq_amd.ops.rvq_encode(z, *st.codes_args(), imp=imp, level=1.0)
    assert torch.equal(ref[0], codes), "stamped build disagrees with the product library"
    s = stamps[: grid * (nq + 1) * 2 * 8].cpu().numpy().reshape(grid, nq + 1, 2, 8).astype(np.int64)
    pro = s[:, nq, 0, :]
    print(f"B={B} nq={nq} T={T}: grid {grid} workgroups x {F} frames")
    print(f"prologue {np.median(pro[:, 1] - pro[:, 0]):.0f} cyc, stages {np.median(pro[:, 2] - pro[:, 1]):.0f}"
          f" cyc, epilogue {np.median(pro[:, 3] - pro[:, 2]):.0f} cyc (wave 0 medians)")
    names = ["deferred", "prefetch", "scan", "barrier1", "S2 argmin", "S2 next e", "barrier2"]
    for w, tag in ((0, "wave0"), (1, "wave7")):
        print(f"{tag}: median cycles per step, per stage")
        for i in range(nq):
            d = np.diff(s[:, i, w, :], axis=1)
            med = np.median(d, axis=0)
            print(f"  stage {i:2d}: " + " ".join(f"{n}={m:6.0f}" for n, m in zip(names, med)) +
                  f"  total {np.median(s[:, i, w, 7] - s[:, i, w, 0]):6.0f}")
    # spread of stage-0 start across workgroups (launch skew)
    st0 = s[:, 0, 0, 0]
    print(f"stage-0 start spread over workgroups: {(st0.max() - st0.min())} cyc; "
          f"end-to-end per WG median {np.median(pro[:, 3] - pro[:, 0]):.0f} cyc")


if __name__ == "__main__":
    main()
