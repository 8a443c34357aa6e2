#!/usr/bin/env python
"""Timeline of a fused RVQ launch (rvq_fused_kernel, or rvq_pt_kernel with --pt) from in-kernel s_memrealtime stamps
(100 MHz, one clock for the whole chip; diagnostic build vrvq_amd/libvrvq_hip_stamps.so, built
with `python -m vrvq_amd.build --stamps`). Thread 0 of every workgroup records:
  projection / chain workgroups: 0 start | 44 z slab in LDS (x3 projection) | 45 projection
      MFMAs done, partial granules issued | 2 thread 0's partials seen (tags valid) | 3 chain
      prologue done | 4 + i end of stage i | 36 epilogue done
  expansion workgroups: 0 start | 1 + i stage i starts (its wait passed) | 40 all stages done |
      41 z_q stored
Prints, in us from the first workgroup's start, the median and max over workgroups."""
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
    ap.add_argument("--no-zqis", action="store_true",
                    help="z_q_is not materialised (the expansion writes z_q only)")
    ap.add_argument("--no-expand-mfma", action="store_true",
                    help="timing experiment: the expansion skips its MFMAs (outputs not checked)")
    ap.add_argument("--pt", action="store_true",
                    help="the launch from the conv's projection partials (vrvq_rvq_encode_part: "
                         "rvq_pt_kernel; partials made here by vrvq_rvq_project)")
    ap.add_argument("--flags", type=int, default=0,
                    help="timing experiment: vrvq_debug_set_fused_flags bits (2: the chain parts "
                         "skip the next stage's codebook fragment loads; outputs not checked)")
    args = ap.parse_args()
    flags = (1 if args.no_expand_mfma else 0) | args.flags
    lib = ctypes.CDLL(os.path.join(HERE, "vrvq_amd", os.environ.get("VRVQ_STAMPS_LIB", "libvrvq_hip_stamps.so")))
    lib.vrvq_rvq_path.restype = ctypes.c_int
    assert lib.vrvq_rvq_path(2) in (1, 2)
    dev = torch.device("cuda:0")
    model = vrvq_amd.DAC_VRVQ(n_codebooks=args.nq)
    load_recipe(model, 0)
    q = model.quantizer.to(dev).eval()
    st = q.stacked()
    B, T, nq = args.batch, args.frames, args.nq
    assert B <= 32, "one launch: at most 32 clips"
    g = torch.Generator(device="cpu").manual_seed(1)
    z = (torch.randn(B, 1024, T, generator=g) * 0.3).to(dev)
    imp = torch.rand(B, T, generator=g).to(dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    codes = torch.empty(B, nq, T, dtype=torch.int64, device=dev)
    lat = torch.empty(B, nq * 8, T, device=dev)
    loss = torch.empty(B, nq, T, device=dev)
    zqis = torch.empty(B, nq, 1024, T, device=dev)
    zq = torch.empty(B, 1024, T, device=dev)
    mask = torch.empty(B, nq, T, device=dev)
    n = ctypes.c_longlong(0)
    assert lib.vrvq_rvq_workspace(B, T, nq, ctypes.byref(n)) == 0
    ws = torch.empty((n.value + 3) // 4, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    grid = 2 * B * 8
    stamps = torch.zeros(grid * 64, dtype=torch.int64, device=dev)

    assert args.pt or T <= 96, "rvq_fused_kernel: T <= 96"

    if args.pt:
        part = torch.empty(8, B * T, nq * 8, device=dev)
        assert lib.vrvq_rvq_project(P(z), B, 1024, T, nq, 8, P(st.w_in_t), P(part), stream) == 0
        n2 = ctypes.c_longlong(0)
        assert lib.vrvq_rvq_workspace_part(B, T, nq, 1024, ctypes.byref(n2)) == 0
        wsp = torch.empty((n2.value + 3) // 4, device=dev)
        F_env = int(os.environ.get("VRVQ_RVQ_PT_F", "0"))
        F = min(F_env, T) if 1 <= F_env <= 16 else min(16, T)  # pt_frames_per_part
        P_parts = (T + F - 1) // F
        n_fb = (T + 95) // 96
        grid = B * (P_parts + 8 * n_fb)
        stamps = torch.zeros(grid * 64, dtype=torch.int64, device=dev)

    def run(with_stamps):
        lib.vrvq_debug_set_fused_stamps(P(stamps) if with_stamps else None)
        if args.pt:
            rc = lib.vrvq_rvq_encode_part(P(part), B, 1024, T, nq, 1024, 8, P(st.b_in), P(st.cb),
                                          P(st.cbf), P(st.c2), P(st.w_out), P(st.b_out),
                                          P(st.mcol), P(st.qb), P(imp), ctypes.c_float(1.0),
                                          P(codes), P(lat), P(loss),
                                          None if args.no_zqis else P(zqis), P(zq), P(mask),
                                          P(wsp), ctypes.c_longlong(wsp.numel() * 4), stream)
            assert rc == 0, rc
            return
        rc = lib.vrvq_rvq_encode(P(z), B, 1024, T, nq, 1024, 8, P(st.w_in_t), P(st.b_in),
                                 P(st.cb), P(st.cbf), P(st.c2), P(st.w_out), P(st.b_out),
                                 P(st.mcol), P(st.qb), P(imp), ctypes.c_float(1.0), P(codes),
                                 P(lat), P(loss), None if args.no_zqis else P(zqis), P(zq),
                                 P(mask), P(ws),
                                 ctypes.c_longlong(ws.numel() * 4), stream)
        assert rc == 0, rc

    for _ in range(5):
        run(False)
    run(True)
    torch.cuda.synchronize()
    if flags:
        lib.vrvq_debug_set_fused_flags(flags)
        stamps.zero_()
        for _ in range(5):
            run(False)
        run(True)
        torch.cuda.synchronize()
        lib.vrvq_debug_set_fused_flags(0)
        print(f"fused flags {flags} (timing experiment: 1 expansion MFMAs skipped, 2 chain "
              "codebook stream skipped)")
    if args.pt:
        ref = vrvq_amd.ops.rvq_encode_part(part, T, st.b_in, st.cb, st.cbf, st.c2, st.w_out,
                                           st.b_out, st.mcol, st.qb, imp=imp, level=1.0)
    else:
        ref = vrvq_amd.ops.rvq_encode(z, *st.codes_args(), imp=imp, level=1.0)
    nocheck = os.environ.get("VRVQ_STAMPS_NOCHECK") == "1"  # timing-only experiment builds
    assert nocheck or flags or torch.equal(ref[0], codes), "stamped build disagrees with the product library"
    if flags:
        zq.copy_(ref[4])
    assert nocheck or torch.equal(ref[4], zq), "stamped build disagrees with the product library"
    if args.no_zqis:
        print("z_q_is not materialised")
    s = stamps.cpu().numpy().reshape(grid, 64).astype(np.int64)
    t0 = s[:, 0].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731
    npc = B * (P_parts if args.pt else 8)
    pc, ex = s[:npc], s[npc:]

    def row(name, v):
        v = us(v)
        print(f"  {name:34s} median {np.median(v):7.2f}  max {v.max():7.2f}  min {v.min():7.2f}")

    print(f"B={B} nq={nq} T={T}: {len(pc)} chain + {len(ex)} expansion workgroups (us)")
    print("projection / chain workgroups")
    row("start", pc[:, 0])
    if not args.pt:
        row("z slab in LDS", pc[:, 44])
        row("projection MFMAs + stores issued", pc[:, 45])
        row("clip's partials seen (thread 0)", pc[:, 2])
    row("prologue done", pc[:, 3])
    for i in range(nq):
        row(f"stage {i} end", pc[:, 4 + i])
    row("epilogue done", pc[:, 36])
    print("expansion workgroups")
    row("start", ex[:, 0])
    for i in range(nq):
        if i < 8:
            row(f"stage {i} slice seen ({'loader' if args.pt else 'thread 0'})", ex[:, 56 + i])
        row(f"stage {i} start", ex[:, 1 + i])
        if i < 8:
            row(f"stage {i} stores issued (thread 0)", ex[:, 48 + i])
    row("stages done", ex[:, 40])
    row("z_q stored", ex[:, 41])
    end = max(us(pc[:, 36]).max(), us(ex[:, 41]).max())
    print(f"last workgroup done at {end:.2f} us")


if __name__ == "__main__":
    main()
