#!/usr/bin/env python
"""Micro-bench of the RVQ operator alone (torch.ops.vrvq.rvq_encode: project -> chain ->
expand) at BASELINE shapes, for rocprofv3 kernel traces / PMC passes and quick timing with HIP
events on the launch stream. Prints the median per-call time and the algorithmic HBM rate
(bytes per SURVEY.md §8(d), the same formula as bench.py)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import vrvq_amd  # noqa: E402
from vrvq_amd import ops  # noqa: E402
from vrvq_amd.recipe import load_recipe  # noqa: E402


def rvq_bytes(B, T, nq, D=1024, d=8, N=1024, from_partials=False):
    """bench.py's count: SURVEY §8(d); from_partials (path pt) reads the 8 channel-split in_proj
    partials instead of z, and not W_in."""
    inp = 8 * nq * d * 4 if from_partials else D * 4
    per_frame = inp + 4 + nq * D * 4 + D * 4 + nq * 8 + nq * d * 4 + nq * 4 + nq * 4
    return B * T * per_frame + nq * 4 * ((0 if from_partials else d * D) + d + 2 * N * d +
                                         D * d + D)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--nq", type=int, default=8)
    ap.add_argument("--frames", type=int, default=87)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-zqis", action="store_true", help="want_z_q_is=False (z_q only)")
    ap.add_argument("--variants", default="3,2", help="projection kernel variants to time (2,3)")
    ap.add_argument("--paths", default="pt,2,1",
                    help="RVQ launch structures to time (pt: the launch from the conv's projection "
                         "partials, the eval encode's; on channel-major z: 2 fused, 1 three "
                         "launches)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    model = vrvq_amd.DAC_VRVQ(n_codebooks=args.nq)
    load_recipe(model, 0)
    q = model.quantizer.to(dev).eval()
    st = q.stacked()
    g = torch.Generator(device="cpu").manual_seed(1)
    z = (torch.randn(args.batch, 1024, args.frames, generator=g) * 0.3).to(dev)
    imp = torch.rand(args.batch, args.frames, generator=g).to(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    run = lambda: ops.rvq_encode(z, *st.codes_args(), imp=imp, level=1.0,  # noqa: E731
                                 want_z_q_is=not args.no_zqis)
    from vrvq_amd import _lib
    part = torch.empty(8, args.batch * args.frames, args.nq * 8, device=dev)
    import ctypes
    _lib.call("vrvq_rvq_project", ctypes.c_void_p(z.data_ptr()), args.batch, 1024, args.frames,
              args.nq, 8, ctypes.c_void_p(st.w_in_t.data_ptr()), ctypes.c_void_p(part.data_ptr()),
              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    run_pt = lambda: ops.rvq_encode_part(part, args.frames, st.b_in, st.cb, st.cbf, st.c2,  # noqa: E731
                                         st.w_out, st.b_out, st.mcol, st.qb, imp=imp, level=1.0,
                                         want_z_q_is=not args.no_zqis)
    runs = []
    for p in args.paths.split(","):
        if p == "pt":
            runs.append((p, 0))
        else:
            runs += [(int(p), int(x)) for x in args.variants.split(",")]
    for path, v in runs:
        if path == "pt":
            run = run_pt
            _lib.rvq_path(2)  # (a numeric path left at 1 would select pt's two-launch form)
        else:
            run = lambda: ops.rvq_encode(z, *st.codes_args(), imp=imp, level=1.0,  # noqa: E731
                                         want_z_q_is=not args.no_zqis)
            _lib.rvq_project_variant(v)
            _lib.rvq_path(path)
        ts = []
        for it in range(args.iters):
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            if it >= min(5, args.iters - 1):
                ts.append(e0.elapsed_time(e1) * 1e3)
        med = sorted(ts)[len(ts) // 2]
        # back to back: the host enqueues ahead of the GPU, as inside bench.py's step
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        b2b = e0.elapsed_time(e1) * 1e3 / args.iters
        # the fused launches' own duration (HIP events in their dispatch packets)
        _lib.rvq_timing_read()
        _lib.rvq_timing(True)
        for _ in range(args.iters):
            run()
        torch.cuda.synchronize()
        kms, kn = _lib.rvq_timing_read()
        _lib.rvq_timing(False)
        byt = rvq_bytes(args.batch, args.frames, args.nq, from_partials=path == "pt")
        tag = "rvq_encode no z_q_is" if args.no_zqis else "rvq_encode"
        print(f"path {path} projection v{v} B={args.batch} nq={args.nq} T={args.frames}: {tag} median "
              f"{med:.1f} us (min {min(ts):.1f}), {byt / med / 1e3:.0f} GB/s algorithmic "
              f"({byt / med / 1e3 / 8000:.3f} of 8 TB/s), {byt / 1e6:.1f} MB; back to back "
              f"{b2b:.1f} us/call ({byt / b2b / 1e3 / 8000:.3f})"
              + (f"; kernel {kms * 1e3:.1f} us x {kn // args.iters} launches/call "
                 f"({byt / (kms * 1e3 * (kn // args.iters)) / 1e3 / 8000:.3f})" if kn else ""))


if __name__ == "__main__":
    main()
