#!/usr/bin/env python
"""Micro-bench of the RVQ kernels alone at BASELINE shapes — the single-launch vrvq_rvq_fused
and the two-kernel path (rvq_codes + rvq_expand) — for rocprofv3 kernel traces / PMC passes
and quick A/B timing with HIP events.  --only fused|pair limits what is launched."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import vrvq_amd  # noqa: E402
from vrvq_amd import ops  # noqa: E402
from vrvq_amd.recipe import load_recipe  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--nq", type=int, default=8)
    ap.add_argument("--frames", type=int, default=87)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", choices=["encode", "fused", "pair", "split", "all"], default="all")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    model = vrvq_amd.DAC_VRVQ(n_codebooks=args.nq)
    load_recipe(model, 0)
    q = model.quantizer.to(dev).eval()
    st = q.stacked()
    g = torch.Generator(device="cpu").manual_seed(1)
    z = (torch.randn(args.batch, 1024, args.frames, generator=g) * 0.3).to(dev)
    imp = torch.rand(args.batch, args.frames, generator=g).to(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(10)]
    tf, tc, te, tp, tch, tx, ts = [], [], [], [], [], [], []
    for it in range(args.iters):
        ev[4].record()
        if args.only in ("encode", "all"):
            B, D, T = z.shape
            part = ops.rvq_project(z, st.w_in_t)
            ev[5].record()
            _, _, _, zst2, _ = ops.rvq_chain(part, B, T, st.b_in, st.qb, st.mcol, st.cb, st.cbn,
                                             st.c2, imp, 1.0)
            ev[6].record()
            ops.rvq_expand(zst2, st.w_out, st.b_out, imp, 1.0, want_mask=False)
        else:
            ev[5].record(); ev[6].record()
        ev[7].record()
        ev[0].record()
        if args.only in ("fused", "all"):
            ops.rvq_fused(z, *st.codes_args(), imp=imp, level=1.0)
        ev[1].record()
        if args.only in ("pair", "all"):
            codes, latents, loss_pf, zst = ops.rvq_codes(z, *st.codes_args())
        ev[2].record()
        if args.only in ("pair", "all"):
            ops.rvq_expand(zst, st.w_out, st.b_out, imp, 1.0)
        ev[3].record()
        ev[8].record()
        if args.only in ("split", "all"):
            ops.rvq_split(z, *st.codes_args(), imp=imp, level=1.0)
        ev[9].record()
        torch.cuda.synchronize()
        if it >= 5:
            tf.append(ev[0].elapsed_time(ev[1]) * 1e3)
            tc.append(ev[1].elapsed_time(ev[2]) * 1e3)
            te.append(ev[2].elapsed_time(ev[3]) * 1e3)
            tp.append(ev[4].elapsed_time(ev[5]) * 1e3)
            tch.append(ev[5].elapsed_time(ev[6]) * 1e3)
            tx.append(ev[6].elapsed_time(ev[7]) * 1e3)
            ts.append(ev[8].elapsed_time(ev[9]) * 1e3)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    byt = args.batch * args.frames * (1024 * 4 * (2 + args.nq) + 4 + args.nq * (8 + 32 + 8))
    enc = med(tp) + med(tch) + med(tx)
    print(f"B={args.batch} nq={args.nq} T={args.frames}: encode path {enc:.1f} us "
          f"({byt / enc / 1e3:.0f} GB/s algorithmic) = project {med(tp):.1f} + chain "
          f"{med(tch):.1f} + expand {med(tx):.1f} us")
    print(f"B={args.batch} nq={args.nq} T={args.frames}: fused median {med(tf):.1f} us "
          f"({byt / med(tf) / 1e3:.0f} GB/s algorithmic); codes {med(tc):.1f} us, "
          f"expand {med(te):.1f} us")
    if args.only in ("split", "all"):
        print(f"B={args.batch} nq={args.nq} T={args.frames}: split median {med(ts):.1f} us "
              f"({byt / med(ts) / 1e3:.0f} GB/s algorithmic)")
        if args.only == "all":
            a = ops.rvq_fused(z, *st.codes_args(), imp=imp, level=1.0)
            b = ops.rvq_split(z, *st.codes_args(), imp=imp, level=1.0)
            torch.cuda.synchronize()
            agree = (a[0] == b[0]).float().mean().item()
            dz = (a[3] - b[3]).abs().max().item()
            print(f"  split vs fused: codes agree {agree:.6f}, z_q_is max |diff| {dz:.3e}, "
                  f"error flag {ops.rvq_split_error(dev)}")

if __name__ == "__main__":
    main()
