#!/usr/bin/env python
"""Micro-bench of the RVQ kernels alone (rvq_codes + rvq_expand) at BASELINE shapes, for
rocprofv3 kernel traces / PMC passes and quick A/B timing with HIP events."""
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
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    model = vrvq_amd.DAC_VRVQ(n_codebooks=args.nq)
    load_recipe(model, 0)
    q = model.quantizer.to(dev).eval()
    st = q.stacked()
    g = torch.Generator(device="cpu").manual_seed(1)
    z = (torch.randn(args.batch, 1024, args.frames, generator=g) * 0.3).to(dev)
    imp = torch.rand(args.batch, args.frames, generator=g).to(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tc, te = [], []
    for it in range(args.iters):
        ev[0].record()
        codes, latents, loss_pf, zst = ops.rvq_codes(z, *st.codes_args())
        ev[1].record()
        ops.rvq_expand(zst, st.w_out, st.b_out, imp, 1.0)
        ev[2].record()
        torch.cuda.synchronize()
        if it >= 5:
            tc.append(ev[0].elapsed_time(ev[1]) * 1e3)
            te.append(ev[1].elapsed_time(ev[2]) * 1e3)
    tc.sort(); te.sort()
    print(f"B={args.batch} nq={args.nq} T={args.frames}: codes median {tc[len(tc)//2]:.1f} us, "
          f"expand median {te[len(te)//2]:.1f} us")


if __name__ == "__main__":
    main()
