#!/usr/bin/env python
"""Single-layer micro-bench of the conv kernels (HIP events; use under rocprofv3 for PMC).

    python tools/conv_bench.py --cin 384 --cout 384 --t 5568 --k 7 --dil 3 --batch 32
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vrvq_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=384)
    ap.add_argument("--cout", type=int, default=384)
    ap.add_argument("--t", type=int, default=5568)
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--dil", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--res", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--convt", type=int, default=0, help="transposed conv with this stride")
    ap.add_argument("--ru", action="store_true",
                    help="fused ResidualUnit (k7 dil --dil, k1, skip) with cin channels")
    ap.add_argument("--snake-in", action="store_true", help="Snake on load (consumer side)")
    ap.add_argument("--no-snake-out", action="store_true", help="no producer-side Snake output")
    ap.add_argument("--raw", action="store_true",
                    help="also write the raw output next to the Snake one (encoder blocks)")
    ap.add_argument("--x3", action="store_true", help="the bf16x3 split path (csrc/conv_x3.h)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(args.batch, args.cin, args.t, generator=g) - 0.5).to(dev)
    alpha = (torch.rand(args.cin, generator=g) + 0.5).to(dev)
    inv = ops.snake_inv_alpha(alpha)
    a_in, i_in = (alpha, inv) if args.snake_in else (None, None)
    ao = (torch.rand(args.cout, generator=g) + 0.5).to(dev)
    osn = None if args.no_snake_out else (ao, ops.snake_inv_alpha(ao))
    if args.ru:
        C = args.cin
        w7 = (torch.randn(C, C, 7, generator=g) * 0.02).to(dev)
        w1 = (torch.randn(C, C, 1, generator=g) * 0.02).to(dev)
        wp7, cp = ops.pack_conv1d_weight(w7)
        wp1, _ = ops.pack_conv1d_weight(w1)
        b = torch.zeros(C, device=dev)
        x_snk = x.clone()  # snake1(x) in the model; any values time the same
        osn = (ao[:C].contiguous(), ops.snake_inv_alpha(ao[:C].contiguous()))
        w73 = ops.pack_x3_weight(wp7, 7) if args.x3 else None
        w13 = ops.pack_x3_weight(wp1, 1) if args.x3 else None
        fn = lambda: ops.residual_unit(x, x_snk, args.dil, wp7, b, alpha, inv, wp1, b, cp,
                                       out_snake=osn, want_raw=True, w7_x3=w73, w1_x3=w13)
        flops = 2.0 * args.batch * C * C * 8 * args.t
    elif args.convt:
        w = (torch.randn(args.cin, args.cout, 2 * args.convt, generator=g) * 0.02).to(dev)
        wp, cp = ops.pack_convt1d_weight(w, args.convt)
        b = torch.zeros(args.cout, device=dev)
        w3 = ops.pack_x3_weight(wp, 2) if args.x3 else None
        fn = lambda: ops.conv_transpose1d(x, wp, args.cout, cp, args.convt, b, a_in, i_in,
                                          out_snake=osn, want_raw=True, w_x3=w3)
        flops = 2.0 * args.batch * args.cin * args.cout * 2 * args.convt * args.t
    else:
        w = (torch.randn(args.cout, args.cin, args.k, generator=g) * 0.02).to(dev)
        wp, cp = ops.pack_conv1d_weight(w)
        b = torch.zeros(args.cout, device=dev)
        pad = (args.k - 1) * args.dil // 2 if args.stride == 1 else (args.stride + 1) // 2
        tout = (args.t + 2 * pad - args.dil * (args.k - 1) - 1) // args.stride + 1
        res = torch.randn(args.batch, args.cout, tout, device=dev) if args.res else None
        w3 = None
        if args.x3:
            w3 = (ops.pack_x3_weight(wp, args.k) if args.stride == 1 else
                  ops.pack_x3_strided_weight(w, args.stride))
        fn = lambda: ops.conv1d(x, wp, args.cout, cp, args.k, args.stride, pad, args.dil, b, a_in,
                                i_in, res, out_snake=osn, want_raw=args.raw or args.res or osn is None,
                                w_x3=w3)
        flops = 2.0 * args.batch * args.cin * args.cout * args.k * tout
    for _ in range(3):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(args.iters):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    med = ts[len(ts) // 2]
    print(f"{vars(args)}: median {med*1e3:.1f} us, {flops / med / 1e9:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
