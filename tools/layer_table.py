#!/usr/bin/env python
"""Per-layer conv efficiency from a rocprofv3 kernel trace.

Runs the model's forward on CPU with the ops layer replaced by shape-only fakes to get the
conv launch sequence (Cin, Cout, k, stride, dil, Tout), then matches it against the last step's
conv dispatches in a rocprofv3 --kernel-trace CSV and prints FLOPs, time and TFLOP/s per layer.

    python tools/layer_table.py gpurun_out/prof_X/run_kernel_trace.csv [--batch 32]
"""
import argparse
import csv
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vrvq_amd import ops  # noqa: E402

CALLS = []


def _fake():
    def conv1d(x, wp, cout, cout_pad, k, stride=1, pad=0, dil=1, bias=None, alpha=None,
               inv_alpha=None, residual=None, epilogue=0, out_snake=None, want_raw=True,
               w_x3=None):
        B, cin, tin = x.shape
        tout = (tin + 2 * pad - dil * (k - 1) - 1) // stride + 1
        CALLS.append(("conv", cin, cout, k, stride, dil, tout, B,
                      2.0 * B * cout * tout * cin * k, residual is not None))
        y = torch.empty(B, cout, tout)
        if out_snake is None:
            return y
        return y, torch.empty_like(y)

    def conv1d_proj(x, wp, cout, k, w3in, nq, pad=0, dil=1, bias=None, alpha=None,
                    inv_alpha=None, w_x3=None, want_z=False):
        B, cin, tin = x.shape
        tout = tin + 2 * pad - dil * (k - 1)
        CALLS.append(("conv", cin, cout, k, 1, dil, tout, B, 2.0 * B * cout * tout * cin * k,
                      False))
        return torch.empty(8, B * tout, 8 * nq), (torch.empty(B, cout, tout) if want_z else None)

    def convt(x, wp, cout, cout_pad, stride, bias=None, alpha=None, inv_alpha=None,
              out_snake=None, want_raw=True, pad=-1, w_x3=None):
        B, cin, tin = x.shape
        CALLS.append(("convT", cin, cout, 2 * stride, stride, 1, tin * stride, B,
                      2.0 * B * cin * cout * tin * 2 * stride, False))
        y = torch.empty(B, cout, tin * stride)
        if out_snake is None:
            return y
        return y, torch.empty_like(y)

    def residual_unit(x, x_snk, dil, w7, b7, alpha2, inv_alpha2, w1, b1, cout_pad,
                      out_snake=None, want_raw=True, w7_x3=None, w1_x3=None):
        B, C, T = x.shape
        CALLS.append(("RU", C, C, 7, 1, dil, T, B, 2.0 * B * C * T * C * 8, True))
        y = torch.empty(B, C, T)
        return y if out_snake is None else (y, torch.empty_like(y))

    ops.conv1d = conv1d
    ops.conv_transpose1d = convt
    ops.residual_unit = residual_unit
    ops.weight_norm = lambda g, v: v
    ops.snake_inv_alpha = lambda a: a
    ops.pack_conv1d_weight = lambda w: (w, 128)
    ops.pack_convt1d_weight = lambda w, s: (w, 128)
    ops.pack_x3_weight = lambda w, k: w
    ops.codebook_prep = lambda cb: (cb, cb[..., 0])

    def rvq_codes(z, w_in_t, b_in, cb, cbn, c2, w_out, b_out):
        B, D, T = z.shape
        nq = cb.shape[0]
        return (torch.zeros(B, nq, T, dtype=torch.long), torch.empty(B, nq * 8, T),
                torch.empty(B, nq, T), torch.empty(B, nq, T, 8))

    def rvq_expand(zst, w_out, b_out, imp=None, level=1.0, want_z_q_is=True, want_mask=True):
        B, nq, T, d = zst.shape
        D = w_out.shape[1]
        return torch.empty(B, nq, D, T), torch.empty(B, D, T), torch.empty(B, nq, T)

    def rvq_fused(z, w_in_t, b_in, cb, cbn, c2, w_out, b_out, imp=None, level=1.0,
                  want_z_q_is=True, want_mask=True):
        B, D, T = z.shape
        nq = cb.shape[0]
        return (torch.zeros(B, nq, T, dtype=torch.long), torch.empty(B, nq * 8, T),
                torch.empty(B, nq, T), torch.empty(B, nq, D, T), torch.empty(B, D, T),
                torch.empty(B, nq, T))

    def rvq_encode(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, imp=None, level=1.0,
                   want_z_q_is=True, want_mask=True):
        B, D, T = z.shape
        nq = cb.shape[0]
        return (torch.zeros(B, nq, T, dtype=torch.long), torch.empty(B, nq * 8, T),
                torch.empty(B, nq, T), torch.empty(B, nq, D, T) if want_z_q_is else None,
                torch.empty(B, D, T), torch.empty(B, nq, T) if want_mask else None)

    def rvq_encode_part(part, T, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, imp=None, level=1.0,
                        want_z_q_is=True, want_mask=True):
        B = part.shape[1] // T
        nq, D = cb.shape[0], w_out.shape[1]
        return (torch.zeros(B, nq, T, dtype=torch.long), torch.empty(B, nq * 8, T),
                torch.empty(B, nq, T), torch.empty(B, nq, D, T) if want_z_q_is else None,
                torch.empty(B, D, T), torch.empty(B, nq, T) if want_mask else None)

    ops.rvq_encode = rvq_encode
    ops.rvq_encode_part = rvq_encode_part
    ops.conv1d_proj = conv1d_proj
    ops.rvq_pack_w_in = lambda w: w
    ops.rvq_frag = lambda cbn: cbn
    ops.rvq_codes = rvq_codes
    ops.rvq_expand = rvq_expand
    ops.rvq_fused = rvq_fused
    ops.rvq_cross_prep = lambda wi, wo, bo: (torch.zeros(wi.shape[0], wi.shape[0], 8, 8),
                                             torch.zeros(wi.shape[0], 8))
    ops.masked_loss = lambda l, m: torch.zeros(())
    ops.imp_mask = lambda *a, **k: None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--nq", type=int, default=8)
    args = ap.parse_args()
    _fake()
    import vrvq_amd
    m = vrvq_amd.DAC_VRVQ(n_codebooks=args.nq).eval()
    with torch.no_grad():
        m(torch.zeros(args.batch, 1, 44100), 44100, None, 1.0)
    rows = list(csv.DictReader(open(args.trace)))
    conv = []
    for r in rows:
        if "conv_splitk_epilogue_kernel" in r["Kernel_Name"] and conv:
            # a split-K layer (conv.hip launch_splitk): its K parts and their epilogue launch,
            # stream-ordered, timed as one layer from the first start to the epilogue's end
            conv[-1] = dict(conv[-1], End_Timestamp=r["End_Timestamp"])
        elif any(k in r["Kernel_Name"] for k in ("conv_mfma_kernel", "conv_small", "conv_cout1",
                                                   "conv_cin1", "ru_fused_kernel")):
            conv.append(r)
    step = conv[-len(CALLS):]
    tot_t = tot_f = 0.0
    # %pk against the ceiling of the path the kernel runs: the x3 split-bf16 MFMA (template
    # flag true: bf16 dense peak / 6 = 419.4 TF/s of fp32 work) or the fp32-input MFMA (157.3)
    print(f"{'layer':42s} {'kernel':34s} {'us':>9s} {'GFLOP':>8s} {'TF/s':>7s} {'%pk':>5s}")
    for c, r in zip(CALLS, step):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        kn = r["Kernel_Name"]
        i = kn.find("<")
        pre = ("mfma" if "mfma" in kn else "ru" if "ru_fused" in kn else
               "cout1" if "cout1" in kn else "cin1" if "cin1" in kn else "small")
        targs = [t.strip() for t in kn[i + 1:kn.find(">")].split(",")] if i >= 0 else []
        # conv_mfma_kernel<BM, BN, WM, NW, KS, X3[, PH]>, ru_fused_kernel<C, BN, WM, NW, X3>
        x3 = ((pre == "mfma" and len(targs) >= 6 and targs[5] == "true") or
              (pre == "ru" and len(targs) >= 5 and targs[4] == "true"))
        kn = pre + kn[i:kn.find(">") + 1] if i >= 0 else pre
        tf = c[8] / (us * 1e-6) / 1e12
        tot_t += us
        tot_f += c[8]
        desc = (f"RU {c[1]} k7+k1 d{c[5]} T{c[6]} (fused)" if c[0] == "RU" else
                f"{c[0]} {c[1]}->{c[2]} k{c[3]} s{c[4]} d{c[5]} T{c[6]}{' +res' if c[9] else ''}")
        pk = 419.4 if x3 else 157.3
        print(f"{desc:42s} {kn:34s} {us:9.1f} {c[8]/1e9:8.1f} {tf:7.1f} {tf/pk*100:5.1f}")
    print(f"total conv: {tot_t/1e3:.2f} ms, {tot_f/1e12:.3f} TFLOP, {tot_f/(tot_t*1e-6)/1e12:.1f} TF/s")


if __name__ == "__main__":
    main()
