"""Training step of the VRVQ generator on gfx950 kernels.

The reference trains with PyTorch autograd over its modules (scripts/train.py:262-330:
generator forward in train mode, losses, backward, grad-norm clip, AdamW). Here every
generator op of that graph is a torch.autograd.Function whose forward AND backward run in
libvrvq_hip.so (include/vrvq.h, "Training step"); PyTorch provides the tape, the caching
allocator and the optimizer:

  SnakeConv   Snake1d -> WNConv1d / WNConvTranspose1d (+ residual, + Tanh / Sigmoid)
              forward: weight-norm fold + the MFMA conv kernels of the inference path;
              backward: activation backward, bias sums, weight gradient (split-K MFMA GEMM,
              Snake applied while staging), weight-norm backward, input gradient through the
              adjoint conv on the same forward kernels (flipped weights / polyphase ConvT /
              strided conv) and Snake backward (dx, dalpha).
  MaskSte     the training-mode importance mask: random-level STE rows, quantizer-dropout rows,
              full-codebook rows (models/quantize.py:374-414, models/utils.py:11-61).
  RvqTrain    the residual quantizer over all stages with the straight-through estimator,
              commitment and codebook losses (models/quantize.py:42-79, 353-423); backward in
              the 8-dim latent space (csrc/rvq_train.hip).

Random draws (levels, dropout counts) come from torch's global CPU generator in the
reference's order, so a seeded step draws bit-identical values.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import ops

# Forward and adjoint convs of the training step on the bf16x3 split MFMA path (csrc/conv_x3.h:
# fp32-accurate; the weights change every step, so their split planes are packed per call).
# VRVQ_TRAIN_X3=0 keeps them on the fp32-input MFMA (A/B).
TRAIN_X3 = ops.X3 and os.environ.get("VRVQ_TRAIN_X3", "1") != "0"


def _x3(wp: torch.Tensor, k: int) -> Optional[torch.Tensor]:
    """Split planes of a packed weight for a stride-1 conv (k taps) or a polyphase ConvT (k=2)."""
    return ops.pack_x3_weight(wp, k) if TRAIN_X3 and k in ops.X3_TAPS else None


def _x3s(w: torch.Tensor, k: int, stride: int) -> Optional[torch.Tensor]:
    """Split planes of a strided conv's phase-split weight (k = 2s, s a power of two)."""
    ok = TRAIN_X3 and ops.X3_STRIDED and k == 2 * stride and stride & (stride - 1) == 0
    return ops.pack_x3_strided_weight(w, stride) if ok and w.shape[1] >= 8 else None


def _c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None else t.contiguous()


# ============================================================================ convolutions
class _SnakeConv(torch.autograd.Function):
    """y = epi(conv(snake(x); w = weight_norm(g, v)) + bias (+ residual))."""

    @staticmethod
    def forward(ctx, x, alpha, g, v, bias, residual, spec):
        kind, cout, k, stride, pad, dil, epi = spec
        x = x.contiguous()
        w = ops.weight_norm(g.detach().contiguous(), v.detach().contiguous())
        inv = ops.snake_inv_alpha(alpha.detach()) if alpha is not None else None
        a = alpha.detach() if alpha is not None else None
        b = bias.detach()
        if kind == "conv":
            wp, cp = ops.pack_conv1d_weight(w)
            y = ops.conv1d(x, wp, cout, cp, k, stride, pad, dil, bias=b, alpha=a, inv_alpha=inv,
                           residual=_c(residual.detach()) if residual is not None else None,
                           epilogue=epi, w_x3=_x3(wp, k) if stride == 1 else _x3s(w, k, stride))
        else:
            wp, cp = ops.pack_convt1d_weight(w, stride)
            y = ops.conv_transpose1d(x, wp, cout, cp, stride, bias=b, alpha=a, inv_alpha=inv,
                                     w_x3=_x3(wp, 2))
        ctx.spec = spec
        ctx.has_alpha = alpha is not None
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, a, inv, g.detach(), v.detach(), w, y if epi else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        kind, cout, k, stride, pad, dil, epi = ctx.spec
        x, a, inv, g, v, w, y = ctx.saved_tensors
        gy = gy.contiguous()
        if epi:
            gy = ops.act_backward(y, gy, epi)
        snake = (a, inv) if ctx.has_alpha else None
        need_x = ctx.needs_input_grad[0]
        need_a = ctx.has_alpha and ctx.needs_input_grad[1]
        db = ops.bias_grad(gy) if ctx.needs_input_grad[4] else None
        dg = dv = None
        if ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            if kind == "conv":
                dw = ops.conv1d_wgrad(gy, x, k, stride, pad, dil, snake_x=snake)
            else:  # y[co][t s - p + j] += W[ci][co][j] xs[ci][t]
                dw = ops.conv1d_wgrad(x, gy, k, stride, pad, 1, snake_a=snake)
            dg, dv = ops.weight_norm_backward(g.contiguous(), v.contiguous(), dw)
        dx = dalpha = None
        if need_x or need_a:
            cin = x.shape[1]
            if kind == "conv" and stride == 1:
                wf, cpf = ops.pack_conv1d_flip(w)
                dxs = ops.conv1d(gy, wf, cin, cpf, k, 1, dil * (k - 1) - pad, dil, w_x3=_x3(wf, k))
            elif kind == "conv":  # strided conv: adjoint is the polyphase ConvTranspose1d
                wt, cpt = ops.pack_convt1d_weight(w, stride)
                dxs = ops.conv_transpose1d(gy, wt, cin, cpt, stride, w_x3=_x3(wt, 2))
            else:  # ConvTranspose1d: adjoint is the strided conv with the same weight array
                wc, cpc = ops.pack_conv1d_weight(w)
                dxs = ops.conv1d(gy, wc, cin, cpc, k, stride, pad, 1, w_x3=_x3s(w, k, stride))
            if dxs.shape != x.shape:
                raise RuntimeError(f"adjoint conv shape {tuple(dxs.shape)} != {tuple(x.shape)}")
            if ctx.has_alpha:
                dx, dalpha = ops.snake_backward(x, a, inv, dxs, want_dx=need_x)
            else:
                dx = dxs
        dres = gy if ctx.has_res else None
        return dx, dalpha, dg, dv, db, dres, None


def conv(layer, x, snake=None, residual=None, epilogue: int = ops.EPI_NONE):
    """Differentiable Snake1d -> WNConv1d / WNConvTranspose1d (vrvq_amd.layers modules)."""
    from .layers import WNConvTranspose1d
    kind = "convt" if isinstance(layer, WNConvTranspose1d) else "conv"
    spec = (kind, layer.out_channels, layer.kernel_size[0], layer.stride[0], layer.padding[0],
            layer.dilation[0], int(epilogue))
    alpha = snake.alpha.reshape(-1) if snake is not None else None
    return _SnakeConv.apply(x, alpha, layer.weight_g.reshape(-1), layer.weight_v, layer.bias,
                            residual, spec)


def residual_unit(ru, x):
    """models/layers.py:52-68 (the residual add in the k=1 conv's epilogue)."""
    h = conv(ru.block[1], x, snake=ru.block[0])
    return conv(ru.block[3], h, snake=ru.block[2], residual=x)


def encoder_forward(enc, x):
    """models/dac_vrvq.py:19-48 -> (z, feat)."""
    blocks = enc.block
    n = len(blocks)
    x = conv(blocks[0], x)
    for i in range(1, n - 2):
        eb = blocks[i].block
        for j in range(3):
            x = residual_unit(eb[j], x)
        x = conv(eb[4], x, snake=eb[3])
    feat = x
    return conv(blocks[n - 1], x, snake=blocks[n - 2]), feat


def decoder_forward(dec, z):
    """models/dac_vrvq.py:51-80."""
    layers = dec.model
    n = len(layers)
    x = conv(layers[0], z)
    for i in range(1, n - 3):
        db = layers[i].block
        x = conv(db[1], x, snake=db[0])
        for j in range(2, 5):
            x = residual_unit(db[j], x)
    return conv(layers[n - 2], x, snake=layers[n - 3], epilogue=ops.EPI_TANH)


def imp_subnet_forward(net, feat):
    """models/importance_subnet.py:38-45 -> (B, 1, T) in (0, 1)."""
    x = feat.detach() if net.detach_input else feat
    x = conv(net.in_block[1], x, snake=net.in_block[0])
    last = len(net.blocks) - 1
    for i, blk in enumerate(net.blocks):
        x = conv(blk[1], x, snake=blk[0], epilogue=ops.EPI_SIGMOID if i == last else ops.EPI_NONE)
    return x


# ============================================================================ quantizer
class _MaskSte(torch.autograd.Function):
    """Training mask rows: [0, n_imps) STE of the scaled importance, then n_drop dropout rows,
    then full-codebook rows (gradient only through the first block)."""

    @staticmethod
    def forward(ctx, imp, levels, dropout, nq, alpha, n_imps, n_drop):
        # levels None: imp is already the scaled map x of generate_mask_ste(x, nq, alpha)
        B, T = imp.shape[0], imp.shape[-1]
        imp2 = imp.detach().reshape(B, T).contiguous()
        mask = ops.mask_ste(imp2, levels, dropout, nq, alpha, n_imps, n_drop)
        ctx.save_for_backward(imp2, levels)
        ctx.cfg = (alpha, n_imps, tuple(imp.shape))
        return mask

    @staticmethod
    def backward(ctx, dmask):
        imp2, levels = ctx.saved_tensors
        alpha, n_imps, shape = ctx.cfg
        dimp = ops.mask_ste_backward(imp2, levels, dmask.contiguous(), alpha, n_imps)
        return dimp.reshape(shape), None, None, None, None, None, None


class _RvqTrain(torch.autograd.Function):
    """All stages of the residual quantizer with the straight-through estimator:
    (z, mask, in_proj g/v/b, out_proj g/v/b, codebooks) -> (z_q, commitment_loss,
    codebook_loss, codes, latents). Losses are (loss * mask).sum(1).mean() over the per-frame
    per-stage MSE (models/quantize.py:70-71, 422-423)."""

    @staticmethod
    def forward(ctx, z, mask, g_in, v_in, b_in, g_out, v_out, b_out, cb):
        nq, _n, d = cb.shape
        D = z.shape[1]
        z = z.contiguous()
        mask = mask.detach().contiguous()
        # in_proj rows (nq*d, D), out_proj rows (nq*D, d): weight norm per conv output channel
        w_in = ops.weight_norm(g_in.detach().contiguous(), v_in.detach().contiguous())
        w_in_t = w_in.reshape(nq, d, D).transpose(1, 2).contiguous()
        w_out = ops.weight_norm(g_out.detach().contiguous(),
                                v_out.detach().contiguous()).reshape(nq, D, d)
        cbd = cb.detach().contiguous()
        cbn, c2 = ops.codebook_prep(cbd)
        cbf = ops.rvq_frag(cbn)
        b_in_d, b_out_d = b_in.detach().contiguous(), b_out.detach().contiguous()
        mcol, qb = ops.rvq_cross_prep(w_in_t, w_out, b_out_d)
        codes, lat, loss_pf, zst, z_q = ops.rvq_encode_train(z, w_in_t, b_in_d, cbd, cbf, c2,
                                                             w_out, b_out_d, mcol, qb, mask)
        commit = ops.masked_loss(loss_pf, mask)
        ctx.save_for_backward(z, zst, lat, codes, mask, w_in_t, w_out, b_out_d, mcol, cbd,
                              g_in.detach(), v_in.detach(), g_out.detach(), v_out.detach())
        ctx.mark_non_differentiable(codes, lat)
        return z_q, commit, commit.clone(), codes, lat

    @staticmethod
    def backward(ctx, dzq, gc, gcb, _codes, _lat):
        (z, zst, lat, codes, mask, w_in_t, w_out, b_out, mcol, cb, g_in, v_in, g_out,
         v_out) = ctx.saved_tensors
        nq, D, d = w_out.shape
        zero = None
        if dzq is None:
            dzq = torch.zeros_like(z)
        if gc is None or gcb is None:
            zero = torch.zeros((), device=z.device, dtype=torch.float32)
        gc = zero if gc is None else gc.contiguous()
        gcb = zero if gcb is None else gcb.contiguous()
        dz, dmask, dw_in, db_in, dw_out, db_out, dcb = ops.rvq_backward(
            dzq.contiguous(), gc, gcb, z, zst, lat, codes, mask, w_in_t, w_out, b_out, mcol, cb)
        dg_in, dv_in = ops.weight_norm_backward(g_in.contiguous(), v_in.contiguous(),
                                                dw_in.reshape(nq * d, D))
        dg_out, dv_out = ops.weight_norm_backward(g_out.contiguous(), v_out.contiguous(),
                                                  dw_out.reshape(nq * D, d))
        return dz, dmask, dg_in, dv_in, db_in, dg_out, dv_out, db_out, dcb


def _stage_params(quantizers):
    """Stacked (differentiable) per-stage parameters in the kernels' layouts: in_proj g
    (nq*d,), v (nq*d, D), b (nq, d); out_proj g (nq*D,), v (nq*D, d), b (nq, D); codebooks
    (nq, N, d). torch.stack / reshape route the gradients back to the per-stage Parameters."""
    g_in = torch.cat([q.in_proj.weight_g.reshape(-1) for q in quantizers])
    v_in = torch.cat([q.in_proj.weight_v.reshape(q.in_proj.out_channels, -1) for q in quantizers])
    b_in = torch.stack([q.in_proj.bias for q in quantizers])
    g_out = torch.cat([q.out_proj.weight_g.reshape(-1) for q in quantizers])
    v_out = torch.cat([q.out_proj.weight_v.reshape(q.out_proj.out_channels, -1)
                       for q in quantizers])
    b_out = torch.stack([q.out_proj.bias for q in quantizers])
    cb = torch.stack([q.codebook.weight for q in quantizers])
    return g_in, v_in, b_in, g_out, v_out, b_out, cb


def _rvq(quantizers, z, mask):
    return _RvqTrain.apply(z, mask, *_stage_params(quantizers))


def draw_levels(q, B: int) -> torch.Tensor:
    """random_levels of models/quantize.py:377-384 (torch CPU generator, (B, 1, 1))."""
    if q.level_dist == "uniform":
        return torch.rand((B, 1, 1)) * (q.level_max - q.level_min) + q.level_min
    if q.level_dist == "log_uniform":
        lv = torch.rand((B, 1, 1)) * (math.log(q.level_max) - math.log(q.level_min)) + \
            math.log(q.level_min)
        return torch.exp(lv)
    raise ValueError("Invalid level_dist")


def vbr_forward(q, z, feat):
    """VBRResidualVectorQuantize.forward in training mode (models/quantize.py:328-443)."""
    B, D, T = z.shape
    nq = q.n_codebooks
    if not q.level_min < q.level_max:
        raise AssertionError("level_min must be < level_max")
    imp_map = imp_subnet_forward(q.imp_subnet, feat)                      # (B, 1, T)
    levels = draw_levels(q, B)
    dropout = torch.randint(1, nq + 1, (B, 1, 1))
    n_full = int(B * q.full_codebook_rate)
    n_drop = int(B * q.quantizer_dropout)
    n_imps = int(B) - n_full - n_drop
    dev = z.device
    mask = _MaskSte.apply(imp_map, levels.reshape(B).to(dev).contiguous(),
                          dropout.reshape(B).to(dev).contiguous(), nq, float(q.imp2mask_alpha),
                          n_imps, n_drop)
    z_q, commit, cbl, codes, lat = _rvq(q.quantizers, z, mask)
    return {"z_q": z_q, "z_q_is": None, "codes": codes, "latents": lat,
            "commitment_loss": commit, "codebook_loss": cbl,
            "imp_map": imp_map[:n_imps], "mask_imp": mask,
            "random_levels": levels, "dropout": dropout}


def mask_ste(x: torch.Tensor, nq: int, alpha: float = 1.0) -> torch.Tensor:
    """generate_mask_ste(x, nq, alpha) of models/utils.py:45-53 with its backward: x (B, 1, T)
    the scaled importance map; forward the hard mask, backward d logcosh(alpha, x - n) / dx."""
    if x.dim() != 3 or x.shape[1] != 1:
        raise RuntimeError(f"generate_mask_ste: x must be (B, 1, T), got {tuple(x.shape)}")
    return _MaskSte.apply(x, None, None, int(nq), float(alpha), int(x.shape[0]), 0)


def vbr_cbr_forward(q, z, n_quantizers: int):
    """VBRResidualVectorQuantize.forward in training mode with n_quantizers given (CBR mode,
    models/quantize.py:346-414): every stage runs, the importance rows of the mask are ones
    (no level draw, no importance map), then the dropout and full-codebook rows. The only draw
    is the dropout randint (:406). n_quantizers < Nq raises here. In the reference 2 <= n < Nq
    is a shape mismatch at :421 and n = 0 fails at torch.stack, but n = 1 broadcasts the one
    stage against the (B, Nq, T) mask (z_q = sum of the mask rows * z_q_0): that value is a
    known difference."""
    B, D, T = z.shape
    nq = q.n_codebooks
    if int(n_quantizers) < nq:
        raise RuntimeError(
            f"VBRResidualVectorQuantize in CBR mode needs n_quantizers >= n_codebooks "
            f"({n_quantizers} < {nq}), as in the reference")
    dropout = torch.randint(1, nq + 1, (B, 1, 1))
    n_full = int(B * q.full_codebook_rate)
    n_drop = int(B * q.quantizer_dropout)
    n_imps = int(B) - n_full - n_drop
    dev = z.device
    # rows < n_imps: mask_imp = ones (:400) -- the STE of the constant map x = nq is 1 exactly
    ones = torch.full((B, T), float(nq), device=dev)
    mask = ops.mask_ste(ones, None, dropout.reshape(B).to(dev).contiguous(), nq, 1.0,
                        max(n_imps, 0), n_drop)
    z_q, commit, cbl, codes, lat = _rvq(q.quantizers, z, mask)
    return {"z_q": z_q, "z_q_is": None, "codes": codes, "latents": lat,
            "commitment_loss": commit, "codebook_loss": cbl, "imp_map": None,
            "mask_imp": mask, "dropout": dropout}


def cbr_forward(q, z):
    """ResidualVectorQuantize.forward in training mode (models/quantize.py:165-214): the first
    int(B * quantizer_dropout) rows use randint(1, nq + 1) stages, the others all stages."""
    B, D, T = z.shape
    nq = q.n_codebooks
    dropout = torch.randint(1, nq + 1, (B,))
    n_drop = int(B * q.quantizer_dropout)
    # row b keeps stages i < dropout[b]: the hard-mask rows of mask_ste with (dropout - 1)
    mask = ops.mask_ste(torch.zeros(B, T, device=z.device), torch.ones(B, device=z.device),
                        (dropout - 1).to(z.device).contiguous(), nq, 1.0, 0, n_drop)
    z_q, commit, cbl, codes, lat = _rvq(q.quantizers, z, mask)
    return {"z_q": z_q, "codes": codes, "latents": lat, "commitment_loss": commit,
            "codebook_loss": cbl, "dropout": dropout}
