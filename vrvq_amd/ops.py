"""Tensor-level wrappers over the C-ABI (include/vrvq.h).

PyTorch is used here only for device memory (the caching allocator) and the current HIP
stream; every value is computed by libvrvq_hip.so. Inputs must be contiguous fp32 tensors on
one GPU — anything else raises (there is no CPU or eager-PyTorch fallback).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import _lib

EPI_NONE, EPI_TANH, EPI_SIGMOID = 0, 1, 2


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _chk(t: Optional[torch.Tensor], name: str, dtype=torch.float32, device=None):
    if t is None:
        return
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: vrvq_amd kernels run on the GPU only (got device {t.device})")
    if t.dtype != dtype:
        raise RuntimeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise RuntimeError(f"{name}: tensor must be contiguous")
    if device is not None and t.device != device:
        raise RuntimeError(f"{name}: on {t.device}, expected {device}")


def round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


# ----------------------------------------------------------------------------- weights
def weight_norm(g: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """w = v * (g / ||v||) with the norm over all dims but 0 (torch weight_norm, dim=0)."""
    _chk(g, "g"); _chk(v, "v", device=g.device)
    rows = v.shape[0]
    cols = v.numel() // rows
    if g.numel() != rows:
        raise RuntimeError("weight_norm: g must have one entry per row of v")
    w = torch.empty_like(v)
    _lib.call("vrvq_weight_norm", _p(g), _p(v), rows, cols, _p(w), _stream(v))
    return w


def snake_inv_alpha(alpha: torch.Tensor) -> torch.Tensor:
    _chk(alpha, "alpha")
    inv = torch.empty_like(alpha)
    _lib.call("vrvq_snake_inv_alpha", _p(alpha), alpha.numel(), _p(inv), _stream(alpha))
    return inv


def codebook_prep(cb: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-normalised codebook and its squared row norms ([..., N, d] -> cbn, c2[..., N])."""
    _chk(cb, "codebook")
    dim = cb.shape[-1]
    rows = cb.numel() // dim
    cbn = torch.empty_like(cb)
    c2 = torch.empty(cb.shape[:-1], device=cb.device, dtype=torch.float32)
    _lib.call("vrvq_codebook_prep", _p(cb), rows, dim, _p(cbn), _p(c2), _stream(cb))
    return cbn, c2


def pack_conv1d_weight(w: torch.Tensor) -> Tuple[torch.Tensor, int]:
    _chk(w, "w")
    cout, cin, k = w.shape
    cout_pad = round_up(cout, 128)
    wp = torch.empty((cin, k, cout_pad), device=w.device, dtype=torch.float32)
    _lib.call("vrvq_pack_conv1d_weight", _p(w), cout, cin, k, cout_pad, _p(wp), _stream(w))
    return wp, cout_pad


def pack_convt1d_weight(w: torch.Tensor, stride: int) -> Tuple[torch.Tensor, int]:
    _chk(w, "w")
    cin, cout, k = w.shape
    if k != 2 * stride:
        raise RuntimeError("conv_transpose1d: kernel_size must be 2*stride (DecoderBlock)")
    cout_pad = round_up(cout * stride, 128)
    wp = torch.empty((cin, 2, cout_pad), device=w.device, dtype=torch.float32)
    _lib.call("vrvq_pack_convt1d_weight", _p(w), cin, cout, stride, cout_pad, _p(wp), _stream(w))
    return wp, cout_pad


# ----------------------------------------------------------------------------- convs
def conv1d(x: torch.Tensor, w_packed: torch.Tensor, cout: int, cout_pad: int, k: int,
           stride: int = 1, pad: int = 0, dil: int = 1, bias: Optional[torch.Tensor] = None,
           alpha: Optional[torch.Tensor] = None, inv_alpha: Optional[torch.Tensor] = None,
           residual: Optional[torch.Tensor] = None, epilogue: int = EPI_NONE,
           out_snake: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, want_raw: bool = True):
    """y = epi(residual + conv1d(snake(x)) + bias) on the MFMA implicit-GEMM kernel.

    out_snake = (alpha_next, inv_alpha_next) also produces snake_next(y) from the epilogue
    (the next layer's Snake). Returns y, or (y | None, snake_next(y)) when out_snake is given
    (y is None when want_raw is False)."""
    _chk(x, "x"); dev = x.device
    for t, n in ((w_packed, "w_packed"), (bias, "bias"), (alpha, "alpha"),
                 (inv_alpha, "inv_alpha"), (residual, "residual")):
        _chk(t, n, device=dev)
    if x.dim() != 3:
        raise RuntimeError("conv1d: x must be (B, C, T)")
    B, cin, tin = x.shape
    tout = (tin + 2 * pad - dil * (k - 1) - 1) // stride + 1
    if tout <= 0:
        raise RuntimeError("conv1d: input too short")
    if residual is not None and tuple(residual.shape) != (B, cout, tout):
        raise RuntimeError("conv1d: residual shape must equal the output shape")
    if alpha is not None and inv_alpha is None:
        raise RuntimeError("conv1d: snake needs inv_alpha")
    ao, io, ys = _out_snake(out_snake, (B, cout, tout), dev)
    y = torch.empty((B, cout, tout), device=dev, dtype=torch.float32) \
        if (want_raw or out_snake is None) else None
    _lib.call("vrvq_conv1d", _p(x), B, cin, tin, _p(alpha), _p(inv_alpha), _p(w_packed), cout,
              cout_pad, k, stride, pad, dil, _p(bias), _p(residual), int(epilogue), _p(y), tout,
              _p(ao), _p(io), _p(ys), _stream(x))
    return y if out_snake is None else (y, ys)


def _out_snake(out_snake, shape, dev):
    if out_snake is None:
        return None, None, None
    ao, io = out_snake
    _chk(ao, "alpha_out", device=dev); _chk(io, "inv_alpha_out", device=dev)
    if ao.numel() != shape[1] or io.numel() != shape[1]:
        raise RuntimeError("out_snake: one alpha per output channel")
    return ao, io, torch.empty(shape, device=dev, dtype=torch.float32)


def conv_transpose1d(x: torch.Tensor, w_packed: torch.Tensor, cout: int, cout_pad: int,
                     stride: int, bias: Optional[torch.Tensor] = None,
                     alpha: Optional[torch.Tensor] = None,
                     inv_alpha: Optional[torch.Tensor] = None,
                     out_snake: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                     want_raw: bool = True):
    """Polyphase ConvTranspose1d (k = 2*stride); out_snake / want_raw as in conv1d."""
    _chk(x, "x"); dev = x.device
    for t, n in ((w_packed, "w_packed"), (bias, "bias"), (alpha, "alpha"), (inv_alpha, "inv_alpha")):
        _chk(t, n, device=dev)
    B, cin, tin = x.shape
    p = (stride + 1) // 2
    tout = (tin - 1) * stride - 2 * p + 2 * stride
    ao, io, ys = _out_snake(out_snake, (B, cout, tout), dev)
    y = torch.empty((B, cout, tout), device=dev, dtype=torch.float32) \
        if (want_raw or out_snake is None) else None
    _lib.call("vrvq_conv_transpose1d", _p(x), B, cin, tin, _p(alpha), _p(inv_alpha),
              _p(w_packed), cout, cout_pad, stride, _p(bias), _p(y), _p(ao), _p(io), _p(ys),
              _stream(x))
    return y if out_snake is None else (y, ys)


RU_FUSED_CHANNELS = (64, 96, 128, 192, 256)


def residual_unit(x, x_snk, dil: int, w7, b7, alpha2, inv_alpha2, w1, b1, cout_pad: int,
                  out_snake: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                  want_raw: bool = True):
    """Fused ResidualUnit: x + conv1(snake2(conv7_dil(x_snk))) in one launch (include/vrvq.h,
    vrvq_residual_unit). Returns y, or (y | None, snake_next(y)) when out_snake is given."""
    _chk(x, "x"); dev = x.device
    for t, n in ((x_snk, "x_snk"), (w7, "w7"), (b7, "b7"), (alpha2, "alpha2"),
                 (inv_alpha2, "inv_alpha2"), (w1, "w1"), (b1, "b1")):
        _chk(t, n, device=dev)
    B, C, T = x.shape
    if tuple(x_snk.shape) != (B, C, T):
        raise RuntimeError("residual_unit: x_snk must have the shape of x")
    ao, io, ys = _out_snake(out_snake, (B, C, T), dev)
    y = torch.empty((B, C, T), device=dev, dtype=torch.float32) \
        if (want_raw or out_snake is None) else None
    _lib.call("vrvq_residual_unit", _p(x), _p(x_snk), B, C, T, int(dil), _p(w7), _p(b7),
              _p(alpha2), _p(inv_alpha2), _p(w1), _p(b1), int(cout_pad), _p(y), _p(ao), _p(io),
              _p(ys), _stream(x))
    return y if out_snake is None else (y, ys)


# ----------------------------------------------------------------------------- RVQ
def rvq_codes(z, w_in_t, b_in, cb, cbn, c2, w_out, b_out):
    """Sequential residual chain over nq = w_in_t.shape[0] stages.

    Returns codes int64 [B,nq,T], latents [B,nq*d,T], loss_pf [B,nq,T], zst [B,nq,T,d].
    """
    _chk(z, "z"); dev = z.device
    for t, n in ((w_in_t, "w_in_t"), (b_in, "b_in"), (cb, "cb"), (cbn, "cbn"), (c2, "c2"),
                 (w_out, "w_out"), (b_out, "b_out")):
        _chk(t, n, device=dev)
    B, D, T = z.shape
    nq, N, d = cb.shape
    codes = torch.empty((B, nq, T), device=dev, dtype=torch.int64)
    latents = torch.empty((B, nq * d, T), device=dev, dtype=torch.float32)
    loss_pf = torch.empty((B, nq, T), device=dev, dtype=torch.float32)
    zst = torch.empty((B, nq, T, d), device=dev, dtype=torch.float32)
    _lib.call("vrvq_rvq_codes", _p(z), B, D, T, nq, N, d, _p(w_in_t), _p(b_in), _p(cb), _p(cbn),
              _p(c2), _p(w_out), _p(b_out), _p(codes), _p(latents), _p(loss_pf), _p(zst),
              _stream(z))
    return codes, latents, loss_pf, zst


def rvq_expand(zst, w_out, b_out, imp=None, level: float = 1.0, want_z_q_is: bool = True,
               want_mask: bool = True):
    """z_q_is / masked z_q / mask from the straight-through vectors (HBM-streaming kernel)."""
    _chk(zst, "zst"); dev = zst.device
    _chk(w_out, "w_out", device=dev); _chk(b_out, "b_out", device=dev); _chk(imp, "imp", device=dev)
    B, nq, T, d = zst.shape
    D = w_out.shape[1]
    z_q_is = torch.empty((B, nq, D, T), device=dev, dtype=torch.float32) if want_z_q_is else None
    z_q = torch.empty((B, D, T), device=dev, dtype=torch.float32)
    mask = torch.empty((B, nq, T), device=dev, dtype=torch.float32) if want_mask else None
    _lib.call("vrvq_rvq_expand", _p(zst), B, D, T, nq, d, _p(w_out), _p(b_out), _p(imp),
              float(level), _p(z_q_is), _p(z_q), _p(mask), _stream(zst))
    return z_q_is, z_q, mask


def rvq_gather(codes: torch.Tensor, cb: torch.Tensor, want_zst: bool = True,
               want_z_p: bool = True):
    """decode_code of every stage (models/quantize.py:81-85): raw codebook rows for int64 codes
    [B,nq,T] over the stacked codebooks cb [nq',N,d] (nq <= nq'). Returns (zst [B,nq,T,d],
    z_p [B,nq*d,T]); an out-of-range code raises IndexError, as F.embedding does."""
    _chk(codes, "codes", dtype=torch.int64); dev = codes.device
    _chk(cb, "cb", device=dev)
    if codes.dim() != 3:
        raise RuntimeError("rvq_gather: codes must be (B, n_codebooks, T)")
    B, nq, T = codes.shape
    if nq > cb.shape[0]:
        raise RuntimeError(f"rvq_gather: {nq} codebooks requested, {cb.shape[0]} available")
    _, N, d = cb.shape
    zst = torch.empty((B, nq, T, d), device=dev, dtype=torch.float32) if want_zst else None
    z_p = torch.empty((B, nq * d, T), device=dev, dtype=torch.float32) if want_z_p else None
    err = torch.zeros(1, device=dev, dtype=torch.int32)
    _lib.call("vrvq_rvq_gather", _p(codes), B, nq, T, _p(cb), N, d, _p(zst), _p(z_p), _p(err),
              _stream(codes))
    if int(err.item()) != 0:
        raise IndexError(f"code out of range for codebook size {N}")
    return zst, z_p


def rvq_cross_prep(w_in_t, w_out, b_out):
    """M_ij = W_in[i] W_out[j] blocks (mcol [nq][nq][8][8]) and Qb [nq][8] of the projected
    chain (once per weight version)."""
    _chk(w_in_t, "w_in_t"); dev = w_in_t.device
    _chk(w_out, "w_out", device=dev); _chk(b_out, "b_out", device=dev)
    nq, D, d = w_in_t.shape
    mcol = torch.empty((nq, nq, d, d), device=dev, dtype=torch.float32)
    qb = torch.empty((nq, d), device=dev, dtype=torch.float32)
    _lib.call("vrvq_rvq_cross_prep", _p(w_in_t), _p(w_out), _p(b_out), nq, D, d, _p(mcol),
              _p(qb), _stream(w_in_t))
    return mcol, qb


def rvq_project(z, w_in_t):
    """in_proj of every stage over z, as 8 channel-split partials [8, B*T, nq*8]."""
    _chk(z, "z"); dev = z.device
    _chk(w_in_t, "w_in_t", device=dev)
    B, D, T = z.shape
    nq, _, d = w_in_t.shape
    part = torch.empty((8, B * T, nq * d), device=dev, dtype=torch.float32)
    _lib.call("vrvq_rvq_project", _p(z), B, D, T, nq, d, _p(w_in_t), _p(part), _stream(z))
    return part


def rvq_chain(part, B, T, b_in, qb, mcol, cb, cbn, c2, imp=None, level: float = 1.0,
              want_mask: bool = True):
    """8-dim residual chain: codes, latents, loss_pf, zst, mask (see include/vrvq.h)."""
    _chk(part, "part"); dev = part.device
    for t_, n_ in ((b_in, "b_in"), (qb, "qb"), (mcol, "mcol"), (cb, "cb"), (cbn, "cbn"),
                   (c2, "c2")):
        _chk(t_, n_, device=dev)
    _chk(imp, "imp", device=dev)
    nq, N, d = cb.shape
    codes = torch.empty((B, nq, T), device=dev, dtype=torch.int64)
    latents = torch.empty((B, nq * d, T), device=dev, dtype=torch.float32)
    loss_pf = torch.empty((B, nq, T), device=dev, dtype=torch.float32)
    zst = torch.empty((B, nq, T, d), device=dev, dtype=torch.float32)
    mask = torch.empty((B, nq, T), device=dev, dtype=torch.float32) if want_mask else None
    _lib.call("vrvq_rvq_chain", _p(part), B, T, nq, N, d, _p(b_in), _p(qb), _p(mcol), _p(cb),
              _p(cbn), _p(c2), _p(imp), float(level), _p(codes), _p(latents), _p(loss_pf),
              _p(zst), _p(mask), _stream(part))
    return codes, latents, loss_pf, zst, mask


def rvq_encode(z, st, imp=None, level: float = 1.0, want_z_q_is: bool = True,
               want_mask: bool = True):
    """The production RVQ path: projection GEMM -> 8-dim chain -> HBM expansion (three
    launches). `st` is a model._Stacked (folded, stacked stage weights + cross terms).
    Returns codes, latents, loss_pf, z_q_is (or None), z_q, mask (or None)."""
    B, D, T = z.shape
    part = rvq_project(z, st.w_in_t)
    codes, latents, loss_pf, zst, mask = rvq_chain(part, B, T, st.b_in, st.qb, st.mcol, st.cb,
                                                   st.cbn, st.c2, imp, level, want_mask)
    z_q_is, z_q, _ = rvq_expand(zst, st.w_out, st.b_out, imp, level, want_z_q_is=want_z_q_is,
                                want_mask=False)
    return codes, latents, loss_pf, z_q_is, z_q, mask


def rvq_fused(z, w_in_t, b_in, cb, cbn, c2, w_out, b_out, imp=None, level: float = 1.0,
              want_z_q_is: bool = True, want_mask: bool = True):
    """Residual chain + z_q_is stream + importance gating in one launch (vrvq_rvq_fused).

    Returns codes int64 [B,nq,T], latents [B,nq*d,T], loss_pf [B,nq,T], z_q_is [B,nq,D,T] (or
    None), z_q [B,D,T], mask [B,nq,T] (or None).
    """
    _chk(z, "z"); dev = z.device
    for t, n in ((w_in_t, "w_in_t"), (b_in, "b_in"), (cb, "cb"), (cbn, "cbn"), (c2, "c2"),
                 (w_out, "w_out"), (b_out, "b_out")):
        _chk(t, n, device=dev)
    _chk(imp, "imp", device=dev)
    B, D, T = z.shape
    nq, N, d = cb.shape
    codes = torch.empty((B, nq, T), device=dev, dtype=torch.int64)
    latents = torch.empty((B, nq * d, T), device=dev, dtype=torch.float32)
    loss_pf = torch.empty((B, nq, T), device=dev, dtype=torch.float32)
    z_q_is = torch.empty((B, nq, D, T), device=dev, dtype=torch.float32) if want_z_q_is else None
    z_q = torch.empty((B, D, T), device=dev, dtype=torch.float32)
    mask = torch.empty((B, nq, T), device=dev, dtype=torch.float32) if want_mask else None
    _lib.call("vrvq_rvq_fused", _p(z), B, D, T, nq, N, d, _p(w_in_t), _p(b_in), _p(cb), _p(cbn),
              _p(c2), _p(w_out), _p(b_out), _p(imp), float(level), _p(codes), _p(latents),
              _p(loss_pf), _p(z_q_is), _p(z_q), _p(mask), _stream(z))
    return codes, latents, loss_pf, z_q_is, z_q, mask


_split_ws = {}  # device index -> zero-filled workspace of vrvq_rvq_split (left zero by every launch)


def _split_workspace(dev: torch.device, B: int, T: int) -> torch.Tensor:
    n = ctypes.c_longlong(0)
    _lib.call("vrvq_rvq_split_workspace", B, T, ctypes.byref(n))
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ws = _split_ws.get(key)
    if ws is None or ws.numel() < n.value:
        ws = torch.zeros(max(n.value, 1 << 20), device=dev, dtype=torch.uint8)
        _split_ws[key] = ws
    return ws


def rvq_split_error(dev: torch.device) -> bool:
    """True if a vrvq_rvq_split launch on `dev` timed out in a group exchange (its outputs are
    invalid); re-zeroes the workspace. Synchronises the device."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ws = _split_ws.get(key)
    if ws is None:
        return False
    bad = bool(ws[:4].any().item())
    if bad:
        ws.zero_()
    return bad


def rvq_split(z, w_in_t, b_in, cb, cbn, c2, w_out, b_out, imp=None, level: float = 1.0,
              want_z_q_is: bool = True, want_mask: bool = True):
    """Channel-split single launch (vrvq_rvq_split): the outputs of rvq_fused, computed by
    groups of 8 workgroups exchanging 8-dim partials / argmin candidates through L2."""
    _chk(z, "z"); dev = z.device
    for t, n in ((w_in_t, "w_in_t"), (b_in, "b_in"), (cb, "cb"), (cbn, "cbn"), (c2, "c2"),
                 (w_out, "w_out"), (b_out, "b_out")):
        _chk(t, n, device=dev)
    _chk(imp, "imp", device=dev)
    B, D, T = z.shape
    nq, N, d = cb.shape
    codes = torch.empty((B, nq, T), device=dev, dtype=torch.int64)
    latents = torch.empty((B, nq * d, T), device=dev, dtype=torch.float32)
    loss_pf = torch.empty((B, nq, T), device=dev, dtype=torch.float32)
    z_q_is = torch.empty((B, nq, D, T), device=dev, dtype=torch.float32) if want_z_q_is else None
    z_q = torch.empty((B, D, T), device=dev, dtype=torch.float32)
    mask = torch.empty((B, nq, T), device=dev, dtype=torch.float32) if want_mask else None
    ws = _split_workspace(dev, B, T)
    _lib.call("vrvq_rvq_split", _p(z), B, D, T, nq, N, d, _p(w_in_t), _p(b_in), _p(cb), _p(cbn),
              _p(c2), _p(w_out), _p(b_out), _p(imp), float(level), _p(codes), _p(latents),
              _p(loss_pf), _p(z_q_is), _p(z_q), _p(mask), _p(ws), ws.numel(), _stream(z))
    return codes, latents, loss_pf, z_q_is, z_q, mask


def masked_loss(loss_pf: torch.Tensor, mask: Optional[torch.Tensor]) -> torch.Tensor:
    _chk(loss_pf, "loss_pf"); _chk(mask, "mask", device=loss_pf.device)
    B, nq, T = loss_pf.shape
    out = torch.empty((), device=loss_pf.device, dtype=torch.float32)
    _lib.call("vrvq_masked_loss", _p(loss_pf), _p(mask), B, nq, T, _p(out), _stream(loss_pf))
    return out


def scale_imp(imp: torch.Tensor, a: float, c: float) -> torch.Tensor:
    _chk(imp, "imp")
    s = torch.empty_like(imp)
    _lib.call("vrvq_scale_imp", _p(imp), imp.numel(), float(a), float(c), _p(s), _stream(imp))
    return s


def mask_hard(s: torch.Tensor, nq: int) -> torch.Tensor:
    """s: (B, 1, T) scaled importance -> (B, nq, T) {0,1} mask."""
    _chk(s, "x")
    B, T = s.shape[0], s.shape[-1]
    if s.numel() != B * T:
        raise RuntimeError("generate_mask_hard: x must be (B, 1, T)")
    mask = torch.empty((B, nq, T), device=s.device, dtype=torch.float32)
    _lib.call("vrvq_mask_hard", _p(s), B, T, int(nq), _p(mask), _stream(s))
    return mask


def masked_sum(z_q_is: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    _chk(z_q_is, "z_q_is"); _chk(mask, "mask", device=z_q_is.device)
    B, nq, D, T = z_q_is.shape
    if tuple(mask.shape) != (B, nq, T):
        raise RuntimeError("masked_sum: mask must be (B, nq, T)")
    z_q = torch.empty((B, D, T), device=z_q_is.device, dtype=torch.float32)
    _lib.call("vrvq_masked_sum", _p(z_q_is), _p(mask), B, nq, D, T, _p(z_q), _stream(z_q_is))
    return z_q


def bpf(mask: torch.Tensor, bits: torch.Tensor) -> torch.Tensor:
    _chk(mask, "mask"); _chk(bits, "bits", device=mask.device)
    B, nq, T = mask.shape
    if bits.numel() != nq:
        raise RuntimeError("cal_bpf_from_mask: one bit count per codebook")
    out = torch.empty((), device=mask.device, dtype=torch.float32)
    _lib.call("vrvq_bpf", _p(mask), _p(bits), B, nq, T, _p(out), _stream(mask))
    return out
