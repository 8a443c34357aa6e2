"""Tensor-level API of the hot path: thin wrappers over the PyTorch-ROCm custom operators
`torch.ops.vrvq.*` (TORCH_LIBRARY(vrvq) in csrc/torch_ops.cpp, over the C-ABI of
include/vrvq.h).

PyTorch supplies device memory (the caching allocator) and the current HIP stream only; every
value is computed by libvrvq_hip.so. The ops check their inputs (contiguous, fp32 / int64, one
GPU) and raise RuntimeError otherwise — there is no CPU or eager-PyTorch fallback: a missing
library raises at import of this module's first op. Each op has a fake (meta) kernel below, so
shapes propagate under FakeTensorMode / torch.compile, and none synchronises the host, so a
sequence of them can be captured in a torch.cuda.CUDAGraph.
"""
from __future__ import annotations

import os
import threading
from typing import Optional, Tuple

import torch

EPI_NONE, EPI_TANH, EPI_SIGMOID = 0, 1, 2

_HERE = os.path.dirname(os.path.abspath(__file__))
TORCH_LIB_PATH = os.environ.get("VRVQ_TORCH_LIB") or os.path.join(_HERE, "libvrvq_torch.so")
_lock = threading.Lock()
_loaded = False


def load_ops():
    """Load libvrvq_torch.so (once): registers torch.ops.vrvq.* and their fake kernels."""
    global _loaded
    if _loaded:
        return torch.ops.vrvq
    with _lock:
        if not _loaded:
            if not os.path.exists(TORCH_LIB_PATH):
                raise RuntimeError(
                    f"vrvq_amd: operator library {TORCH_LIB_PATH} is missing; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
            torch.ops.load_library(TORCH_LIB_PATH)
            _register_fakes()
            _loaded = True
    return torch.ops.vrvq


def _ops():
    return torch.ops.vrvq if _loaded else load_ops()


def _none(t: torch.Tensor) -> Optional[torch.Tensor]:
    """Ops return a 0-element tensor for an output that was not requested."""
    return None if t.numel() == 0 and t.dim() == 1 else t


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def conv_out_len(tin: int, k: int, stride: int, pad: int, dil: int) -> int:
    return (tin + 2 * pad - dil * (k - 1) - 1) // stride + 1


def convt_out_len(tin: int, stride: int, pad: int = -1) -> int:
    p = (stride + 1) // 2 if pad < 0 else pad
    return (tin - 1) * stride - 2 * p + 2 * stride


# ----------------------------------------------------------------------------- weights
def weight_norm(g: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """w = v * (g / ||v||) with the norm over all dims but 0 (torch weight_norm, dim=0)."""
    return _ops().weight_norm(g, v)


def snake_inv_alpha(alpha: torch.Tensor) -> torch.Tensor:
    return _ops().snake_inv_alpha(alpha)


def codebook_prep(cb: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-normalised codebook and its squared row norms ([..., N, d] -> cbn, c2[..., N])."""
    return _ops().codebook_prep(cb)


def pack_conv1d_weight(w: torch.Tensor) -> Tuple[torch.Tensor, int]:
    wp = _ops().pack_conv1d_weight(w)
    return wp, wp.shape[2]


def pack_convt1d_weight(w: torch.Tensor, stride: int) -> Tuple[torch.Tensor, int]:
    wp = _ops().pack_convt1d_weight(w, int(stride))
    return wp, wp.shape[2]


# ----------------------------------------------------------------------------- convs
def conv1d(x: torch.Tensor, w_packed: torch.Tensor, cout: int, cout_pad: int, k: int,
           stride: int = 1, pad: int = 0, dil: int = 1, bias: Optional[torch.Tensor] = None,
           alpha: Optional[torch.Tensor] = None, inv_alpha: Optional[torch.Tensor] = None,
           residual: Optional[torch.Tensor] = None, epilogue: int = EPI_NONE,
           out_snake: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, want_raw: bool = True,
           w_x3: Optional[torch.Tensor] = None):
    """y = epi(residual + conv1d(snake(x)) + bias) on the MFMA implicit-GEMM kernel.

    out_snake = (alpha_next, inv_alpha_next) also produces snake_next(y) from the epilogue
    (the next layer's Snake). Returns y, or (y | None, snake_next(y)) when out_snake is given
    (y is None when want_raw is False). w_x3 = pack_x3_weight(w_packed, k) selects the bf16x3
    split MFMA path for stride-1 convs (include/vrvq.h)."""
    if w_packed.dim() != 3 or w_packed.shape[1] != k or w_packed.shape[2] != cout_pad:
        raise RuntimeError("conv1d: w_packed must be (Cin, k, cout_pad)")
    ao, io = out_snake if out_snake is not None else (None, None)
    y, ys = _ops().snake_conv1d(x, w_packed, int(cout), int(stride), int(pad), int(dil), bias,
                                alpha, inv_alpha, residual, int(epilogue), ao, io, bool(want_raw),
                                w_x3)
    return _none(y) if out_snake is None else (_none(y), ys)


def conv1d_proj(x: torch.Tensor, w_packed: torch.Tensor, cout: int, k: int, w3in: torch.Tensor,
                nq: int, pad: int = 0, dil: int = 1, bias: Optional[torch.Tensor] = None,
                alpha: Optional[torch.Tensor] = None, inv_alpha: Optional[torch.Tensor] = None,
                w_x3: Optional[torch.Tensor] = None, want_z: bool = False):
    """conv1d(snake(x)) + bias (stride 1, cout 1024: the encoder's last conv) with the in_proj of
    all nq RVQ stages in its epilogue (include/vrvq.h vrvq_conv1d_proj). Returns (part, z):
    part (8, B*T, 8 nq) = rvq_project's channel-split partials, bit for bit, and z (B, 1024, T)
    when want_z (else None). w3in = rvq_pack_w_in(w_in_t)."""
    if w_packed.dim() != 3 or w_packed.shape[1] != k:
        raise RuntimeError("conv1d_proj: w_packed must be (Cin, k, cout_pad)")
    part, z = _ops().snake_conv1d_proj(x, w_packed, int(cout), int(pad), int(dil), bias, alpha,
                                       inv_alpha, w_x3, w3in, int(nq), bool(want_z))
    return part, _none(z)


def conv_transpose1d(x: torch.Tensor, w_packed: torch.Tensor, cout: int, cout_pad: int,
                     stride: int, bias: Optional[torch.Tensor] = None,
                     alpha: Optional[torch.Tensor] = None,
                     inv_alpha: Optional[torch.Tensor] = None,
                     out_snake: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                     want_raw: bool = True, pad: int = -1,
                     w_x3: Optional[torch.Tensor] = None):
    """Polyphase ConvTranspose1d (k = 2*stride); out_snake / want_raw as in conv1d. pad -1 is
    the DecoderBlock's ceil(stride / 2), 0 the padding=False window of the chunked codec."""
    ao, io = out_snake if out_snake is not None else (None, None)
    y, ys = _ops().snake_conv_transpose1d(x, w_packed, int(cout), int(stride), bias, alpha,
                                          inv_alpha, ao, io, bool(want_raw), int(pad), w_x3)
    return _none(y) if out_snake is None else (_none(y), ys)


RU_FUSED_CHANNELS = tuple(int(c) for c in os.environ.get("VRVQ_RU_FUSED", "64,96,128,256").split(",") if c)

# The bf16x3 split MFMA path (include/vrvq.h, csrc/conv_x3.h) for the stride-1 convs of the
# inference path; VRVQ_CONV_X3=0 keeps every conv on the fp32-input MFMA (A/B and tests).
X3 = os.environ.get("VRVQ_CONV_X3", "1") != "0"
X3_TAPS = (1, 2, 3, 7)
RU256_SPLIT = os.environ.get("VRVQ_RU256_SPLIT", "1") != "0"
# The strided encoder convs (k = 2s) on the x3 path through the phase-split view (vrvq_conv1d);
# VRVQ_CONV_X3_STRIDED=0 keeps them on the fp32-input MFMA's strided window (A/B).
X3_STRIDED = os.environ.get("VRVQ_CONV_X3_STRIDED", "1") != "0"


def x3_size(cin: int, k: int, cout_pad: int) -> int:
    ck = 32 if k == 1 else 16 if k <= 3 else 8
    no = k * ck // 8
    return -(-cin // ck) * 3 * (no + (no & 1)) * cout_pad * 8


def pack_x3_weight(w_packed: torch.Tensor, k: int) -> torch.Tensor:
    """bf16 planes of a packed conv weight ([Cin][k][cout_pad]; k = 2 for the polyphase
    ConvTranspose1d) for the x3 path: int16 storage, x3_size(...) elements."""
    return _ops().pack_x3_weight(w_packed, int(k))


def pack_x3_strided_weight(w: torch.Tensor, stride: int) -> torch.Tensor:
    """x3 planes for a strided conv (w: (Cout, Cin, 2*stride), stride a power of two): the
    planes of W'[co][c*s + r][j] = W[co][c][j*s + r], the 2-tap weight of the stride-1 conv over
    the phase-split view of x that vrvq_conv1d runs when given w_x3 for stride > 1."""
    co, ci, k = w.shape
    s = int(stride)
    if k != 2 * s or s < 2 or s & (s - 1):
        raise RuntimeError("pack_x3_strided_weight: kernel must be 2*stride, stride a power of 2")
    wv = w.reshape(co, ci, 2, s).permute(0, 1, 3, 2).reshape(co, ci * s, 2).contiguous()
    wp, _ = pack_conv1d_weight(wv)
    return pack_x3_weight(wp, 2)


def residual_unit(x, x_snk, dil: int, w7, b7, alpha2, inv_alpha2, w1, b1, cout_pad: int,
                  out_snake: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                  want_raw: bool = True, w7_x3: Optional[torch.Tensor] = None,
                  w1_x3: Optional[torch.Tensor] = None):
    """Fused ResidualUnit: x + conv1(snake2(conv7_dil(x_snk))) in one launch (include/vrvq.h,
    vrvq_residual_unit). Returns y, or (y | None, snake_next(y)) when out_snake is given."""
    ao, io = out_snake if out_snake is not None else (None, None)
    y, ys = _ops().residual_unit(x, x_snk, int(dil), w7, b7, alpha2, inv_alpha2, w1, b1, ao, io,
                                 bool(want_raw), w7_x3, w1_x3)
    return _none(y) if out_snake is None else (_none(y), ys)


# ----------------------------------------------------------------------------- RVQ
def rvq_cross_prep(w_in_t, w_out, b_out):
    """M_ij = W_in[i] W_out[j] blocks (mcol [nq][nq][8][8]) and Qb [nq][8] of the projected
    chain (once per weight version)."""
    return _ops().rvq_cross_prep(w_in_t, w_out, b_out)


def rvq_frag(cbn):
    """The normalised codebooks in the chain's MFMA fragment order (once per weight version)."""
    return _ops().rvq_frag(cbn)


def rvq_encode(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, imp=None,
               level: float = 1.0, want_z_q_is: bool = True, want_mask: bool = True):
    """The residual quantizer over all nq = cb.shape[0] stages + importance gating
    (VBRResidualVectorQuantize.forward, models/quantize.py:328-443): projection, 8-dim chain
    and expansion (include/vrvq.h, vrvq_rvq_encode).

    Returns codes int64 [B,nq,T], latents [B,nq*d,T], loss_pf [B,nq,T], z_q_is [B,nq,D,T] (or
    None), z_q [B,D,T], mask [B,nq,T] (or None)."""
    codes, lat, loss, zqis, zq, mask = _ops().rvq_encode(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out,
                                                       mcol, qb, imp, float(level),
                                                       bool(want_z_q_is), bool(want_mask))
    return codes, lat, loss, _none(zqis), zq, _none(mask)


def rvq_pack_w_in(w_in_t: torch.Tensor) -> torch.Tensor:
    """W_in planes (bf16 x3 split, MFMA fragment order) for conv1d_proj, once per weight
    version (include/vrvq.h vrvq_rvq_pack_w_in)."""
    return _ops().rvq_pack_w_in(w_in_t)


def rvq_encode_part(part, frames, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, imp=None,
                    level: float = 1.0, want_z_q_is: bool = True, want_mask: bool = True):
    """rvq_encode from conv1d_proj's partials (8, B*T, 8 nq): one launch per group of resident
    clips (include/vrvq.h vrvq_rvq_encode_part), or the chain + expansion launches where a clip
    does not fit it. Same outputs as rvq_encode's three launches, bit for bit."""
    codes, lat, loss, zqis, zq, mask = _ops().rvq_encode_part(part, int(frames), b_in, cb, cbf,
                                                            c2, w_out, b_out, mcol, qb, imp,
                                                            float(level), bool(want_z_q_is),
                                                            bool(want_mask))
    return codes, lat, loss, _none(zqis), zq, _none(mask)


def rvq_check_error(like: torch.Tensor, sync: bool = True) -> int:
    """Timeout code of an earlier fused RVQ launch (0: none), cleared once read; sync waits for
    the current stream first (the RVQ ops also raise on a pending code at their next call)."""
    return int(_ops().rvq_check_error(like, bool(sync)))


def rvq_gather(codes: torch.Tensor, cb: torch.Tensor, check: bool = True):
    """decode_code of every stage (models/quantize.py:81-85): raw codebook rows for int64 codes
    [B,nq,T] over the stacked codebooks cb [nq',N,d] (nq <= nq'). Returns (zst [B,nq,T,d],
    z_p [B,nq*d,T]). An out-of-range code raises IndexError, as F.embedding does — that check
    reads a device flag (one host sync); it is skipped inside CUDA-graph capture and when
    check=False."""
    zst, z_p, err = _ops().rvq_gather(codes, cb)
    if check and not _capturing() and int(err.item()) != 0:
        raise IndexError(f"code out of range for codebook size {cb.shape[1]}")
    return zst, z_p


def rvq_nearest(latents, cbn, c2, nq: int) -> torch.Tensor:
    """decode_latents of stages 0..nq-1 on their own latents (from_latents): codes int64
    [B, nq, T]."""
    return _ops().rvq_nearest(latents, cbn, c2, int(nq))


def rvq_expand(zst, w_out, b_out, imp=None, level: float = 1.0, want_z_q_is: bool = True,
               want_mask: bool = True):
    """z_q_is / masked z_q / mask from the straight-through vectors (HBM-streaming kernel)."""
    zqis, zq, mask = _ops().rvq_expand(zst, w_out, b_out, imp, float(level), bool(want_z_q_is),
                                       bool(want_mask))
    return _none(zqis), zq, _none(mask)


def masked_loss(loss_pf: torch.Tensor, mask: Optional[torch.Tensor]) -> torch.Tensor:
    return _ops().masked_loss(loss_pf, mask)


def scale_imp(imp: torch.Tensor, a: float, c: float) -> torch.Tensor:
    return _ops().scale_imp(imp, float(a), float(c))


def mask_hard(s: torch.Tensor, nq: int) -> torch.Tensor:
    """s: (B, 1, T) scaled importance -> (B, nq, T) {0,1} mask."""
    return _ops().imp_mask(s, int(nq))


def masked_sum(z_q_is: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    return _ops().masked_sum(z_q_is, mask)


def bpf(mask: torch.Tensor, bits: torch.Tensor) -> torch.Tensor:
    return _ops().bpf(mask, bits)


# ----------------------------------------------------------------------------- training step
# Backward operators of the generator (include/vrvq.h "Training step"; vrvq_amd/train.py).
def conv1d_wgrad(a, x, k: int, stride: int = 1, pad: int = 0, dil: int = 1,
                 snake_a: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                 snake_x: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """out[m][c][k] = sum_{b,t} snake_a(a)[b][m][t] * snake_x(x)[b][c][t*stride - pad + k*dil]
    (split-K MFMA GEMM, fixed reduction order)."""
    aa, ia = snake_a if snake_a is not None else (None, None)
    ax, ix = snake_x if snake_x is not None else (None, None)
    return _ops().conv1d_wgrad(a, x, int(k), int(stride), int(pad), int(dil), aa, ia, ax, ix)


def snake_backward(x, alpha, inv_alpha, grad, want_dx: bool = True):
    """Snake1d backward: (dx or None, dalpha [C])."""
    dx, da = _ops().snake_backward(x, alpha, inv_alpha, grad, bool(want_dx))
    return _none(dx), da


def bias_grad(grad: torch.Tensor) -> torch.Tensor:
    return _ops().bias_grad(grad)


def act_backward(y: torch.Tensor, grad: torch.Tensor, epilogue: int) -> torch.Tensor:
    return _ops().act_backward(y, grad, int(epilogue))


def weight_norm_backward(g, v, dw):
    """(dg, dv) of w = v * (g / ||v||) (norm over all dims but 0)."""
    return _ops().weight_norm_backward(g, v, dw)


def pack_conv1d_flip(w: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """Packed adjoint (flipped, transposed) weight of a stride-1 Conv1d."""
    wp = _ops().pack_conv1d_flip(w)
    return wp, wp.shape[2]


def mask_ste(imp, levels, dropout, nq: int, alpha: float, n_imps: int, n_drop: int):
    """Training-mode mask (models/quantize.py:377-414): importance STE rows, dropout rows,
    full-codebook rows."""
    return _ops().mask_ste(imp, levels, dropout, int(nq), float(alpha), int(n_imps), int(n_drop))


def mask_ste_backward(imp, levels, dmask, alpha: float, n_imps: int):
    return _ops().mask_ste_backward(imp, levels, dmask, float(alpha), int(n_imps))


def rvq_encode_train(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, mask):
    """Training-mode quantizer forward: (codes, latents, loss_pf, zst, z_q) with z_q masked by
    the given mask values."""
    return _ops().rvq_encode_train(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, mask)


def rvq_backward(dz_q, g_commit, g_codebook, z, zst, latents, codes, mask, w_in_t, w_out, b_out,
                 mcol, cb):
    """(dz, dmask, dw_in [nq,d,D], db_in, dw_out [nq,D,d], db_out, dcb)."""
    return _ops().rvq_backward(dz_q, g_commit, g_codebook, z, zst, latents, codes, mask, w_in_t,
                               w_out, b_out, mcol, cb)


# ----------------------------------------------------------------------------- fake kernels
def _register_fakes():
    """Shape functions of every op (FakeTensorMode / meta / torch.compile tracing)."""
    reg = torch.library.register_fake

    def f32(t, shape):
        return t.new_empty(shape, dtype=torch.float32)

    def none(t):
        return t.new_empty((0,))

    @reg("vrvq::weight_norm")
    def _(g, v):
        return torch.empty_like(v)

    @reg("vrvq::snake_inv_alpha")
    def _(alpha):
        return torch.empty_like(alpha)

    @reg("vrvq::codebook_prep")
    def _(cb):
        return torch.empty_like(cb), f32(cb, cb.shape[:-1])

    @reg("vrvq::pack_conv1d_weight")
    def _(w):
        cout, cin, k = w.shape
        return f32(w, (cin, k, round_up(cout, 128)))

    @reg("vrvq::pack_x3_weight")
    def _(w_packed, k):
        cin, _k, cout_pad = w_packed.shape
        return torch.empty(x3_size(cin, k, cout_pad), dtype=torch.int16, device=w_packed.device)

    @reg("vrvq::pack_convt1d_weight")
    def _(w, stride):
        cin, cout, _k = w.shape
        return f32(w, (cin, 2, round_up(cout * stride, 128 if 128 % stride == 0 else 192)))

    def pair(x, shape, ao, want_raw):
        ys = f32(x, shape) if ao is not None else none(x)
        y = f32(x, shape) if (want_raw or ao is None) else none(x)
        return y, ys

    @reg("vrvq::snake_conv1d")
    def _(x, w_packed, cout, stride, pad, dil, bias, alpha, inv_alpha, residual, epilogue,
          alpha_out, inv_alpha_out, want_raw, w_x3=None):
        B, _c, tin = x.shape
        tout = conv_out_len(tin, w_packed.shape[1], stride, pad, dil)
        return pair(x, (B, cout, tout), alpha_out, want_raw)

    @reg("vrvq::snake_conv_transpose1d")
    def _(x, w_packed, cout, stride, bias, alpha, inv_alpha, alpha_out, inv_alpha_out, want_raw,
          pad=-1, w_x3=None):
        B, _c, tin = x.shape
        tout = convt_out_len(tin, stride, pad)
        return pair(x, (B, cout, tout), alpha_out, want_raw)

    @reg("vrvq::residual_unit")
    def _(x, x_snk, dil, w7, b7, alpha2, inv_alpha2, w1, b1, alpha_out, inv_alpha_out, want_raw,
          w7_x3=None, w1_x3=None):
        return pair(x, tuple(x.shape), alpha_out, want_raw)

    @reg("vrvq::rvq_cross_prep")
    def _(w_in_t, w_out, b_out):
        nq, _D, d = w_in_t.shape
        return f32(w_in_t, (nq, nq, d, d)), f32(w_in_t, (nq, d))

    @reg("vrvq::rvq_frag")
    def _(cbn):
        return torch.empty_like(cbn)

    @reg("vrvq::rvq_encode")
    def _(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, imp, level, want_z_q_is,
          want_mask):
        B, D, T = z.shape
        nq, _n, d = cb.shape
        return (z.new_empty((B, nq, T), dtype=torch.int64), f32(z, (B, nq * d, T)),
                f32(z, (B, nq, T)), f32(z, (B, nq, D, T)) if want_z_q_is else none(z),
                f32(z, (B, D, T)), f32(z, (B, nq, T)) if want_mask else none(z))

    @reg("vrvq::rvq_pack_w_in")
    def _(w_in_t):
        nq = w_in_t.shape[0]
        return w_in_t.new_empty((32 * 3 * ((nq * 8 + 15) // 16) * 64 * 8,), dtype=torch.int16)

    @reg("vrvq::snake_conv1d_proj")
    def _(x, w_packed, cout, pad, dil, bias, alpha, inv_alpha, w_x3, w3in, nq, want_z):
        B, _c, tin = x.shape
        T = conv_out_len(tin, w_packed.shape[1], 1, pad, dil)
        return f32(x, (8, B * T, nq * 8)), (f32(x, (B, cout, T)) if want_z else none(x))

    @reg("vrvq::rvq_encode_part")
    def _(part, frames, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, imp, level, want_z_q_is,
          want_mask):
        T = frames
        B = part.shape[1] // T
        nq, _n, d = cb.shape
        D = w_out.shape[1]
        return (part.new_empty((B, nq, T), dtype=torch.int64), f32(part, (B, nq * d, T)),
                f32(part, (B, nq, T)), f32(part, (B, nq, D, T)) if want_z_q_is else none(part),
                f32(part, (B, D, T)), f32(part, (B, nq, T)) if want_mask else none(part))

    @reg("vrvq::rvq_gather")
    def _(codes, cb):
        B, nq, T = codes.shape
        d = cb.shape[2]
        return (f32(cb, (B, nq, T, d)), f32(cb, (B, nq * d, T)),
                codes.new_empty((1,), dtype=torch.int32))

    @reg("vrvq::rvq_nearest")
    def _(latents, cbn, c2, nq):
        return latents.new_empty((latents.shape[0], nq, latents.shape[2]), dtype=torch.int64)

    @reg("vrvq::rvq_expand")
    def _(zst, w_out, b_out, imp, level, want_z_q_is, want_mask):
        B, nq, T, _d = zst.shape
        D = w_out.shape[1]
        return (f32(zst, (B, nq, D, T)) if want_z_q_is else none(zst), f32(zst, (B, D, T)),
                f32(zst, (B, nq, T)) if want_mask else none(zst))

    @reg("vrvq::masked_loss")
    def _(loss_pf, mask):
        return f32(loss_pf, ())

    @reg("vrvq::scale_imp")
    def _(imp, a, c):
        return torch.empty_like(imp)

    @reg("vrvq::imp_mask")
    def _(s, nq):
        return f32(s, (s.shape[0], nq, s.shape[-1]))

    @reg("vrvq::masked_sum")
    def _(z_q_is, mask):
        B, _nq, D, T = z_q_is.shape
        return f32(z_q_is, (B, D, T))

    @reg("vrvq::bpf")
    def _(mask, bits):
        return f32(mask, ())

    @reg("vrvq::pack_counts")
    def _(mask):
        B, _nq, T = mask.shape
        return (mask.new_empty((B, T), dtype=torch.int32),
                mask.new_empty((B + 1,), dtype=torch.int64),
                mask.new_empty((1,), dtype=torch.int32))

    @reg("vrvq::pack_codes")
    def _(codes, counts, clip_off, total, ncode):
        return (codes.new_empty((total,), dtype=torch.int16),
                codes.new_empty((1,), dtype=torch.int32))

    @reg("vrvq::unpack_offsets")
    def _(counts):
        return counts.new_empty((counts.shape[0] + 1,), dtype=torch.int64)

    @reg("vrvq::unpack_codes")
    def _(packed, counts, clip_off, n_codebooks):
        B, T = counts.shape
        return (counts.new_empty((B, n_codebooks, T), dtype=torch.int64),
                counts.new_empty((B, n_codebooks, T), dtype=torch.float32))

    @reg("vrvq::conv1d_wgrad")
    def _(a, x, k, stride, pad, dil, alpha_a, inv_alpha_a, alpha, inv_alpha):
        return f32(a, (a.shape[1], x.shape[1], k))

    @reg("vrvq::snake_backward")
    def _(x, alpha, inv_alpha, grad, want_dx):
        return (torch.empty_like(x) if want_dx else none(x)), f32(x, (x.shape[1],))

    @reg("vrvq::bias_grad")
    def _(grad):
        return f32(grad, (grad.shape[1],))

    @reg("vrvq::act_backward")
    def _(y, grad, epilogue):
        return torch.empty_like(y)

    @reg("vrvq::weight_norm_backward")
    def _(g, v, dw):
        return torch.empty_like(g), torch.empty_like(v)

    @reg("vrvq::pack_conv1d_flip")
    def _(w):
        cout, cin, k = w.shape
        return f32(w, (cout, k, round_up(cin, 128)))

    @reg("vrvq::mask_ste")
    def _(imp, levels, dropout, nq, alpha, n_imps, n_drop):
        return f32(imp, (imp.shape[0], nq, imp.shape[-1]))

    @reg("vrvq::mask_ste_backward")
    def _(imp, levels, dmask, alpha, n_imps):
        return torch.empty_like(imp)

    @reg("vrvq::rvq_encode_train")
    def _(z, w_in_t, b_in, cb, cbf, c2, w_out, b_out, mcol, qb, mask):
        B, D, T = z.shape
        nq, _n, d = cb.shape
        return (z.new_empty((B, nq, T), dtype=torch.int64), f32(z, (B, nq * d, T)),
                f32(z, (B, nq, T)), f32(z, (B, nq, T, d)), f32(z, (B, D, T)))

    @reg("vrvq::rvq_backward")
    def _(dz_q, g_commit, g_codebook, z, zst, latents, codes, mask, w_in_t, w_out, b_out, mcol,
          cb):
        nq, D, d = w_in_t.shape
        return (torch.empty_like(z), torch.empty_like(mask), f32(z, (nq, d, D)), f32(z, (nq, d)),
                f32(z, (nq, D, d)), f32(z, (nq, D)), torch.empty_like(cb))
