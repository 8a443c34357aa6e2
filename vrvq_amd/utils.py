"""Importance-map gating and rate helpers (reference: models/utils.py:45-73,
scripts/inference.py:88-112) on gfx950 kernels."""
from __future__ import annotations

import math
from typing import Sequence

import torch

from . import ops


def _as_scaled(x: torch.Tensor) -> torch.Tensor:
    if x.dtype != torch.float32:
        raise RuntimeError("importance map must be float32")
    return x.contiguous()


def generate_mask_hard(x: torch.Tensor, nq: int) -> torch.Tensor:
    """mask[b, n, t] = 1.0 if x[b, 0, t] - n >= 0 else 0.0   (models/utils.py:55-61)."""
    return ops.mask_hard(_as_scaled(x), nq)


def generate_mask_ste(x: torch.Tensor, nq: int, alpha: float = 1) -> torch.Tensor:
    """Straight-through mask (models/utils.py:45-53): x (B, 1, T) the scaled importance map.

    Forward: mask_smooth + (mask_quant - mask_smooth).detach(), which equals the hard mask
    exactly in fp32 (for q = 0 it is s + (-s) = 0; for q = 1, s >= 0.5 and 1 - s is exact by
    Sterbenz). Backward (when x requires grad): d/dx of the log-cosh smooth step
    logcosh(alpha, x - n) (models/utils.py:11-32), summed over the nq rows. Both run in the
    mask STE kernels (include/vrvq.h vrvq_mask_ste with levels = NULL)."""
    from . import train
    x = _as_scaled(x)
    if x.requires_grad and torch.is_grad_enabled():
        return train.mask_ste(x, nq, float(alpha))
    return ops.mask_hard(x, nq)


def scale_importance(imp_map: torch.Tensor, a: float, c: float = 1.0) -> torch.Tensor:
    """(imp_map * a) * c with fp32 roundings (see include/vrvq.h vrvq_scale_imp)."""
    return ops.scale_imp(_as_scaled(imp_map), a, c)


def cal_bpf_from_mask(mask: torch.Tensor, bits_per_codebook: Sequence[float]) -> float:
    """Bits per frame: sum(mask * bits[n]) / (B * T), returned as a Python float like the
    reference's `.item()` (models/utils.py:64-73)."""
    return float(cal_bpf_tensor(mask, bits_per_codebook).item())


def cal_bpf_tensor(mask: torch.Tensor, bits_per_codebook: Sequence[float]) -> torch.Tensor:
    """Same as cal_bpf_from_mask but returns a 0-d device tensor (no host sync)."""
    bits = torch.as_tensor(list(bits_per_codebook), dtype=torch.float32).to(mask.device)
    return ops.bpf(mask.contiguous(), bits)


def masked_sum(z_q_is: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """z_q = sum_i z_q_is[:, i] * mask[:, i, None, :]   (scripts/inference.py:99-100)."""
    return ops.masked_sum(z_q_is.contiguous(), mask.contiguous())


def check_errors(device=None) -> None:
    """End-of-work check for the fused RVQ launches' bounded in-kernel waits (include/vrvq.h
    vrvq_rvq_pending_error): synchronises the device, then raises RuntimeError if any launch
    completed by now timed out (its outputs were poisoned: codes -1, NaN z_q). The RVQ ops also
    raise on such a code at their next call; a one-shot caller (a single encode, the last call of
    a sweep) calls this after its own work instead. Clears the code it reports."""
    from . import _lib
    torch.cuda.synchronize(device)
    code = _lib.rvq_pending_error()
    if code:
        raise RuntimeError(
            f"vrvq: a fused RVQ launch timed out in an in-kernel hand-off (code {code}: "
            f"{'projection partials' if code == 1 else 'stage rows'}); its outputs are invalid "
            "(codes -1, NaN)")


def sweep_latents(imp_map: torch.Tensor, z_q_is: torch.Tensor, levels: Sequence[float],
                  n_q: int):
    """Per level: hard mask of imp_map * (level * Nq) and the masked sum of z_q_is
    (scripts/inference.py:95-100). Returns (masks, z_q stacked level-major as (L*B, D, T))."""
    masks = [generate_mask_hard(scale_importance(imp_map, level * n_q, 1.0), n_q)
             for level in levels]
    return masks, torch.cat([masked_sum(z_q_is, m) for m in masks])


def level_sweep(model, audio: torch.Tensor, levels: Sequence[float], bits_per_codebook: int = 10,
                decode: bool = True, max_decode_clips: int | None = None):
    """The reference's VBR level sweep (scripts/inference.py:88-112) without file I/O.

    Encodes once (level 1), then for each level: hard mask of imp_map * (level * Nq),
    masked sum of z_q_is, bpf and kbps. The levels' z_q are decoded as batches of up to
    `max_decode_clips` clips (default: all L*B at once, the fastest; the reference decodes level
    by level, so a cap of B keeps its peak decoder memory). Clips are independent, but a conv's
    tile choice can depend on the batch size, so the per-level recon agrees with a per-level
    decode within fp32 rounding, not bit for bit (tests/test_gpu_parity.py checks the batched
    recon against the reference's per-level fixtures). Returns a list of dicts."""
    n_q = model.n_codebooks
    with torch.no_grad():
        x = model.preprocess(audio, model.sample_rate)
        enc = model.encode(x, n_quantizers=None, level=1)
        masks, z_all = sweep_latents(enc["imp_map"], enc["z_q_is"], levels, n_q)
        recon_all = None
        if decode:
            cap = max_decode_clips or z_all.shape[0]
            if cap < 1:
                raise ValueError("max_decode_clips must be >= 1")
            recon_all = torch.cat([model.decode(z_all[i:i + cap])
                                   for i in range(0, z_all.shape[0], cap)])
    check_errors(audio.device)  # the sweep's one encode: a timed-out hand-off raises here
    B = audio.shape[0]
    out = []
    for li, level in enumerate(levels):
        mask = masks[li]
        bpf = cal_bpf_from_mask(mask, [bits_per_codebook] * n_q)
        kbps = bpf * math.floor(model.sample_rate / model.hop_length) / 1000
        recon = recon_all[li * B:(li + 1) * B] if decode else None
        out.append({"level": level, "level_scaled": level * n_q, "mask": mask,
                    "z_q": z_all[li * B:(li + 1) * B], "recon": recon, "bpf": bpf, "kbps": kbps})
    return out
