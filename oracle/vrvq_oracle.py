"""CPU oracle: a numpy float32 restatement of the reference VRVQ hot path.

TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module, and only as the checker / the timed CPU baseline — never as the
product path (vrvq_amd has no CPU fallback).

Pinned against the reference: tests/test_oracle.py checks it against the golden fixtures in
tests/golden/ (produced by tests/golden/make_golden.py, which runs the reference PyTorch CPU
path itself): codes bit-exact, floats within 1e-4 relative.

Every function cites the reference (lixinghe1999/VRVQ) file:line it restates. The state dict
is a mapping name -> np.float32 array with the reference's parameter names.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np

F32 = np.float32


# --------------------------------------------------------------------------- primitives
def weight_norm(g: np.ndarray, v: np.ndarray) -> np.ndarray:
    """torch weight_norm(dim=0): v * (g / ||v||), norm over all dims but 0
    (models/layers.py:17-22)."""
    n = np.sqrt(np.sum(v.astype(np.float64) ** 2, axis=tuple(range(1, v.ndim)), keepdims=True))
    return (v * (g / n.astype(F32))).astype(F32)


def snake(x: np.ndarray, alpha: np.ndarray) -> np.ndarray:
    """x + (alpha + 1e-9)^-1 * sin(alpha * x)^2   (models/layers.py:26-32)."""
    alpha = alpha.reshape(1, -1, 1).astype(F32)
    inv = (F32(1.0) / (alpha + F32(1e-9))).astype(F32)
    s = np.sin(alpha * x).astype(F32)
    return (x + inv * (s * s)).astype(F32)


def conv1d(x: np.ndarray, w: np.ndarray, b: Optional[np.ndarray], stride: int = 1,
           pad: int = 0, dil: int = 1) -> np.ndarray:
    """nn.Conv1d: y[b,co,t] = bias[co] + sum_{ci,k} w[co,ci,k] x[b,ci,t*s - p + k*d]."""
    B, cin, tin = x.shape
    cout, _, K = w.shape
    tout = (tin + 2 * pad - dil * (K - 1) - 1) // stride + 1
    xp = np.zeros((B, cin, tin + 2 * pad), F32)
    xp[:, :, pad:pad + tin] = x
    y = np.zeros((B, cout, tout), F32)
    for bi in range(B):
        for k in range(K):
            s0 = k * dil
            # contiguous copy: numpy's matmul leaves BLAS for strided operands
            xs = np.ascontiguousarray(xp[bi, :, s0: s0 + (tout - 1) * stride + 1: stride])
            y[bi] += np.ascontiguousarray(w[:, :, k]) @ xs
    if b is not None:
        y += b.reshape(1, -1, 1)
    return y


def conv_transpose1d(x: np.ndarray, w: np.ndarray, b: Optional[np.ndarray], stride: int,
                     pad: int) -> np.ndarray:
    """nn.ConvTranspose1d, weight (Cin, Cout, K): y[t*s - p + k] += x[t] w[:, :, k]."""
    B, cin, tin = x.shape
    _, cout, K = w.shape
    full = (tin - 1) * stride + K
    y = np.zeros((B, cout, full), F32)
    for bi in range(B):
        xb = np.ascontiguousarray(x[bi])
        for k in range(K):
            y[bi, :, k: k + (tin - 1) * stride + 1: stride] += np.ascontiguousarray(w[:, :, k].T) @ xb
    tout = full - 2 * pad
    y = y[:, :, pad: pad + tout]
    if b is not None:
        y = y + b.reshape(1, -1, 1)
    return np.ascontiguousarray(y, dtype=F32)


def sigmoid(x):
    return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(F32)


# --------------------------------------------------------------------------- model pieces
class Oracle:
    """Forward pass of DAC_VRVQ (models/dac_vrvq.py:83-252) on a reference-named state dict."""

    def __init__(self, sd: Dict[str, np.ndarray], encoder_dim=64, encoder_rates=(2, 4, 8, 8),
                 latent_dim=None, decoder_dim=1536, decoder_rates=(8, 8, 4, 2), n_codebooks=9,
                 codebook_size=1024, codebook_dim=8, model_type="VBR", sample_rate=44100,
                 **_ignored):
        self.sd = {k: np.asarray(v, F32) for k, v in sd.items()}
        self.encoder_rates = list(encoder_rates)
        self.decoder_rates = list(decoder_rates)
        self.encoder_dim = encoder_dim
        self.decoder_dim = decoder_dim
        self.latent_dim = latent_dim or encoder_dim * 2 ** len(encoder_rates)
        self.n_codebooks = n_codebooks
        self.codebook_dim = codebook_dim
        self.model_type = model_type
        self.sample_rate = sample_rate
        self.hop_length = int(np.prod(encoder_rates))
        self._w = {}

    def w(self, prefix: str) -> np.ndarray:
        if prefix not in self._w:
            self._w[prefix] = weight_norm(self.sd[prefix + ".weight_g"], self.sd[prefix + ".weight_v"])
        return self._w[prefix]

    def conv(self, x, prefix, stride=1, pad=0, dil=1):
        return conv1d(x, self.w(prefix), self.sd[prefix + ".bias"], stride, pad, dil)

    def snake(self, x, prefix):
        return snake(x, self.sd[prefix + ".alpha"])

    # models/layers.py:52-68
    def residual_unit(self, x, p, dil):
        y = self.snake(x, p + ".block.0")
        y = self.conv(y, p + ".block.1", pad=3 * dil, dil=dil)
        y = self.snake(y, p + ".block.2")
        y = self.conv(y, p + ".block.3")
        return (x + y).astype(F32)

    # models/layers.py:71-89
    def encoder_block(self, x, p, stride):
        for i, d in enumerate((1, 3, 9)):
            x = self.residual_unit(x, f"{p}.block.{i}", d)
        x = self.snake(x, p + ".block.3")
        return self.conv(x, p + ".block.4", stride=stride, pad=math.ceil(stride / 2))

    # models/layers.py:92-110
    def decoder_block(self, x, p, stride):
        x = self.snake(x, p + ".block.0")
        q = p + ".block.1"
        x = conv_transpose1d(x, self.w(q), self.sd[q + ".bias"], stride, math.ceil(stride / 2))
        for i, d in zip((2, 3, 4), (1, 3, 9)):
            x = self.residual_unit(x, f"{p}.block.{i}", d)
        return x

    # models/dac_vrvq.py:39-48
    def encoder(self, x):
        x = self.conv(x, "encoder.block.0", pad=3)
        for i, s in enumerate(self.encoder_rates):
            x = self.encoder_block(x, f"encoder.block.{i + 1}", s)
        feat = x
        n = len(self.encoder_rates) + 1
        x = self.snake(x, f"encoder.block.{n}")
        return self.conv(x, f"encoder.block.{n + 1}", pad=1), feat

    # models/dac_vrvq.py:79-80
    def decoder(self, z):
        x = self.conv(z, "decoder.model.0", pad=3)
        for i, s in enumerate(self.decoder_rates):
            x = self.decoder_block(x, f"decoder.model.{i + 1}", s)
        n = len(self.decoder_rates) + 1
        x = self.snake(x, f"decoder.model.{n}")
        x = self.conv(x, f"decoder.model.{n + 1}", pad=3)
        return np.tanh(x).astype(F32)

    # models/importance_subnet.py:38-45
    def imp_subnet(self, feat):
        p = "quantizer.imp_subnet"
        x = self.snake(feat, p + ".in_block.0")
        x = self.conv(x, p + ".in_block.1", pad=1)
        i = 0
        while f"{p}.blocks.{i}.0.alpha" in self.sd:
            x = self.snake(x, f"{p}.blocks.{i}.0")
            x = self.conv(x, f"{p}.blocks.{i}.1", pad=1)
            i += 1
        return sigmoid(x)

    # models/quantize.py:42-103 (one stage)
    def vq_stage(self, residual, i):
        p = f"quantizer.quantizers.{i}"
        z_e = self.conv(residual, p + ".in_proj")                     # (B, d, T)
        B, d, T = z_e.shape
        enc = z_e.transpose(0, 2, 1).reshape(-1, d)                    # (B*T, d)
        cb = self.sd[p + ".codebook.weight"]
        en = enc / np.maximum(np.sqrt(np.sum(enc * enc, 1, keepdims=True)), F32(1e-12))
        cn = cb / np.maximum(np.sqrt(np.sum(cb * cb, 1, keepdims=True)), F32(1e-12))
        dist = (np.sum(en * en, 1, keepdims=True) - 2 * en @ cn.T) + np.sum(cn * cn, 1, keepdims=True).T
        idx = np.argmax(-dist, axis=1).reshape(B, T)                   # first index on ties
        z_q = cb[idx].transpose(0, 2, 1).astype(F32)                   # raw codebook rows
        loss = np.mean((z_e - z_q) ** 2, axis=1).astype(F32)           # (B, T)
        z_st = (z_e + (z_q - z_e)).astype(F32)
        z_q_i = self.conv(z_st, p + ".out_proj")
        return z_q_i, loss, idx.astype(np.int64), z_e

    # models/quantize.py:217-249 (ResidualVectorQuantize.from_codes): decode_code (:81-85,
    # raw codebook rows) -> out_proj per stage, z_q = sum in stage order; with `mask` the
    # masked sum of scripts/inference.py:99-100 (VBR).
    def from_codes(self, codes, mask=None):
        B, n, T = codes.shape
        z_p, z_q_is = [], []
        for i in range(n):
            p = f"quantizer.quantizers.{i}"
            cb = self.sd[p + ".codebook.weight"]
            zp = cb[codes[:, i]].transpose(0, 2, 1).astype(F32)         # (B, d, T)
            z_p.append(zp)
            z_q_is.append(self.conv(zp, p + ".out_proj"))
        z_q_is = np.stack(z_q_is, axis=1)
        if mask is None:
            z_q = np.zeros(z_q_is[:, 0].shape, F32)
            for i in range(n):
                z_q = z_q + z_q_is[:, i]
        else:
            z_q = masked_sum(z_q_is, mask)
        return z_q, np.concatenate(z_p, axis=1), z_q_is

    # models/quantize.py:251-285 (ResidualVectorQuantize.from_latents): per whole stage of the
    # latents, decode_latents (:87-103) on the stage's own slice (no residual), out_proj, sum.
    def from_latents(self, latents):
        B, C, T = latents.shape
        n = min(C // 8, self.n_codebooks)
        z_q = np.zeros((B, self.sd["quantizer.quantizers.0.out_proj.bias"].shape[0], T), F32)
        z_p, codes = [], []
        for i in range(n):
            p = f"quantizer.quantizers.{i}"
            enc = latents[:, 8 * i: 8 * i + 8].transpose(0, 2, 1).reshape(-1, 8)
            cb = self.sd[p + ".codebook.weight"]
            en = enc / np.maximum(np.sqrt(np.sum(enc * enc, 1, keepdims=True)), F32(1e-12))
            cn = cb / np.maximum(np.sqrt(np.sum(cb * cb, 1, keepdims=True)), F32(1e-12))
            dist = (np.sum(en * en, 1, keepdims=True) - 2 * en @ cn.T) + np.sum(cn * cn, 1, keepdims=True).T
            idx = np.argmax(-dist, axis=1).reshape(B, T)
            zp = cb[idx].transpose(0, 2, 1).astype(F32)
            z_p.append(zp)
            codes.append(idx.astype(np.int64))
            z_q = z_q + self.conv(zp, p + ".out_proj")
        return z_q, np.concatenate(z_p, axis=1), np.stack(codes, axis=1)

    # models/quantize.py:328-443 (eval) and :136-214 (CBR eval)
    def quantize(self, z, n_quantizers=None, feat=None, level=1.0):
        nq = self.n_codebooks
        if self.model_type == "CBR":
            n = nq if n_quantizers is None else min(n_quantizers, nq)
        else:
            n = nq
        residual = z
        z_q_is, losses, codes, lat = [], [], [], []
        for i in range(n):
            z_q_i, loss, idx, z_e = self.vq_stage(residual, i)
            z_q_is.append(z_q_i)
            residual = (residual - z_q_i).astype(F32)
            losses.append(loss)
            codes.append(idx)
            lat.append(z_e)
        zqis = np.stack(z_q_is, 1)
        L = np.stack(losses, 1)
        out = {"codes": np.stack(codes, 1), "latents": np.concatenate(lat, 1)}
        if self.model_type == "CBR":
            out["z_q"] = np.sum(zqis, 1).astype(F32)
            out["commitment_loss"] = F32(sum(np.mean(L[:, i]) for i in range(n)))
            return out
        if n_quantizers is None:
            imp = self.imp_subnet(feat)
            s = (imp * F32(level)).astype(F32) * F32(nq)
            mask = generate_mask_hard(s, nq)
        else:
            imp, mask = None, np.ones((z.shape[0], nq, z.shape[2]), F32)
        out["z_q"] = masked_sum(zqis, mask)
        out["z_q_is"] = zqis
        out["commitment_loss"] = F32(np.mean(np.sum(L * mask, 1)))
        out["imp_map"] = imp
        out["mask_imp"] = mask
        return out

    # models/dac_vrvq.py:164-173
    def preprocess(self, audio):
        L = audio.shape[-1]
        pad = math.ceil(L / self.hop_length) * self.hop_length - L
        return np.pad(audio, ((0, 0), (0, 0), (0, pad))).astype(F32)

    # models/dac_vrvq.py:222-252
    def forward(self, audio, n_quantizers=None, level=1.0):
        L = audio.shape[-1]
        x = self.preprocess(audio)
        z, feat = self.encoder(x)
        q = self.quantize(z, n_quantizers, feat, level)
        y = self.decoder(q["z_q"])
        q["audio"] = y[..., :L]
        q["z"] = z
        q["feat"] = feat
        return q


# --------------------------------------------------------------------------- gating helpers
def generate_mask_hard(s: np.ndarray, nq: int) -> np.ndarray:
    """mask[b,n,t] = (s[b,0,t] - n >= 0)   (models/utils.py:55-61)."""
    n = np.arange(nq, dtype=F32).reshape(1, nq, 1)
    return ((s - n) >= 0).astype(F32)


def masked_sum(z_q_is: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """sum_i z_q_is[:, i] * mask[:, i, None]   (models/quantize.py:420-421)."""
    acc = np.zeros(z_q_is[:, 0].shape, F32)
    for i in range(z_q_is.shape[1]):
        acc = acc + z_q_is[:, i] * mask[:, i, None, :]
    return acc


def cal_bpf_from_mask(mask: np.ndarray, bits_per_codebook: List[float]) -> float:
    """sum(mask * bits) / (B*T)   (models/utils.py:64-73)."""
    bits = np.asarray(bits_per_codebook, F32).reshape(1, -1, 1)
    return float(np.sum(mask * bits, dtype=np.float64) / (mask.shape[0] * mask.shape[2]))


def pack_codes(codes: np.ndarray, mask: np.ndarray):
    """Variable-length packing (vrvq_amd/codes_io.py; no reference
    counterpart — the reference's DACFile, models/dac_base.py:19-58, stores every code): per
    clip, per frame, the codes of the stages whose mask is 1, in stage order. Returns
    (packed uint16, counts (B, T) int32)."""
    B, nq, T = codes.shape
    on = mask != 0
    counts = on.sum(1).astype(np.int32)
    packed = codes.transpose(0, 2, 1)[on.transpose(0, 2, 1)].astype(np.uint16)
    return packed, counts
