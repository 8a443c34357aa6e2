"""CPU baseline: a pure-PyTorch (CPU) restatement of the reference VRVQ forward.

TEST INFRASTRUCTURE ONLY, like oracle/vrvq_oracle.py: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it — never the product path (vrvq_amd has no CPU
fallback). It is the timed CPU baseline BASELINE.md plans for the GPU host (the reference's own
Python cannot travel there): the same op sequence as the reference on torch's CPU kernels
(MKLDNN convolutions, the same Snake / weight-norm / RVQ expressions), written functionally over
a reference-named state dict. tests/test_oracle.py pins it against the reference-generated
golden fixtures (codes bit-exact, floats within 1e-5 relative).

Every function cites the reference (lixinghe1999/VRVQ) file:line it restates.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F


class TorchRef:
    """DAC_VRVQ forward (models/dac_vrvq.py:83-252) on torch CPU tensors."""

    def __init__(self, sd: Dict[str, np.ndarray], encoder_rates=(2, 4, 8, 8),
                 decoder_rates=(8, 8, 4, 2), n_codebooks=9, model_type="VBR", **_ignored):
        self.p = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
        self.encoder_rates = list(encoder_rates)
        self.decoder_rates = list(decoder_rates)
        self.n_codebooks = n_codebooks
        self.model_type = model_type
        self.hop = int(np.prod(encoder_rates))
        # padding=False (models/dac_base.py:68-84, the chunked codec): encoder / decoder convs
        # unpadded, residual skips centre-cropped (models/layers.py:65-67)
        self.valid = False
        # weight norm folded once (the reference recomputes it in a pre-hook every forward:
        # the same expression, models/layers.py:17-22 -> torch._weight_norm over dims != 0)
        self.w = {}
        for k in self.p:
            if k.endswith(".weight_g"):
                pre = k[: -len(".weight_g")]
                self.w[pre] = torch._weight_norm(self.p[pre + ".weight_v"], self.p[k], 0)

    # models/layers.py:26-32
    def snake(self, x, pre):
        alpha = self.p[pre + ".alpha"]
        return x + (alpha + 1e-9).reciprocal() * torch.sin(alpha * x).pow(2)

    def conv(self, x, pre, stride=1, pad=0, dil=1):
        return F.conv1d(x, self.w[pre], self.p[pre + ".bias"], stride, pad, dil)

    # models/layers.py:52-68
    def residual_unit(self, x, pre, dil):
        y = self.conv(self.snake(x, pre + ".block.0"), pre + ".block.1", pad=self._p(3 * dil),
                      dil=dil)
        y = self.conv(self.snake(y, pre + ".block.2"), pre + ".block.3")
        pad = (x.shape[-1] - y.shape[-1]) // 2
        if pad > 0:
            x = x[..., pad:-pad]
        return x + y

    def _p(self, pad):
        return 0 if self.valid else pad

    # models/dac_vrvq.py:39-48 with models/layers.py:71-89
    def encoder(self, x):
        x = self.conv(x, "encoder.block.0", pad=self._p(3))
        for i, s in enumerate(self.encoder_rates):
            pre = f"encoder.block.{i + 1}"
            for j, d in enumerate((1, 3, 9)):
                x = self.residual_unit(x, f"{pre}.block.{j}", d)
            x = self.conv(self.snake(x, pre + ".block.3"), pre + ".block.4", stride=s,
                          pad=self._p(math.ceil(s / 2)))
        feat = x
        n = len(self.encoder_rates) + 1
        z = self.conv(self.snake(x, f"encoder.block.{n}"), f"encoder.block.{n + 1}", pad=self._p(1))
        p = (feat.shape[-1] - z.shape[-1]) // 2  # padding=False: feat cropped to z's frames
        return z, (feat[..., p:feat.shape[-1] - p] if p > 0 else feat)

    # models/dac_vrvq.py:79-80 with models/layers.py:92-110
    def decoder(self, z):
        x = self.conv(z, "decoder.model.0", pad=self._p(3))
        for i, s in enumerate(self.decoder_rates):
            pre = f"decoder.model.{i + 1}"
            q = pre + ".block.1"
            x = F.conv_transpose1d(self.snake(x, pre + ".block.0"), self.w[q], self.p[q + ".bias"],
                                   stride=s, padding=self._p(math.ceil(s / 2)))
            for j, d in zip((2, 3, 4), (1, 3, 9)):
                x = self.residual_unit(x, f"{pre}.block.{j}", d)
        n = len(self.decoder_rates) + 1
        x = self.conv(self.snake(x, f"decoder.model.{n}"), f"decoder.model.{n + 1}",
                      pad=self._p(3))
        return torch.tanh(x)

    # models/importance_subnet.py:38-45
    def imp_subnet(self, feat):
        pre = "quantizer.imp_subnet"
        x = self.conv(self.snake(feat, pre + ".in_block.0"), pre + ".in_block.1", pad=1)
        i = 0
        while f"{pre}.blocks.{i}.0.alpha" in self.p:
            x = self.conv(self.snake(x, f"{pre}.blocks.{i}.0"), f"{pre}.blocks.{i}.1", pad=1)
            i += 1
        return torch.sigmoid(x)

    # models/quantize.py:42-103 (one stage, eval)
    def vq_stage(self, residual, i):
        pre = f"quantizer.quantizers.{i}"
        z_e = self.conv(residual, pre + ".in_proj")
        B, d, T = z_e.shape
        enc = F.normalize(z_e.permute(0, 2, 1).reshape(B * T, d))
        cb = self.p[pre + ".codebook.weight"]
        cbn = F.normalize(cb)
        dist = enc.pow(2).sum(1, keepdim=True) - 2 * enc @ cbn.t() + cbn.pow(2).sum(1, keepdim=True).t()
        idx = (-dist).max(1)[1].reshape(B, T)
        z_q = F.embedding(idx, cb).transpose(1, 2)
        loss = F.mse_loss(z_e, z_q, reduction="none").mean(1)
        z_q = z_e + (z_q - z_e)
        return self.conv(z_q, pre + ".out_proj"), loss, idx, z_e

    # models/quantize.py:328-443 (VBR, eval) and :136-214 (CBR, eval)
    def quantize(self, z, feat, level=1.0):
        nq = self.n_codebooks
        residual = z
        z_q_is, losses, codes, lat = [], [], [], []
        for i in range(nq):
            z_q_i, loss, idx, z_e = self.vq_stage(residual, i)
            residual = residual - z_q_i
            z_q_is.append(z_q_i)
            losses.append(loss)
            codes.append(idx)
            lat.append(z_e)
        z_q_is = torch.stack(z_q_is, 1)
        L = torch.stack(losses, 1)
        out = {"codes": torch.stack(codes, 1), "latents": torch.cat(lat, 1), "z_q_is": z_q_is}
        if self.model_type == "CBR":
            out["z_q"] = z_q_is.sum(1)
            out["mask_imp"] = None
            out["imp_map"] = None
            return out
        imp = self.imp_subnet(feat)
        s = imp * level * nq
        mask = (s - torch.arange(nq, dtype=torch.float32)[None, :, None] >= 0).float()
        out["z_q"] = (z_q_is * mask[:, :, None, :]).sum(1)
        out["commitment_loss"] = (L * mask).sum(1).mean()
        out["imp_map"] = imp
        out["mask_imp"] = mask
        return out

    # models/dac_vrvq.py:222-252
    @torch.no_grad()
    def forward(self, audio: torch.Tensor, level: float = 1.0):
        L = audio.shape[-1]
        x = F.pad(audio, (0, math.ceil(L / self.hop) * self.hop - L))
        z, feat = self.encoder(x)
        q = self.quantize(z, feat, level)
        q["audio"] = self.decoder(q["z_q"])[..., :L]
        return q
