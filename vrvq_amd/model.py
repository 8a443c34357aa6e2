"""Drop-in DAC_VRVQ codec (reference: models/dac_vrvq.py, models/quantize.py,
models/importance_subnet.py, models/dac_base.py) on gfx950 kernels.

Same constructor kwargs (the `DAC_VRVQ.*` keys of conf/*.yml), same state_dict keys, same
`preprocess / encode / decode / forward` signatures and output dicts. All arithmetic runs in
libvrvq_hip.so (see ops.py); the modules here hold parameters and orchestrate launches.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Union

import numpy as np
import torch
import torch.nn as nn

from . import ops, train
from .layers import (DecoderBlock, EncoderBlock, ResidualUnit, Snake1d, WNConv1d,
                     WNConvTranspose1d, _param_key)


# ============================================================================ encoder / decoder
class Encoder(nn.Module):
    """models/dac_vrvq.py:19-48. forward(x, return_feat) -> z or (z, feat)."""

    def __init__(self, d_model: int = 64, strides: List[int] = [2, 4, 8, 8], latent_dim: int = 512):
        super().__init__()
        blocks = [WNConv1d(1, d_model, kernel_size=7, padding=3)]
        for stride in strides:
            d_model *= 2
            blocks += [EncoderBlock(d_model, stride=stride)]
        blocks += [Snake1d(d_model), WNConv1d(d_model, latent_dim, kernel_size=3, padding=1)]
        self.block = nn.Sequential(*blocks)
        self.valid = False  # padding=False (CodecMixin.padding): unpadded convs

    def forward(self, x, return_feat: bool = False, project: Optional["_Stacked"] = None):
        """project (a quantizer's stacked stage weights): z comes back as a ProjectedZ -- the last conv's epilogue projects it onto every
        stage's in_proj (include/vrvq.h vrvq_conv1d_proj) and z itself is not written."""
        if self.training:  # autograd path (vrvq_amd/train.py)
            if self.valid:
                raise NotImplementedError("padding=False is an inference (compress) mode")
            out, feat = train.encoder_forward(self, x)
            return (out, feat) if return_feat else out
        n = len(self.block)
        if self.valid:
            # Unpadded convs change every length, so the per-module forms run (Snake in each
            # conv's prologue, residual units with the centre-cropped skip).
            x = self.block[0](x)
            for i in range(1, n - 2):
                x = self.block[i](x)
            out = self.block[n - 1](x, snake=self.block[n - 2])
            # the unpadded k3 conv leaves z 2 frames shorter than feat: feat is centre-cropped
            # to z's frames so the importance map gates the frames it was computed for
            p = (x.shape[-1] - out.shape[-1]) // 2
            feat = x[..., p:x.shape[-1] - p].contiguous() if p > 0 else x
            return (out, feat) if return_feat else out
        # Chained launches: every conv's epilogue also writes the next Snake's output, so each
        # activation is evaluated once per element (include/vrvq.h, producer-side Snake).
        x, x_snk = self.block[0](x, out_snake=self.block[1].entry_snake())
        for i in range(1, n - 2):
            last = i == n - 3
            nxt = None if last else self.block[i + 1].entry_snake()
            r = self.block[i].run(x, x_snk, nxt, want_raw=True)
            x, x_snk = (r, None) if last else r
        feat = x  # output of block index n-3 (the last EncoderBlock), models/dac_vrvq.py:43-44
        if project is not None:
            nq = project.b_in.shape[0]
            part, _ = self.block[n - 1].forward_proj(x, project.w3in(), nq, snake=self.block[n - 2])
            B = x.shape[0]
            out = ProjectedZ(part, B, self.block[n - 1].out_channels, part.shape[1] // B, nq)
        else:
            out = self.block[n - 1](x, snake=self.block[n - 2])
        return (out, feat) if return_feat else out


class Decoder(nn.Module):
    """models/dac_vrvq.py:51-80: conv k7, DecoderBlocks, Snake, conv k7, Tanh (fused)."""

    def __init__(self, input_channel, channels, rates, d_out: int = 1):
        super().__init__()
        layers = [WNConv1d(input_channel, channels, kernel_size=7, padding=3)]
        output_dim = channels
        for i, stride in enumerate(rates):
            input_dim = channels // 2 ** i
            output_dim = channels // 2 ** (i + 1)
            layers += [DecoderBlock(input_dim, output_dim, stride)]
        layers += [Snake1d(output_dim), WNConv1d(output_dim, d_out, kernel_size=7, padding=3),
                   nn.Tanh()]
        self.model = nn.Sequential(*layers)
        self.valid = False  # padding=False (CodecMixin.padding): unpadded convs

    def forward(self, x):
        if self.training:
            if self.valid:
                raise NotImplementedError("padding=False is an inference (decompress) mode")
            return train.decoder_forward(self, x)
        n = len(self.model)
        if self.valid:
            x = self.model[0](x)
            for i in range(1, n - 3):
                x = self.model[i](x)
            return self.model[n - 2](x, snake=self.model[n - 3], epilogue=ops.EPI_TANH)
        _, x_snk = self.model[0](x, out_snake=self.model[1].entry_snake(), want_raw=False)
        for i in range(1, n - 3):
            nxt = self.model[n - 3] if i == n - 4 else self.model[i + 1].entry_snake()
            _, x_snk = self.model[i].run(x_snk, nxt, want_raw=False)
        return self.model[n - 2](x_snk, epilogue=ops.EPI_TANH)


# ============================================================================ importance subnet
class ImportanceSubnet(nn.Module):
    """models/importance_subnet.py:6-45: [Snake, WN k3 conv] x 6 then Sigmoid (fused)."""

    def __init__(self, d_input, d_feat, intermediate_channels: list = [512, 128, 32, 8],
                 out_channels=1, detach_input: bool = False):
        super().__init__()
        self.in_block = nn.Sequential(Snake1d(d_input),
                                      WNConv1d(d_input, d_feat, kernel_size=3, padding=1))
        in_ch = [d_feat] + list(intermediate_channels)
        out_ch = list(intermediate_channels) + [out_channels]
        self.blocks = nn.ModuleList([
            nn.Sequential(Snake1d(in_ch[i]), WNConv1d(in_ch[i], out_ch[i], kernel_size=3, padding=1))
            for i in range(len(in_ch))
        ])
        self.act_fn = nn.Sigmoid()
        self.detach_input = detach_input  # detaches the input in training (no grad to feat)

    def forward(self, x_in):
        if self.training:
            return train.imp_subnet_forward(self, x_in)
        x = self.in_block[1](x_in, snake=self.in_block[0])
        last = len(self.blocks) - 1
        for i, blk in enumerate(self.blocks):
            x = blk[1](x, snake=blk[0], epilogue=ops.EPI_SIGMOID if i == last else ops.EPI_NONE)
        return x  # (B, 1, T) in (0, 1)


# ============================================================================ quantizers
class VectorQuantize(nn.Module):
    """Factorised, L2-normalised VQ stage (models/quantize.py:21-103)."""

    def __init__(self, input_dim: int, codebook_size: int, codebook_dim: int):
        super().__init__()
        self.codebook_size = codebook_size
        self.codebook_dim = codebook_dim
        self.in_proj = WNConv1d(input_dim, codebook_dim, kernel_size=1)
        self.out_proj = WNConv1d(codebook_dim, input_dim, kernel_size=1)
        self.codebook = nn.Embedding(codebook_size, codebook_dim)

    def forward(self, z, loss_per_frame: bool = False):
        """Single-stage quantisation (the fused RVQ kernels with nq = 1).

        Returns z_q, commitment_loss, codebook_loss, indices, z_e as the reference does
        (losses per frame (B, T) if loss_per_frame else per item (B,))."""
        st = _stack_stages([self], z.device)
        codes, latents, loss_pf, _, z_q, _ = _rvq_encode(z, st, want_z_q_is=False,
                                                          want_mask=False)
        loss = loss_pf[:, 0, :]
        if not loss_per_frame:
            loss = loss.mean(1)
        return z_q, loss, loss.clone(), codes[:, 0, :], latents


# The eval encode hands z to the quantizer as its stage projections: the encoder's last conv
# computes every stage's in_proj in its epilogue (vrvq_conv1d_proj) and the quantizer runs from
# those partials (vrvq_rvq_encode_part: no z read, no projection in front of the chain).
# VRVQ_RVQ_PROJ=0 (A/B): z (B, D, T) and vrvq_rvq_encode.
RVQ_PROJ = os.environ.get("VRVQ_RVQ_PROJ", "1") != "0"


class ProjectedZ:
    """The encoder's z as the eval quantizer consumes it: the in_proj of every stage, computed in
    the last conv's epilogue (include/vrvq.h vrvq_conv1d_proj) as (8, B*T, 8 nq) channel-split
    partials -- rvq_project's values bit for bit. z (B, D, T) itself is not materialised; `shape`
    is its shape."""

    def __init__(self, part: torch.Tensor, B: int, D: int, T: int, nq: int):
        self.part = part
        self.shape = torch.Size((B, D, T))
        self.nq = nq

    def dim(self) -> int:
        return 3

    @property
    def device(self):
        return self.part.device


def _rvq_encode(z, st, **kw):
    """ops.rvq_encode_part for a ProjectedZ, else ops.rvq_encode."""
    if isinstance(z, ProjectedZ):
        if z.nq != st.b_in.shape[0]:
            raise RuntimeError(f"ProjectedZ holds {z.nq} stages' projections, the quantizer "
                               f"runs {st.b_in.shape[0]}")
        return ops.rvq_encode_part(z.part, z.shape[2], st.b_in, st.cb, st.cbf, st.c2, st.w_out,
                                   st.b_out, st.mcol, st.qb, **kw)
    return ops.rvq_encode(z.contiguous(), *st.codes_args(), **kw)


class _Stacked:
    """Per-stage RVQ weights folded and stacked in the kernels' layouts."""

    def __init__(self, quantizers, device):
        w_in_t, b_in, cb, w_out, b_out = [], [], [], [], []
        for q in quantizers:
            wi = q.in_proj.folded_weight()                       # (d, D, 1)
            w_in_t.append(wi.reshape(wi.shape[0], wi.shape[1]).t())
            b_in.append(q.in_proj.bias.detach())
            cb.append(q.codebook.weight.detach())
            wo = q.out_proj.folded_weight()                      # (D, d, 1)
            w_out.append(wo.reshape(wo.shape[0], wo.shape[1]))
            b_out.append(q.out_proj.bias.detach())
        self.w_in_t = torch.stack(w_in_t).contiguous()
        self.b_in = torch.stack(b_in).contiguous()
        self.cb = torch.stack(cb).contiguous()
        self.cbn, self.c2 = ops.codebook_prep(self.cb)
        self.cbf = ops.rvq_frag(self.cbn)  # the chain's MFMA fragment order
        self.w_out = torch.stack(w_out).contiguous()
        self.b_out = torch.stack(b_out).contiguous()
        # cross terms of the projected chain (include/vrvq.h, vrvq_rvq_cross_prep)
        self.mcol, self.qb = ops.rvq_cross_prep(self.w_in_t, self.w_out, self.b_out)

    def codes_args(self):
        return (self.w_in_t, self.b_in, self.cb, self.cbf, self.c2, self.w_out, self.b_out,
                self.mcol, self.qb)

    def w3in(self):
        """W_in planes of the encoder conv's projection epilogue (packed on first use)."""
        if getattr(self, "_w3in", None) is None:
            self._w3in = ops.rvq_pack_w_in(self.w_in_t)
        return self._w3in

    def prefix(self, n):
        """The first n stages (a CBR prefix), built once per n."""
        cache = self.__dict__.setdefault("_prefixes", {})
        if n not in cache:
            s = _Stacked.__new__(_Stacked)
            s._w3in = None
            for k in ("w_in_t", "b_in", "cb", "cbn", "cbf", "c2", "w_out", "b_out", "qb"):
                setattr(s, k, getattr(self, k)[:n].contiguous())
            s.mcol = self.mcol[:n, :n].contiguous()
            cache[n] = s
        return cache[n]


def _stack_stages(quantizers, device):
    return _Stacked(quantizers, device)


class ResidualVectorQuantize(nn.Module):
    """CBR residual VQ (models/quantize.py:106-285)."""

    def __init__(self, input_dim: int = 512, n_codebooks: int = 9, codebook_size: int = 1024,
                 codebook_dim: Union[int, list] = 8, quantizer_dropout: float = 0.0):
        super().__init__()
        if isinstance(codebook_dim, int):
            codebook_dim = [codebook_dim for _ in range(n_codebooks)]
        self.n_codebooks = n_codebooks
        self.codebook_dim = codebook_dim
        self.codebook_size = codebook_size
        self.quantizers = nn.ModuleList([
            VectorQuantize(input_dim, codebook_size, codebook_dim[i]) for i in range(n_codebooks)
        ])
        self.quantizer_dropout = quantizer_dropout
        self._stack_cache = None

    def stacked(self) -> _Stacked:
        params = []
        for q in self.quantizers:
            params += [q.in_proj.weight_g, q.in_proj.weight_v, q.in_proj.bias, q.codebook.weight,
                       q.out_proj.weight_g, q.out_proj.weight_v, q.out_proj.bias]
        key = _param_key(*params)
        if self._stack_cache is None or self._stack_cache[0] != key:
            self._stack_cache = (key, _Stacked(self.quantizers, params[0].device))
        return self._stack_cache[1]

    def forward(self, z, n_quantizers: int = None):
        if self.training:  # quantizer dropout, autograd (models/quantize.py:175-199)
            return train.cbr_forward(self, z.contiguous())
        n = self.n_codebooks if n_quantizers is None else min(int(n_quantizers), self.n_codebooks)
        st = self.stacked()
        if n < self.n_codebooks:
            st = st.prefix(n)
        codes, latents, loss_pf, _, z_q, _ = _rvq_encode(z, st, want_z_q_is=False,
                                                          want_mask=False)
        loss = ops.masked_loss(loss_pf, None)  # sum_i mean_{b,t} loss_i (mask all-true in eval)
        return {"z_q": z_q, "codes": codes, "latents": latents,
                "commitment_loss": loss, "codebook_loss": loss.clone()}

    def from_codes(self, codes: torch.Tensor, return_z_q_is: bool = False):
        """Codes -> continuous latents (models/quantize.py:217-249): per stage the raw codebook
        row (decode_code, :81-85), out_proj, summed over the stages in order. Runs as two
        launches: vrvq_rvq_gather (codes -> z_p rows) and vrvq_rvq_expand (out_proj + sum, no
        gating). Returns (z_q, z_p, codes[, z_q_is]) like the reference."""
        return self._from_codes(codes, return_z_q_is, None)

    def _from_codes(self, codes, return_z_q_is, mask):
        if not isinstance(codes, torch.Tensor) or codes.dim() != 3:
            raise RuntimeError("from_codes: codes must be a (B, n_codebooks, T) tensor")
        n = codes.shape[1]
        if n > self.n_codebooks:  # the reference indexes self.quantizers[i]: IndexError
            raise IndexError(f"{n} codebooks in codes, the model has {self.n_codebooks}")
        st = self.stacked()
        codes = codes.contiguous()
        zst, z_p = ops.rvq_gather(codes, st.cb)
        want_is = return_z_q_is or mask is not None
        z_q_is, z_q, _ = ops.rvq_expand(zst, st.w_out[:n], st.b_out[:n], None, 1.0,
                                        want_z_q_is=want_is, want_mask=False)
        if mask is not None:
            z_q = ops.masked_sum(z_q_is, mask.contiguous())
        if return_z_q_is:
            return z_q, z_p, codes, z_q_is
        return z_q, z_p, codes

    def from_latents(self, latents: torch.Tensor):
        """Unquantised latents -> (z_q, z_p, codes) (models/quantize.py:251-285): the stages
        whose 8 channels fit in latents.shape[1] each pick the nearest normalised codeword of
        their own slice (decode_latents, no residual chain: vrvq_rvq_nearest), then the raw
        rows (rvq_gather) go through out_proj and are summed (rvq_expand)."""
        if not isinstance(latents, torch.Tensor) or latents.dim() != 3:
            raise RuntimeError("from_latents: latents must be a (B, N*d, T) tensor")
        dims = np.cumsum([0] + [self.quantizers[0].codebook_dim] * self.n_codebooks)
        n = int(np.where(dims <= latents.shape[1])[0].max())
        if n == 0:  # the reference's torch.cat of an empty list
            raise RuntimeError("from_latents: fewer channels than one codebook_dim")
        st = self.stacked()
        lat = latents.contiguous()
        codes = ops.rvq_nearest(lat, st.cbn, st.c2, n)
        zst, z_p = ops.rvq_gather(codes, st.cb, check=False)
        _, z_q, _ = ops.rvq_expand(zst, st.w_out[:n], st.b_out[:n], None, 1.0,
                                   want_z_q_is=False, want_mask=False)
        return z_q, z_p, codes


class VBRResidualVectorQuantize(ResidualVectorQuantize):
    """Variable-bitrate RVQ with importance-map gating (models/quantize.py:288-449)."""

    def __init__(self, *, input_dim: int = 512, n_codebooks: int = 9, codebook_size: int = 1024,
                 codebook_dim: Union[int, list] = 8, quantizer_dropout: float = 0.0,
                 full_codebook_rate: float = 0.5, level_min: float, level_max: float,
                 level_dist: str = "uniform", detach_imp_map_input: bool = False,
                 imp2mask_alpha: float = 1.0):
        super().__init__(input_dim=input_dim, n_codebooks=n_codebooks, codebook_size=codebook_size,
                         codebook_dim=codebook_dim, quantizer_dropout=quantizer_dropout)
        self.full_codebook_rate = full_codebook_rate
        self.level_min = level_min
        self.level_max = level_max
        self.level_dist = level_dist
        self.detach_imp_map_input = detach_imp_map_input
        self.imp2mask_alpha = imp2mask_alpha
        self.imp_subnet = ImportanceSubnet(d_input=input_dim, d_feat=input_dim,
                                           intermediate_channels=[512, 128, 32, 8], out_channels=1,
                                           detach_input=detach_imp_map_input)

    def forward(self, z: torch.Tensor, n_quantizers: int = None, feat_enc: torch.Tensor = None,
                level: float = None, want_z_q_is: bool = True):
        if n_quantizers is None and level is None:
            raise AssertionError("level must be specified in VBR mode")
        if self.training:
            if n_quantizers is not None:  # CBR mode: ones + dropout / full rows (:397-414)
                return train.vbr_cbr_forward(self, z.contiguous(), n_quantizers)
            # random levels / dropout / full-codebook rows, autograd (models/quantize.py:374-414)
            return train.vbr_forward(self, z.contiguous(), feat_enc.contiguous())
        B, D, T = z.shape
        nq = self.n_codebooks
        if n_quantizers is None:
            if level is None:
                raise AssertionError("level must be specified in VBR mode")
            mode = "VBR"
        else:
            mode = "CBR"
            if int(n_quantizers) < nq:
                # The reference stacks n_quantizers z_q_i against an (B, Nq, T) mask of ones at
                # models/quantize.py:421: 2 <= n < Nq is a shape mismatch there,
                # n = 0 fails at torch.stack, and n = 1 broadcasts to z_q = (sum of the Nq mask
                # rows) * z_q_0. All three raise here (n = 1 is a known difference).
                raise RuntimeError(
                    f"VBRResidualVectorQuantize in CBR mode needs n_quantizers >= n_codebooks "
                    f"({n_quantizers} < {nq}), as in the reference")
        st = self.stacked()
        if mode == "VBR":
            imp_map = self.imp_subnet(feat_enc.contiguous())                 # (B, 1, T)
            imp, lvl = imp_map.reshape(B, T), float(level)
        else:
            imp_map, imp, lvl = None, None, 1.0
        # residual chain, z_q_is stream, importance mask, masked z_q
        codes, latents, loss_pf, z_q_is, z_q, mask = _rvq_encode(
            z, st, imp=imp, level=lvl, want_z_q_is=want_z_q_is)
        loss = ops.masked_loss(loss_pf, mask)
        return {
            "z_q": z_q,
            "z_q_is": z_q_is,
            "codes": codes,
            "latents": latents,
            "commitment_loss": loss,
            "codebook_loss": loss.clone(),
            "imp_map": imp_map,
            "mask_imp": mask,
        }

    def from_codes(self, codes: torch.Tensor, return_z_q_is=False, mask_imp=None):
        """VBR codes -> z_q (the reference raises NotImplementedError at
        models/quantize.py:445-446). Every stage's z_q_i as in ResidualVectorQuantize.from_codes;
        with `mask_imp` (B, Nq, T) — the encode dict's mask — z_q is the masked sum of
        scripts/inference.py:99-100, without it the plain sum over the given stages."""
        return self._from_codes(codes, return_z_q_is, mask_imp)

    def from_latents(self, latents: torch.Tensor):
        raise NotImplementedError


# ============================================================================ codec
class CodecMixin:
    """Delay / output-length bookkeeping of models/dac_base.py:61-127."""

    @property
    def padding(self):
        if not hasattr(self, "_padding"):
            self._padding = True
        return self._padding

    @padding.setter
    def padding(self, value):
        """models/dac_base.py:68-84: padding=False zeroes every encoder / decoder conv's padding
        (kept in `original_padding`), True restores it. The importance subnet keeps its "same"
        k3 padding: zeroed, its imp_map would be 12 frames shorter than z and the reference
        fails at the mask product (models/quantize.py:421)."""
        assert isinstance(value, bool)
        for part in (self.encoder, self.decoder):
            for layer in part.modules():
                if not isinstance(layer, (WNConv1d, WNConvTranspose1d)):
                    continue
                if value:
                    if hasattr(layer, "original_padding"):
                        layer.padding = layer.original_padding
                else:
                    if not hasattr(layer, "original_padding") or layer.padding != (0,):
                        layer.original_padding = layer.padding
                    layer.padding = tuple(0 for _ in layer.padding)
            part.valid = not value
        self._padding = value

    def _conv_layers(self):
        return [m for m in self.modules() if isinstance(m, (WNConv1d, WNConvTranspose1d))]

    def compress(self, audio_path_or_signal, win_duration: float = 1.0, verbose: bool = False,
                 normalize_db: float = -16, n_quantizers: int = None, **kw):
        """models/dac_base.py:130-240 (the body after the reference's NotImplementedError at
        :161): chunked encode to a DACFile on the HIP path — vrvq_amd/codec.py."""
        from .codec import compress
        return compress(self, audio_path_or_signal, win_duration, verbose, normalize_db,
                        n_quantizers, **kw)

    def decompress(self, obj, verbose: bool = False, **kw):
        """models/dac_base.py:243-304 (after the reference's raise at :264): DACFile -> audio
        (vrvq_amd/codec.py)."""
        from .codec import decompress
        return decompress(self, obj, verbose, **kw)

    def get_delay(self, layers=None):
        """models/dac_base.py:86-110 over every conv in self.modules() (as the reference), or
        over `layers`."""
        layers = self._conv_layers() if layers is None else layers
        l_out = self.get_output_length(0, layers)
        L = l_out
        for layer in reversed(layers):
            d, k, s = layer.dilation[0], layer.kernel_size[0], layer.stride[0]
            if isinstance(layer, WNConvTranspose1d):
                L = ((L - d * (k - 1) - 1) / s) + 1
            else:
                L = (L - 1) * s + d * (k - 1) + 1
            L = math.ceil(L)
        return (L - l_out) // 2

    def get_output_length(self, input_length, layers=None):
        """models/dac_base.py:112-127."""
        L = input_length
        for layer in (self._conv_layers() if layers is None else layers):
            d, k, s = layer.dilation[0], layer.kernel_size[0], layer.stride[0]
            if isinstance(layer, WNConv1d):
                L = ((L - d * (k - 1) - 1) / s) + 1
            else:
                L = (L - 1) * s + d * (k - 1) + 1
            L = math.floor(L)
        return L

    def codec_layers(self):
        """The convs a chunked window passes through: encoder then decoder. The reference's
        get_delay / get_output_length also walk the quantizer (its importance subnet's six k3
        convs take 12 frames = 6144 samples off the length and 3072 off the delay), which
        would misplace every window of a VBR model; for a CBR model the two lists give the
        same numbers."""
        return [m for part in (self.encoder, self.decoder) for m in part.modules()
                if isinstance(m, (WNConv1d, WNConvTranspose1d))]


class DAC_VRVQ(nn.Module, CodecMixin):
    """Drop-in for models/dac_vrvq.py:83-252 (`DAC_VRVQ`)."""

    def __init__(self, encoder_dim: int = 64, encoder_rates: List[int] = [2, 4, 8, 8],
                 latent_dim: int = None, decoder_dim: int = 1536,
                 decoder_rates: List[int] = [8, 8, 4, 2], n_codebooks: int = 9,
                 codebook_size: Union[int, list] = 1024, codebook_dim: Union[int, list] = 8,
                 quantizer_dropout: float = 0.0, sample_rate: int = 44100,
                 model_type: str = "VBR", full_codebook_rate: float = 0.0,
                 level_min: float = None, level_max: float = None, level_dist: str = "uniform",
                 detach_imp_map_input: bool = False, imp2mask_alpha: float = 1.0):
        super().__init__()
        self.encoder_dim = encoder_dim
        self.encoder_rates = encoder_rates
        self.decoder_dim = decoder_dim
        self.decoder_rates = decoder_rates
        self.sample_rate = sample_rate
        if latent_dim is None:
            latent_dim = encoder_dim * (2 ** len(encoder_rates))
        self.latent_dim = latent_dim
        self.hop_length = int(np.prod(encoder_rates))
        self.encoder = Encoder(encoder_dim, encoder_rates, latent_dim)
        self.n_codebooks = n_codebooks
        self.codebook_size = codebook_size
        self.codebook_dim = codebook_dim
        self.model_type = model_type
        if model_type == "CBR":
            self.quantizer = ResidualVectorQuantize(input_dim=latent_dim, n_codebooks=n_codebooks,
                                                    codebook_size=codebook_size,
                                                    codebook_dim=codebook_dim,
                                                    quantizer_dropout=quantizer_dropout)
        elif model_type == "VBR":
            self.quantizer = VBRResidualVectorQuantize(
                input_dim=latent_dim, n_codebooks=n_codebooks, codebook_size=codebook_size,
                codebook_dim=codebook_dim, quantizer_dropout=quantizer_dropout,
                full_codebook_rate=full_codebook_rate, level_min=level_min, level_max=level_max,
                level_dist=level_dist, detach_imp_map_input=detach_imp_map_input,
                imp2mask_alpha=imp2mask_alpha)
        else:
            raise ValueError(f"Invalid RVQ model_type: {model_type}")
        self.decoder = Decoder(latent_dim, decoder_dim, decoder_rates)
        self.delay = self.get_delay()

    @property
    def device(self):
        return next(self.parameters()).device

    def preprocess(self, audio_data, sample_rate):
        """Right-pad to a multiple of hop_length (models/dac_vrvq.py:164-173)."""
        if sample_rate is None:
            sample_rate = self.sample_rate
        assert sample_rate == self.sample_rate
        length = audio_data.shape[-1]
        right_pad = math.ceil(length / self.hop_length) * self.hop_length - length
        return nn.functional.pad(audio_data, (0, right_pad))

    def encode(self, audio_data: torch.Tensor, n_quantizers: int = None, level: int = 1,
               want_z_q_is: bool = True):
        """models/dac_vrvq.py:176-213. Returns the quantizer's output dict.

        `want_z_q_is=False` skips materialising the (B, Nq, D, T) per-codebook tensor when the
        caller does not need it (it is ~90 % of the quantizer's HBM traffic); the default keeps
        the reference's dict."""
        ev = not self.training and not self.encoder.valid
        # the projection epilogue computes the stages the quantizer runs: all of them, or a CBR
        # prefix (n_quantizers < Nq; a VBR model raises for one in its quantizer)
        proj = RVQ_PROJ and ev
        if proj:
            st = self.quantizer.stacked()
            nq = self.n_codebooks if n_quantizers is None else int(n_quantizers)
            if self.model_type == "CBR" and 1 <= nq < self.n_codebooks:
                st = st.prefix(nq)
            z, feat = self.encoder(audio_data.contiguous(), return_feat=True, project=st)
        else:
            z, feat = self.encoder(audio_data.contiguous(), return_feat=True)
        if self.model_type == "CBR":
            return self.quantizer(z, n_quantizers)
        return self.quantizer(z, n_quantizers, feat, level, want_z_q_is=want_z_q_is)

    def decode(self, z: torch.Tensor):
        """models/dac_vrvq.py:215-220."""
        return self.decoder(z.contiguous())

    def forward(self, audio_data: torch.Tensor, sample_rate: int = None, n_quantizers: int = None,
                level: int = 1):
        """models/dac_vrvq.py:222-252."""
        length = audio_data.shape[-1]
        audio_data = self.preprocess(audio_data, sample_rate)
        out = self.encode(audio_data, n_quantizers, level) if self.model_type == "VBR" \
            else self.encode(audio_data, n_quantizers)
        z_q = out["z_q"]
        x = self.decode(z_q)
        return {
            "audio": x[..., :length],
            "z": z_q,
            "codes": out["codes"],
            "latents": out["latents"],
            "vq/commitment_loss": out["commitment_loss"],
            "vq/codebook_loss": out["codebook_loss"],
            "imp_map": out.get("imp_map", None),
            "mask_imp": out.get("mask_imp", None),
        }
