"""Multi-period / multi-scale / multi-resolution discriminator of the training step
(reference models/discriminator.py:30-220, the DAC discriminator) on PyTorch-ROCm.

SURVEY.md §8f row 1 keeps the discriminator and the losses on PyTorch (rocBLAS / MIOpen
convolutions): they are not on the codec's hot path, and their reference depends on audiotools
(absent here), so their parity is unpinned. The parameter tree (and state_dict keys) follows
the reference — `discriminators.<i>.convs.<j>.0.weight_g` etc. — so reference checkpoints load.
"""
from __future__ import annotations

import math
import os
from typing import List, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.utils import weight_norm

BANDS = [(0.0, 0.1), (0.1, 0.25), (0.25, 0.5), (0.5, 0.75), (0.75, 1.0)]


def _wn(conv: nn.Module, act: bool):
    """weight_norm'd conv, followed by LeakyReLU(0.1) when act (models/discriminator.py:14-27)."""
    conv = weight_norm(conv)
    return nn.Sequential(conv, nn.LeakyReLU(0.1)) if act else conv


def _run(layers, x, fmap: list):
    for layer in layers:
        x = layer(x)
        fmap.append(x)
    return x


# (cin, cout, kernel, stride, padding) of each MPD 2-D conv (over (frames, period) planes)
_MPD_LAYERS = [(1, 32, 3), (32, 128, 3), (128, 512, 3), (512, 1024, 3), (1024, 1024, 1)]


# The period discriminators' (k, 1) Conv2d run as Conv1d over the folded batch (B * period, C,
# frames): the same sums per output element (each column is an independent 1-D signal); the
# feature maps are then laid out (B * period, C, frames), which every use of them (means and
# elementwise L1 between real and fake, losses.GANLoss) is invariant to. VRVQ_MPD_1D=0: the
# reference's Conv2d over (B, C, frames, period).
MPD_1D = os.environ.get("VRVQ_MPD_1D", "1") != "0"
# ... and as plain GEMMs (hipBLASLt fp32) over a channels-last (B * period, frames, C) layout:
# the k-tap windows of the strided conv gathered once (unfold), no layout transposes between
# layers (VRVQ_MPD_GEMM=0: F.conv1d, MIOpen).
MPD_GEMM = os.environ.get("VRVQ_MPD_GEMM", "1") != "0"


def _conv1d_cl(h: torch.Tensor, w: torch.Tensor, bias, stride: int, pad: int) -> torch.Tensor:
    """Conv1d on channels-last h (N, L, C) with w (Cout, C, k): (N, Lout, Cout), the k windows
    of stride `stride` flattened (tap, channel) against w laid out (Cout, k, C)."""
    n, _, c = h.shape
    cout, _, k = w.shape
    hp = F.pad(h, (0, 0, pad, pad))
    win = hp.unfold(1, k, stride)                      # (N, Lout, C, k) view
    lout = win.shape[1]
    cols = win.transpose(2, 3).reshape(n * lout, k * c)  # (tap, channel) per row: one copy
    wm = w.permute(0, 2, 1).reshape(cout, k * c)
    y = torch.addmm(bias, cols, wm.t()) if bias is not None else cols @ wm.t()
    return y.reshape(n, lout, cout)


class MPD(nn.Module):
    """Period discriminator: the waveform folded into `period` columns (:30-65)."""

    def __init__(self, period: int):
        super().__init__()
        self.period = period
        self.convs = nn.ModuleList([_wn(nn.Conv2d(ci, co, (5, 1), (s, 1), padding=(2, 0)), True)
                                    for ci, co, s in _MPD_LAYERS])
        self.conv_post = _wn(nn.Conv2d(1024, 1, (3, 1), padding=(1, 0)), False)

    def to_reference_layout(self, fmap: torch.Tensor, batch: int) -> torch.Tensor:
        """One map of forward() in the reference's (B, C, frames, period) layout (a view where
        the folded layouts allow; the values are unchanged)."""
        if fmap.dim() == 4:  # already the Conv2d form (VRVQ_MPD_1D=0)
            return fmap
        p = self.period
        if MPD_GEMM:  # (B * p, frames, C)
            return fmap.reshape(batch, p, fmap.shape[1], fmap.shape[2]).permute(0, 3, 2, 1)
        return fmap.reshape(batch, p, fmap.shape[1], fmap.shape[2]).permute(0, 2, 3, 1)

    def forward(self, x):
        t = x.shape[-1]
        x = F.pad(x, (0, self.period - t % self.period), mode="reflect")
        b, c, n = x.shape
        x = x.reshape(b, c, n // self.period, self.period)
        fmap: list = []
        if MPD_1D:
            # (B, C, frames, period) -> (B * period, C, frames) or channels-last (.., frames, C)
            h = x.permute(0, 3, 1, 2).reshape(b * self.period, c, n // self.period)
            if MPD_GEMM:
                h = h.transpose(1, 2)
            for layer in list(self.convs) + [self.conv_post]:
                conv = layer[0] if isinstance(layer, nn.Sequential) else layer
                w = torch._weight_norm(conv.weight_v, conv.weight_g, 0)[..., 0]
                if MPD_GEMM:
                    h = _conv1d_cl(h, w, conv.bias, conv.stride[0], conv.padding[0])
                else:
                    h = F.conv1d(h, w, conv.bias, stride=conv.stride[0], padding=conv.padding[0])
                if layer is not self.conv_post:
                    h = F.leaky_relu(h, 0.1)
                fmap.append(h)
            return fmap
        x = _run(self.convs, x, fmap)
        fmap.append(self.conv_post(x))
        return fmap


# (cin, cout, kernel, stride, groups, padding) of each MSD 1-D conv
_MSD_LAYERS = [(1, 16, 15, 1, 1, 7), (16, 64, 41, 4, 4, 20), (64, 256, 41, 4, 16, 20),
               (256, 1024, 41, 4, 64, 20), (1024, 1024, 41, 4, 256, 20), (1024, 1024, 5, 1, 1, 2)]


class MSD(nn.Module):
    """Scale discriminator on the waveform resampled to sample_rate // rate (:68-98). Only
    rate 1 (no resampling) is supported here; the reference configs use rates = []."""

    def __init__(self, rate: int = 1, sample_rate: int = 44100):
        super().__init__()
        if rate != 1:
            raise NotImplementedError("MSD resampling (rate != 1) needs audiotools' resampler")
        self.convs = nn.ModuleList([
            _wn(nn.Conv1d(ci, co, k, s, groups=g, padding=p), True)
            for ci, co, k, s, g, p in _MSD_LAYERS])
        self.conv_post = _wn(nn.Conv1d(1024, 1, 3, 1, padding=1), False)
        self.sample_rate = sample_rate
        self.rate = rate

    def forward(self, x):
        fmap: list = []
        x = _run(self.convs, x, fmap)
        fmap.append(self.conv_post(x))
        return fmap


def stft(x: torch.Tensor, window_length: int, hop_length: int, match_stride: bool = False,
         padding_type: str = "reflect") -> torch.Tensor:
    """Complex STFT with audiotools' AudioSignal.stft conventions (periodic Hann window,
    center=True; match_stride pads so frames align with the hop and drops 2 frames per side).
    x (B, C, T) -> (B, C, F, frames)."""
    if match_stride:
        if hop_length != window_length // 4:
            raise ValueError("match_stride needs hop_length == window_length // 4")
        n = x.shape[-1]
        right = math.ceil(n / hop_length) * hop_length - n
        pad = (window_length - hop_length) // 2
        x = F.pad(x, (pad, pad + right), mode=padding_type)
    B, C, T = x.shape
    win = torch.hann_window(window_length, device=x.device, dtype=x.dtype)
    s = torch.stft(x.reshape(B * C, T), n_fft=window_length, hop_length=hop_length, window=win,
                   center=True, pad_mode=padding_type, return_complex=True)
    s = s.reshape(B, C, s.shape[-2], s.shape[-1])
    return s[..., 2:-2] if match_stride else s


class MRD(nn.Module):
    """Complex multi-band spectrogram discriminator (:104-175)."""

    def __init__(self, window_length: int, hop_factor: float = 0.25, sample_rate: int = 44100,
                 bands: Sequence[Tuple[float, float]] = BANDS):
        super().__init__()
        self.window_length = window_length
        self.hop_length = int(window_length * hop_factor)
        self.sample_rate = sample_rate
        n_bins = window_length // 2 + 1
        self.bands = [(int(lo * n_bins), int(hi * n_bins)) for lo, hi in bands]
        ch = 32

        def stack():
            spec = [(2, (3, 9), (1, 1), (1, 4)), (ch, (3, 9), (1, 2), (1, 4)),
                    (ch, (3, 9), (1, 2), (1, 4)), (ch, (3, 9), (1, 2), (1, 4)),
                    (ch, (3, 3), (1, 1), (1, 1))]
            return nn.ModuleList([_wn(nn.Conv2d(ci, ch, k, s, padding=p), True)
                                  for ci, k, s, p in spec])

        self.band_convs = nn.ModuleList([stack() for _ in self.bands])
        self.conv_post = _wn(nn.Conv2d(ch, 1, (3, 3), (1, 1), padding=(1, 1)), False)

    def forward(self, x):
        spec = torch.view_as_real(stft(x, self.window_length, self.hop_length, True))
        # (B, 1, F, frames, 2) -> (B, 2, frames, F)
        spec = spec[:, 0].permute(0, 3, 2, 1)
        fmap: list = []
        outs = [_run(layers, spec[..., lo:hi], fmap)
                for (lo, hi), layers in zip(self.bands, self.band_convs)]
        fmap.append(self.conv_post(torch.cat(outs, dim=-1)))
        return fmap


class Discriminator(nn.Module):
    """MPD(periods) + MSD(rates) + MRD(fft_sizes) on peak-normalised, DC-removed audio
    (models/discriminator.py:178-220). forward(x) -> list (per discriminator) of feature maps,
    the last one the logits.

    Feature-map layout: with VRVQ_MPD_1D / VRVQ_MPD_GEMM on (the default) each
    period discriminator's maps are (B * period, frames, C) -- the channels-last folded batch its
    GEMMs run on -- where the reference returns (B, C, frames, period). The values are the same
    and every consumer in the training step (means, elementwise L1 between the real and the fake
    maps: losses.GANLoss) is layout-invariant; a consumer that indexes the maps (hooks, per-layer
    comparisons against reference fixtures) takes MPD.to_reference_layout(map, B) or runs with
    VRVQ_MPD_1D=0 (the reference's Conv2d layout). MSD / MRD maps keep the reference layout."""

    def __init__(self, rates: List[int] = [], periods: List[int] = [2, 3, 5, 7, 11],
                 fft_sizes: List[int] = [2048, 1024, 512], sample_rate: int = 44100,
                 bands: Sequence[Tuple[float, float]] = BANDS):
        super().__init__()
        discs: List[nn.Module] = [MPD(p) for p in periods]
        discs += [MSD(r, sample_rate=sample_rate) for r in rates]
        discs += [MRD(f, sample_rate=sample_rate, bands=bands) for f in fft_sizes]
        self.discriminators = nn.ModuleList(discs)

    @staticmethod
    def preprocess(y):
        y = y - y.mean(dim=-1, keepdim=True)
        return 0.8 * y / (y.abs().max(dim=-1, keepdim=True)[0] + 1e-9)

    def forward(self, x):
        x = self.preprocess(x)
        return [d(x) for d in self.discriminators]
