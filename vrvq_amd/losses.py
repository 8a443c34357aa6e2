"""Generator / discriminator losses of the training step (reference models/loss.py:19-447) on
PyTorch-ROCm, over plain (B, 1, T) waveform tensors instead of audiotools AudioSignals.

Parity unpinned (audiotools and librosa are absent here): the STFT follows
audiotools' AudioSignal.stft conventions (discriminator.stft) and the mel filterbank is a
restatement of librosa.filters.mel (Slaney mel scale, Slaney area normalisation), which is what
audiotools' mel_spectrogram calls.
"""
from __future__ import annotations

import functools
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .discriminator import stft


# ------------------------------------------------------------------ mel filterbank
def _hz_to_mel(f):
    """Slaney mel scale: linear below 1 kHz, logarithmic above (librosa htk=False)."""
    f = np.asarray(f, np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep,
                    mels)


def _mel_to_hz(m):
    m = np.asarray(m, np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


@functools.lru_cache(maxsize=64)
def mel_filters(sr: int, n_fft: int, n_mels: int, fmin: float = 0.0,
                fmax: Optional[float] = None) -> np.ndarray:
    """Triangular mel filters (n_mels, 1 + n_fft // 2), area-normalised (librosa norm='slaney')."""
    fmax = sr / 2.0 if fmax is None else float(fmax)
    fft_f = np.linspace(0.0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft_f[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0.0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


def mel_spectrogram(x, sr: int, n_mels: int, window_length: int, hop_length: int,
                    fmin: float = 0.0, fmax: Optional[float] = None):
    """|STFT| projected on the mel filters: (B, C, T) -> (B, C, n_mels, frames)."""
    mag = stft(x, window_length, hop_length).abs()
    fb = torch.from_numpy(mel_filters(sr, 2 * (mag.shape[2] - 1), n_mels, fmin, fmax)).to(mag)
    return torch.einsum("mf,bcft->bcmt", fb, mag)


# ------------------------------------------------------------------ losses
class L1Loss(nn.Module):
    """models/loss.py:19-56 on waveforms."""

    def __init__(self, weight: float = 1.0):
        super().__init__()
        self.weight = weight

    def forward(self, x, y):
        return F.l1_loss(x, y)


class MultiScaleSTFTLoss(nn.Module):
    """models/loss.py:168-254: L1 of log10(|X|^pow clamped) (+ mag_weight * L1 of |X|) per
    window length (hop = window / 4)."""

    def __init__(self, window_lengths: Sequence[int] = (2048, 512), clamp_eps: float = 1e-5,
                 mag_weight: float = 1.0, log_weight: float = 1.0, pow: float = 2.0,
                 weight: float = 1.0):
        super().__init__()
        self.window_lengths = list(window_lengths)
        self.clamp_eps, self.mag_weight, self.log_weight = clamp_eps, mag_weight, log_weight
        self.pow, self.weight = pow, weight

    def forward(self, x, y):
        loss = 0.0
        for w in self.window_lengths:
            xm = stft(x, w, w // 4).abs()
            ym = stft(y, w, w // 4).abs()
            loss = loss + self.log_weight * F.l1_loss(
                xm.clamp(self.clamp_eps).pow(self.pow).log10(),
                ym.clamp(self.clamp_eps).pow(self.pow).log10())
            loss = loss + self.mag_weight * F.l1_loss(xm, ym)
        return loss


class MelSpectrogramLoss(nn.Module):
    """models/loss.py:257-401 (levels=None branch); defaults are conf/base.yml's
    (7 scales, n_mels 5..320, windows 32..2048, pow 1, mag_weight 0)."""

    def __init__(self, n_mels: Sequence[int] = (5, 10, 20, 40, 80, 160, 320),
                 window_lengths: Sequence[int] = (32, 64, 128, 256, 512, 1024, 2048),
                 clamp_eps: float = 1e-5, mag_weight: float = 0.0, log_weight: float = 1.0,
                 pow: float = 1.0, weight: float = 1.0, mel_fmin: Sequence[float] = None,
                 mel_fmax: Sequence[Optional[float]] = None, sample_rate: int = 44100):
        super().__init__()
        self.n_mels = list(n_mels)
        self.window_lengths = list(window_lengths)
        self.mel_fmin = list(mel_fmin) if mel_fmin is not None else [0.0] * len(self.n_mels)
        self.mel_fmax = list(mel_fmax) if mel_fmax is not None else [None] * len(self.n_mels)
        self.clamp_eps, self.mag_weight, self.log_weight = clamp_eps, mag_weight, log_weight
        self.pow, self.weight, self.sample_rate = pow, weight, sample_rate

    def forward(self, x, y):
        loss = 0.0
        for n, w, lo, hi in zip(self.n_mels, self.window_lengths, self.mel_fmin, self.mel_fmax):
            xm = mel_spectrogram(x, self.sample_rate, n, w, w // 4, lo, hi)
            ym = mel_spectrogram(y, self.sample_rate, n, w, w // 4, lo, hi)
            loss = loss + self.log_weight * F.l1_loss(
                xm.clamp(self.clamp_eps).pow(self.pow).log10(),
                ym.clamp(self.clamp_eps).pow(self.pow).log10())
            if self.mag_weight:
                loss = loss + self.mag_weight * F.l1_loss(xm, ym)
        return loss


class GANLoss(nn.Module):
    """Least-squares GAN + feature matching (models/loss.py:404-447)."""

    def __init__(self, discriminator: nn.Module):
        super().__init__()
        self.discriminator = discriminator

    def forward(self, fake, real):
        return self.discriminator(fake), self.discriminator(real)

    def discriminator_loss(self, fake, real):
        d_fake, d_real = self.forward(fake.clone().detach(), real)
        loss = 0.0
        for f, r in zip(d_fake, d_real):
            loss = loss + torch.mean(f[-1] ** 2) + torch.mean((1 - r[-1]) ** 2)
        return loss

    def generator_loss(self, fake, real):
        d_fake, d_real = self.forward(fake, real)
        loss_g = 0.0
        for f in d_fake:
            loss_g = loss_g + torch.mean((1 - f[-1]) ** 2)
        loss_feat = 0.0
        for f, r in zip(d_fake, d_real):
            for a, b in zip(f[:-1], r[:-1]):
                loss_feat = loss_feat + F.l1_loss(a, b.detach())
        return loss_g, loss_feat
