"""NN primitives of the VRVQ codec with the reference's parameter layout, run on gfx950 kernels.

Mirrors models/layers.py (reference): Snake1d (:35-41), WNConv1d (:17-18),
WNConvTranspose1d (:21-22), ResidualUnit (:52-68), EncoderBlock (:71-89),
DecoderBlock (:92-110). Parameters keep the reference's names and shapes
(`weight_g`, `weight_v`, `bias`, `alpha`) so a reference `state_dict` loads with
`strict=True`; the modules' forward passes go through the fused HIP kernels in `ops`
(Snake is fused into the following convolution, the residual add into the k=1 conv's
epilogue). Weight norm is folded once per parameter version, not per forward.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn

from . import ops


def _param_key(*ps):
    return tuple((p.device, p.data_ptr(), p._version) for p in ps)


class Snake1d(nn.Module):
    """Snake activation parameters (models/layers.py:35-41); applied inside the next conv."""

    def __init__(self, channels: int):
        super().__init__()
        self.channels = channels
        self.alpha = nn.Parameter(torch.ones(1, channels, 1))
        self._cache = None

    def prepared(self):
        """(alpha[C], 1/(alpha+1e-9)[C]) on the parameter's device."""
        key = _param_key(self.alpha)
        if self._cache is None or self._cache[0] != key:
            a = self.alpha.detach().reshape(-1).contiguous()
            self._cache = (key, a, ops.snake_inv_alpha(a))
        return self._cache[1], self._cache[2]

    def forward(self, x):  # standalone use (not on the fused path)
        raise RuntimeError("Snake1d is fused into the following convolution in vrvq_amd; "
                           "call the owning block instead")


def _wn_init(weight_v: torch.Tensor, fan_in: int, out_dim0: int):
    # PyTorch default Conv init (kaiming_uniform a=sqrt(5) -> U(-1/sqrt(fan_in), +)),
    # then weight_norm's g = ||v||: the effective init of the reference (its
    # trunc_normal_ init_weights is discarded by the weight_norm pre-hook).
    bound = 1.0 / math.sqrt(fan_in)
    with torch.no_grad():
        weight_v.uniform_(-bound, bound)
        g = weight_v.reshape(out_dim0, -1).norm(dim=1)
    return g


class WNConv1d(nn.Module):
    """Weight-normalised Conv1d (models/layers.py:17-18), fused Snake prologue."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1,
                 padding: int = 0, dilation: int = 1):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = (kernel_size,)
        self.stride = (stride,)
        self.padding = (padding,)
        self.dilation = (dilation,)
        # Registration order bias, weight_g, weight_v = the reference's state_dict order
        # (torch weight_norm re-registers g and v after the conv's bias).
        self.bias = nn.Parameter(torch.zeros(out_channels))  # init_weights zeroes conv biases
        v = torch.empty(out_channels, in_channels, kernel_size)
        g = _wn_init(v, in_channels * kernel_size, out_channels)
        self.weight_g = nn.Parameter(g.reshape(out_channels, 1, 1).clone())
        self.weight_v = nn.Parameter(v)
        self._cache = None
        self._cache_x3 = None

    def folded_weight(self) -> torch.Tensor:
        """w = v * (g / ||v||) in the reference layout (Cout, Cin, k)."""
        return ops.weight_norm(self.weight_g.detach().contiguous(), self.weight_v.detach().contiguous())

    def prepared(self):
        key = _param_key(self.weight_g, self.weight_v)
        if self._cache is None or self._cache[0] != key:
            wp, cout_pad = ops.pack_conv1d_weight(self.folded_weight())
            self._cache = (key, wp, cout_pad)
        return self._cache[1], self._cache[2]

    def prepared_x3(self):
        """bf16 planes of the packed weight for the x3 MFMA path, or None (fp32-input MFMA
        path): stride-1 k in {1, 3, 7} with >= 8 input channels, and the strided encoder convs
        (k = 2s, s a power of two) as a stride-1 k = 2 conv over the phase-split view of x,
        whose weight is W'[co][c*s + r][j] = W[co][c][j*s + r] (include/vrvq.h vrvq_conv1d)."""
        k, s = self.kernel_size[0], self.stride[0]
        if not ops.X3 or self.in_channels < 8:
            return None
        strided = (s > 1 and k == 2 * s and s & (s - 1) == 0 and ops.X3_STRIDED)
        if not ((s == 1 and k in ops.X3_TAPS) or strided):
            return None
        key = _param_key(self.weight_g, self.weight_v)
        if self._cache_x3 is None or self._cache_x3[0] != key:
            if strided:
                self._cache_x3 = (key, ops.pack_x3_strided_weight(self.folded_weight(), s))
            else:
                wp, _ = self.prepared()
                self._cache_x3 = (key, ops.pack_x3_weight(wp, k))
        return self._cache_x3[1]

    def forward(self, x: torch.Tensor, snake: Optional[Snake1d] = None,
                residual: Optional[torch.Tensor] = None, epilogue: int = ops.EPI_NONE,
                out_snake: Optional[Snake1d] = None, want_raw: bool = True):
        """conv(snake(x)) (+ residual, epilogue). With out_snake (the consumer's Snake1d)
        returns (y or None, out_snake(y)) computed in the same epilogue."""
        wp, cout_pad = self.prepared()
        alpha = inv = None
        if snake is not None:
            alpha, inv = snake.prepared()
        return ops.conv1d(x, wp, self.out_channels, cout_pad, self.kernel_size[0],
                          self.stride[0], self.padding[0], self.dilation[0],
                          bias=self.bias.detach(), alpha=alpha, inv_alpha=inv,
                          residual=residual, epilogue=epilogue,
                          out_snake=None if out_snake is None else out_snake.prepared(),
                          want_raw=want_raw, w_x3=self.prepared_x3())

    def forward_proj(self, x: torch.Tensor, w3in: torch.Tensor, nq: int,
                     snake: Optional[Snake1d] = None, want_z: bool = False):
        """conv(snake(x)) + bias (stride 1, 1024 outputs) with the in_proj of nq RVQ stages in
        the epilogue (include/vrvq.h vrvq_conv1d_proj): returns (part, z or None), part the
        (8, B*T, 8 nq) channel-split projection partials rvq_encode_part takes."""
        if self.stride[0] != 1:
            raise RuntimeError("forward_proj: stride-1 convs only")
        wp, _ = self.prepared()
        alpha = inv = None
        if snake is not None:
            alpha, inv = snake.prepared()
        return ops.conv1d_proj(x, wp, self.out_channels, self.kernel_size[0], w3in, nq,
                               self.padding[0], self.dilation[0], bias=self.bias.detach(),
                               alpha=alpha, inv_alpha=inv, w_x3=self.prepared_x3(),
                               want_z=want_z)


class WNConvTranspose1d(nn.Module):
    """Weight-normalised ConvTranspose1d (models/layers.py:21-22); norm over dim 0 = Cin."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1,
                 padding: int = 0):
        super().__init__()
        if kernel_size != 2 * stride or padding != math.ceil(stride / 2):
            raise ValueError("WNConvTranspose1d: only the DecoderBlock geometry "
                             "(kernel 2*stride, padding ceil(stride/2)) is implemented")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = (kernel_size,)
        self.stride = (stride,)
        self.padding = (padding,)
        self.dilation = (1,)
        self.bias = nn.Parameter(torch.zeros(out_channels))
        v = torch.empty(in_channels, out_channels, kernel_size)
        g = _wn_init(v, out_channels * kernel_size, in_channels)
        self.weight_g = nn.Parameter(g.reshape(in_channels, 1, 1).clone())
        self.weight_v = nn.Parameter(v)
        self._cache = None
        self._cache_x3 = None

    def folded_weight(self) -> torch.Tensor:
        return ops.weight_norm(self.weight_g.detach().contiguous(), self.weight_v.detach().contiguous())

    def prepared(self):
        key = _param_key(self.weight_g, self.weight_v)
        if self._cache is None or self._cache[0] != key:
            wp, cout_pad = ops.pack_convt1d_weight(self.folded_weight(), self.stride[0])
            self._cache = (key, wp, cout_pad)
        return self._cache[1], self._cache[2]

    def prepared_x3(self):
        """bf16 planes of the polyphase weight (2 taps) for the x3 MFMA path, or None."""
        if not (ops.X3 and self.in_channels >= 8):
            return None
        wp, _ = self.prepared()
        key = _param_key(self.weight_g, self.weight_v)
        if self._cache_x3 is None or self._cache_x3[0] != key:
            self._cache_x3 = (key, ops.pack_x3_weight(wp, 2))
        return self._cache_x3[1]

    def forward(self, x: torch.Tensor, snake: Optional[Snake1d] = None,
                out_snake: Optional[Snake1d] = None, want_raw: bool = True):
        wp, cout_pad = self.prepared()
        alpha = inv = None
        if snake is not None:
            alpha, inv = snake.prepared()
        return ops.conv_transpose1d(x, wp, self.out_channels, cout_pad, self.stride[0],
                                    bias=self.bias.detach(), alpha=alpha, inv_alpha=inv,
                                    out_snake=None if out_snake is None else out_snake.prepared(),
                                    want_raw=want_raw, pad=self.padding[0],
                                    w_x3=self.prepared_x3())


class ResidualUnit(nn.Module):
    """x + conv1(snake(conv7_dil(snake(x))))  (models/layers.py:52-68)."""

    fused = True  # class-level switch (tests / A-B timing): single-launch form where supported

    def __init__(self, dim: int = 16, dilation: int = 1):
        super().__init__()
        pad = ((7 - 1) * dilation) // 2
        self.block = nn.Sequential(
            Snake1d(dim),
            WNConv1d(dim, dim, kernel_size=7, dilation=dilation, padding=pad),
            Snake1d(dim),
            WNConv1d(dim, dim, kernel_size=1),
        )

    def forward(self, x):
        y = self.block[1](x, snake=self.block[0])
        # centre crop of the skip (:65-67): only with padding=False (the chunked codec), where
        # the k7 conv runs unpadded; with "same" padding it never triggers.
        pad = (x.shape[-1] - y.shape[-1]) // 2
        if pad > 0:
            x = x[..., pad:-pad].contiguous()
        return self.block[3](y, snake=self.block[2], residual=x)

    def runs_fused(self) -> bool:
        C = self.block[1].in_channels
        return self.fused and C in ops.RU_FUSED_CHANNELS and not (C == 256 and ops.X3 and
                                                                 ops.RU256_SPLIT)

    def run(self, x: torch.Tensor, x_snk: torch.Tensor, out_snake: Snake1d, want_raw: bool):
        """Chained form: x_snk = block[0](x) was produced by the previous layer's epilogue.
        For C in ops.RU_FUSED_CHANNELS one launch (vrvq_residual_unit: block[2](h) stays in
        LDS); otherwise the k7 conv writes only block[2](h) (h has no other consumer) and the
        k1 conv adds the skip. Either way the output is (y if want_raw, out_snake(y)) (bit for
        bit the same where both forms run the k7 with the same K chunking; the two-launch k7 on
        the 64 x 256 pair tiles -- M >= 128, T >= 640 -- sums in another order). The default
        fused set is C = 64 / 96 / 128 (and C = 256 without the x3 weights): C = 192 runs as two
        launches since the 192-row x3 k1 tiles (+2.8 % end to end,
        profiles/r04z_ru_fusion_ab.txt)."""
        # C = 256 with the x3 weights: the two launches (k7 on the x3 path at 128-row tiles,
        # then k1 + skip) beat the fused kernel, whose 256-row x3 weight stage does not fit
        # twice per CU and therefore keeps the fp32 MFMA (profiles/r02zi_bench_ab.txt)
        if self.runs_fused():
            w7, cp7 = self.block[1].prepared()
            w1, cp1 = self.block[3].prepared()
            a2, ia2 = self.block[2].prepared()
            return ops.residual_unit(x, x_snk, self.block[1].dilation[0], w7,
                                     self.block[1].bias.detach(), a2, ia2, w1,
                                     self.block[3].bias.detach(), cp7,
                                     out_snake=out_snake.prepared(), want_raw=want_raw,
                                     w7_x3=self.block[1].prepared_x3(),
                                     w1_x3=self.block[3].prepared_x3())
        return self.run_two_launch(x, x_snk, out_snake, want_raw)

    def run_two_launch(self, x, x_snk, out_snake: Snake1d, want_raw: bool):
        _, h_snk = self.block[1](x_snk, out_snake=self.block[2], want_raw=False)
        return self.block[3](h_snk, residual=x, out_snake=out_snake, want_raw=want_raw)


class EncoderBlock(nn.Module):
    """3 residual units (dil 1, 3, 9), Snake, strided conv k=2s (models/layers.py:71-89)."""

    def __init__(self, dim: int = 16, stride: int = 1):
        super().__init__()
        self.block = nn.Sequential(
            ResidualUnit(dim // 2, dilation=1),
            ResidualUnit(dim // 2, dilation=3),
            ResidualUnit(dim // 2, dilation=9),
            Snake1d(dim // 2),
            WNConv1d(dim // 2, dim, kernel_size=2 * stride, stride=stride,
                     padding=math.ceil(stride / 2)),
        )

    def forward(self, x):
        for i in range(3):
            x = self.block[i](x)
        return self.block[4](x, snake=self.block[3])

    def entry_snake(self) -> Snake1d:
        return self.block[0].block[0]

    def run(self, x: torch.Tensor, x_snk: torch.Tensor, out_snake: Optional[Snake1d],
            want_raw: bool):
        """Chained form (see ResidualUnit.run); returns what block[4] returns."""
        for i in range(3):
            nxt = self.block[i + 1].block[0] if i < 2 else self.block[3]
            x, x_snk = self.block[i].run(x, x_snk, nxt, want_raw=i < 2)
        return self.block[4](x_snk, out_snake=out_snake, want_raw=want_raw)


class DecoderBlock(nn.Module):
    """Snake, ConvTranspose k=2s (x s upsampling), 3 residual units (models/layers.py:92-110)."""

    def __init__(self, input_dim: int = 16, output_dim: int = 8, stride: int = 1):
        super().__init__()
        self.block = nn.Sequential(
            Snake1d(input_dim),
            WNConvTranspose1d(input_dim, output_dim, kernel_size=2 * stride, stride=stride,
                              padding=math.ceil(stride / 2)),
            ResidualUnit(output_dim, dilation=1),
            ResidualUnit(output_dim, dilation=3),
            ResidualUnit(output_dim, dilation=9),
        )

    def forward(self, x):
        x = self.block[1](x, snake=self.block[0])
        for i in range(2, 5):
            x = self.block[i](x)
        return x

    def entry_snake(self) -> Snake1d:
        return self.block[0]

    def run(self, x_snk: torch.Tensor, out_snake: Snake1d, want_raw: bool = False):
        """Chained form: x_snk = block[0](x) from the previous epilogue; returns
        (y or None, out_snake(y))."""
        x, x_snk = self.block[1](x_snk, out_snake=self.block[2].block[0], want_raw=True)
        for i in range(2, 5):
            last = i == 4
            nxt = out_snake if last else self.block[i + 1].block[0]
            x, x_snk = self.block[i].run(x, x_snk, nxt, want_raw=want_raw if last else True)
        return x, x_snk
