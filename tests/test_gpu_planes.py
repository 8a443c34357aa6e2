"""The bf16 "planes" hand-over between a producing epilogue and the k7 planes tile
(include/vrvq.h vrvq_conv1d_ex, csrc/conv_pl.h). Needs an MI355X.

Bar: the planes hold exactly the split the x3 staging makes of the same fp32 snake values, and
the planes tile runs the register-staged pair tile's MFMA sequence, so every output is BIT-
identical to the fp32 hand-over -- layer by layer and over the whole chained encoder / decoder
(the reference fixtures pin that path in test_gpu_parity.py)."""
import numpy as np
import pytest
import torch

import vrvq_amd
from conftest import rel_err
from vrvq_amd import layers, ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _unplanes(p):
    """planes (B, 3, C/8, T, 8) int16 -> the fp32 values h + m + l (B, C, T)."""
    u = p.to(torch.int32) & 0xFFFF
    f = (u << 16).view(torch.float32)  # bf16 -> fp32 bit pattern
    v = f[:, 0].double() + f[:, 1].double() + f[:, 2].double()
    B, C8, T, _ = v.shape
    return v.permute(0, 1, 3, 2).reshape(B, C8 * 8, T)


def _layer(cin, cout, k, dil, seed):
    gen = torch.Generator().manual_seed(seed)
    conv = layers.WNConv1d(cin, cout, kernel_size=k, dilation=dil, padding=(k - 1) * dil // 2)
    sn_in, sn_out = layers.Snake1d(cin), layers.Snake1d(cout)
    with torch.no_grad():
        conv.bias.copy_(torch.randn(cout, generator=gen) * 0.1)
        sn_in.alpha.copy_(torch.rand(1, cin, 1, generator=gen) + 0.5)
        sn_out.alpha.copy_(torch.rand(1, cout, 1, generator=gen) + 0.5)
    return conv.to(DEV), sn_in.to(DEV), sn_out.to(DEV), gen


@pytest.mark.parametrize("B,C,T,dil", [(2, 192, 1000, 1), (1, 256, 700, 3), (2, 384, 640, 9),
                                       (1, 768, 87, 9), (3, 128, 2000, 3), (1, 512, 256, 1),
                                       (1, 192, 5000, 9)])
def test_planes_epilogue_and_k7_tile_bit_identical(B, C, T, dil):
    """A k1 + skip producer writing snake(y) as planes (== the split of its fp32 snake(y)), and
    the k7 planes tile consuming them (== the pair tile on fp32 snake(y)): y, snake2(h) equal."""
    k1, sn_a, sn_b, gen = _layer(C, C, 1, 1, B * C + T)
    k7, _, sn_h, _ = _layer(C, C, 7, dil, C + dil)
    x = torch.randn(B, C, T, generator=gen).to(DEV)
    res = torch.randn(B, C, T, generator=gen).to(DEV)
    y32, ys32 = k1(x, snake=sn_a, residual=res, out_snake=sn_b, want_raw=True)
    y_p, ysp = k1(x, snake=sn_a, residual=res, out_snake=sn_b, want_raw=True, ys_planes=True)
    torch.cuda.synchronize()
    assert ysp.dtype == torch.int16 and ysp.shape == (B, 3, C // 8, T, 8)
    assert torch.equal(y_p, y32)
    assert torch.equal(_unplanes(ysp).float(), ys32)  # h + m + l is the fp32 value, exactly
    # the k7 consumer: planes input vs fp32 snake(x) input. From T = 640 the fp32 input runs
    # the pair tile too (the model's C >= 192 layers all have T >= 696): bit-identical; below,
    # another tile's K order: within fp32 rounding
    _, h32 = k7(ys32, out_snake=sn_h, want_raw=False)
    _, h_p = k7(ysp, out_snake=sn_h, want_raw=False)
    torch.cuda.synchronize()
    if T >= 640:
        assert torch.equal(h_p, h32)
    else:
        assert rel_err(h_p.cpu().numpy(), h32.cpu().numpy()) < 1e-5
    # and a planes-in, planes-out chain step
    y_pp, h_pp = k7(ysp, out_snake=sn_h, want_raw=True, ys_planes=True)
    torch.cuda.synchronize()
    assert torch.equal(_unplanes(h_pp).float(), h_p)


@pytest.mark.parametrize("cin,cout,s,T", [(1536, 768, 8, 87), (768, 384, 8, 100), (384, 192, 4, 333)])
def test_convtranspose_planes_epilogue(cin, cout, s, T):
    """The ConvTranspose epilogue's planes (the decoder blocks' first residual unit input)."""
    gen = torch.Generator().manual_seed(cin + T)
    ct = layers.WNConvTranspose1d(cin, cout, kernel_size=2 * s, stride=s, padding=(s + 1) // 2)
    sn_in, sn_out = layers.Snake1d(cin), layers.Snake1d(cout)
    with torch.no_grad():
        ct.bias.copy_(torch.randn(cout, generator=gen) * 0.1)
        sn_out.alpha.copy_(torch.rand(1, cout, 1, generator=gen) + 0.5)
    ct, sn_in, sn_out = ct.to(DEV), sn_in.to(DEV), sn_out.to(DEV)
    x = torch.randn(2, cin, T, generator=gen).to(DEV)
    y32, ys32 = ct(x, snake=sn_in, out_snake=sn_out, want_raw=True)
    y_p, ysp = ct(x, snake=sn_in, out_snake=sn_out, want_raw=True, ys_planes=True)
    torch.cuda.synchronize()
    assert torch.equal(y_p, y32)
    assert torch.equal(_unplanes(ysp).float(), ys32)


def test_planes_input_shape_errors():
    conv, _, sn, _ = _layer(64, 96, 7, 1, 3)  # cout 96: not a planes-tile shape
    p = torch.zeros(1, 3, 8, 100, 8, dtype=torch.int16, device=DEV)
    with pytest.raises(RuntimeError):
        conv(p, out_snake=sn, want_raw=True)


def test_chained_model_planes_bit_identical(manifest):
    """The whole chained encoder + decoder (every C >= 192 residual unit's k7 on the planes
    tile, its producers writing planes) against VRVQ_CONV_PLANES=0: every output bit-identical."""
    from test_gpu_parity import model_for, t
    from conftest import load_golden
    g = load_golden("golden_nq8")
    model = model_for(manifest, "golden_nq8")
    x = t(g["audio_in"])
    prev = layers.PLANES
    try:
        with torch.no_grad():
            layers.PLANES = True
            a = model(x, 44100, None, 1)
            layers.PLANES = False
            b = model(x, 44100, None, 1)
    finally:
        layers.PLANES = prev
    torch.cuda.synchronize()
    for k in ("audio", "z", "codes", "latents", "imp_map", "mask_imp"):
        assert torch.equal(a[k], b[k]), k
