"""Chunked compress / decompress (reference models/dac_base.py:130-304).

The reference raises NotImplementedError before its compress / decompress bodies run (:161,
:264), so there are no reference outputs: parity is against a CPU restatement of that body
(`_ref_compress` / `_ref_decompress` below over oracle/torch_ref.py in padding=False mode) —
parity unpinned w.r.t. the reference itself. Codes and masks bit-exact, audio <= 1e-4 rel."""
import math

import numpy as np
import pytest
import torch

import vrvq_amd
from conftest import rel_err
from oracle.torch_ref import TorchRef
from vrvq_amd.codec import AudioSignal, ensure_max_of_audio, loudness, normalize
from vrvq_amd.recipe import load_recipe, recipe_state_dict, shapes_of

SR = 44100
KW = dict(encoder_dim=64, encoder_rates=[2, 4, 8, 8], decoder_dim=1536,
          decoder_rates=[8, 8, 4, 2], n_codebooks=8, codebook_size=1024, codebook_dim=8,
          quantizer_dropout=1.0, sample_rate=SR)


def _signal(n, seed, nch=1):
    g = np.random.default_rng(seed)
    t = np.arange(n) / SR
    x = 0.3 * np.sin(2 * np.pi * 220 * t) + 0.05 * g.standard_normal((nch, n))
    return torch.tensor(x, dtype=torch.float32)[None]


# ------------------------------------------------------------------------------ CPU
def test_loudness_kat():
    """BS.1770 / EBU Tech 3341 case 1: a stereo 997 Hz sine at -23 dBFS reads -23 LUFS (+-0.1);
    mono is 3.01 dB lower; silence floors at -70; normalize reaches its target."""
    t = np.arange(3 * SR) / SR
    a = 10 ** (-23 / 20)
    x = torch.tensor(a * np.sin(2 * np.pi * 997 * t), dtype=torch.float32)[None, None]
    assert abs(float(loudness(x.repeat(1, 2, 1), SR)) + 23.0) < 0.1
    assert abs(float(loudness(x, SR)) + 26.01) < 0.1
    assert float(loudness(torch.zeros(2, 1, 5000), SR)[1]) == -70.0
    y = normalize(_signal(2 * SR, 1), SR, -16.0)
    assert abs(float(loudness(y, SR)) + 16.0) < 1e-3
    z = ensure_max_of_audio(torch.tensor([[[0.5, -3.0, 1.5]]]))
    assert torch.allclose(z, torch.tensor([[[0.5 / 3, -1.0, 0.5]]]))


def test_padding_setter_and_window_lengths():
    """padding=False zeroes every encoder / decoder conv padding and restores it; the
    unpadded CPU restatement's encoder / decoder lengths agree with get_output_length."""
    model = vrvq_amd.DAC_VRVQ(**KW)
    pads = [(n, l.padding) for n, l in model.named_modules() if hasattr(l, "original_padding")
            or type(l).__name__ in ("WNConv1d", "WNConvTranspose1d")]
    model.padding = False
    assert model.encoder.valid and model.decoder.valid
    for n, l in model.encoder.named_modules():
        if type(l).__name__ in ("WNConv1d", "WNConvTranspose1d"):
            assert l.padding == (0,), n
    assert model.quantizer.imp_subnet.in_block[1].padding == (1,)
    model.padding = True
    assert [(n, l.padding) for n, l in model.named_modules() if type(l).__name__ in
            ("WNConv1d", "WNConvTranspose1d")] == [(n, p) for n, p in pads]
    tr = TorchRef(recipe_state_dict(shapes_of(model.state_dict()), 0), **KW)
    tr.valid = True
    n = int(math.ceil(SR / 512) * 512)
    z, feat = tr.encoder(torch.zeros(1, 1, n))
    y = tr.decoder(z)
    assert y.shape[-1] == model.get_output_length(n, model.codec_layers())
    assert z.shape[-1] == feat.shape[-1]
    # the reference's own numbers (all modules) stay the drop-in's
    assert model.delay == model.get_delay() and model.get_output_length(n) == y.shape[-1] - 6144


def test_unpadded_window_length_is_hop():
    """Each unpadded window decodes to exactly `hop` samples, so the decoded windows tile the
    signal without gaps or overlaps (models/dac_base.py:204-208 with :278-284)."""
    model = vrvq_amd.DAC_VRVQ(**KW)
    tr = TorchRef(recipe_state_dict(shapes_of(model.state_dict()), 0), **KW)
    layers = model.codec_layers()
    tr.valid = True
    for n in (87 * 512, 100 * 512):
        with torch.no_grad():
            y = tr.decoder(tr.encoder(torch.zeros(1, 1, n))[0])
        assert y.shape[-1] == model.get_output_length(n, layers)
    assert model.get_delay(layers) == 7904 and model.delay == 10976


def test_wav_roundtrip(tmp_path):
    x = _signal(4000, 3, nch=2).clamp(-1, 1)
    p = AudioSignal(x, SR).save(tmp_path / "a.wav")
    s = AudioSignal.load(p)
    assert s.sample_rate == SR and s.audio_data.shape == x.shape
    assert float((s.audio_data - x).abs().max()) < 1.0 / 32767 + 1e-6


def test_decompress_rejects_out_of_range_codes():
    """A code >= codebook_size is the VBR mask marker only for a VBR quantizer (== size); a CBR
    model, a larger code or a negative one is a corrupt container: ValueError naming the code,
    raised before any decode."""
    from vrvq_amd.codes_io import DACFile
    codes = torch.zeros(1, 8, 10, dtype=torch.long)
    codes[0, 3, 4] = 1024

    def dac(c):
        return DACFile(codes=c, chunk_length=10, original_length=5120,
                       input_db=np.array([-20.0], np.float32), channels=1, sample_rate=SR,
                       padding=True, dac_version="1.0.0")
    cbr = vrvq_amd.DAC_VRVQ(**{**KW, "model_type": "CBR"})
    with pytest.raises(ValueError, match="VBR mask marker"):
        cbr.decompress(dac(codes))
    vbr = vrvq_amd.DAC_VRVQ(**KW)
    for v in (1025, -1):
        c = codes.clone()
        c[0, 3, 4] = v
        with pytest.raises(ValueError, match=f"code {v} is out of range"):
            vbr.decompress(dac(c))


# ------------------------------------------------------------------------------ restatement
def _ref_compress(tr: TorchRef, model, audio, win_duration, level=1.0, normalize_db=-16.0):
    """models/dac_base.py:162-240 on the CPU restatement (VBR masks carried as codebook_size)."""
    nb, nac, nt = audio.shape
    x = normalize(audio, SR, normalize_db)
    x = ensure_max_of_audio(x).reshape(nb * nac, 1, nt)
    if nt / SR <= win_duration:
        tr.valid, n_samples, hop = False, nt, nt
    else:
        tr.valid = True
        layers = model.codec_layers()
        d = model.get_delay(layers)
        x = torch.nn.functional.pad(x, (d, d))
        n_samples = int(math.ceil(int(win_duration * SR) / 512) * 512)
        hop = model.get_output_length(n_samples, layers)
    codes = []
    for i in range(0, nt, hop):
        c = x[..., i:i + n_samples]
        c = torch.nn.functional.pad(c, (0, n_samples - c.shape[-1]))
        c = torch.nn.functional.pad(c, (0, int(math.ceil(c.shape[-1] / 512) * 512) - c.shape[-1]))
        z, feat = tr.encoder(c)
        q = tr.quantize(z, feat, level)
        codes.append(q["codes"].masked_fill(q["mask_imp"] == 0, model.codebook_size))
    tr.valid = False
    return torch.cat(codes, -1), n_samples


def _ref_decompress(tr: TorchRef, model, codes, chunk_length, valid, input_db, n_orig):
    tr.valid = valid
    out = []
    for i in range(0, codes.shape[-1], chunk_length):
        c = codes[..., i:i + chunk_length]
        mask = (c < model.codebook_size)
        z = 0
        for s in range(c.shape[1]):
            pre = f"quantizer.quantizers.{s}"
            idx = torch.where(mask[:, s], c[:, s], torch.zeros_like(c[:, s]))
            zq = torch.nn.functional.embedding(idx, tr.p[pre + ".codebook.weight"]).transpose(1, 2)
            z = z + tr.conv(zq, pre + ".out_proj") * mask[:, s, None, :].float()
        out.append(tr.decoder(z))
    tr.valid = False
    r = torch.cat(out, -1)
    r = normalize(r, SR, torch.as_tensor(input_db).reshape(-1))
    return r[..., :n_orig]


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("seconds,win", [(2.6, 1.0), (0.7, 1.0)])
def test_compress_decompress_vs_restatement(tmp_path, seconds, win):
    dev = torch.device("cuda:0")
    model = vrvq_amd.DAC_VRVQ(**KW)
    load_recipe(model, 0)
    model = model.to(dev).eval()
    tr = TorchRef(recipe_state_dict(shapes_of(model.state_dict()), 0), **KW)
    audio = _signal(int(seconds * SR), 7)
    dac = model.compress(audio, win_duration=win, max_batch=2)
    ref_codes, _ = _ref_compress(tr, model, audio, win)
    assert dac.padding == (seconds <= win)
    assert model.padding is True and not model.encoder.valid  # restored
    np.testing.assert_array_equal(dac.codes.numpy(), ref_codes.numpy())
    assert int((dac.codes == model.codebook_size).sum()) > 0  # VBR masks reached the container
    assert abs(float(dac.input_db[0]) - float(loudness(audio, SR)[0])) < 1e-6
    path = dac.save(tmp_path / "x")
    sig = model.decompress(path)
    assert sig.audio_data.shape == audio.shape
    ref = _ref_decompress(tr, model, ref_codes, dac.chunk_length, not dac.padding,
                          dac.input_db, audio.shape[-1])
    assert rel_err(sig.audio_data.cpu().numpy(), ref.numpy()) < 1e-4
