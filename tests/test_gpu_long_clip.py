"""The reference inference driver's own shape (scripts/inference.py:58-70, 88-112): ONE 10-s clip
(L = 441,000 samples, T = 862 frames: the frame-major fused RVQ with 54 chain parts per clip),
encoded once and swept over the driver's 12 levels. Needs an MI355X.

Bars (TOL = 1e-4 relative for floats, as in test_gpu_parity.py): codes bit-exact, imp_map / latents /
z_q_is / z_q / audio within TOL of the numpy oracle; per level, the hard mask bit-exact and bpf
equal to the formula on the oracle's mask; recon within TOL at the two ends of the sweep."""
import numpy as np
import pytest
import torch

import vrvq_amd
from conftest import rel_err
from vrvq_amd.recipe import load_recipe, recipe_state_dict, synthetic_audio

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-4
L10 = 441000
LEVELS12 = (0.2, 0.3, 0.4, 0.5, 0.6, 0.8, 1, 1.2, 1.5, 2, 2.5, 3)  # inference.py:69
_run = {}


def _long(manifest):
    if "r" in _run:
        return _run["r"]
    from oracle.vrvq_oracle import Oracle
    kw = manifest["golden_nq8"]["kwargs"]
    model = vrvq_amd.DAC_VRVQ(**kw)
    load_recipe(model, 0)
    model = model.to(DEV).eval()
    audio = synthetic_audio(1, L10, seed=10)
    x = torch.from_numpy(audio).to(DEV)
    with torch.no_grad():
        out = model(x, 44100, None, 1)
        sweep = vrvq_amd.level_sweep(model, x, LEVELS12, max_decode_clips=4)
    torch.cuda.synchronize()
    sd = recipe_state_dict({k: tuple(v.shape) for k, v in model.state_dict().items()}, 0)
    o = Oracle(sd, **kw)
    ref = o.forward(audio, None, 1.0)
    _run["r"] = (model, out, sweep, o, ref)
    return _run["r"]


def test_ten_second_clip_vs_oracle(manifest):
    _model, out, _sweep, _o, ref = _long(manifest)
    assert out["codes"].shape == (1, 8, 862) and out["audio"].shape == (1, 1, L10)
    codes = out["codes"].cpu().numpy()
    bad = np.argwhere(codes != ref["codes"])
    assert bad.size == 0, f"codes differ at (clip, stage, frame) {bad[:8].tolist()}"
    np.testing.assert_array_equal(out["mask_imp"].cpu().numpy(), ref["mask_imp"])
    for k, rk in (("imp_map", "imp_map"), ("latents", "latents"), ("z", "z_q"),
                  ("audio", "audio")):
        assert rel_err(out[k].cpu().numpy(), ref[rk]) < TOL, k


def test_ten_second_clip_twelve_level_sweep(manifest):
    from oracle.vrvq_oracle import cal_bpf_from_mask as bpf_np, generate_mask_hard as mask_np
    from oracle.vrvq_oracle import masked_sum as msum_np
    model, _out, sweep, o, ref = _long(manifest)
    nq = model.n_codebooks
    assert [r["level"] for r in sweep] == list(LEVELS12)
    for r in sweep:
        lv = float(r["level"])
        m_ref = mask_np((ref["imp_map"] * np.float32(lv * nq)).astype(np.float32), nq)
        mask = r["mask"].cpu().numpy()
        np.testing.assert_array_equal(mask, m_ref)
        assert r["bpf"] == pytest.approx(bpf_np(m_ref, [10] * nq), rel=1e-6)
        assert r["kbps"] == pytest.approx(r["bpf"] * 86 / 1000, rel=1e-12)
        assert rel_err(r["z_q"].cpu().numpy(), msum_np(ref["z_q_is"], m_ref)) < TOL
    for r in (sweep[0], sweep[-1]):  # the sweep's two ends through the oracle decoder
        m_ref = mask_np((ref["imp_map"] * np.float32(float(r["level"]) * nq)).astype(np.float32),
                        nq)
        y = o.decoder(msum_np(ref["z_q_is"], m_ref))
        assert rel_err(r["recon"].cpu().numpy(), y) < TOL
