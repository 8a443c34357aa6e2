"""Host-side drop-in surface (no GPU): config loading, state_dict layout, delay bookkeeping,
weight recipe, and loud failure off-GPU."""
import os

import numpy as np
import pytest
import torch

import vrvq_amd
from vrvq_amd.config import load_config, model_kwargs
from vrvq_amd.recipe import load_recipe, recipe_state_dict, shapes_of

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.parametrize("rel,nq", [("conf/base.yml", 8), ("conf/base_24kbps.yml", 28),
                                    ("conf/vrvq/vrvq_a2.yml", 28), ("conf/vrvq/vrvq_a2_dt.yml", 8),
                                    ("conf/original_dac/cbr.yml", 8)])
def test_shipped_configs(rel, nq):
    kw = model_kwargs(load_config(os.path.join(REPO, rel)))
    assert kw["n_codebooks"] == nq
    assert kw["encoder_rates"] == [2, 4, 8, 8] and kw["decoder_rates"] == [8, 8, 4, 2]


def test_configs_match_reference(manifest):
    """Our loader on our conf/ files gives the kwargs the generator read from the reference's."""
    for rel, kw_ref in manifest["yml_kwargs"].items():
        kw = model_kwargs(load_config(os.path.join(REPO, rel)))
        assert kw == kw_ref, rel


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree only in the build container")
def test_loader_on_reference_tree(manifest):
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        for rel, kw_ref in manifest["yml_kwargs"].items():
            assert model_kwargs(load_config(os.path.join(REF, rel))) == kw_ref
    finally:
        os.chdir(cwd)


@pytest.mark.parametrize("name", ["golden_nq8", "golden_nq28", "golden_nq32", "golden_cbr"])
def test_state_dict_and_delay(manifest, name):
    m = manifest[name]
    model = vrvq_amd.DAC_VRVQ(**m["kwargs"])
    sd = model.state_dict()
    assert list(sd.keys()) == list(m["state_dict"].keys())
    assert {k: list(v.shape) for k, v in sd.items()} == m["state_dict"]
    assert model.delay == m["delay"]
    assert sum(p.numel() for p in model.parameters()) == m["n_params"]
    assert model.hop_length == 512 and model.latent_dim == 1024


def test_recipe_deterministic_and_strict(manifest):
    shapes = {k: tuple(v) for k, v in manifest["golden_nq8"]["state_dict"].items()}
    a = recipe_state_dict(shapes, 0)
    b = recipe_state_dict(shapes, 0)
    c = recipe_state_dict(shapes, 1)
    k = "decoder.model.1.block.1.weight_v"
    assert np.array_equal(a[k], b[k]) and not np.array_equal(a[k], c[k])
    model = vrvq_amd.DAC_VRVQ(**manifest["golden_nq8"]["kwargs"])
    load_recipe(model, 0)
    assert torch.equal(model.state_dict()[k], torch.from_numpy(a[k]))


def test_reference_checkpoint_roundtrip(manifest, tmp_path):
    """A reference-layout checkpoint {'state_dict': ...} loads strictly (scripts/inference.py:45-46)."""
    kw = manifest["golden_nq8"]["kwargs"]
    src = vrvq_amd.DAC_VRVQ(**kw)
    load_recipe(src, 3)
    p = tmp_path / "weights.pth"
    torch.save({"state_dict": src.state_dict()}, p)
    dst = vrvq_amd.DAC_VRVQ(**kw)
    dst.load_state_dict(torch.load(p, map_location="cpu", weights_only=True)["state_dict"], strict=True)
    for k, v in src.state_dict().items():
        assert torch.equal(v, dst.state_dict()[k])


def test_cpu_tensors_fail_loudly():
    model = vrvq_amd.DAC_VRVQ(n_codebooks=2).eval()
    x = torch.zeros(1, 1, 1024)
    with pytest.raises(RuntimeError, match="GPU"):
        model.encode(model.preprocess(x, 44100))


def test_training_mode_cpu_fails_loudly():
    """Training mode runs the autograd kernels (vrvq_amd/train.py): on CPU tensors they raise
    instead of falling back to a CPU implementation."""
    model = vrvq_amd.DAC_VRVQ(n_codebooks=2, level_min=0.5, level_max=2.0)
    model.train()
    with pytest.raises(RuntimeError, match="GPU"):
        model.quantizer(torch.zeros(1, 1024, 4), None, torch.zeros(1, 1024, 4), 1)
    with pytest.raises(RuntimeError, match="GPU"):  # VBR quantizer in CBR mode, training
        model.quantizer(torch.zeros(1, 1024, 4), 2, torch.zeros(1, 1024, 4), None)
    with pytest.raises(RuntimeError, match="n_quantizers >= n_codebooks"):
        model.quantizer(torch.zeros(1, 1024, 4), 1, torch.zeros(1, 1024, 4), None)


def test_invalid_model_type():
    with pytest.raises(ValueError):
        vrvq_amd.DAC_VRVQ(model_type="XYZ")


def test_preprocess_pads_to_hop():
    model = vrvq_amd.DAC_VRVQ(n_codebooks=2)
    y = model.preprocess(torch.ones(2, 1, 44100), 44100)
    assert y.shape[-1] == 44544 and float(y[..., 44100:].abs().sum()) == 0.0
    with pytest.raises(AssertionError):
        model.preprocess(torch.ones(1, 1, 10), 16000)
