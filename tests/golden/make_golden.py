#!/usr/bin/env python
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE PyTorch CPU path.

Run in the build container only (the reference is not shipped to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--ref /root/reference]

The reference (lixinghe1999/VRVQ) is imported from its source tree with stub modules for the
three third-party packages that are absent here and that the hot path does not use
arithmetically: `audiotools` (only `ml.BaseModel`, an nn.Module base with a
`device` property, and the `AudioSignal` name), `torchmetrics` (imported, unused on the path)
and nothing else. Weights come from vrvq_amd.recipe (name-seeded PCG64), so the GPU tests can
regenerate identical weights without a checkpoint. Outputs are .npz fixtures (inputs and
expected outputs: data only) plus a JSON manifest.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types
from collections import namedtuple

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vrvq_amd.recipe import recipe_state_dict, shapes_of, synthetic_audio  # noqa: E402

LEVELS = [0.25, 0.5, 1.0, 2.0]
MASK_KAT_S = [0.0, 1.0, 2.0, 7.0, 8.0, -0.5, 3.9999999, 4.5, 27.0, 31.9999]


def install_stubs():
    at = types.ModuleType("audiotools")
    ml = types.ModuleType("audiotools.ml")

    class BaseModel(torch.nn.Module):
        @property
        def device(self):
            return next(self.parameters()).device

    ml.BaseModel = BaseModel
    at.ml = ml
    at.AudioSignal = type("AudioSignal", (), {})
    at.STFTParams = namedtuple("STFTParams", ["window_length", "hop_length", "window_type",
                                              "match_stride", "padding_type"],
                                 defaults=(None, None, None, None, None))
    sys.modules["audiotools"] = at
    sys.modules["audiotools.ml"] = ml
    sys.modules["torchmetrics"] = types.ModuleType("torchmetrics")


def load_ref(ref_root):
    install_stubs()
    sys.path.insert(0, ref_root)
    from models.dac_vrvq import DAC_VRVQ  # noqa: E402
    from models import utils as ref_utils  # noqa: E402
    return DAC_VRVQ, ref_utils


def yml_kwargs(ref_root, rel):
    sys.path.insert(0, REPO)
    from vrvq_amd.config import load_config, model_kwargs
    cwd = os.getcwd()
    os.chdir(ref_root)  # argbind resolves $include relative to the working directory
    try:
        return model_kwargs(load_config(os.path.join(ref_root, rel)))
    finally:
        os.chdir(cwd)


def build(DAC, kw, seed=0):
    torch.manual_seed(0)
    m = DAC(**kw)
    sd = m.state_dict()
    rec = recipe_state_dict(shapes_of(sd), seed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in rec.items()}, strict=True)
    m.eval()
    return m


def top2_gap(z_e_list, quantizers):
    """Min (second - best) distance over frames, per stage (argmin stability diagnostic)."""
    gaps = []
    for ze, q in zip(z_e_list, quantizers):
        enc = torch.nn.functional.normalize(ze.permute(0, 2, 1).reshape(-1, ze.shape[1]))
        cb = torch.nn.functional.normalize(q.codebook.weight)
        dist = enc.pow(2).sum(1, keepdim=True) - 2 * enc @ cb.t() + cb.pow(2).sum(1, keepdim=True).t()
        s = torch.sort(dist, dim=1).values
        gaps.append(float((s[:, 1] - s[:, 0]).min()))
    return gaps


def sweep(model, ref_utils, x_pad, enc, n_q):
    """scripts/inference.py:95-112 without SI-SDR / file output."""
    out = {}
    imp_map = enc["imp_map"]
    for li, level in enumerate(LEVELS):
        level_scaled = level * n_q
        imp_scaled = imp_map * level_scaled
        mask = ref_utils.generate_mask_hard(imp_scaled, nq=n_q)
        z_q = torch.sum(enc["z_q_is"] * mask[:, :, None, :], dim=1, keepdim=False)
        with torch.no_grad():
            recon = model.decode(z_q)
        bpf = ref_utils.cal_bpf_from_mask(mask, bits_per_codebook=[10] * n_q)
        kbps = bpf * np.floor(model.sample_rate / model.hop_length) / 1000
        out[f"sweep{li}_mask"] = mask.numpy()
        out[f"sweep{li}_zq_norm"] = z_q.norm(dim=1).numpy()
        out[f"sweep{li}_recon_s8"] = recon[..., ::8].numpy()
        out[f"sweep{li}_bpf"] = np.float64(bpf)
        out[f"sweep{li}_kbps"] = np.float64(kbps)
        s = imp_scaled.numpy().astype(np.float64)
        out[f"sweep{li}_tie_margin"] = np.float64(np.min(np.abs(s - np.round(s))))
    return out


def model_fixture(DAC, ref_utils, kw, batch, name, manifest, n_quantizers=None, full_z=True):
    model = build(DAC, kw)
    audio = synthetic_audio(batch, 44100, seed=1234)
    x = torch.from_numpy(audio)
    res = {"audio_in": audio}
    with torch.no_grad():
        xp = model.preprocess(x, 44100)
        z, feat = model.encoder(xp, return_feat=True)
        if model.model_type == "VBR":
            enc = model.quantizer(z, n_quantizers, feat, 1)
        else:
            enc = model.quantizer(z, n_quantizers)
        fwd = model(x, 44100, n_quantizers, 1) if model.model_type == "VBR" else model(x, 44100, n_quantizers)
        # per-stage latents for the argmin-gap diagnostic
        nlat = enc["latents"].shape[1] // 8
        ze_list = [enc["latents"][:, 8 * i: 8 * i + 8] for i in range(nlat)]
        gaps = top2_gap(ze_list, model.quantizer.quantizers)
    if full_z:
        res["z"] = z.numpy()
        res["feat"] = feat.numpy()
    res["codes"] = enc["codes"].numpy()
    res["latents"] = enc["latents"].numpy()
    res["z_q"] = enc["z_q"].numpy()
    res["commitment_loss"] = np.float32(enc["commitment_loss"].item())
    res["codebook_loss"] = np.float32(enc["codebook_loss"].item())
    if enc.get("imp_map") is not None:
        res["imp_map"] = enc["imp_map"].numpy()
    if enc.get("mask_imp") is not None:
        res["mask_imp"] = enc["mask_imp"].numpy()
    if enc.get("z_q_is") is not None:
        zqis = enc["z_q_is"]
        res["z_q_is_norm"] = zqis.norm(dim=(2, 3)).numpy()
        res["z_q_is_s16"] = zqis[:, :, ::16, :].numpy()
    res["audio_out"] = fwd["audio"].numpy()
    if model.model_type == "VBR" and n_quantizers is None:
        res.update(sweep(model, ref_utils, xp, enc, model.n_codebooks))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
    imp = enc.get("imp_map")
    manifest[name] = {
        "kwargs": kw, "batch": batch, "length": 44100, "audio_seed": 1234, "weight_seed": 0,
        "n_quantizers": n_quantizers, "delay": int(model.delay),
        "min_top2_gap_per_stage": gaps,
        "imp_range": [float(imp.min()), float(imp.max())] if imp is not None else None,
        "n_params": int(sum(p.numel() for p in model.parameters())),
        "state_dict": {k: list(v.shape) for k, v in model.state_dict().items()},
    }
    print(name, "gap", min(gaps), "imp", manifest[name]["imp_range"], "delay", model.delay)
    return model


def rvq_stress_fixture(DAC, kw, name, manifest, batch=4, frames=50, seed=7):
    """RVQ unit at random latents (many frames): z, feat -> quantizer outputs."""
    model = build(DAC, kw)
    g = torch.Generator().manual_seed(seed)
    z = torch.randn(batch, model.latent_dim, frames, generator=g) * 0.5
    feat = torch.randn(batch, model.latent_dim, frames, generator=g) * 0.5
    with torch.no_grad():
        enc = model.quantizer(z, None, feat, 1)
        nlat = enc["latents"].shape[1] // 8
        gaps = top2_gap([enc["latents"][:, 8 * i: 8 * i + 8] for i in range(nlat)],
                        model.quantizer.quantizers)
    res = {"z": z.numpy(), "feat": feat.numpy(), "codes": enc["codes"].numpy(),
           "latents": enc["latents"].numpy(), "z_q": enc["z_q"].numpy(),
           "imp_map": enc["imp_map"].numpy(), "mask_imp": enc["mask_imp"].numpy(),
           "commitment_loss": np.float32(enc["commitment_loss"].item()),
           "z_q_is_norm": enc["z_q_is"].norm(dim=(2, 3)).numpy()}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
    manifest[name] = {"kwargs": kw, "batch": batch, "frames": frames, "z_seed": seed,
                      "weight_seed": 0, "min_top2_gap_per_stage": gaps,
                      "state_dict": {k: list(v.shape) for k, v in model.state_dict().items()}}
    print(name, "gap", min(gaps))


def from_codes_fixture(DAC, kw, name, manifest, batch=2, frames=40, seed=5, vbr=False):
    """codes -> z_q / z_p / z_q_is / audio. CBR: the reference's own
    ResidualVectorQuantize.from_codes (models/quantize.py:217-249). VBR (whose from_codes raises
    NotImplementedError in the reference): the same per-stage decode_code + out_proj of the
    reference's quantizers and the masked sum of scripts/inference.py:99-100."""
    model = build(DAC, kw)
    q = model.quantizer
    nq, N = len(q.quantizers), q.quantizers[0].codebook_size
    g = torch.Generator().manual_seed(seed)
    codes = torch.randint(0, N, (batch, nq, frames), generator=g, dtype=torch.int64)
    codes[0, :, 0] = 0
    codes[-1, :, -1] = N - 1
    res = {"codes": codes.numpy()}
    with torch.no_grad():
        if not vbr:
            z_q, z_p, _, z_q_is = q.from_codes(codes, return_z_q_is=True)
        else:
            z_p = torch.cat([qi.decode_code(codes[:, i]) for i, qi in enumerate(q.quantizers)], 1)
            z_q_is = torch.stack([qi.out_proj(qi.decode_code(codes[:, i]))
                                  for i, qi in enumerate(q.quantizers)], dim=1)
            s = torch.rand(batch, 1, frames, generator=g) * nq
            mask = torch.stack([(s[:, 0] - i >= 0).float() for i in range(nq)], dim=1)
            z_q = torch.sum(z_q_is * mask[:, :, None, :], dim=1, keepdim=False)
            res["mask"] = mask.numpy()
        audio = model.decode(z_q)
    res.update(z_q=z_q.numpy(), z_p=z_p.numpy(), z_q_is=z_q_is.numpy(), audio=audio.numpy())
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
    manifest[name] = {"kwargs": kw, "batch": batch, "frames": frames, "codes_seed": seed,
                      "weight_seed": 0, "vbr": vbr,
                      "state_dict": {k: list(v.shape) for k, v in model.state_dict().items()}}
    print(name, "nq", nq, "audio", tuple(audio.shape))


def mask_kat(ref_utils, manifest):
    s = torch.tensor(MASK_KAT_S, dtype=torch.float32).reshape(1, 1, -1)
    out = {}
    for nq in (8, 28, 32):
        m = ref_utils.generate_mask_hard(s, nq)
        out[str(nq)] = {"mask": m[0].tolist(), "bpf10": ref_utils.cal_bpf_from_mask(m, [10] * nq)}
    ste = ref_utils.generate_mask_ste(s.clone(), 8, alpha=2.0)
    out["ste8_alpha2"] = ste[0].tolist()
    manifest["mask_kat"] = {"s": [float(v) for v in s.reshape(-1)], "results": out}


def from_latents_fixture(DAC, kw, name, manifest, batch=2, frames=40, seed=21):
    """ResidualVectorQuantize.from_latents (models/quantize.py:251-285) of the reference on
    random latents: all 8 stages, and a 43-channel input (5 whole stages, 3 channels ignored)."""
    model = build(DAC, kw)
    q = model.quantizer
    g = torch.Generator().manual_seed(seed)
    res = {}
    for tag, ch in (("full", 8 * len(q.quantizers)), ("part", 43)):
        lat = torch.randn(batch, ch, frames, generator=g) * 0.7
        with torch.no_grad():
            z_q, z_p, codes = q.from_latents(lat)
        res.update({f"{tag}_latents": lat.numpy(), f"{tag}_z_q": z_q.numpy(),
                    f"{tag}_z_p": z_p.numpy(), f"{tag}_codes": codes.numpy()})
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
    manifest[name] = {"kwargs": kw, "batch": batch, "frames": frames, "latents_seed": seed,
                      "weight_seed": 0,
                      "state_dict": {k: list(v.shape) for k, v in model.state_dict().items()}}
    print(name, "codes", res["full_codes"].shape, res["part_codes"].shape)


def from_codes_all(DAC, ref, manifest):
    from_latents_fixture(DAC, yml_kwargs(ref, "conf/original_dac/cbr.yml"), "golden_from_latents_cbr",
                         manifest)
    from_codes_fixture(DAC, yml_kwargs(ref, "conf/original_dac/cbr.yml"), "golden_from_codes_cbr",
                       manifest)
    from_codes_fixture(DAC, yml_kwargs(ref, "conf/base.yml"), "golden_from_codes_vbr", manifest,
                       seed=6, vbr=True)


def dac_file_fixture(ref_root):
    """A .dac file written by the reference's own DACFile.save (models/dac_base.py:31-47)."""
    from models.dac_base import DACFile
    g = torch.Generator().manual_seed(3)
    codes = torch.randint(0, 1024, (1, 8, 25), generator=g)
    f = DACFile(codes=codes, chunk_length=25, original_length=12345,
                input_db=torch.tensor([-17.25]), channels=1, sample_rate=44100, padding=True,
                dac_version="1.0.0")
    path = f.save(os.path.join(HERE, "ref_written"))
    np.savez(os.path.join(HERE, "ref_written_expect.npz"), codes=codes.numpy())
    print("dac file", path)


TRAIN_SAMPLES = 256   # gradient elements kept per parameter tensor (evenly spaced)
TRAIN_FULL = 4096     # parameter tensors up to this size keep their whole gradient
TRAIN_LAMBDAS = {"waveform": 1.0, "commitment": 0.25, "codebook": 1.0, "rate": 2.0}


def grad_sample_index(numel):
    return np.unique(np.linspace(0, numel - 1, min(numel, TRAIN_SAMPLES)).round().astype(np.int64))


def train_fixture(DAC, kw, name, manifest, batch, seed, length=16758, audio_seed=4321):
    """Generator gradients of one training step (scripts/train.py:262-330) under the reference's
    own autograd: model.train(), the training-mode quantizer (random levels, dropout and
    full-codebook rows drawn from torch's global CPU generator after torch.manual_seed(seed)),
    and a surrogate generator loss with the vrvq_a2 weights of the terms that reach the
    generator without a discriminator:
        L = mean|audio - x| + 0.25 commitment + 1.0 codebook + 2.0 mean(imp_map)
    (plain L1 in place of the audiotools L1Loss; mel/STFT/GAN terms are out of the fixture).
    The components are called in DAC_VRVQ.forward's order (models/dac_vrvq.py:222-252) so the
    intermediate gradients (z_q, z, feat) can be retained."""
    model = build(DAC, kw)
    model.train()
    audio = synthetic_audio(batch, length, seed=audio_seed)
    x = torch.from_numpy(audio)
    nq = model.n_codebooks
    torch.manual_seed(seed)
    draws_levels = torch.rand((batch, 1, 1))
    draws_dropout = torch.randint(1, nq + 1, (batch, 1, 1))
    torch.manual_seed(seed)
    xp = model.preprocess(x, 44100)
    z, feat = model.encoder(xp, return_feat=True)
    z.retain_grad()
    feat.retain_grad()
    enc = model.quantizer(z, None, feat, 1)
    zq = enc["z_q"]
    zq.retain_grad()
    y = model.decode(zq)[..., :length]
    lam = TRAIN_LAMBDAS
    terms = {"waveform": (y - x).abs().mean(), "commitment": enc["commitment_loss"],
             "codebook": enc["codebook_loss"], "rate": enc["imp_map"].mean()}
    loss = sum(lam[k] * v for k, v in terms.items())
    loss.backward()
    res = {"audio_in": audio, "audio_out": y.detach().numpy(), "codes": enc["codes"].numpy(),
           "mask_imp": enc["mask_imp"].detach().numpy(),
           "imp_map": enc["imp_map"].detach().numpy(), "loss": np.float64(loss.item()),
           "draws_levels": draws_levels.numpy(), "draws_dropout": draws_dropout.numpy(),
           "grad_z_q": zq.grad.numpy(), "grad_z": z.grad.numpy(), "grad_feat": feat.grad.numpy()}
    for k, v in terms.items():
        res["term_" + k] = np.float64(v.item())
    norms, params = {}, []
    for pname, p in model.named_parameters():
        g = p.grad.detach().reshape(-1).double()
        norms[pname] = float(g.norm())
        params.append(pname)
        if g.numel() <= TRAIN_FULL:
            res["g_full/" + pname] = g.float().numpy()
        else:
            res["g_s/" + pname] = g[torch.from_numpy(grad_sample_index(g.numel()))].float().numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
    n_full = int(batch * model.quantizer.full_codebook_rate)
    n_drop = int(batch * model.quantizer.quantizer_dropout)
    manifest[name] = {"kwargs": kw, "batch": batch, "length": length, "audio_seed": audio_seed,
                      "weight_seed": 0, "rng_seed": seed, "lambdas": lam,
                      "rows": {"imp": batch - n_full - n_drop, "dropout": n_drop, "full": n_full},
                      "grad_norms": norms, "params": params,
                      "sample_rule": f"linspace(0, numel-1, min(numel, {TRAIN_SAMPLES})) rounded, "
                                     f"unique; tensors <= {TRAIN_FULL} elements kept whole"}
    print(name, "loss", loss.item(), {k: float(v) for k, v in terms.items()},
          "rows", manifest[name]["rows"])


def discriminator_fixture(ref_root, manifest):
    """State-dict layout of the reference Discriminator (models/discriminator.py:178-220) and
    its feature-map shapes for a short input: the training step's discriminator must load
    reference checkpoints."""
    from models.discriminator import Discriminator
    torch.manual_seed(0)
    d = Discriminator()
    x = torch.from_numpy(synthetic_audio(1, 4410, seed=99))
    try:
        with torch.no_grad():
            fm = d(x)
        shapes = [[list(t.shape) for t in f] for f in fm]
    except Exception as e:  # MRD needs audiotools' STFT (stubbed here): keys only
        print("discriminator forward unavailable with stubs:", type(e).__name__)
        shapes = None
    manifest["discriminator"] = {"state_dict": {k: list(v.shape) for k, v in d.state_dict().items()},
                                 "fmap_shapes_4410": shapes}


def train_all(DAC, ref, manifest):
    discriminator_fixture(ref, manifest)
    a2 = yml_kwargs(ref, "conf/vrvq/vrvq_a2.yml")
    train_fixture(DAC, a2, "golden_train_a2", manifest, batch=2, seed=2024)
    # all three row kinds of the training quantizer (importance / dropout / full codebook)
    train_fixture(DAC, dict(a2, quantizer_dropout=0.25), "golden_train_a2_rows", manifest,
                  batch=4, seed=77)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=os.environ.get("VRVQ_REFERENCE", "/root/reference"))
    ap.add_argument("--only", choices=["from_codes", "dac_file", "train"], default=None,
                    help="regenerate only these fixtures and merge them into manifest.json")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    DAC, ref_utils = load_ref(args.ref)
    if args.only == "dac_file":
        dac_file_fixture(args.ref)
        return
    if args.only in ("from_codes", "train"):
        with open(os.path.join(HERE, "manifest.json")) as f:
            manifest = json.load(f)
        (from_codes_all if args.only == "from_codes" else train_all)(DAC, args.ref, manifest)
        with open(os.path.join(HERE, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1, default=float)
        return
    manifest = {"generator": "tests/golden/make_golden.py", "torch": torch.__version__,
                "reference": "lixinghe1999/VRVQ @ 2025-07-25 (/root/reference)",
                "levels": LEVELS}
    base = yml_kwargs(args.ref, "conf/base.yml")
    k24 = yml_kwargs(args.ref, "conf/base_24kbps.yml")
    cbr = yml_kwargs(args.ref, "conf/original_dac/cbr.yml")
    a2 = yml_kwargs(args.ref, "conf/vrvq/vrvq_a2.yml")
    manifest["yml_kwargs"] = {"conf/base.yml": base, "conf/base_24kbps.yml": k24,
                              "conf/original_dac/cbr.yml": cbr, "conf/vrvq/vrvq_a2.yml": a2}
    model_fixture(DAC, ref_utils, base, 2, "golden_nq8", manifest)
    model_fixture(DAC, ref_utils, k24, 1, "golden_nq28", manifest)
    k32 = dict(k24, n_codebooks=32)
    model_fixture(DAC, ref_utils, k32, 1, "golden_nq32", manifest)
    model_fixture(DAC, ref_utils, cbr, 1, "golden_cbr", manifest, full_z=False)
    model_fixture(DAC, ref_utils, cbr, 1, "golden_cbr_n4", manifest, n_quantizers=4, full_z=False)
    rvq_stress_fixture(DAC, base, "golden_rvq_stress_nq8", manifest)
    rvq_stress_fixture(DAC, k32, "golden_rvq_stress_nq32", manifest, batch=2, frames=40, seed=11)
    mask_kat(ref_utils, manifest)
    from_codes_all(DAC, args.ref, manifest)
    train_all(DAC, args.ref, manifest)
    dac_file_fixture(args.ref)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, default=float)


if __name__ == "__main__":
    main()
