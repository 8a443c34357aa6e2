"""Training-step host logic on CPU (no GPU): the PyTorch-ROCm discriminator and losses of
vrvq_amd.trainer (parity unpinned: audiotools / librosa are absent), the batch sharding, and
the data-parallel path — DistributedDataParallel over a world_size-2 `gloo` group standing in
for RCCL — on the discriminator update of train_step (scripts/train.py:286-297)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vrvq_amd.discriminator import Discriminator, stft
from vrvq_amd.losses import GANLoss, MelSpectrogramLoss, MultiScaleSTFTLoss, mel_filters
from vrvq_amd.trainer import reduce_metrics, shard


def test_discriminator_state_dict_matches_reference(manifest):
    ref = manifest["discriminator"]["state_dict"]
    mine = {k: list(v.shape) for k, v in Discriminator().state_dict().items()}
    assert mine == ref


def test_discriminator_forward_shapes():
    torch.manual_seed(0)
    d = Discriminator()
    fm = d(torch.randn(2, 1, 4410) * 0.1)
    assert len(fm) == 8
    assert [len(f) for f in fm] == [6] * 5 + [26] * 3
    for p, f in zip([2, 3, 5, 7, 11], fm[:5]):
        # period discriminators: channels-last over the folded batch (B * period, frames, 1)
        assert f[-1].shape[0] == 2 * p and f[-1].shape[2] == 1
    for f in fm[5:]:
        assert f[-1].shape[0] == 2 and f[-1].shape[1] == 1
    for f in fm:
        assert all(torch.isfinite(t).all() for t in f)


def test_mpd_folded_gemm_matches_conv2d(monkeypatch):
    """The folded channels-last GEMM form of a period discriminator holds the reference's
    Conv2d feature maps (models/discriminator.py:30-65), element for element."""
    import vrvq_amd.discriminator as D

    torch.manual_seed(1)
    mpd = D.MPD(3)
    x = torch.randn(2, 1, 997) * 0.1
    fm = mpd(x)
    monkeypatch.setattr(D, "MPD_1D", False)
    ref = mpd(x)
    assert len(fm) == len(ref) == 6
    for a, r in zip(fm, ref):
        b, c, frames, p = r.shape
        got = a.reshape(b, p, frames, c).permute(0, 3, 2, 1)
        torch.testing.assert_close(got, r, rtol=1e-4, atol=1e-6)
        # the documented converter gives the same view
        assert torch.equal(mpd.to_reference_layout(a, b), got)
        assert mpd.to_reference_layout(r, b) is r


def test_stft_match_stride_frames():
    x = torch.randn(1, 1, 44100)
    s = stft(x, 2048, 512, match_stride=True)
    assert s.shape == (1, 1, 1025, 44100 // 512 + 1)  # ceil(T / hop) frames, aligned to the hop
    s2 = stft(x, 512, 128)
    assert s2.shape == (1, 1, 257, 44100 // 128 + 1)


def test_mel_filters_properties():
    for n_mels, n_fft in ((5, 32), (80, 512), (320, 2048)):
        w = mel_filters(44100, n_fft, n_mels)
        assert w.shape == (n_mels, n_fft // 2 + 1)
        assert (w >= 0).all()
        peaks = w.argmax(1)
        assert (np.diff(peaks) >= 0).all()               # centres increase with the mel index
    # Slaney area normalisation: each triangle integrates to ~1 (in Hz units * 2 / width)
    w = mel_filters(44100, 4096, 40).astype(np.float64)
    df = 44100 / 4096
    area = w.sum(1) * df
    np.testing.assert_allclose(area, 1.0, rtol=0.05)


def test_losses_zero_on_identical_and_positive_otherwise():
    torch.manual_seed(1)
    x = torch.randn(2, 1, 8192) * 0.1
    y = x + torch.randn_like(x) * 0.05
    for loss in (MultiScaleSTFTLoss(), MelSpectrogramLoss()):
        assert float(loss(x, x)) == pytest.approx(0.0, abs=1e-6)
        assert float(loss(x, y)) > 0
    torch.manual_seed(0)
    g = GANLoss(Discriminator())
    lg, lf = g.generator_loss(y, x)
    ld = g.discriminator_loss(y, x)
    assert torch.isfinite(lg) and torch.isfinite(lf) and torch.isfinite(ld)


def test_shard_covers_batch():
    for gb, w in ((256, 8), (10, 3), (5, 8)):
        idx = [i for r in range(w) for i in shard(gb, r, w)]
        assert idx == list(range(gb))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from torch.nn.parallel import DistributedDataParallel as DDP
        torch.manual_seed(0)
        d_local = Discriminator(periods=[2, 3], fft_sizes=[512])
        torch.manual_seed(0)
        d = DDP(Discriminator(periods=[2, 3], fft_sizes=[512]))
        gen = torch.Generator().manual_seed(5)
        real = torch.randn(2 * world, 1, 2048, generator=gen) * 0.1
        fake = torch.randn(2 * world, 1, 2048, generator=gen) * 0.1
        mine = shard(2 * world, rank, world)
        loss = GANLoss(d).discriminator_loss(fake[mine.start:mine.stop], real[mine.start:mine.stop])
        loss.backward()
        # expected: mean over the ranks' shards of the local (non-DDP) gradients
        want = None
        for r in range(world):
            d_local.zero_grad()
            s = shard(2 * world, r, world)
            GANLoss(d_local).discriminator_loss(fake[s.start:s.stop], real[s.start:s.stop]).backward()
            g = [p.grad.clone() for p in d_local.parameters()]
            want = g if want is None else [a + b for a, b in zip(want, g)]
        want = [a / world for a in want]
        err = max(float((p.grad - w).abs().max() / (w.abs().max() + 1e-30))
                  for p, w in zip(d.parameters(), want))
        m = reduce_metrics({"adv/disc_loss": loss.detach(), "x": torch.tensor(float(rank))})
        q.put((rank, err, m["x"]))
    finally:
        dist.destroy_process_group()


def test_ddp_gradient_allreduce_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, xm in res:
        assert err < 1e-5, (rank, err)
        assert xm == pytest.approx(0.5)


def test_a2_kwargs_match_reference_config(manifest):
    from vrvq_amd.config import A2_KWARGS
    assert A2_KWARGS == manifest["yml_kwargs"]["conf/vrvq/vrvq_a2.yml"]


def test_unknown_lambda_key_raises():
    """scripts/train.py:319 sums every lambda key: a misspelt key is a KeyError, raised before
    any work; the VBR rate keys only where the generator has an importance subnet (a CBR model
    has no rate term: a KeyError in the reference too)."""
    from vrvq_amd.trainer import LAMBDAS_A2, check_lambdas
    check_lambdas(LAMBDAS_A2)
    check_lambdas({"mel/loss": 15.0, "vq/rate_loss": 2.0})
    with pytest.raises(KeyError, match="rate_loss"):
        check_lambdas({"mel/loss": 15.0, "vq/rate_loss": 2.0}, has_rate=False)
    with pytest.raises(KeyError, match="mel/los"):
        check_lambdas({**LAMBDAS_A2, "mel/los": 1.0})
