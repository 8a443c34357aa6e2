"""The VRVQ training step (scripts/train.py:117-229 `load`, :262-335 `train_loop`) on MI355X.

Generator: vrvq_amd.DAC_VRVQ in train mode — every op forward and backward in the HIP kernels
(vrvq_amd/train.py). Discriminator and losses: PyTorch-ROCm (vrvq_amd/discriminator.py,
vrvq_amd/losses.py; parity unpinned). Optimisers: torch AdamW + ExponentialLR with the
reference's settings (conf/base.yml: lr 1e-4, betas (0.8, 0.99), gamma 0.999996), grad-norm
clipping 10 (discriminator) / 1e3 (generator).

Data parallel: one process per GPU, `torch.distributed` over RCCL ("nccl" backend) — the
generator and discriminator wrapped in DistributedDataParallel, whose bucketed gradient
all-reduce over xGMI overlaps the backward pass (scripts/train.py:181-182 accel.prepare_model).
Each rank trains on its own shard of the global batch (global_batch / world_size clips).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP

from .discriminator import Discriminator
from .losses import GANLoss, L1Loss, MelSpectrogramLoss, MultiScaleSTFTLoss
from .model import DAC_VRVQ

# conf/vrvq/vrvq_a2.yml lambdas
LAMBDAS_A2 = {"mel/loss": 15.0, "adv/feat_loss": 2.0, "adv/gen_loss": 1.0,
              "vq/commitment_loss": 0.25, "vq/codebook_loss": 1.0, "vq/rate_loss": 2.0}


@dataclass
class State:
    """scripts/train.py:117-135."""
    generator: torch.nn.Module
    optimizer_g: torch.optim.Optimizer
    scheduler_g: torch.optim.lr_scheduler.LRScheduler
    discriminator: torch.nn.Module
    optimizer_d: torch.optim.Optimizer
    scheduler_d: torch.optim.lr_scheduler.LRScheduler
    stft_loss: MultiScaleSTFTLoss
    mel_loss: MelSpectrogramLoss
    gan_loss: GANLoss
    waveform_loss: L1Loss


def unwrap(m: torch.nn.Module) -> torch.nn.Module:
    return m.module if isinstance(m, DDP) else m


def build_state(generator: DAC_VRVQ, device: torch.device, ddp: bool = False,
                discriminator: Optional[Discriminator] = None, lr: float = 1e-4,
                betas=(0.8, 0.99), gamma: float = 0.999996,
                mel_kwargs: Optional[dict] = None) -> State:
    """scripts/train.py:138-229 without checkpoint resume / datasets."""
    gen = generator.to(device)
    disc = (discriminator or Discriminator()).to(device)
    if ddp:
        ids = [device.index] if device.type == "cuda" else None
        gen = DDP(gen, device_ids=ids)
        disc = DDP(disc, device_ids=ids)
    opt_g = torch.optim.AdamW(gen.parameters(), lr=lr, betas=betas)
    opt_d = torch.optim.AdamW(disc.parameters(), lr=lr, betas=betas)
    return State(generator=gen, optimizer_g=opt_g,
                 scheduler_g=torch.optim.lr_scheduler.ExponentialLR(opt_g, gamma),
                 discriminator=disc, optimizer_d=opt_d,
                 scheduler_d=torch.optim.lr_scheduler.ExponentialLR(opt_d, gamma),
                 stft_loss=MultiScaleSTFTLoss(), mel_loss=MelSpectrogramLoss(**(mel_kwargs or {})),
                 gan_loss=GANLoss(disc), waveform_loss=L1Loss())


LOSS_KEYS = ("adv/disc_loss", "stft/loss", "mel/loss", "waveform/loss", "adv/gen_loss",
             "adv/feat_loss", "vq/commitment_loss", "vq/codebook_loss")
RATE_KEYS = ("vq/rate_loss", "vq/rate_loss_scaled")


def check_lambdas(lambdas: Dict[str, float], has_rate: bool = True) -> None:
    """scripts/train.py:319 sums `v * output[k]` over every lambda key, so a key with no loss
    term is a KeyError there; raised here before any work. The rate terms exist only for a
    generator with an importance subnet (has_rate): on a CBR model they are KeyErrors too."""
    known = set(LOSS_KEYS) | (set(RATE_KEYS) if has_rate else set())
    missing = [k for k in lambdas if k not in known]
    if missing:
        raise KeyError(f"train_step: lambda keys with no loss term: {missing}")


def train_step(state: State, audio: torch.Tensor, lambdas: Dict[str, float] = LAMBDAS_A2,
               sample_rate: int = 44100) -> Dict[str, torch.Tensor]:
    """One iteration of scripts/train.py:262-335 on a (B, 1, T) batch already on the device:
    generator forward (train mode), discriminator update, generator losses + update. Returns the
    loss / norm tensors (device tensors: no host sync here)."""
    gen, disc = state.generator, state.discriminator
    check_lambdas(lambdas, hasattr(unwrap(gen).quantizer, "imp_subnet"))
    gen.train()
    disc.train()
    n_codebooks = unwrap(gen).n_codebooks
    out: Dict[str, torch.Tensor] = {}
    g = gen(audio, sample_rate)
    recons = g["audio"]
    imp_map = g["imp_map"]

    out["adv/disc_loss"] = state.gan_loss.discriminator_loss(recons, audio)
    state.optimizer_d.zero_grad(set_to_none=True)
    out["adv/disc_loss"].backward()
    out["other/grad_norm_d"] = torch.nn.utils.clip_grad_norm_(disc.parameters(), 10.0)
    state.optimizer_d.step()
    state.scheduler_d.step()

    out["stft/loss"] = state.stft_loss(recons, audio)
    out["mel/loss"] = state.mel_loss(recons, audio)
    out["waveform/loss"] = state.waveform_loss(recons, audio)
    out["adv/gen_loss"], out["adv/feat_loss"] = state.gan_loss.generator_loss(recons, audio)
    out["vq/commitment_loss"] = g["vq/commitment_loss"]
    out["vq/codebook_loss"] = g["vq/codebook_loss"]
    if imp_map is not None:
        out["vq/rate_loss"] = imp_map.mean()
        out["vq/rate_loss_scaled"] = out["vq/rate_loss"] * n_codebooks
    out["loss"] = sum(v * out[k] for k, v in lambdas.items())

    state.optimizer_g.zero_grad(set_to_none=True)
    out["loss"].backward()
    out["other/grad_norm_g"] = torch.nn.utils.clip_grad_norm_(gen.parameters(), 1e3)
    state.optimizer_g.step()
    state.scheduler_g.step()
    return out


def shard(global_batch: int, rank: int, world: int) -> range:
    """Clips of the global batch that `rank` trains on (equal shards; the remainder goes to the
    first ranks)."""
    base, rem = divmod(global_batch, world)
    lo = rank * base + min(rank, rem)
    return range(lo, lo + base + (1 if rank < rem else 0))


def reduce_metrics(out: Dict[str, torch.Tensor]) -> Dict[str, float]:
    """Mean of every scalar over the ranks (one all-reduce of a packed vector)."""
    keys = sorted(k for k, v in out.items() if torch.is_tensor(v) and v.numel() == 1)
    vec = torch.stack([out[k].detach().float().reshape(()) for k in keys])
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)
        vec = vec / dist.get_world_size()
    return dict(zip(keys, vec.tolist()))


def clip_length(seconds: float, sample_rate: int = 44100) -> int:
    """Samples of an AudioDataset excerpt (conf/dataset.yml train duration 0.38 s)."""
    return int(math.floor(seconds * sample_rate))
