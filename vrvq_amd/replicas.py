"""Data-parallel replica runner for the encode -> RVQ -> decode path (one process per GPU).

Clips are independent in the reference (`scripts/inference.py:88-112` loops over files; every
op in `models/dac_vrvq.py:164-252` is per clip), so the path shards as replicas: each rank owns
its own batch of clips and there is no collective on the data path. The only collectives are
reporting ones: a barrier before and after a timed region and an all_reduce(MAX) of the
per-rank wall time, so the reported time is that of the slowest rank (weak scaling); and one
all_reduce(SUM) of [audio seconds, bits, frames], so the job-wide bits per
frame equals cal_bpf_from_mask (models/utils.py:64-73) over the concatenated batch.

Backend-agnostic: `nccl` (RCCL over xGMI) on the GPU box, `gloo` in the CPU tests
(tests/test_replicas.py, world_size 2).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist


def shard_seed(base: int, rank: int) -> int:
    """Seed of rank `rank`'s synthetic clips: every rank draws a distinct batch."""
    return base + rank


def shard_range(n_items: int, rank: int, world: int) -> range:
    """Contiguous share of `n_items` clips for `rank` (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world or n_items < 0:
        raise ValueError(f"bad shard request: n_items={n_items} rank={rank} world={world}")
    q, r = divmod(n_items, world)
    lo = rank * q + min(rank, r)
    return range(lo, lo + q + (1 if rank < r else 0))


@dataclass
class TimedResult:
    seconds: float          # max over ranks of the timed region
    local_seconds: float    # this rank's own timed region
    steps: int
    world: int
    last: object            # the last step's output (this rank)


def _distributed() -> bool:
    return dist.is_available() and dist.is_initialized()


def max_over_ranks(x: float, device: Optional[torch.device] = None) -> float:
    """all_reduce(MAX) of a per-rank float (identity without a process group)."""
    if not _distributed() or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device: Optional[torch.device] = None):
    """all_reduce(SUM) of a per-rank list of floats in float64 (identity without a group)."""
    vals = [float(v) for v in values]
    if not _distributed() or dist.get_world_size() == 1:
        return vals
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


@dataclass
class RateReport:
    """Job-wide totals of one level of the VBR sweep (scripts/inference.py:110-112)."""
    audio_seconds: float
    bits: float
    frames: float
    frames_per_second: int  # floor(sample_rate / hop_length)

    @property
    def bpf(self) -> float:
        return self.bits / self.frames

    @property
    def kbps(self) -> float:
        return self.bpf * self.frames_per_second / 1000


def job_rate(audio_seconds: float, bits: float, frames: float, frames_per_second: int,
             device: Optional[torch.device] = None) -> RateReport:
    """Per-rank [audio_s, Σ mask·bits, B·T] -> job-wide RateReport (one SUM all-reduce)."""
    a, b, f = sum_over_ranks([audio_seconds, bits, frames], device)
    return RateReport(a, b, f, int(frames_per_second))


def timed_steps(step: Callable[[], object], steps: int, warmup: int,
                sync: Callable[[], None] = lambda: None,
                device: Optional[torch.device] = None,
                on_start: Callable[[], None] = lambda: None,
                on_stop: Callable[[], None] = lambda: None) -> TimedResult:
    """`warmup` untimed steps, then exactly `steps` timed steps bracketed by
    barrier + `sync()` on both sides; returns the max over ranks of the timed region."""
    if steps < 1 or warmup < 0:
        raise ValueError(f"steps must be >= 1 and warmup >= 0 (got {steps}, {warmup})")
    multi = _distributed() and dist.get_world_size() > 1
    world = dist.get_world_size() if _distributed() else 1
    for _ in range(warmup):
        step()
    sync()
    if multi:
        dist.barrier()
    sync()
    on_start()
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    sync()
    if multi:
        dist.barrier()
    t1 = time.perf_counter()
    on_stop()
    local = t1 - t0
    return TimedResult(seconds=max_over_ranks(local, device), local_seconds=local, steps=steps,
                       world=world, last=out)


def throughput(units_per_rank_step: float, res: TimedResult) -> float:
    """Whole-job rate: the units every rank processed over the slowest rank's time."""
    return units_per_rank_step * res.steps * res.world / res.seconds
