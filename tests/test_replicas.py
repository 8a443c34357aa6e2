"""N>1 path of the replica runner (vrvq_amd/replicas.py) on CPU: world_size-2 `gloo` process
groups stand in for RCCL. Covers what bench.py relies on for `--gpus N`: distinct clip shards per
rank, barrier-bracketed timing with the MAX over ranks, and the whole-job throughput formula."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vrvq_amd.replicas import (job_rate, shard_range, shard_seed, sum_over_ranks, throughput,
                               timed_steps, TimedResult)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import time

        from vrvq_amd.recipe import synthetic_audio
        audio = synthetic_audio(2, 512, seed=shard_seed(1234, rank))
        calls = []

        def step():
            calls.append(1)
            time.sleep(0.02 * (rank + 1))   # rank 1 is the slow one
            return float(audio.sum())

        res = timed_steps(step, steps=3, warmup=2)
        # every rank holds its own shard: gather the clip checksums
        sums = [None] * world
        dist.all_gather_object(sums, res.last)
        # job-wide bpf from per-rank mask sums (SUM all-reduce) == bpf of the concatenated batch
        import numpy as np
        from oracle.vrvq_oracle import cal_bpf_from_mask, generate_mask_hard
        rng = np.random.default_rng(7)
        s_all = (rng.random((2 * world, 1, 11)) * 10).astype(np.float32)
        mine = s_all[2 * rank: 2 * rank + 2]
        mask = generate_mask_hard(mine, 8)
        rep = job_rate(2.0, float((mask * 10).sum()), mask.shape[0] * mask.shape[2], 86)
        want = cal_bpf_from_mask(generate_mask_hard(s_all, 8), [10] * 8)
        tot = sum_over_ranks([rank + 1.0])
        q.put((rank, res.seconds, res.local_seconds, res.world, len(calls), sums,
               rep.bpf, want, rep.audio_seconds, rep.kbps, tot))
    finally:
        dist.destroy_process_group()


def test_timed_steps_two_ranks_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got.sort()
    maxes = {g[1] for g in got}
    assert len(maxes) == 1, "every rank must report the same (max) time"
    t_max = maxes.pop()
    assert t_max == pytest.approx(max(g[2] for g in got))
    assert t_max >= 3 * 0.04                      # the slow rank's 3 timed steps
    for rank, _, _, w, ncalls, sums, bpf, want, audio_s, kbps, tot in got:
        assert w == world and ncalls == 5         # 2 warmup + exactly 3 timed
        assert sums[0] != sums[1]                 # distinct shards per rank
        assert bpf == pytest.approx(want, rel=1e-12)
        assert audio_s == 2.0 * world and kbps == pytest.approx(bpf * 86 / 1000)
        assert tot == [3.0]


def test_shard_range_partitions():
    for n in (0, 1, 7, 32, 33):
        for world in (1, 2, 3, 8):
            parts = [shard_range(n, r, world) for r in range(world)]
            flat = [i for p in parts for i in p]
            assert flat == list(range(n))
            assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def test_single_process_and_throughput():
    res = timed_steps(lambda: 1, steps=4, warmup=0)
    assert res.world == 1 and res.seconds == res.local_seconds and res.last == 1
    r = TimedResult(seconds=2.0, local_seconds=2.0, steps=10, world=8, last=None)
    assert throughput(32.0, r) == pytest.approx(32 * 10 * 8 / 2.0)
    with pytest.raises(ValueError):
        timed_steps(lambda: 1, steps=0, warmup=0)
