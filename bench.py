#!/usr/bin/env python
"""Throughput bench of the VRVQ hot path on MI355X: audio-sec/s of preprocess -> encode
(Snake/WNConv encoder + RVQ + importance gating) -> decode, batch 32 x 1 s @ 44.1 kHz per GPU
(BASELINE.json configs[1]), synthetic audio resident in HBM, recipe (random-init) weights.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank/GPU)

Multi-GPU: clips shard data-parallel (each rank its own 32 clips, no data-path collective),
weak scaling; the timed region is bracketed by barrier + synchronize and the MAX over ranks is
reported. Rank 0 prints one JSON line, including
  roofline      the single-launch RVQ kernel (vrvq_rvq_fused: residual chain + z_q_is stream +
                importance gating) against HBM, bytes per SURVEY.md §8(d), per-launch
                durations from HIP events recorded on the launch stream inside the timed steps;
  roofline_conv the fp32-MFMA conv stacks against the fp32 matrix peak;
  cpu_baseline  the CPU oracle (numpy, oracle/vrvq_oracle.py) timed on this host on a bounded
                sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense fp32 matrix peak (= vector peak)
CLIP_SAMPLES = 44100
SR = 44100


def rvq_bytes(B: int, T: int, nq: int, D: int = 1024, d: int = 8, N: int = 1024) -> int:
    """Algorithmic HBM bytes of one RVQ launch:
    per frame z read, imp read, z_q_is + z_q writes, codes (int64), latents, mask, loss;
    plus the stage weights (normalised codebook counted once more)."""
    per_frame = D * 4 + 4 + nq * D * 4 + D * 4 + nq * 8 + nq * d * 4 + nq * 4 + nq * 4
    weights = nq * 4 * (d * D + d + 2 * N * d + D * d + D)
    return B * T * per_frame + weights


def rvq_pmc_traffic(kernel: str = "rvq_fused_kernel<4>"):
    """HBM bytes per launch of the RVQ kernel from the newest committed PMC measurement
    (profiles/*_rvq_pmc.json: rocprofv3 FETCH_SIZE + WRITE_SIZE, separate passes, made by
    tools/gpu/pmc_rvq.sh at this workload). bench.py cannot collect PMC counters itself (they
    need their own rocprofv3 passes), so it reports that measurement and names its file."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_rvq_pmc.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    k = d.get("kernels", {}).get(kernel)
    return (int(k["total"]) if k else None), os.path.relpath(files[-1], REPO)


def conv_flops(model, B: int, L: int) -> float:
    """Algorithmic conv FLOPs of one encode+decode (2 * MACs over every conv layer), counted
    from the layer geometry: the implicit GEMM's M x N x K per layer."""
    from vrvq_amd.layers import WNConv1d, WNConvTranspose1d

    flops = 0.0
    T = L
    # walk encoder / imp subnet / decoder in execution order with their time lengths
    def conv_len(T, m):
        k, s, p, d = m.kernel_size[0], m.stride[0], m.padding[0], m.dilation[0]
        return (T + 2 * p - d * (k - 1) - 1) // s + 1

    def acc_conv(m, Tin):
        nonlocal flops
        Tout = conv_len(Tin, m)
        flops += 2.0 * B * m.out_channels * Tout * m.in_channels * m.kernel_size[0]
        return Tout

    enc = model.encoder.block
    T = acc_conv(enc[0], T)
    for i in range(1, len(enc) - 2):
        blk = enc[i].block
        for r in range(3):
            acc_conv(blk[r].block[1], T)
            acc_conv(blk[r].block[3], T)
        T = acc_conv(blk[4], T)
    T = acc_conv(enc[len(enc) - 1], T)
    Tz = T
    if hasattr(model.quantizer, "imp_subnet"):
        sub = model.quantizer.imp_subnet
        acc_conv(sub.in_block[1], Tz)
        for b in sub.blocks:
            acc_conv(b[1], Tz)
    dec = model.decoder.model
    T = acc_conv(dec[0], Tz)
    for i in range(1, len(dec) - 3):
        blk = dec[i].block
        ct = blk[1]
        flops += 2.0 * B * ct.in_channels * ct.out_channels * T * ct.kernel_size[0]
        T = T * ct.stride[0]
        for r in range(2, 5):
            acc_conv(blk[r].block[1], T)
            acc_conv(blk[r].block[3], T)
    acc_conv(dec[len(dec) - 2], T)
    return flops


class RvqTimer:
    """HIP-event timing of the RVQ launch (vrvq_rvq_fused), recorded on the stream it runs
    on."""

    KERNELS = ("encode",)

    def __init__(self):
        self.events = []
        self.enabled = False

    def mark(self, tag):
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream())
            self.events.append((tag, e))

    def durations_ms(self):
        torch.cuda.synchronize()
        out = {k: [] for k in self.KERNELS}
        ev = self.events
        for (t0, e0), (t1, e1) in zip(ev, ev[1:]):
            for k in self.KERNELS:
                if t0 == k + "_begin" and t1 == k + "_end":
                    out[k].append(e0.elapsed_time(e1))
        return out


def install_rvq_timer(timer: RvqTimer):
    from vrvq_amd import ops

    def wrap(name):
        orig = getattr(ops, "rvq_" + name)

        def f(*a, **k):
            timer.mark(name + "_begin")
            r = orig(*a, **k)
            timer.mark(name + "_end")
            return r
        setattr(ops, "rvq_" + name, f)

    for k in RvqTimer.KERNELS:
        wrap(k)


def cpu_baseline(kwargs, clips: int):
    """The numpy CPU oracle on a bounded sample (same model/weights, `clips` x 1 s)."""
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        threads = os.cpu_count() or 1
    from oracle.vrvq_oracle import Oracle
    from vrvq_amd.recipe import recipe_state_dict, synthetic_audio
    import vrvq_amd

    shapes = {k: tuple(v.shape) for k, v in vrvq_amd.DAC_VRVQ(**kwargs).state_dict().items()}
    o = Oracle(recipe_state_dict(shapes, 0), **kwargs)
    audio = synthetic_audio(clips, CLIP_SAMPLES, seed=1234)
    o.forward(audio[:1, :, :4096], None, 1.0)  # warm caches / BLAS threads
    t0 = time.perf_counter()
    o.forward(audio, None, 1.0)
    dt = time.perf_counter() - t0
    return {"value": clips * CLIP_SAMPLES / SR / dt, "unit": "audio-sec/s", "cores": int(threads),
            "kind": "port",
            "sample": f"{clips} x 1 s clip(s), full encode+RVQ+decode, numpy oracle, 1 run ({dt:.1f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="clips per GPU")
    ap.add_argument("--n-codebooks", type=int, default=8)
    ap.add_argument("--level", type=float, default=1.0)
    ap.add_argument("--cpu-clips", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    import vrvq_amd
    from vrvq_amd.recipe import load_recipe, synthetic_audio
    from vrvq_amd.replicas import shard_seed, throughput, timed_steps

    kwargs = dict(encoder_dim=64, encoder_rates=[2, 4, 8, 8], decoder_dim=1536,
                  decoder_rates=[8, 8, 4, 2], n_codebooks=args.n_codebooks, codebook_size=1024,
                  codebook_dim=8, quantizer_dropout=1.0, sample_rate=SR)
    model = vrvq_amd.DAC_VRVQ(**kwargs)
    load_recipe(model, seed=0)
    model = model.to(dev).eval()
    audio = synthetic_audio(args.batch, CLIP_SAMPLES, seed=shard_seed(1234, rank))
    audio = torch.from_numpy(audio).to(dev)

    timer = RvqTimer()
    install_rvq_timer(timer)

    def step():
        with torch.no_grad():
            return model(audio, SR, None, args.level)

    def timer_on():
        timer.enabled = True

    def timer_off():
        timer.enabled = False

    res_t = timed_steps(step, args.steps, args.warmup, sync=torch.cuda.synchronize, device=dev,
                        on_start=timer_on, on_stop=timer_off)
    out = res_t.last
    dt = res_t.seconds
    ms_per_step = dt / args.steps * 1e3
    value = throughput(args.batch * CLIP_SAMPLES / SR, res_t)

    durs = timer.durations_ms()
    T = out["codes"].shape[-1]
    byt = rvq_bytes(args.batch, T, args.n_codebooks)
    per = {k: (float(np.mean(v)) if v else float("nan")) for k, v in durs.items()}
    rvq_ms = sum(per.values())
    achieved = byt / (rvq_ms * 1e-3) / 1e9
    flops = conv_flops(model, args.batch, 44544)
    # conv time per step = step time minus the RVQ launches (upper bound on conv kernel time)
    conv_ms = ms_per_step - rvq_ms
    conv_tflops = flops / (conv_ms * 1e-3) / 1e12

    traffic, traffic_src = rvq_pmc_traffic() if (args.batch, args.n_codebooks) == (32, 8) \
        else (None, None)
    if rank == 0:
        res = {
            "metric": "audio-sec/s encode+RVQ+decode, 44.1 kHz batch-32, 1->8 MI355X; RVQ HBM GB/s",
            "value": round(value, 3),
            "unit": "audio-sec/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic uniform audio [-0.5,0.5), recipe random-init weights",
            "config": {"workload": "DAC_VRVQ conf/base.yml VBR, level 1, preprocess+encode+decode "
                                   "(z_q_is materialised)",
                       "model": "DAC_VRVQ base (8 cb)", "global_batch": args.batch * world,
                       "clip_samples": CLIP_SAMPLES, "n_codebooks": args.n_codebooks,
                       "parallelism": f"dp{world} (replicas, no data-path collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "rvq_fused_kernel (residual chain + z_q_is stream + gating)",
                         "bytes_per_launch": byt, "path_us": round(rvq_ms * 1e3, 2),
                         "launch_us": {k: round(v * 1e3, 2) for k, v in per.items()}},
            "roofline_conv": {"bound": "mfma", "achieved": round(conv_tflops, 2),
                              "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": round(conv_tflops / FP32_MFMA_PEAK_TFLOPS, 4),
                              "flops_per_step": flops,
                              "note": "algorithmic conv FLOPs / (step time - RVQ launches)"},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(kwargs, args.cpu_clips)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
