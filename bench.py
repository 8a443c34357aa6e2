#!/usr/bin/env python
"""Throughput bench of the VRVQ hot path on MI355X: audio-sec/s of preprocess -> encode
(Snake/WNConv encoder + RVQ + importance gating) -> decode, batch 32 x 1 s @ 44.1 kHz per GPU
(BASELINE.json configs[1]), synthetic audio resident in HBM, recipe (random-init) weights.

    python bench.py [--gpus N --steps K --warmup W]                 configs[1] (default)
    python bench.py --batch 64 --n-codebooks 32                      configs[2] shape
    python bench.py --sweep [--batch 16]                             configs[4]: VBR level sweep
    python bench.py --gpus N ...          N ranks (this script launches torch.distributed.run)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank/GPU)

Multi-GPU: clips shard data-parallel (each rank its own clips, no data-path collective), weak
scaling; the timed region is bracketed by barrier + synchronize and the MAX over ranks is
reported; the sweep's [audio seconds, bits, frames] are SUM-reduced over ranks (RCCL) so its
bpf / kbps are job-wide. Rank 0 prints one JSON line, including
  roofline      the RVQ path (torch.ops.vrvq.rvq_encode: one fused launch of projection ->
                chain -> expansion) against HBM, bytes per SURVEY.md §8(d), per-launch durations from HIP events
                recorded on the launch stream inside the timed steps; per-kernel split from the
                committed rocprofv3 summary; traffic from the committed PMC passes;
  roofline_conv the conv stacks (fp32 arithmetic: the x3 split-bf16 MFMA path for stride-1
                convs, fp32-input MFMA for the strided ones) against the fp32 matrix peak
                and against the x3 ceiling;
  cpu_baseline  oracle/torch_ref.py (a pure-PyTorch CPU restatement of the reference forward,
                fixture-pinned) timed on this host on a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense fp32 matrix peak (= vector peak)
X3_PEAK_TFLOPS = 2516.6 / 6    # fp32 FLOPs on the bf16 MFMA with the exact 3-way split (6 products)
CLIP_SAMPLES = 44100
SR = 44100
LEVELS = (0.25, 0.5, 1.0, 2.0)
# the reference inference driver's own sweep (scripts/inference.py:58-70: 10-s clips, 12 levels)
LEVELS_INFERENCE = (0.2, 0.3, 0.4, 0.5, 0.6, 0.8, 1.0, 1.2, 1.5, 2.0, 2.5, 3.0)
RVQ_KERNELS = ("rvq_pt_kernel", "rvq_fused_kernel", "rvq_project3_kernel", "rvq_project2_kernel",
               "rvq_chain_kernel", "rvq_expand_kernel")


def rvq_bytes(B: int, T: int, nq: int, D: int = 1024, d: int = 8, N: int = 1024,
              from_partials: bool = True) -> int:
    """Algorithmic HBM bytes of one RVQ pass. SURVEY.md §8(d)'s count per frame: z read, imp
    read, z_q_is + z_q writes, codes (int64), latents, mask, loss; plus the stage weights
    (normalised codebook counted once more). from_partials (the eval encode's path: the encoder's
    last conv computed every stage's in_proj in its epilogue, vrvq_conv1d_proj): the kernel reads
    the 8 channel-split partials (8 x nq d fp32 per frame) instead of z (D fp32), and W_in is the
    conv's read, not the quantizer's."""
    inp = 8 * nq * d * 4 if from_partials else D * 4
    per_frame = inp + 4 + nq * D * 4 + D * 4 + nq * 8 + nq * d * 4 + nq * 4 + nq * 4
    weights = nq * 4 * ((0 if from_partials else d * D) + d + 2 * N * d + D * d + D)
    return B * T * per_frame + weights


def newest(pattern: str, cfg3: bool = False):
    """Newest (by round-tag name) record of the configs[1] shape, or with cfg3=True of the
    configs[2] shape (B=64, 32 codebooks: the *cfg3* files)."""
    files = sorted(f for f in glob.glob(os.path.join(REPO, "profiles", pattern))
                   if ("cfg3" in os.path.basename(f)) == cfg3)
    return files[-1] if files else None


def rvq_pmc_traffic(cfg3: bool = False):
    """HBM bytes per RVQ pass from the newest committed PMC measurement
    (profiles/*_rvq_pmc.json: rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE of the three
    kernels, separate passes, tools/gpu/pmc_rvq.sh at configs[1]). bench.py cannot collect PMC
    counters itself (they need their own rocprofv3 passes), so it reports that file."""
    f = newest("*_rvq_pmc.json", cfg3)
    if f is None:
        return None, None
    d = json.load(open(f))
    return d.get("path_total_bytes"), os.path.relpath(f, REPO)


def rvq_kernel_split(cfg3: bool = False):
    """Per-kernel average duration (us) of the RVQ launches from the newest committed
    rocprofv3 kernel-stats summary (profiles/*_rvq_kernel_stats.csv)."""
    import csv
    f = newest("*_rvq_kernel_stats.csv", cfg3)
    if f is None:
        return None, None
    out = {}
    for r in csv.DictReader(open(f)):
        for k in RVQ_KERNELS:
            if k in r["Name"]:
                out[k] = round(float(r["AverageNs"]) / 1e3, 2)
    if "rvq_pt_kernel" in out:  # the eval path's one launch (the micro-bench's partials come
        out = {"rvq_pt_kernel": out["rvq_pt_kernel"]}  # from rvq_project3_kernel, not timed here)
    return out, os.path.relpath(f, REPO)


def conv_flops(model, B: int, L: int):
    """Algorithmic conv FLOPs (2 * MACs) of one encode (encoder + importance subnet) and one
    decode, counted from the layer geometry: the implicit GEMM's M x N x K per layer."""
    fl = {"enc": 0.0, "dec": 0.0}

    def conv_len(T, m):
        k, s, p, d = m.kernel_size[0], m.stride[0], m.padding[0], m.dilation[0]
        return (T + 2 * p - d * (k - 1) - 1) // s + 1

    def acc(part, m, Tin):
        Tout = conv_len(Tin, m)
        fl[part] += 2.0 * B * m.out_channels * Tout * m.in_channels * m.kernel_size[0]
        return Tout

    enc = model.encoder.block
    T = acc("enc", enc[0], L)
    for i in range(1, len(enc) - 2):
        blk = enc[i].block
        for r in range(3):
            acc("enc", blk[r].block[1], T)
            acc("enc", blk[r].block[3], T)
        T = acc("enc", blk[4], T)
    T = acc("enc", enc[len(enc) - 1], T)
    Tz = T
    if hasattr(model.quantizer, "imp_subnet"):
        sub = model.quantizer.imp_subnet
        acc("enc", sub.in_block[1], Tz)
        for b in sub.blocks:
            acc("enc", b[1], Tz)
    dec = model.decoder.model
    T = acc("dec", dec[0], Tz)
    for i in range(1, len(dec) - 3):
        blk = dec[i].block
        ct = blk[1]
        fl["dec"] += 2.0 * B * ct.in_channels * ct.out_channels * T * ct.kernel_size[0]
        T = T * ct.stride[0]
        for r in range(2, 5):
            acc("dec", blk[r].block[1], T)
            acc("dec", blk[r].block[3], T)
    acc("dec", dec[len(dec) - 2], T)
    return fl["enc"], fl["dec"]


class RvqTimer:
    """HIP-event timing of the RVQ operator (torch.ops.vrvq.rvq_encode: one fused launch at
    these shapes), on the stream it runs on, two ways: the kernel's own duration (a start / stop
    event pair carried in the launch's dispatch, vrvq_rvq_timing: what rocprofv3 reports for the
    kernel) and the operator bracketed by two recorded events (path_us: adds the marker packets'
    cost)."""

    def __init__(self):
        self.events = []
        self.enabled = False
        from vrvq_amd import _lib
        self.lib = _lib

    def start(self):
        self.enabled = True
        self.lib.rvq_timing(True)

    def stop(self):
        self.enabled = False
        self.lib.rvq_timing(False)

    def kernel_ms(self):
        """(mean duration of one fused launch, launches timed, launches per rvq_encode call):
        more than 32 clips run as consecutive launches of up to 32 clips each."""
        torch.cuda.synchronize()
        ms, n = self.lib.rvq_timing_read()
        calls = len(self.events)
        return (ms if n else float("nan")), n, (n / calls if calls else 1.0)

    def install(self):
        from vrvq_amd import ops

        def wrap(orig):
            def timed(*a, **k):
                if not self.enabled:
                    return orig(*a, **k)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(torch.cuda.current_stream())
                r = orig(*a, **k)
                e1.record(torch.cuda.current_stream())
                self.events.append((e0, e1))
                return r
            return timed
        # the eval encode's entry (from the conv's partials, model.py RVQ_PROJ) and the
        # channel-major one of the A/B path (VRVQ_RVQ_PROJ=0)
        ops.rvq_encode_part = wrap(ops.rvq_encode_part)
        ops.rvq_encode = wrap(ops.rvq_encode)

    def mean_ms(self):
        torch.cuda.synchronize()
        v = [a.elapsed_time(b) for a, b in self.events]
        return float(np.mean(v)) if v else float("nan")


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(kwargs, clips: int, runs: int = 3):
    """oracle/torch_ref.py (pure-PyTorch CPU restatement of the reference forward, pinned to the
    reference's fixtures by tests/test_oracle.py) on a bounded sample of the same workload:
    `clips` x 1 s clips, same recipe weights, 1 warm-up then the median of `runs`."""
    from oracle.torch_ref import TorchRef
    from vrvq_amd.recipe import recipe_state_dict, synthetic_audio
    import vrvq_amd

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        shapes = {k: tuple(v.shape) for k, v in vrvq_amd.DAC_VRVQ(**kwargs).state_dict().items()}
        ref = TorchRef(recipe_state_dict(shapes, 0), **kwargs)
        audio = torch.from_numpy(synthetic_audio(clips, CLIP_SAMPLES, seed=1234))
        ref.forward(audio, 1.0)  # warm-up at the timed shape (allocator, MKLDNN primitives)
        ts = []
        for _ in range(runs):
            t0 = time.perf_counter()
            ref.forward(audio, 1.0)
            ts.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev)
    dt = float(np.median(ts))
    return {"value": clips * CLIP_SAMPLES / SR / dt, "unit": "audio-sec/s", "cores": threads,
            "kind": "port", "implementation": "torch-restatement (oracle/torch_ref.py)",
            "cpu_model": cpu_model(), "median_of": runs,
            "sample": f"{clips} x 1 s clips of the same workload (B={clips} of 32), full "
                      f"preprocess+encode+RVQ+decode, torch CPU, 1 warm-up at B={clips}, "
                      f"median of {runs} runs ({', '.join(f'{t:.2f}' for t in ts)} s)"}


def build_model(args, dev):
    import vrvq_amd
    from vrvq_amd.recipe import load_recipe
    kwargs = dict(encoder_dim=64, encoder_rates=[2, 4, 8, 8], decoder_dim=1536,
                  decoder_rates=[8, 8, 4, 2], n_codebooks=args.n_codebooks, codebook_size=1024,
                  codebook_dim=8, quantizer_dropout=1.0, sample_rate=SR)
    model = vrvq_amd.DAC_VRVQ(**kwargs)
    load_recipe(model, seed=0)
    return model.to(dev).eval(), kwargs


TRAIN_CLIP = 16758  # conf/dataset.yml train duration 0.38 s at 44.1 kHz


def train_main(args, world: int, rank: int, dev):
    """configs[3]: the vrvq_a2 training step (scripts/train.py:262-335) with `--batch` clips of
    0.38 s per rank (global batch 256 at 8 GPUs), DDP over RCCL for the gradient all-reduce."""
    import vrvq_amd
    from vrvq_amd.config import A2_KWARGS
    from vrvq_amd.recipe import load_recipe, synthetic_audio
    from vrvq_amd.replicas import shard_seed, sum_over_ranks, throughput, timed_steps
    from vrvq_amd.trainer import LAMBDAS_A2, build_state, train_step
    model = vrvq_amd.DAC_VRVQ(**A2_KWARGS)
    load_recipe(model, seed=0)
    torch.manual_seed(0)
    state = build_state(model, dev, ddp=world > 1)
    audio = torch.from_numpy(synthetic_audio(args.batch, TRAIN_CLIP,
                                             seed=shard_seed(4321, rank))).to(dev)

    def step():
        return train_step(state, audio, LAMBDAS_A2)

    res_t = timed_steps(step, args.steps, args.warmup, sync=torch.cuda.synchronize, device=dev)
    ms = res_t.seconds / args.steps * 1e3
    value = throughput(args.batch * TRAIN_CLIP / SR, res_t)
    losses = {k: round(float(v), 5) for k, v in res_t.last.items()}
    ranks_seen = int(sum_over_ranks([1.0], dev)[0])
    if rank == 0:
        print(json.dumps({
            "metric": "train audio-sec/s (vrvq_a2 generator+discriminator step, 0.38 s clips)",
            "value": round(value, 3), "unit": "audio-sec/s", "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic uniform audio [-0.5,0.5), recipe random-init weights",
            "config": {"workload": "vrvq_a2 training step: generator fwd/bwd on the HIP autograd "
                                   "path, discriminator + mel/stft/GAN losses on PyTorch-ROCm, "
                                   "AdamW, grad clipping",
                       "model": "DAC_VRVQ vrvq_a2 (28 cb) + Discriminator",
                       "global_batch": args.batch * world, "clip_samples": TRAIN_CLIP,
                       "parallelism": f"dp{world} (DDP, RCCL all-reduce)"},
            "losses_last_step_rank0": losses}), flush=True)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """`--gpus N` run started as a plain `python bench.py`: launch N ranks of this script, one
    process per GPU, the way the reference launches its multi-GPU jobs
    (scripts/script_train.sh:33: torch.distributed.run --nproc_per_node). torch.distributed.run
    sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, each rank binds cuda:LOCAL_RANK and joins the
    RCCL process group, and rank 0 prints the job's JSON line. This parent only waits: it never
    initialises the GPU, and it starts the ranks as children (no exec)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return subprocess.call(cmd, env=env)


def selftest_main(args, world: int, rank: int) -> None:
    """The launcher and the timed-region contract without a GPU (tests/test_bench_launcher.py):
    gloo process group, a stub CPU step, barrier-bracketed timing with the MAX over ranks, and
    the count of ranks that ran (a SUM all-reduce), reported by rank 0 as one JSON line."""
    from vrvq_amd.replicas import sum_over_ranks, throughput, timed_steps
    if world > 1:
        dist.init_process_group("gloo")
    x = torch.full((64, 64), 1.0 / 64)

    def step():
        return float((x @ x).sum())

    res_t = timed_steps(step, args.steps, args.warmup)
    ranks_seen = int(sum_over_ranks([1.0])[0])
    if rank == 0:
        print(json.dumps({"metric": "selftest", "value": round(throughput(1.0, res_t), 3),
                          "unit": "steps/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ranks_seen": ranks_seen,
                          "ms_per_step": round(res_t.seconds / args.steps * 1e3, 3)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="clips per GPU (32; sweep 16)")
    ap.add_argument("--n-codebooks", type=int, default=8)
    ap.add_argument("--level", type=float, default=1.0)
    ap.add_argument("--sweep", action="store_true", help="configs[4]: VBR level sweep")
    ap.add_argument("--clip-seconds", type=float, default=1.0,
                    help="clip length (1 s: configs[1..4]; 10 with --batch 1 --sweep: the "
                         "reference inference driver's shape, scripts/inference.py:58-70)")
    ap.add_argument("--levels", default=None,
                    help="sweep levels, comma separated (default: configs[4]'s 0.25,0.5,1,2 for "
                         "1-s clips, inference.py:69's 12 levels for longer clips)")
    ap.add_argument("--max-decode-clips", type=int, default=None,
                    help="sweep: decode the levels' z_q in batches of at most this many clips")
    ap.add_argument("--train", action="store_true",
                    help="configs[3]: vrvq_a2 training step (generator + discriminator + losses, "
                         "DDP over RCCL), 0.38 s clips")
    ap.add_argument("--cpu-clips", type=int, default=32,
                    help="clips of the cpu_baseline sample (BASELINE.md: the full B=32 batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--selftest", action="store_true",
                    help="launcher / timing self-test: gloo on CPU with a stub step, no GPU")
    args = ap.parse_args(argv)
    if args.batch is None:
        args.batch = 16 if args.sweep else 32
    clip = int(round(args.clip_seconds * SR))
    if args.levels:
        levels = tuple(float(v) for v in args.levels.split(","))
    else:
        levels = LEVELS if clip == CLIP_SAMPLES else LEVELS_INFERENCE

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N ranks ourselves. Nothing
        # in this process has touched the GPU (torch.cuda is not initialised by the import).
        sys.exit(launch_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    if args.selftest:
        return selftest_main(args, world, rank)
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    import vrvq_amd
    from vrvq_amd.recipe import synthetic_audio
    from vrvq_amd.replicas import job_rate, shard_seed, sum_over_ranks, throughput, timed_steps

    if args.train:
        train_main(args, world, rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    model, kwargs = build_model(args, dev)
    audio = torch.from_numpy(synthetic_audio(args.batch, clip,
                                             seed=shard_seed(1234, rank))).to(dev)
    timer = RvqTimer()
    timer.install()
    nq = args.n_codebooks
    fps = math.floor(SR / model.hop_length)
    lvl_ev = {"all": []}

    if args.sweep:
        # scripts/inference.py:88-112: encode once (level 1), then per level hard mask,
        # masked sum of z_q_is and bpf (device-side, no host sync inside the step); the four
        # levels' z_q decoded as ONE batch of 4 x B clips (vrvq_amd.level_sweep)
        bits = torch.full((nq,), 10.0, device=dev)
        from vrvq_amd.utils import sweep_latents

        def step():
            with torch.no_grad():
                enc = model.encode(model.preprocess(audio, SR), None, 1.0)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                masks, z_all = sweep_latents(enc["imp_map"], enc["z_q_is"], levels, nq)
                cap = args.max_decode_clips or z_all.shape[0]
                y = torch.cat([model.decode(z_all[i:i + cap])
                               for i in range(0, z_all.shape[0], cap)])
                bpfs = [vrvq_amd.ops.bpf(m, bits) for m in masks]
                e1.record()
                if timer.enabled:
                    lvl_ev["all"].append((e0, e1))
                B = args.batch
                return [(lv, masks[i], bpfs[i], y[i * B:(i + 1) * B])
                        for i, lv in enumerate(levels)]
    else:
        def step():
            with torch.no_grad():
                return model(audio, SR, None, args.level)

    def on():
        timer.start()

    def off():
        timer.stop()

    res_t = timed_steps(step, args.steps, args.warmup, sync=torch.cuda.synchronize, device=dev,
                        on_start=on, on_stop=off)
    vrvq_amd.check_errors(dev)  # end of work: a timed-out RVQ hand-off raises here, not silently
    ms_per_step = res_t.seconds / args.steps * 1e3
    value = throughput(args.batch * clip / SR, res_t)
    T = math.ceil(clip / model.hop_length)
    rvq_ms = timer.mean_ms()
    kern_ms, kern_n, per_call = timer.kernel_ms()
    from_part = vrvq_amd.model.RVQ_PROJ
    byt = rvq_bytes(args.batch, T, nq, from_partials=from_part)
    # the dominant kernel's time per rvq_encode call (the fused launches of the call: one per 32
    # clips); the operator bracket when the shape takes the three launches (no kernel-attached
    # events there)
    dur_ms = kern_ms * per_call if kern_n else rvq_ms
    achieved = byt / (dur_ms * 1e-3) / 1e9
    fl_enc, fl_dec = conv_flops(model, args.batch, T * model.hop_length)
    flops = fl_enc + (len(levels) if args.sweep else 1) * fl_dec
    levels_rep = None
    if args.sweep:
        levels_rep = []
        ms = float(np.mean([a.elapsed_time(b) for a, b in lvl_ev["all"]]))
        for lv, mask, bpf_t, _y in res_t.last:
            rep = job_rate(args.batch * clip / SR, float((mask.double() * 10.0).sum()),
                           mask.shape[0] * mask.shape[2], fps, device=dev)
            levels_rep.append({"level": lv, "bpf": round(rep.bpf, 6), "kbps": round(rep.kbps, 4),
                               "bpf_rank0_kernel": round(float(bpf_t), 6),
                               "decode_ms_all_levels_rank0": round(ms, 3),
                               "decode_audio_sec_per_s_all_levels": round(
                                   len(levels) * rep.audio_seconds / (ms * 1e-3), 2)})
    conv_ms = ms_per_step - rvq_ms
    conv_tflops = flops / (conv_ms * 1e-3) / 1e12
    shape = ({(32, 8): False, (64, 32): True}.get((args.batch, nq))
             if not args.sweep and clip == CLIP_SAMPLES else None)
    traffic, traffic_src = rvq_pmc_traffic(shape) if shape is not None else (None, None)
    split, split_src = rvq_kernel_split(shape) if shape is not None else (None, None)
    ranks_seen = int(sum_over_ranks([1.0], dev)[0])
    if rank == 0:
        lv_txt = ",".join(f"{v:g}" for v in levels)
        workload = (f"DAC_VRVQ conf/base.yml VBR, {args.clip_seconds:g}-s clips, level sweep "
                    f"{{{lv_txt}}}: encode once + per level mask/masked-sum/decode/bpf "
                    "(scripts/inference.py:88-112)"
                    if args.sweep else
                    f"DAC_VRVQ VBR {nq} cb, level {args.level}, {args.clip_seconds:g}-s clips, "
                    "preprocess+encode+decode (z_q_is materialised)")
        res = {
            "metric": "audio-sec/s encode+RVQ+decode, 44.1 kHz batch-32, 1->8 MI355X; RVQ HBM GB/s",
            "value": round(value, 3),
            "unit": "audio-sec/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic uniform audio [-0.5,0.5), recipe random-init weights",
            "config": {"workload": workload, "model": f"DAC_VRVQ base ({nq} cb)",
                       "global_batch": args.batch * world, "clip_samples": clip,
                       "n_codebooks": nq,
                       "parallelism": f"dp{world} (replicas, no data-path collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": ("RVQ path: one torch.ops.vrvq.rvq_encode_part = "
                                    "rvq_pt_kernel per group of resident clips (chain parts sum "
                                    "the 8 channel-split in_proj partials the encoder's last conv "
                                    "wrote in its epilogue, vrvq_conv1d_proj, then the stage "
                                    "chain; expansion workgroups with a loader wave write z_q_is "
                                    "/ z_q; in-launch tagged-granule hand-offs)"
                                    if from_part else
                                    "RVQ path: torch.ops.vrvq.rvq_encode on channel-major z = "
                                    "rvq_fused_kernel per <= 32 clips at T <= 96, else three "
                                    "launches (A/B path, VRVQ_RVQ_PROJ=0)"),
                         "bytes_per_call": byt,
                         "bytes_model": ("SURVEY.md §8(d) with the kernel's input = the 8 "
                                         "channel-split in_proj partials (8 x 8 nq fp32 per "
                                         "frame) instead of z, W_in not read"
                                         if from_part else "SURVEY.md §8(d)"),
                         "bytes_per_call_survey_z_input": rvq_bytes(args.batch, T, nq,
                                                                    from_partials=False),
                         "kernel_us": round(kern_ms * 1e3, 2) if kern_n else None,
                         "kernel_launches_timed": kern_n,
                         "launches_per_call": round(per_call, 3),
                         "path_us": round(rvq_ms * 1e3, 2),
                         "kernel_us_rocprof": split, "kernel_us_source": split_src},
            "roofline_conv": {"bound": "mfma", "achieved": round(conv_tflops, 2),
                              "peak": round(X3_PEAK_TFLOPS, 1), "unit": "TFLOP/s",
                              "frac": round(conv_tflops / X3_PEAK_TFLOPS, 4),
                              "flops_per_step": flops,
                              "note": "algorithmic fp32 conv FLOPs / (step time - RVQ launches) "
                                      "against the x3 ceiling: every MFMA conv runs the x3 path "
                                      "(csrc/conv_x3.h: both operands split exactly into 3 bf16 "
                                      "terms, 6 bf16 MFMAs per fp32 product pair, fp32 "
                                      "accumulate -- fp32-accurate), whose ceiling is the bf16 "
                                      "dense peak / 6 = 419.4 TF/s; the fp32-input MFMA peak "
                                      "(157.3 TF/s) is not this path's bound"},
        }
        if levels_rep is not None:
            res["levels"] = levels_rep
        if world == 1 and not args.no_cpu_baseline and not args.sweep:
            res["cpu_baseline"] = cpu_baseline(kwargs, args.cpu_clips)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
