"""Time the training step's discriminator parts (forward + backward of the GAN losses) at the
configs[3] per-GPU shape: the five period discriminators vs the three spectral ones."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vrvq_amd.discriminator import Discriminator
from vrvq_amd.recipe import synthetic_audio

dev = torch.device("cuda:0")
x = torch.from_numpy(synthetic_audio(32, 16758, seed=1)).to(dev)
y = (x + 0.01 * torch.randn_like(x)).requires_grad_(True)
for name, kw in (("MPD x5", dict(periods=[2, 3, 5, 7, 11], fft_sizes=[])),
                 ("MRD x3", dict(periods=[], fft_sizes=[2048, 1024, 512]))):
    d = Discriminator(**kw).to(dev)
    def step():
        fr = d(y)
        rr = d(x)
        loss = sum(torch.mean((1 - f[-1]) ** 2) for f in fr)
        loss = loss + sum(torch.nn.functional.l1_loss(a, b.detach())
                          for f, r in zip(fr, rr) for a, b in zip(f[:-1], r[:-1]))
        loss.backward()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 5:.1f} ms per generator-side D pass (fwd real+fake, bwd)")
