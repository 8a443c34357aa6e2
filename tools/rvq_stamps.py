#!/usr/bin/env python
"""Per-step timing of the rvq_codes kernel from in-kernel s_memtime stamps (diagnostic build:
`python -m vrvq_amd.build --stamps`, then VRVQ_LIB=vrvq_amd/libvrvq_hip_stamps.so)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("VRVQ_LIB", os.path.join(HERE, "vrvq_amd", "libvrvq_hip_stamps.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vrvq_amd  # noqa: E402
from vrvq_amd import _lib, ops  # noqa: E402
from vrvq_amd.recipe import load_recipe  # noqa: E402

B, NQ, T = int(os.environ.get("B", 32)), int(os.environ.get("NQ", 8)), 87
dev = torch.device("cuda:0")
model = vrvq_amd.DAC_VRVQ(n_codebooks=NQ)
load_recipe(model, 0)
q = model.quantizer.to(dev).eval()
st = q.stacked()
z = (torch.randn(B, 1024, T, generator=torch.Generator().manual_seed(1)) * 0.3).to(dev)
stamps = torch.zeros(4096 * NQ * 8, dtype=torch.int64, device=dev)
_lib.load().vrvq_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
for _ in range(5):
    ops.rvq_codes(z, *st.codes_args())
torch.cuda.synchronize()
s = stamps.cpu().numpy().astype(np.int64)
nblk = int((s.reshape(-1, NQ, 8)[:, 0, 0] != 0).sum())
s = s[: nblk * NQ * 8].reshape(nblk, NQ, 8)
d = np.diff(s, axis=2)  # step durations (cycles)
names = ["dma+in_proj", "reduce_scatter", "dma wait+barrier", "normalize+barrier",
         "distance+argmin+barrier", "gather+barrier", "out_proj"]
print(f"blocks={nblk} stages={NQ}; median cycles per step (over blocks, stages 1..):")
for k, n in enumerate(names):
    print(f"  {n:26s} {np.median(d[:, 1:, k]):8.0f}   (stage0 {np.median(d[:, 0, k]):8.0f})")
tot = s[:, -1, 7] - s[:, 0, 0]
print(f"  per-block total median {np.median(tot):.0f} cycles, max {tot.max()}")
