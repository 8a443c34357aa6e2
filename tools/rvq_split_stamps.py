#!/usr/bin/env python
"""Per-phase timing of the channel-split RVQ kernel (vrvq_rvq_split) from s_memtime stamps taken
by the exchange wave (diagnostic build: VRVQ_LIB=vrvq_amd/libvrvq_hip_stamps.so)."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
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
g = torch.Generator().manual_seed(1)
z = (torch.randn(B, 1024, T, generator=g) * 0.3).to(dev)
imp = torch.rand(B, T, generator=g).to(dev)
stamps = torch.zeros(4096 * NQ * 8, dtype=torch.int64, device=dev)
_lib.load().vrvq_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
for _ in range(5):
    stamps.zero_()
    ops.rvq_split(z, *st.codes_args(), imp=imp, level=1.0)
torch.cuda.synchronize()
s = stamps.cpu().numpy().astype(np.int64).reshape(-1, NQ, 8)
s = s[s[:, 0, 0] != 0]
d = np.diff(s[:, :, :6], axis=2)
names = ["E1 publish + group wait", "gather/normalize + [Q]", "DMA issue + [R] (argmin)",
         "E2 publish + group wait", "final argmin/gather/stores + [U]"]
print(f"workgroups={len(s)} stages={NQ}; median stamp cycles per phase (stages 1..):")
for k, n in enumerate(names):
    print(f"  {n:34s} {np.median(d[:, 1:, k]):8.0f}   (stage0 {np.median(d[:, 0, k]):8.0f})")
print(f"  [P] (out_proj + in_proj)           {np.median(s[:, 1:, 0] - s[:, :-1, 5]):8.0f}")
print(f"  stage period                       {np.median(s[:, 1:, 0] - s[:, :-1, 0]):8.0f}")
tot = s[:, -1, 5] - s[:, 0, 0]
print(f"  first item total median {np.median(tot):.0f}, max {tot.max()}")
