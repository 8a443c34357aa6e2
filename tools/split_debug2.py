"""Diagnostic of vrvq_rvq_split internals (VRVQ_SPLIT_DBG modes; B=1, T=8, nq=2)."""
import os, sys
import torch
sys.path.insert(0, ".")
import vrvq_amd
from vrvq_amd import ops
dev = torch.device("cuda:0")
B, T, nq = 1, 8, 2
gen = torch.Generator().manual_seed(7)
q = vrvq_amd.model.ResidualVectorQuantize(input_dim=1024, n_codebooks=nq, codebook_size=1024, codebook_dim=8)
with torch.no_grad():
    for p in q.parameters():
        p.copy_(torch.randn(p.shape, generator=gen) * (0.05 if p.ndim == 3 else 1.0))
q = q.to(dev).eval()
st = q.stacked()
args = st.codes_args()
w_in_t = args[0]
print("w_in_t", tuple(w_in_t.shape), "cbn", tuple(args[3].shape))
z = (torch.randn(B, 1024, T, generator=gen) * 0.3).to(dev)
b = ops.rvq_split(z, *args)
torch.cuda.synchronize()
lat = b[1].view(B, nq, 8, T)[0, 0]
mode = os.environ.get("VRVQ_SPLIT_DBG")
if mode == "1":
    exp = torch.einsum("ck,ct->kt", w_in_t[0, :128].double(), z[0, :128].double())
    print("own-slice partial: got", lat[:, 0].tolist())
    print("                   exp", exp[:, 0].tolist())
elif mode == "2":
    print("got", lat[:, 0].tolist())
    print("exp", (w_in_t[0, 0, :8] + 1000 * args[3][0, 0, :8]).tolist() if w_in_t.dim() == 3 else "?")
