"""Diagnostic: vrvq_rvq_split vs vrvq_rvq_fused stage by stage (latents = z_e, codes, z_q_is)."""
import sys
import torch
sys.path.insert(0, ".")
import vrvq_amd
from vrvq_amd import ops

dev = torch.device("cuda:0")
for (B, T, nq) in [(1, 8, 2), (2, 87, 8), (32, 87, 8)]:
    gen = torch.Generator().manual_seed(7)
    q = vrvq_amd.model.ResidualVectorQuantize(input_dim=1024, n_codebooks=nq, codebook_size=1024,
                                              codebook_dim=8)
    with torch.no_grad():
        for p in q.parameters():
            p.copy_(torch.randn(p.shape, generator=gen) * (0.05 if p.ndim == 3 else 1.0))
    q = q.to(dev).eval()
    st = q.stacked()
    z = (torch.randn(B, 1024, T, generator=gen) * 0.3).to(dev)
    a = ops.rvq_fused(z, *st.codes_args())
    b = ops.rvq_split(z, *st.codes_args())
    torch.cuda.synchronize()
    err = ops.rvq_split_error(dev)
    la, lb = a[1].view(B, nq, 8, T), b[1].view(B, nq, 8, T)
    print(f"B={B} T={T} nq={nq} err={err}")
    for i in range(nq):
        dl = (la[:, i] - lb[:, i]).abs().max().item()
        ca = (a[0][:, i] == b[0][:, i]).float().mean().item()
        dz = (a[3][:, i] - b[3][:, i]).abs().max().item()
        print(f"  stage {i}: latents max|d| {dl:.3e}  codes agree {ca:.4f}  z_q_is max|d| {dz:.3e}")
    if B == 1:
        print("  fused latents[0,0,:,:4]", la[0, 0, :, :4].flatten()[:8].tolist())
        print("  split latents[0,0,:,:4]", lb[0, 0, :, :4].flatten()[:8].tolist())
        print("  fused codes", a[0][0].tolist())
        print("  split codes", b[0][0].tolist())
