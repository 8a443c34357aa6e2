"""The PyTorch-ROCm custom-operator surface (TORCH_LIBRARY(vrvq) in csrc/torch_ops.cpp).

CPU: the operator library loads, registers every schema SURVEY.md §8(b) names, and its fake
kernels propagate shapes on meta tensors (torch.compile / FakeTensorMode tracing).
GPU: the ops run on the current stream without host syncs, so encode + decode captured in a
torch.cuda.CUDAGraph replays to bit-identical outputs."""
import numpy as np
import pytest
import torch

from vrvq_amd import ops

EXPECTED = ["weight_norm", "snake_inv_alpha", "codebook_prep", "pack_conv1d_weight",
            "pack_convt1d_weight", "snake_conv1d", "snake_conv_transpose1d", "residual_unit",
            "rvq_cross_prep", "rvq_frag", "rvq_encode", "rvq_gather", "rvq_expand", "masked_loss", "scale_imp", "imp_mask",
            "masked_sum", "bpf", "pack_counts", "pack_codes", "unpack_offsets", "unpack_codes"]


def test_ops_registered():
    lib = ops.load_ops()
    for name in EXPECTED:
        op = getattr(lib, name)
        assert op.default._schema.name == f"vrvq::{name}"


def test_fake_kernels_propagate_shapes():
    ops.load_ops()
    m = torch.device("meta")
    vr = torch.ops.vrvq
    x = torch.empty(2, 64, 1000, device=m)
    wp = vr.pack_conv1d_weight(torch.empty(128, 64, 7, device=m))
    assert wp.shape == (64, 7, 128)
    a = torch.empty(64, device=m)
    y, ys = vr.snake_conv1d(x, wp, 128, 1, 9, 3, None, a, a, None, 0, torch.empty(128, device=m),
                            torch.empty(128, device=m), False)
    assert y.shape == (0,) and ys.shape == (2, 128, 1000)
    y, ys = vr.snake_conv1d(x, vr.pack_conv1d_weight(torch.empty(128, 64, 4, device=m)), 128, 2,
                            1, 1, None, None, None, None, 0, None, None, True)
    assert y.shape == (2, 128, 500) and ys.shape == (0,)
    wt = vr.pack_convt1d_weight(torch.empty(64, 32, 16, device=m), 8)
    assert wt.shape == (64, 2, 256)
    y, ys = vr.snake_conv_transpose1d(x, wt, 32, 8, None, a, a, None, None, True)
    assert y.shape == (2, 32, 8000)
    z = torch.empty(3, 1024, 87, device=m)
    cb = torch.empty(8, 1024, 8, device=m)
    w = torch.empty(8, 1024, 8, device=m)
    mcol, qb = vr.rvq_cross_prep(w, w, torch.empty(8, 1024, device=m))
    assert mcol.shape == (8, 8, 8, 8) and qb.shape == (8, 8)
    out = vr.rvq_encode(z, w, torch.empty(8, 8, device=m), cb, cb, torch.empty(8, 1024, device=m),
                        w, torch.empty(8, 1024, device=m), mcol, qb, torch.empty(3, 87, device=m),
                        1.0, True, True)
    assert [tuple(o.shape) for o in out] == [(3, 8, 87), (3, 64, 87), (3, 8, 87),
                                             (3, 8, 1024, 87), (3, 1024, 87), (3, 8, 87)]
    assert out[0].dtype == torch.int64
    zst, zp, err = vr.rvq_gather(torch.empty(3, 4, 87, dtype=torch.int64, device=m), cb)
    assert zst.shape == (3, 4, 87, 8) and zp.shape == (3, 32, 87)
    zqis, zq, mk = vr.rvq_expand(zst, w, torch.empty(8, 1024, device=m), None, 1.0, False, True)
    assert zqis.shape == (0,) and zq.shape == (3, 1024, 87) and mk.shape == (3, 4, 87)
    assert vr.imp_mask(torch.empty(3, 1, 87, device=m), 28).shape == (3, 28, 87)
    assert vr.bpf(torch.empty(3, 8, 87, device=m), torch.empty(8, device=m)).shape == ()


def test_ops_reject_cpu_tensors():
    ops.load_ops()
    with pytest.raises(RuntimeError, match="GPU only"):
        torch.ops.vrvq.snake_inv_alpha(torch.ones(4))


@pytest.mark.gpu
def test_cuda_graph_capture_encode_decode(manifest):
    """encode + decode through torch.ops.vrvq captured in one CUDA graph: replay is
    bit-identical to eager, and replay on new input (copied into the static buffer) equals eager
    on that input."""
    import vrvq_amd
    from vrvq_amd.recipe import load_recipe, synthetic_audio
    dev = torch.device("cuda:0")
    model = vrvq_amd.DAC_VRVQ(**manifest["golden_nq8"]["kwargs"])
    load_recipe(model, 0)
    model = model.to(dev).eval()
    a0 = torch.from_numpy(synthetic_audio(4, 44100, seed=1)).to(dev)
    a1 = torch.from_numpy(synthetic_audio(4, 44100, seed=2)).to(dev)

    def run(x):
        with torch.no_grad():
            enc = model.encode(model.preprocess(x, 44100), None, 1)
            return enc["codes"], enc["z_q"], enc["mask_imp"], model.decode(enc["z_q"])

    eager0, eager1 = run(a0), run(a1)   # also warms the folded-weight caches
    static = a0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run(static)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = run(static)
    g.replay()
    torch.cuda.synchronize()
    for e, o in zip(eager0, outs):
        assert torch.equal(e, o)
    static.copy_(a1)
    g.replay()
    torch.cuda.synchronize()
    for e, o in zip(eager1, outs):
        assert torch.equal(e, o)
    assert not np.array_equal(eager0[0].cpu().numpy(), eager1[0].cpu().numpy())
