"""The frame-major fused RVQ launch (include/vrvq.h vrvq_rvq_encode_fm) and the encoder conv that
feeds it (vrvq_conv1d_fm), through the torch ops over the C-ABI. Needs an MI355X.

Bar: codes and masks bit-exact against a torch fp64 restatement of the quantizer
(models/quantize.py:42-103, 353-421) and against the three-launch path up to fp32 near-ties
(<= 1e-4 of the codes, the bound test_rvq_projection_variants_bit_identical uses for any
reordering of the projection); z_q / z_q_is within 1e-5 relative; a hand-off that times out is
reported loudly (RuntimeError at the next call) and its outputs are poisoned."""
import numpy as np
import pytest
import torch

import vrvq_amd
from conftest import rel_err
from test_gpu_parity import _random_rvq, _rvq_fp64_reference
from vrvq_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _fm_call(z, st, imp, level, zqis=True):
    return ops.rvq_encode_fm(z.transpose(1, 2).contiguous(), st.w3in(), st.b_in, st.cb, st.cbf,
                             st.c2, st.w_out, st.b_out, st.mcol, st.qb, imp=imp, level=level,
                             want_z_q_is=zqis)


@pytest.mark.parametrize("nq,ncode,B,T,vbr", [
    (8, 1024, 3, 87, True), (8, 1024, 2, 1, True), (8, 1024, 2, 13, True), (1, 1024, 4, 87, False),
    (32, 1024, 2, 87, True), (4, 256, 3, 40, True), (4, 512, 2, 87, True), (4, 768, 2, 12, False),
    (28, 1024, 2, 70, True), (8, 1024, 3, 96, True), (8, 1024, 2, 97, True),
    (8, 1024, 2, 128, True), (8, 1024, 2, 129, False), (8, 1024, 2, 200, True),
    (32, 1024, 2, 120, True), (9, 1024, 2, 87, True), (5, 1024, 3, 40, False),
    (12, 1024, 1, 862, True), (8, 1024, 2, 66, True), (8, 1024, 2, 101, True),
    (8, 1024, 2, 94, False), (8, 1024, 2, 3, True), (8, 1024, 2, 35, True)])
def test_rvq_fm_vs_fp64(nq, ncode, B, T, vbr):
    """Every codebook size (N/256 = 1..4), nq 1..32 (odd, > 8), one frame, partial parts,
    T > 96 / 128 (several expansion frame blocks, 16-frame parts; nq = 32 at T = 120 on smaller
    parts to fit the LDS), a 10-s clip (T = 862) and every kind of ragged last quad (T % 4 =
    1..3 inside a frame tile: one shifted 16-B store; at a tile's first quad or T < 4: elementwise
    stores): codes / masks exact vs fp64, z_q_is / z_q
    within 1e-5; z_q is the op's own masked sum of z_q_is bit for bit."""
    q, gen = _random_rvq(nq, ncode, 1000 * nq + T + 7)
    st = q.stacked()
    z = (torch.randn(B, 1024, T, generator=gen) * 0.3).to(DEV)
    imp = torch.rand(B, T, generator=gen).to(DEV) if vbr else None
    level = 0.75
    codes, lat, loss, zqis, zq, mask = _fm_call(z, st, imp, level)
    torch.cuda.synchronize()
    rc, rzqis, rzq, rmask = _rvq_fp64_reference(z, st, imp, level)
    assert (codes.cpu() == rc).float().mean().item() == 1.0
    np.testing.assert_array_equal(mask.cpu().numpy(), rmask.numpy())
    assert rel_err(zqis.cpu().numpy(), rzqis.numpy()) < 1e-5
    assert rel_err(zq.cpu().numpy(), rzq.numpy()) < 1e-5
    assert torch.equal(vrvq_amd.masked_sum(zqis, mask), zq)
    zst, _ = ops.rvq_gather(codes, st.cb)
    zrows = zst.permute(0, 1, 3, 2).reshape(B, nq * 8, T)
    ref_loss = (lat - zrows).pow(2).reshape(B, nq, 8, T).mean(2)
    assert rel_err(loss.cpu().numpy(), ref_loss.cpu().numpy()) < 1e-4
    assert _lib.rvq_sync_error(torch.cuda.current_stream().cuda_stream) == 0


@pytest.mark.parametrize("nq,B,T", [(8, 32, 87), (32, 64, 87), (28, 40, 87), (8, 4, 862)])
def test_rvq_fm_vs_three_launches(nq, B, T):
    """Full configs[1] / configs[2] batches, a ragged batch and 10-s clips: the frame-major launch
    against the three launches on (B, D, T) z -- codes up to fp32 near-ties (a different K order
    of the projection), z_q within 1e-5 over the frames whose codes agree, masks exact."""
    q, gen = _random_rvq(nq, 1024, 17 * nq + T)
    st = q.stacked()
    z = (torch.randn(B, 1024, T, generator=gen) * 0.3).to(DEV)
    imp = torch.rand(B, T, generator=gen).to(DEV)
    prev = _lib.rvq_path(1)
    try:
        want = ops.rvq_encode(z, *st.codes_args(), imp=imp, level=0.8)
    finally:
        _lib.rvq_path(prev)
    got = _fm_call(z, st, imp, 0.8)
    torch.cuda.synchronize()
    same = got[0] == want[0]
    assert same.float().mean().item() > 0.9999
    ok = same.all(dim=1)
    zq_g, zq_w = got[4].permute(0, 2, 1)[ok], want[4].permute(0, 2, 1)[ok]
    assert rel_err(zq_g.cpu().numpy(), zq_w.cpu().numpy()) < 1e-5
    assert torch.equal(got[5], want[5])


def test_rvq_fm_repeats_and_streams_bit_identical():
    """Repeated calls alternating between two streams (one process-wide epoch counter: a call on
    one stream never accepts the other stream's granules) give identical bits every time, under
    a GEMM side load on a third stream; no wait runs out."""
    q, gen = _random_rvq(8, 1024, 4243)
    st = q.stacked()
    z = (torch.randn(32, 1024, 87, generator=gen) * 0.3).to(DEV)
    imp = torch.rand(32, 87, generator=gen).to(DEV)
    want = _fm_call(z, st, imp, 1.0)
    torch.cuda.synchronize()
    s1, s2, side = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.randn(2048, 2048, device=DEV)
    outs = []
    for r in range(6):
        s = s1 if r % 2 == 0 else s2
        s.wait_stream(torch.cuda.current_stream())
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(r % 3 + 1):
                a = (a @ a) * (1.0 / 2048)
        with torch.cuda.stream(s):
            outs.append(_fm_call(z, st, imp, 1.0))
    torch.cuda.synchronize()
    for s in (s1, s2):
        assert _lib.rvq_sync_error(s.cuda_stream) == 0
    for o in outs:
        for x, y in zip(want, o):
            assert (x is None and y is None) or torch.equal(x, y)


def test_rvq_fm_graph_replay():
    """Captured in a CUDA graph (memsets of the sync block and the workspace's granules captured
    before the launch, epoch 1): replays and interleaved eager calls give the same bits."""
    q, gen = _random_rvq(8, 1024, 98)
    st = q.stacked()
    z = (torch.randn(32, 1024, 87, generator=gen) * 0.3).to(DEV)
    imp = torch.rand(32, 87, generator=gen).to(DEV)
    zt = z.transpose(1, 2).contiguous()
    st.w3in()
    want = _fm_call(z, st, imp, 1.0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _fm_call(z, st, imp, 1.0)  # warm-up: the stream's sync block exists before capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = ops.rvq_encode_fm(zt, st.w3in(), st.b_in, st.cb, st.cbf, st.c2, st.w_out, st.b_out,
                                st.mcol, st.qb, imp=imp, level=1.0)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        for x, y in zip(want, out):
            assert (x is None and y is None) or torch.equal(x, y)
        eager = _fm_call(z, st, imp, 1.0)
        torch.cuda.synchronize()
        for x, y in zip(want, eager):
            assert (x is None and y is None) or torch.equal(x, y)


def test_rvq_fm_one_launch_per_resident_group():
    """The fused launch really runs (a 0-capacity occupancy answer would silently
    select another path): one timed launch per call at configs[1], two at B = 64 x nq = 32."""
    for nq, B, want_launches in ((8, 32, 1), (32, 64, None)):
        q, gen = _random_rvq(nq, 1024, 5 + nq)
        st = q.stacked()
        z = (torch.randn(B, 1024, 87, generator=gen) * 0.3).to(DEV)
        _fm_call(z, st, None, 1.0)
        torch.cuda.synchronize()
        _lib.rvq_timing_read()
        prev = _lib.rvq_timing(True)
        try:
            _fm_call(z, st, None, 1.0)
            torch.cuda.synchronize()
            ms, n = _lib.rvq_timing_read()
        finally:
            _lib.rvq_timing(prev)
        assert n >= 1 and ms > 0.0
        if want_launches is not None:
            assert n == want_launches


@pytest.mark.parametrize("path", ["fm", "fused"])
def test_rvq_timeout_is_loud(path):
    """A hand-off wait that runs out (forced: waits bounded at 64 polls, the first chain part /
    projection unit held back) poisons its outputs (codes -1 or NaN z_q) and the NEXT RVQ call
    raises RuntimeError without any synchronisation in between; after the knob is reset a clean
    call succeeds and reports nothing."""
    q, gen = _random_rvq(8, 1024, 31)
    st = q.stacked()
    z = (torch.randn(4, 1024, 87, generator=gen) * 0.3).to(DEV)
    run = (lambda: _fm_call(z, st, None, 1.0)) if path == "fm" else \
        (lambda: ops.rvq_encode(z, *st.codes_args(), level=1.0))
    prev = _lib.rvq_path(2)
    try:
        ref = run()
        torch.cuda.synchronize()
        _lib.rvq_debug(spin_max=64, stall=400)
        bad = run()
        torch.cuda.synchronize()
        _lib.rvq_debug(0, 0)
        poisoned = bool((bad[0] < 0).any()) or bool(torch.isnan(bad[4]).any())
        assert poisoned
        with pytest.raises(RuntimeError, match="timed out"):
            run()
        torch.cuda.synchronize()
        assert ops.rvq_check_error(z, sync=True) in (0, 1, 2)  # drained
        good = run()
        torch.cuda.synchronize()
        assert ops.rvq_check_error(z, sync=True) == 0
        assert torch.equal(good[0], ref[0]) and torch.equal(good[4], ref[4])
    finally:
        _lib.rvq_debug(0, 0)
        _lib.rvq_path(prev)


@pytest.mark.parametrize("B,cin,cout,T,k,pad", [(2, 1024, 1024, 87, 3, 1), (3, 64, 128, 50, 3, 1),
                                                (1, 96, 256, 1000, 7, 3), (2, 512, 64, 33, 1, 0)])
def test_conv1d_fm_matches_conv1d(B, cin, cout, T, k, pad):
    """The frame-major epilogue writes the values of the normal epilogue, transposed, bit for
    bit (with and without the Snake prologue / x3 weights)."""
    gen = torch.Generator().manual_seed(B * cin + T)
    conv = vrvq_amd.layers.WNConv1d(cin, cout, kernel_size=k, padding=pad)
    snake = vrvq_amd.layers.Snake1d(cin)
    with torch.no_grad():
        conv.bias.copy_(torch.randn(cout, generator=gen) * 0.1)
        snake.alpha.copy_(torch.rand(1, cin, 1, generator=gen) + 0.5)
    conv, snake = conv.to(DEV), snake.to(DEV)
    x = torch.randn(B, cin, T, generator=gen).to(DEV)
    for sn in (None, snake):
        y = conv(x, snake=sn)
        yfm = conv.forward_fm(x, snake=sn)
        assert yfm.shape == (B, y.shape[2], cout)
        assert torch.equal(yfm.transpose(1, 2), y)


def test_encode_frame_major_matches_channel_major(manifest):
    """DAC_VRVQ.encode through the frame-major hand-over (default) against VRVQ_RVQ_FM=0's
    (B, D, T) z and the three launches: codes / masks / imp_map exact up to near-ties, z_q
    within 1e-5 (the reference fixtures pin the default path in test_gpu_parity.py)."""
    from test_gpu_parity import model_for, t
    from conftest import load_golden
    g = load_golden("golden_nq8")
    model = model_for(manifest, "golden_nq8")
    x = model.preprocess(t(g["audio_in"]), 44100)
    with torch.no_grad():
        a = model.encode(x, level=1.0)
        prev, vrvq_amd.model.RVQ_FM = vrvq_amd.model.RVQ_FM, False
        try:
            b = model.encode(x, level=1.0)
        finally:
            vrvq_amd.model.RVQ_FM = prev
    torch.cuda.synchronize()
    assert (a["codes"] == b["codes"]).float().mean().item() > 0.9999
    assert torch.equal(a["imp_map"], b["imp_map"])
    assert rel_err(a["z_q"].cpu().numpy(), b["z_q"].cpu().numpy()) < 1e-5
