"""The eval encode's RVQ path: the encoder's last conv with every stage's in_proj in its
epilogue (include/vrvq.h vrvq_conv1d_proj) and the quantizer launched from those partials
(vrvq_rvq_encode_part: rvq_pt_kernel, or the chain + expansion launches when a clip does not
fit the resident grid). Needs an MI355X.

Bar: BIT-IDENTICAL to the three-launch path (vrvq_rvq_project's x3 partials -> chain ->
expansion, vrvq_rvq_path(1)) on every output -- the partials are that projection's values and the
chain sums them in the same split order -- hence codes / masks exact and z_q / z_q_is within the
three-launch path's own tolerance against fp64 (test_gpu_parity.py);
reference fixtures pin DAC_VRVQ.encode on this path in test_gpu_parity.py."""
import ctypes

import numpy as np
import pytest
import torch

import vrvq_amd
from conftest import rel_err
from test_gpu_parity import _random_rvq, _rvq_fp64_reference
from vrvq_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def _conv(cin, k, pad, seed):
    gen = torch.Generator().manual_seed(seed)
    conv = vrvq_amd.layers.WNConv1d(cin, 1024, kernel_size=k, padding=pad)
    snake = vrvq_amd.layers.Snake1d(cin)
    with torch.no_grad():
        conv.bias.copy_(torch.randn(1024, generator=gen) * 0.1)
        snake.alpha.copy_(torch.rand(1, cin, 1, generator=gen) + 0.5)
    return conv.to(DEV), snake.to(DEV), gen


def _project(z, st):
    """vrvq_rvq_project (x3 variant, the three-launch path's first kernel) on channel-major z."""
    B, D, T = z.shape
    nq = st.b_in.shape[0]
    part = torch.empty(8, B * T, nq * 8, device=DEV)
    _lib.call("vrvq_rvq_project", P(z), B, D, T, nq, 8, P(st.w_in_t), P(part),
              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    return part


def _three_launches(z, st, imp, level, zqis=True):
    prev = _lib.rvq_path(1)
    try:
        return ops.rvq_encode(z, *st.codes_args(), imp=imp, level=level, want_z_q_is=zqis)
    finally:
        _lib.rvq_path(prev)


def _part_call(part, T, st, imp, level, zqis=True):
    return ops.rvq_encode_part(part, T, st.b_in, st.cb, st.cbf, st.c2, st.w_out, st.b_out,
                               st.mcol, st.qb, imp=imp, level=level, want_z_q_is=zqis)


def _equal(a, b):
    for x, y in zip(a, b):
        assert (x is None and y is None) or torch.equal(x, y)


@pytest.mark.parametrize("B,cin,T,nq,k,pad", [
    (3, 1024, 87, 8, 3, 1), (2, 1024, 87, 32, 3, 1), (5, 1024, 87, 9, 3, 1), (1, 1024, 862, 8, 3, 1),
    (2, 1024, 1, 8, 3, 1), (3, 1024, 40, 1, 3, 1), (2, 1024, 97, 28, 3, 1), (2, 512, 130, 8, 7, 3),
    (48, 1024, 87, 8, 3, 1)])
def test_conv1d_proj_partials_are_project_bits(B, cin, T, nq, k, pad):
    """The epilogue's partials equal vrvq_rvq_project's on the conv's own z bit for bit (every
    tile width: 32-wide at T = 87, 96-wide at B = 48, 128-wide at T = 862 / 130; one frame; odd
    nq; nq = 1 / 28 / 32), and want_z returns z exactly as the plain conv writes it."""
    conv, snake, gen = _conv(cin, k, pad, 7 * B + T + nq)
    q, _ = _random_rvq(nq, 1024, 11 * nq + T)
    st = q.stacked()
    x = torch.randn(B, cin, T, generator=gen).to(DEV)
    z = conv(x, snake=snake)
    part, zz = conv.forward_proj(x, st.w3in(), nq, snake=snake, want_z=True)
    part2, none = conv.forward_proj(x, st.w3in(), nq, snake=snake)
    want = _project(z, st)
    torch.cuda.synchronize()
    assert none is None and torch.equal(zz, z)
    assert part.shape == (8, B * z.shape[2], nq * 8)
    assert torch.equal(part, want) and torch.equal(part2, want)


@pytest.mark.parametrize("nq,ncode,B,T,vbr", [
    (8, 1024, 32, 87, True), (32, 1024, 64, 87, True), (28, 1024, 40, 87, True),
    (8, 1024, 4, 862, True), (8, 1024, 2, 1, True), (4, 256, 3, 40, True), (4, 512, 2, 87, False),
    (4, 768, 2, 12, True), (9, 1024, 3, 87, True), (8, 1024, 2, 96, True), (8, 1024, 2, 97, True),
    (8, 1024, 2, 129, False), (32, 1024, 2, 120, True), (1, 1024, 4, 87, False),
    (8, 1024, 2, 3, True), (8, 1024, 2, 35, True), (12, 1024, 1, 862, True), (8, 1024, 2, 193, True)])
def test_rvq_part_matches_three_launches(nq, ncode, B, T, vbr):
    """rvq_encode_part from the partials against the three launches on (B, D, T) z: all six
    outputs equal bit for bit (full configs[1] / configs[2] batches, ragged batches, 10-s clips,
    every codebook size, odd nq, one frame, every partial expansion window / tile / quad), and
    codes / masks exact against the fp64 restatement."""
    q, gen = _random_rvq(nq, ncode, 1000 * nq + T + 3)
    st = q.stacked()
    z = (torch.randn(B, 1024, T, generator=gen) * 0.3).to(DEV)
    imp = torch.rand(B, T, generator=gen).to(DEV) if vbr else None
    part = _project(z, st)
    want = _three_launches(z, st, imp, 0.8)
    got = _part_call(part, T, st, imp, 0.8)
    torch.cuda.synchronize()
    _equal(got, want)
    assert torch.equal(vrvq_amd.masked_sum(got[3], got[5]), got[4])
    if B * T <= 400:
        rc, _rzqis, rzq, rmask = _rvq_fp64_reference(z, st, imp, 0.8)
        assert (got[0].cpu() == rc).all()
        np.testing.assert_array_equal(got[5].cpu().numpy(), rmask.numpy())
        assert rel_err(got[4].cpu().numpy(), rzq.numpy()) < 1e-5
    assert _lib.rvq_sync_error(torch.cuda.current_stream().cuda_stream) == 0


def test_rvq_part_runs_fused_and_falls_back():
    """configs[1] takes ONE rvq_pt_kernel launch (timed-launch count); with the resident-clip
    capacity forced to 0 (a clip too long for the grid) or vrvq_rvq_path(1), the chain
    + expansion launches run instead (no timed fused launch) with the same bits; z_q_is off too."""
    q, gen = _random_rvq(8, 1024, 77)
    st = q.stacked()
    z = (torch.randn(32, 1024, 87, generator=gen) * 0.3).to(DEV)
    imp = torch.rand(32, 87, generator=gen).to(DEV)
    part = _project(z, st)
    assert _lib.rvq_fused_clips(87, 8) >= 32
    _part_call(part, 87, st, imp, 1.0)
    torch.cuda.synchronize()
    _lib.rvq_timing_read()
    prev_t = _lib.rvq_timing(True)
    try:
        want = _part_call(part, 87, st, imp, 1.0)
        torch.cuda.synchronize()
        assert _lib.rvq_timing_read()[1] == 1
        prev_c = _lib.rvq_debug_capacity(0)
        try:
            assert _lib.rvq_fused_clips(87, 8) == 0
            fb = _part_call(part, 87, st, imp, 1.0)
            fb_nozqis = _part_call(part, 87, st, imp, 1.0, zqis=False)
            torch.cuda.synchronize()
            assert _lib.rvq_timing_read()[1] == 0
        finally:
            _lib.rvq_debug_capacity(prev_c)
        prev_p = _lib.rvq_path(1)
        try:
            p1 = _part_call(part, 87, st, imp, 1.0)
            torch.cuda.synchronize()
            assert _lib.rvq_timing_read()[1] == 0
        finally:
            _lib.rvq_path(prev_p)
    finally:
        _lib.rvq_timing(prev_t)
    _equal(fb, want)
    _equal(p1, want)
    assert fb_nozqis[3] is None and torch.equal(fb_nozqis[4], want[4])


def test_rvq_part_graph_replay_and_streams():
    """Captured in a CUDA graph (granules and sync block in the workspace, zeroed by captured
    memsets) and run eagerly on two streams under a GEMM side load: identical bits every time."""
    q, gen = _random_rvq(8, 1024, 98)
    st = q.stacked()
    z = (torch.randn(32, 1024, 87, generator=gen) * 0.3).to(DEV)
    imp = torch.rand(32, 87, generator=gen).to(DEV)
    part = _project(z, st)
    want = _part_call(part, 87, st, imp, 1.0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _part_call(part, 87, st, imp, 1.0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = _part_call(part, 87, st, imp, 1.0)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        _equal(out, want)
    s1, s2, side = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.randn(2048, 2048, device=DEV)
    outs = []
    for r in range(4):
        st_ = s1 if r % 2 == 0 else s2
        st_.wait_stream(torch.cuda.current_stream())
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(r + 1):
                a = (a @ a) * (1.0 / 2048)
        with torch.cuda.stream(st_):
            outs.append(_part_call(part, 87, st, imp, 1.0))
    torch.cuda.synchronize()
    for o in outs:
        _equal(o, want)


def test_rvq_part_launch_counts():
    """The fused launch really runs (a 0-capacity occupancy answer would silently
    select another path): one timed launch per call at configs[1], at least one at the configs[2]
    shape (B = 64 x nq = 32)."""
    for nq, B, want_launches in ((8, 32, 1), (32, 64, None)):
        q, gen = _random_rvq(nq, 1024, 5 + nq)
        st = q.stacked()
        z = (torch.randn(B, 1024, 87, generator=gen) * 0.3).to(DEV)
        part = _project(z, st)
        _part_call(part, 87, st, None, 1.0)
        torch.cuda.synchronize()
        _lib.rvq_timing_read()
        prev = _lib.rvq_timing(True)
        try:
            _part_call(part, 87, st, None, 1.0)
            torch.cuda.synchronize()
            ms, n = _lib.rvq_timing_read()
        finally:
            _lib.rvq_timing(prev)
        assert n >= 1 and ms > 0.0
        if want_launches is not None:
            assert n == want_launches


def test_rvq_fused_timeout_is_loud():
    """rvq_encode's fused launch on channel-major z: a hand-off wait that runs out (waits bounded
    at 64 polls, the first projection unit held back) poisons its outputs (codes -1 or NaN z_q)
    and the NEXT RVQ call raises RuntimeError without any synchronisation in between; after the
    knob is reset a clean call succeeds and reports nothing."""
    q, gen = _random_rvq(8, 1024, 31)
    st = q.stacked()
    z = (torch.randn(4, 1024, 87, generator=gen) * 0.3).to(DEV)
    run = lambda: ops.rvq_encode(z, *st.codes_args(), level=1.0)  # noqa: E731
    prev = _lib.rvq_path(2)
    try:
        ref = run()
        torch.cuda.synchronize()
        _lib.rvq_debug(spin_max=64, stall=400)
        bad = run()
        torch.cuda.synchronize()
        _lib.rvq_debug(0, 0)
        assert bool((bad[0] < 0).any()) or bool(torch.isnan(bad[4]).any())
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


def test_rvq_part_timeout_is_loud_for_a_one_shot_caller():
    """A hand-off wait that runs out (waits bounded at 64 polls, the first chain part held back)
    poisons the outputs, and a ONE-SHOT caller learns it from vrvq_amd.check_errors() (RuntimeError
    after its own sync) -- no later RVQ call needed; a clean call afterwards reports nothing."""
    q, gen = _random_rvq(8, 1024, 31)
    st = q.stacked()
    z = (torch.randn(4, 1024, 87, generator=gen) * 0.3).to(DEV)
    part = _project(z, st)
    ref = _part_call(part, 87, st, None, 1.0)
    torch.cuda.synchronize()
    vrvq_amd.check_errors()
    _lib.rvq_debug(spin_max=64, stall=400)
    try:
        bad = _part_call(part, 87, st, None, 1.0)
    finally:
        _lib.rvq_debug(0, 0)
    with pytest.raises(RuntimeError, match="timed out"):
        vrvq_amd.check_errors()
    assert bool((bad[0] < 0).any()) or bool(torch.isnan(bad[4]).any())
    good = _part_call(part, 87, st, None, 1.0)
    vrvq_amd.check_errors()
    _equal(good, ref)


def test_encode_projected_matches_channel_major(manifest):
    """DAC_VRVQ.encode on the default path (projection epilogue + rvq_encode_part) against the
    channel-major z path (VRVQ_RVQ_PROJ=0: rvq_encode) -- every output of the dict
    bit for bit -- and against itself with the fused launch's capacity forced to 0 (the two-launch
    fallback a clip too long for the grid takes)."""
    from test_gpu_parity import model_for, t
    from conftest import load_golden
    g = load_golden("golden_nq8")
    model = model_for(manifest, "golden_nq8")
    x = model.preprocess(t(g["audio_in"]), 44100)
    m = vrvq_amd.model
    with torch.no_grad():
        a = model.encode(x, level=1.0)
        prev, m.RVQ_PROJ = m.RVQ_PROJ, False
        try:
            b = model.encode(x, level=1.0)
        finally:
            m.RVQ_PROJ = prev
        prev_c = _lib.rvq_debug_capacity(0)
        try:
            c = model.encode(x, level=1.0)
        finally:
            _lib.rvq_debug_capacity(prev_c)
    torch.cuda.synchronize()
    for key in a:
        if a[key] is None:
            assert b[key] is None and c[key] is None
            continue
        assert torch.equal(a[key], b[key]), key
        assert torch.equal(a[key], c[key]), key


def test_encode_cbr_prefix_projected_matches_channel_major():
    """A CBR model's encode with n_quantizers < Nq projects only the prefix's stages in the conv
    epilogue (the stacked prefix, cached per n): the dict equals the channel-major z path's bit
    for bit, for several prefixes and the full set."""
    model = vrvq_amd.DAC_VRVQ(n_codebooks=8, model_type="CBR").to(DEV).eval()
    gen = torch.Generator().manual_seed(5)
    x = model.preprocess((torch.rand(2, 1, 44100, generator=gen) * 2 - 1).to(DEV), 44100)
    m = vrvq_amd.model
    with torch.no_grad():
        for n in (1, 4, 7, 8, None):
            a = model.encode(x, n)
            prev, m.RVQ_PROJ = m.RVQ_PROJ, False
            try:
                b = model.encode(x, n)
            finally:
                m.RVQ_PROJ = prev
            torch.cuda.synchronize()
            for key in a:
                assert (a[key] is None and b[key] is None) or torch.equal(a[key], b[key]), (n, key)
