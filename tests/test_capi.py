"""The C-ABI library (no GPU needed): it loads, exports every function include/vrvq.h declares,
the ctypes table matches the header, and host-side argument checks reject bad calls before
any launch."""
import ctypes
import os
import re

import pytest

from vrvq_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "vrvq.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decls = {}
    for m in re.finditer(r"(?:const\s+char\s*\*|int)\s+(vrvq_\w+)\s*\(([^)]*)\)\s*;", src):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        decls[m.group(1)] = args
    return decls


def test_header_parsed():
    decls = header_functions()
    assert "vrvq_rvq_encode" in decls and "vrvq_conv1d" in decls and len(decls) >= 16


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name


def test_ctypes_table_matches_header():
    decls = header_functions()
    for name, args in decls.items():
        if name in _lib.SIGNATURES:
            assert len(_lib.SIGNATURES[name]) == len(args), name
        else:
            assert name in _lib.EXTRA, f"{name} declared but not bound"
            assert len(_lib.EXTRA[name][0]) == len(args), name
    assert set(_lib.SIGNATURES) | set(_lib.EXTRA) == set(decls)


def test_status_strings_and_version():
    lib = _lib.load()
    assert lib.vrvq_status_string(0) == b"ok"
    assert b"invalid argument" in lib.vrvq_status_string(10001)
    assert lib.vrvq_version() >= 100


def test_argument_errors_raise_before_launch():
    lib = _lib.load()
    # null pointers -> VRVQ_ERR_ARG, returned by the host-side check (no GPU touched)
    assert lib.vrvq_weight_norm(None, None, 4, 4, None, None) == 10001
    assert lib.vrvq_conv1d(None, 1, 1, 8, None, None, None, None, 1, 128, 3, 1, 1, 1, None,
                           None, 0, None, 8, None, None, None, None) == 10001
    assert lib.vrvq_rvq_encode(*([None] + [1] * 6 + [None] * 10 + [1.0] + [None] * 7 +
                                 [0, None])) == 10001
    n = ctypes.c_longlong(0)
    assert lib.vrvq_rvq_workspace(32, 87, 8, ctypes.byref(n)) == 0
    # partials as tagged granules (8 B each, the fused launch) + the larger of the zst rows
    # (B T nq d floats) and the fused launch's tagged stage granules (B nq 8 parts x 16 frames
    # x d x 8 B), then the sync block a captured fused launch takes from the workspace (2052
    # words, rounded up to 256 B)
    sync = (2052 * 4 + 255) // 256 * 256
    assert n.value == (2 * 8 * 32 * 87 * 64 + max(32 * 87 * 8 * 8, 32 * 8 * 8 * 16 * 8 * 2)) * 4 \
        + sync
    assert lib.vrvq_rvq_path(7) == 10001 and lib.vrvq_rvq_path(0) in (1, 2)
    # the quantizer from the conv's partials: the larger of the captured launch's stage granules
    # (B nq ceil(87 / 16) parts x 16 frames x d x 8 B, + the sync block) and the two-launch
    # fallback's zst rows
    assert lib.vrvq_rvq_workspace_part(32, 87, 8, 1024, ctypes.byref(n)) == 0
    assert n.value == max(32 * 8 * 6 * 16 * 8 * 8 + sync, 32 * 8 * 87 * 8 * 4)
    assert lib.vrvq_rvq_workspace_part(32, 87, 33, 1024, ctypes.byref(n)) == 10002
    assert lib.vrvq_rvq_encode_part(*([None] + [1] * 6 + [None] * 9 + [1.0] + [None] * 7 +
                                      [0, None])) == 10001
    assert lib.vrvq_conv1d_proj(None, 1, 1024, 87, None, None, None, None, 1024, 1024, 3, 1, 1,
                                None, None, 87, None, 8, None, None, 0, None) == 10001
    # the projection epilogue serves the 1024-channel latent only
    assert lib.vrvq_conv1d_proj(p16 := ctypes.c_void_p(16), 1, 512, 87, None, None, p16, None,
                                512, 512, 3, 1, 1, None, None, 87, p16, 8, p16, None, 0,
                                None) == 10002
    with pytest.raises(RuntimeError, match="invalid argument"):
        _lib.call("vrvq_bpf", None, None, 1, 1, 1, None, None)
    # geometry mismatch (tout inconsistent with the conv formula)
    p = ctypes.c_void_p(16)
    assert lib.vrvq_conv1d(p, 1, 4, 100, None, None, p, None, 4, 128, 7, 1, 3, 1, None, None,
                           0, p, 99, None, None, None, None) == 10001
    # producer-side snake without its alpha
    assert lib.vrvq_conv1d(p, 1, 4, 100, None, None, p, None, 4, 128, 7, 1, 3, 1, None, None,
                           0, None, 100, None, None, p, None) == 10001
    # split-K workspace of the deep-K T <= 96 layers (conv.hip splitk_parts): S parts x B x
    # M / 128 tiles x 128 x 96 fp32, S = 4 capped at chunks / 8 -- a function of the layer,
    # not of the batch
    def ws(*shape):
        assert lib.vrvq_conv1d_workspace(*shape, ctypes.byref(n)) == 0
        return n.value
    tile = 128 * 96 * 4
    assert ws(32, 512, 696, 1024, 16, 8, 4, 1, 1) == 4 * 32 * 8 * tile   # 512 -> 1024 s8
    assert ws(1, 512, 696, 1024, 16, 8, 4, 1, 1) == 4 * 1 * 8 * tile
    assert ws(32, 1024, 87, 1024, 3, 1, 1, 1, 1) == 4 * 32 * 8 * tile    # ImportanceSubnet k3
    assert ws(32, 1024, 87, 512, 3, 1, 1, 1, 1) == 4 * 32 * 4 * tile
    assert ws(32, 512, 87, 128, 3, 1, 1, 1, 1) == 4 * 32 * 1 * tile
    assert ws(32, 128, 87, 128, 3, 1, 1, 1, 1) == 0                      # 8 chunks: none
    assert ws(32, 1024, 87, 1536, 7, 1, 3, 1, 1) == 4 * 32 * 12 * tile   # decoder k7
    assert ws(32, 128, 87, 32, 3, 1, 1, 1, 1) == 0                       # M < 128
    assert ws(32, 1024, 87, 1024, 3, 1, 1, 1, 0) == 0                    # fp32-input path
    assert ws(32, 384, 5568, 384, 7, 1, 3, 1, 1) == 0                    # long rows
    assert lib.vrvq_conv1d_ws(p16, 1, 1024, 87, None, None, p16, p16, 1024, 1024, 3, 1, 1, 1,
                              None, None, 0, p16, 87, None, None, None, p16, 16, None) == 10001
    # x3 weight size: chunks x 3 planes x padded octets x cout_pad x 8 bf16
    assert lib.vrvq_x3_weight_size(384, 7, 384, ctypes.byref(n)) == 0
    assert n.value == 48 * 3 * 8 * 384 * 8
    assert lib.vrvq_x3_weight_size(384, 5, 384, ctypes.byref(n)) == 10002
