"""Code containers (vrvq_amd/codes_io.py) on CPU: the reference-compatible
.dac container (a file written by the reference's own DACFile.save is a committed fixture) and
the numpy packing oracle. The GPU packing kernels are checked in test_gpu_parity.py."""
import os
import pickle

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.vrvq_oracle import generate_mask_hard, pack_codes
from vrvq_amd.codes_io import DACFile


def test_load_reference_written_dac():
    f = DACFile.load(os.path.join(GOLDEN, "ref_written.dac"))
    want = np.load(os.path.join(GOLDEN, "ref_written_expect.npz"))["codes"]
    np.testing.assert_array_equal(f.codes.numpy(), want)
    assert f.codes.dtype == torch.int64
    assert (f.original_length, f.sample_rate, f.chunk_length, f.channels, f.padding) == \
        (12345, 44100, 25, 1, True)
    assert f.dac_version == "1.0.0"
    assert float(np.asarray(f.input_db).reshape(-1)[0]) == -17.25


def test_dac_roundtrip_and_byte_layout(tmp_path):
    codes = torch.randint(0, 1024, (1, 8, 25), generator=torch.Generator().manual_seed(3))
    f = DACFile(codes=codes, chunk_length=25, original_length=12345,
                input_db=torch.tensor([-17.25]), channels=1, sample_rate=44100, padding=True,
                dac_version="1.0.0")
    p = f.save(tmp_path / "x")
    assert p.suffix == ".dac"
    g = DACFile.load(p)
    assert torch.equal(g.codes, codes)
    # same bytes as the reference's writer for the same content
    assert p.read_bytes() == open(os.path.join(GOLDEN, "ref_written.dac"), "rb").read()


def test_dac_load_refuses_foreign_objects(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    p = tmp_path / "evil.dac"
    with open(p, "wb") as fh:
        np.save(fh, np.array({"codes": Evil(), "metadata": {}}, dtype=object), allow_pickle=True)
    with pytest.raises(pickle.UnpicklingError):
        DACFile.load(p)


def test_dac_version_check(tmp_path):
    p = tmp_path / "v.dac"
    with open(p, "wb") as fh:
        np.save(fh, np.array({"codes": np.zeros((1, 2, 3), np.uint16),
                              "metadata": {"dac_version": "0.9"}}, dtype=object))
    with pytest.raises(RuntimeError):
        DACFile.load(p)


def test_pack_oracle_properties():
    rng = np.random.default_rng(0)
    B, nq, T = 3, 8, 50
    codes = rng.integers(0, 1024, (B, nq, T)).astype(np.int64)
    s = (rng.random((B, 1, T)) * (nq + 1) - 0.5).astype(np.float32)
    mask = generate_mask_hard(s, nq)
    packed, counts = pack_codes(codes, mask)
    assert packed.dtype == np.uint16 and packed.size == int(mask.sum())
    np.testing.assert_array_equal(counts, mask.sum(1))
    # decode by hand: frame-major, stage-minor
    k = 0
    for b in range(B):
        for t in range(T):
            for i in range(counts[b, t]):
                assert packed[k] == codes[b, i, t]
                k += 1
