"""Code containers either side of the path.

* `DACFile` — the reference's `.dac` container (`models/dac_base.py:19-58`): same fields, same
  on-disk layout (an `np.save`d dict holding uint16 codes + metadata, dac_version "1.0.0"), so
  files round-trip with the reference. Loading uses a restricted unpickler that only rebuilds
  numpy arrays / scalars and plain containers, never arbitrary objects.
* `pack_codes` / `unpack_codes` — variable-length packing of VBR codes by their importance mask
  on the GPU (`vrvq_pack_*` kernels, include/vrvq.h): only the codes whose mask is 1 are kept,
  frame-major, plus one count per frame. `save_packed` / `load_packed` store that as a
  pickle-free `.npz` (uint16 stream, uint8 counts, JSON metadata).
"""
from __future__ import annotations

import io
import json
import pickle
from dataclasses import dataclass
from pathlib import Path
from typing import Tuple

import numpy as np
import torch

from .ops import _ops

SUPPORTED_VERSIONS = ["1.0.0"]
MAX_CODEBOOKS = 255  # counts are stored as uint8 (save_packed)


# ----------------------------------------------------------------------------- GPU packing
def pack_codes(codes: torch.Tensor, mask: torch.Tensor, codebook_size: int = 1024
               ) -> Tuple[torch.Tensor, torch.Tensor]:
    """codes (B, Nq, T) int64 + prefix-shaped mask (B, Nq, T) -> (packed uint16 stream as int16
    storage, counts (B, T) int32). Raises ValueError for a non-prefix mask column and
    IndexError for a code outside [0, codebook_size). The packed length is data-dependent, so
    this synchronises the host once (like torch.nonzero)."""
    if codes.dim() != 3 or mask.shape != codes.shape:
        raise RuntimeError("pack_codes: codes and mask must both be (B, Nq, T)")
    if codes.shape[1] > MAX_CODEBOOKS:
        raise ValueError(f"pack_codes: at most {MAX_CODEBOOKS} codebooks")
    counts, off, err = _ops().pack_counts(mask)
    B = codes.shape[0]
    total = int(off[B].item())
    if int(err.item()) == 1:
        raise ValueError("pack_codes: mask is not prefix-shaped (a 1 after a 0 along Nq)")
    packed, err2 = _ops().pack_codes(codes, counts, off, total, int(codebook_size))
    if total and int(err2.item()) == 2:
        raise IndexError(f"pack_codes: code outside [0, {codebook_size})")
    return packed, counts


def unpack_codes(packed: torch.Tensor, counts: torch.Tensor, n_codebooks: int
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Inverse of pack_codes: -> codes (B, Nq, T) int64 (0 where masked), mask (B, Nq, T).
    n_codebooks must be the value the stream was packed with (load_packed returns it in the
    metadata); a stream whose counts exceed it, or whose length disagrees with the counts,
    raises ValueError."""
    if not 0 < int(n_codebooks) <= MAX_CODEBOOKS:
        raise ValueError(f"unpack_codes: n_codebooks must be in [1, {MAX_CODEBOOKS}]")
    if packed.dim() != 1:
        raise ValueError("unpack_codes: packed must be a 1-D stream")
    if counts.dim() != 2:
        raise ValueError("unpack_codes: counts must be (B, T)")
    if int(counts.min()) < 0 or int(counts.max()) > n_codebooks:
        raise ValueError(f"unpack_codes: counts outside [0, {n_codebooks}]")
    off = _ops().unpack_offsets(counts)
    B = counts.shape[0]
    if int(off[B].item()) != packed.numel():
        raise ValueError(f"unpack_codes: stream holds {packed.numel()} codes, counts say "
                         f"{int(off[B].item())}")
    return _ops().unpack_codes(packed, counts, off, int(n_codebooks))


def save_packed(path, packed: torch.Tensor, counts: torch.Tensor, n_codebooks: int,
                **metadata) -> Path:
    """Pickle-free container of a packed stream: packed (uint16), counts (uint8), metadata."""
    path = Path(path).with_suffix(".vrvq.npz")
    meta = dict(metadata, n_codebooks=int(n_codebooks), dac_version=SUPPORTED_VERSIONS[-1])
    np.savez(path, packed=packed.cpu().numpy().view(np.uint16),
             counts=counts.cpu().numpy().astype(np.uint8), metadata=np.array(json.dumps(meta)))
    return path


def load_packed(path, device="cuda"):
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(str(z["metadata"]))
        if meta.get("dac_version") not in SUPPORTED_VERSIONS:
            raise RuntimeError(f"{path}: unsupported version {meta.get('dac_version')}")
        packed = torch.from_numpy(z["packed"].view(np.int16).copy()).to(device)
        counts = torch.from_numpy(z["counts"].astype(np.int32)).to(device)
    return packed, counts, meta


# ----------------------------------------------------------------------------- .dac files
class _ArrayUnpickler(pickle.Unpickler):
    """Rebuilds only what `np.save` of a dict of arrays / scalars / plain values contains."""
    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
                ("numpy", "ndarray"), ("numpy", "dtype")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f".dac file references {module}.{name}: refused")


@dataclass
class DACFile:
    """models/dac_base.py:19-58 (same fields, same file layout)."""
    codes: torch.Tensor
    chunk_length: int
    original_length: int
    input_db: object
    channels: int
    sample_rate: int
    padding: bool
    dac_version: str

    def save(self, path) -> Path:
        input_db = self.input_db
        if isinstance(input_db, torch.Tensor):
            input_db = input_db.detach().cpu().numpy()
        artifacts = {
            "codes": self.codes.detach().cpu().numpy().astype(np.uint16),
            "metadata": {
                "input_db": np.asarray(input_db).astype(np.float32),
                "original_length": self.original_length,
                "sample_rate": self.sample_rate,
                "chunk_length": self.chunk_length,
                "channels": self.channels,
                "padding": self.padding,
                "dac_version": SUPPORTED_VERSIONS[-1],
            },
        }
        path = Path(path).with_suffix(".dac")
        with open(path, "wb") as f:
            np.save(f, artifacts)
        return path

    @classmethod
    def load(cls, path) -> "DACFile":
        with open(path, "rb") as f:
            version = np.lib.format.read_magic(f)
            read = (np.lib.format.read_array_header_1_0 if version == (1, 0)
                    else np.lib.format.read_array_header_2_0)
            shape, _, dtype = read(f)
            if dtype != np.dtype(object) or shape != ():
                raise RuntimeError(f"{path}: not a .dac container")
            artifacts = _ArrayUnpickler(io.BytesIO(f.read())).load()
        if not isinstance(artifacts, np.ndarray) or artifacts.shape != ():
            raise RuntimeError(f"{path}: not a .dac container")
        artifacts = artifacts[()]
        if artifacts["metadata"].get("dac_version", None) not in SUPPORTED_VERSIONS:
            raise RuntimeError(
                f"Given file {path} can't be loaded with this version of descript-audio-codec.")
        codes = torch.from_numpy(artifacts["codes"].astype(int))
        return cls(codes=codes, **artifacts["metadata"])
