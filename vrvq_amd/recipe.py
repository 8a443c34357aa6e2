"""Portable, name-seeded weight recipe shared by the golden-fixture generator (which loads it
into the reference model), the CPU oracle and the GPU path, so all three run bit-identical
weights without shipping checkpoints (no pretrained VRVQ weights exist offline).

Each tensor is drawn from its own PCG64 stream seeded by (seed, crc32(name)), so the recipe
depends only on parameter names and shapes — not on module construction order or RNG state:
  weight_v         U(-1/sqrt(fan_in), 1/sqrt(fan_in))      (torch's default Conv init)
  weight_g         ||v|| (per dim-0 slice) * U(0.8, 1.25)
  bias             U(-1/sqrt(fan_in), 1/sqrt(fan_in))      (fan_in of the sibling weight_v)
  alpha            U(0.5, 2.0)
  codebook.weight  N(0, 1)                                  (nn.Embedding default)
The importance subnet's last conv gain is multiplied by IMP_SPREAD and its bias set to
IMP_BIAS (calibrated once on the recipe weights + synthetic audio: pre-bias logits are
-0.065 +- 0.005, so logits become ~N(0, 2^2)) so imp_map spreads over (0, 1) instead of
collapsing to ~0.5, which would put the mask thresholds exactly on integer level*Nq ties
(SURVEY.md §7 "Mask threshold ties at random init").
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Tuple

import numpy as np

IMP_SPREAD = 400.0
IMP_BIAS = 26.0
IMP_SPREAD_KEY = "quantizer.imp_subnet.blocks.4.1.weight_g"
IMP_BIAS_KEY = "quantizer.imp_subnet.blocks.4.1.bias"


def _rng(name: str, seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())]))


def _fan_in(shape) -> int:
    return int(np.prod(shape[1:]))


def recipe_tensor(name: str, shape: Tuple[int, ...], shapes: Dict[str, Tuple[int, ...]],
                  seed: int = 0) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    leaf = name.rsplit(".", 1)[-1]
    rng = _rng(name, seed)
    if leaf == "weight_v":
        b = 1.0 / np.sqrt(_fan_in(shape))
        return rng.uniform(-b, b, size=shape).astype(np.float32)
    if leaf == "weight_g":
        vname = name[: -len("weight_g")] + "weight_v"
        v = recipe_tensor(vname, shapes[vname], shapes, seed)
        norm = np.sqrt(np.sum(v.astype(np.float64) ** 2, axis=tuple(range(1, v.ndim))))
        g = norm * rng.uniform(0.8, 1.25, size=norm.shape)
        if name == IMP_SPREAD_KEY:
            g = g * IMP_SPREAD
        return g.reshape(shape).astype(np.float32)
    if leaf == "bias":
        if name == IMP_BIAS_KEY:
            return np.full(shape, IMP_BIAS, dtype=np.float32)
        vname = name[: -len("bias")] + "weight_v"
        vshape = shapes.get(vname)
        fan = _fan_in(vshape) if vshape is not None else shape[0]
        b = 1.0 / np.sqrt(fan)
        return rng.uniform(-b, b, size=shape).astype(np.float32)
    if leaf == "alpha":
        return rng.uniform(0.5, 2.0, size=shape).astype(np.float32)
    if name.endswith("codebook.weight"):
        return rng.standard_normal(size=shape).astype(np.float32)
    raise KeyError(f"recipe: no rule for parameter {name}")


def recipe_state_dict(shapes: Dict[str, Tuple[int, ...]], seed: int = 0) -> Dict[str, np.ndarray]:
    """name -> float32 array for every entry of `shapes` (a state_dict's name -> shape)."""
    shapes = {k: tuple(int(s) for s in v) for k, v in shapes.items()}
    return {k: recipe_tensor(k, v, shapes, seed) for k, v in shapes.items()}


def shapes_of(state_dict) -> Dict[str, Tuple[int, ...]]:
    return {k: tuple(v.shape) for k, v in state_dict.items()}


def load_recipe(model, seed: int = 0) -> None:
    """Fill a torch module's parameters from the recipe (strict: every key must have a rule)."""
    import torch

    sd = model.state_dict()
    rec = recipe_state_dict(shapes_of(sd), seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in rec.items()}, strict=True)


def synthetic_audio(batch: int, length: int, seed: int = 1234) -> np.ndarray:
    """Seeded uniform audio in [-0.5, 0.5), shape (B, 1, L), float32."""
    rng = np.random.Generator(np.random.PCG64([int(seed), 0xA0D10]))
    return rng.uniform(-0.5, 0.5, size=(batch, 1, length)).astype(np.float32)
