"""ctypes binding of the C-ABI in include/vrvq.h (libvrvq_hip.so, built in-tree for gfx950).

The library is the product: every arithmetic op of the hot path runs in it. There is no
fallback — if the library is missing or a call fails, a RuntimeError is raised.
"""
from __future__ import annotations

import ctypes
import os
import threading

LIB_NAME = "libvrvq_hip.so"
LIB_PATH = os.environ.get("VRVQ_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float

# name -> argtypes (restype is int status unless noted). Mirrors include/vrvq.h exactly;
# tests/test_capi.py checks this table against the header and the exported symbols.
SIGNATURES = {
    "vrvq_weight_norm": [_P, _P, _I, _I, _P, _P],
    "vrvq_snake_inv_alpha": [_P, _I, _P, _P],
    "vrvq_snake": [_P, _I, _I, _I, _P, _P, _P, _P],
    "vrvq_phase_split": [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P],
    "vrvq_codebook_prep": [_P, _I, _I, _P, _P, _P],
    "vrvq_conv1d": [_P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _I, _P, _I,
                    _P, _P, _P, _P],
    "vrvq_conv1d_workspace": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "vrvq_conv1d_ws": [_P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _I, _P,
                       _I, _P, _P, _P, _P, ctypes.c_longlong, _P],
    "vrvq_conv1d_proj": [_P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _I, _P, _I,
                         _P, _P, ctypes.c_longlong, _P],
    "vrvq_x3_weight_size": [_I, _I, _I, _P],
    "vrvq_pack_x3_weight": [_P, _I, _I, _I, _P, _P],
    "vrvq_pack_conv1d_weight": [_P, _I, _I, _I, _I, _P, _P],
    "vrvq_residual_unit": [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P,
                           _P, _P, _P],
    "vrvq_conv_transpose1d": [_P, _I, _I, _I, _P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "vrvq_conv_transpose1d_pad": [_P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P,
                                  _P, _P],
    "vrvq_pack_convt1d_weight": [_P, _I, _I, _I, _I, _P, _P],
    "vrvq_rvq_cross_prep": [_P, _P, _P, _I, _I, _I, _P, _P, _P],
    "vrvq_rvq_frag": [_P, _I, _I, _I, _P, _P],
    "vrvq_rvq_workspace": [_I, _I, _I, _P],
    "vrvq_rvq_encode": [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F,
                        _P, _P, _P, _P, _P, _P, _P, ctypes.c_longlong, _P],
    "vrvq_rvq_w_in_planes_size": [_I, _I, _I, _P],
    "vrvq_rvq_pack_w_in": [_P, _I, _I, _I, _P, _P],
    "vrvq_rvq_workspace_part": [_I, _I, _I, _I, _P],
    "vrvq_rvq_encode_part": [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F,
                             _P, _P, _P, _P, _P, _P, _P, ctypes.c_longlong, _P],
    "vrvq_rvq_fused_clips": [_I, _I, _I, _P],
    "vrvq_rvq_project": [_P, _I, _I, _I, _I, _I, _P, _P, _P],
    "vrvq_rvq_chain": [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P,
                       _P],
    "vrvq_rvq_expand": [_P, _I, _I, _I, _I, _I, _P, _P, _P, _F, _P, _P, _P, _P],
    "vrvq_rvq_gather": [_P, _I, _I, _I, _P, _I, _I, _P, _P, _P, _P],
    "vrvq_masked_loss": [_P, _P, _I, _I, _I, _P, _P],
    "vrvq_mask_hard": [_P, _I, _I, _I, _P, _P],
    "vrvq_scale_imp": [_P, _I, _F, _F, _P, _P],
    "vrvq_masked_sum": [_P, _P, _I, _I, _I, _I, _P, _P],
    "vrvq_bpf": [_P, _P, _I, _I, _I, _P, _P],
    "vrvq_pack_counts": [_P, _I, _I, _I, _P, _P, _P, _P, _P],
    "vrvq_pack_codes": [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P],
    "vrvq_unpack_offsets": [_P, _I, _I, _P, _P, _P],
    "vrvq_unpack_codes": [_P, _P, _P, _I, _I, _I, _P, _P, _P],
    "vrvq_rvq_nearest": [_P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _P],
    # training step
    "vrvq_wgrad_plan": [_I, _I, _I, _I, _I, _P, _P],
    "vrvq_conv1d_wgrad": [_P, _I, _I, _I, _P, _P, _P, _I, _I, _P, _P, _I, _I, _I, _I, _I, _P,
                          ctypes.c_longlong, _P, _P],
    "vrvq_snake_backward_workspace": [_I, _I, _I, _P],
    "vrvq_snake_backward": [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P, ctypes.c_longlong, _P],
    "vrvq_bias_grad_workspace": [_I, _I, _I, _P],
    "vrvq_bias_grad": [_P, _I, _I, _I, _P, _P, ctypes.c_longlong, _P],
    "vrvq_act_backward": [_P, _P, ctypes.c_longlong, _I, _P, _P],
    "vrvq_weight_norm_backward": [_P, _P, _P, _I, _I, _P, _P, _P],
    "vrvq_pack_conv1d_flip": [_P, _I, _I, _I, _I, _P, _P],
    "vrvq_mask_ste": [_P, _P, _P, _I, _I, _I, _F, _I, _I, _P, _P],
    "vrvq_mask_ste_backward": [_P, _P, _P, _I, _I, _I, _F, _I, _P, _P],
    "vrvq_rvq_expand_masked": [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "vrvq_rvq_backward_workspace": [_I, _I, _I, _P],
    "vrvq_rvq_backward": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P,
                          _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, ctypes.c_longlong, _P],
}
EXTRA = {"vrvq_status_string": ([_I], ctypes.c_char_p), "vrvq_version": ([], _I),
         "vrvq_rvq_project_variant": ([_I], _I), "vrvq_rvq_path": ([_I], _I),
         "vrvq_rvq_sync_error": ([_P, _P], _I), "vrvq_rvq_timing": ([_I], _I),
         "vrvq_rvq_timing_read": ([_P, _P], _I), "vrvq_rvq_pending_error": ([_P], _I),
         "vrvq_rvq_debug": ([ctypes.c_uint, ctypes.c_uint], _I),
         "vrvq_rvq_debug_capacity": ([_I], _I)}

_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    """Load libvrvq_hip.so (once). Raises RuntimeError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"vrvq_amd: HIP library {LIB_PATH} is missing; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = _I
        for name, (argtypes, restype) in EXTRA.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = restype
        _lib = lib
    return _lib


def call(name: str, *args) -> None:
    """Invoke a C-ABI entry point; raise RuntimeError with the library's message on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.vrvq_status_string(rc)
        raise RuntimeError(f"{name} failed ({rc}): {msg.decode() if msg else 'unknown'}")


def rvq_path(path: int = 0) -> int:
    """Select the RVQ launch structure (2: one fused launch where the shape allows, default; 1:
    three launches; 0: query). Returns the previous path. Same outputs bit for bit."""
    prev = load().vrvq_rvq_path(path)
    if prev not in (1, 2):
        raise RuntimeError(f"vrvq_rvq_path({path}) failed ({prev})")
    return prev


def rvq_sync_error(stream: int) -> int:
    """Timeout code recorded by a fused RVQ launch on `stream` (0: none); clears it."""
    code = ctypes.c_int(0)
    call("vrvq_rvq_sync_error", ctypes.c_void_p(stream), ctypes.byref(code))
    return code.value


def rvq_pending_error() -> int:
    """Timeout code of any fused RVQ launch completed by now (0: none), no synchronisation;
    clears it."""
    code = ctypes.c_int(0)
    call("vrvq_rvq_pending_error", ctypes.byref(code))
    return code.value


def rvq_debug(spin_max: int = 0, stall: int = 0) -> None:
    """Test hook: bound every later fused launch's waits at spin_max polls (0: default) and delay
    its first chain part by stall x s_sleep(127)."""
    call("vrvq_rvq_debug", ctypes.c_uint(spin_max), ctypes.c_uint(stall))


def rvq_fused_clips(frames: int, nq: int, ncode: int = 1024) -> int:
    """Clips one fused launch from the conv's partials holds resident (0: the two-launch form
    runs; include/vrvq.h vrvq_rvq_fused_clips)."""
    n = ctypes.c_int(0)
    call("vrvq_rvq_fused_clips", frames, nq, ncode, ctypes.byref(n))
    return n.value


def rvq_debug_capacity(clips: int) -> int:
    """Test hook: cap the clips per fused launch from partials (0 forces the two launches, -1
    removes the cap). Returns the previous cap."""
    return int(load().vrvq_rvq_debug_capacity(int(clips)))


def rvq_timing(on: bool) -> bool:
    """Attach HIP start / stop events to every fused RVQ launch (kernel duration on its stream)
    while on. Returns the previous setting."""
    return bool(load().vrvq_rvq_timing(1 if on else 0))


def rvq_timing_read():
    """(mean kernel ms, launches) of the launches recorded since the last read."""
    ms, n = ctypes.c_float(0.0), ctypes.c_int(0)
    call("vrvq_rvq_timing_read", ctypes.byref(ms), ctypes.byref(n))
    return float(ms.value), int(n.value)


def rvq_project_variant(variant: int = 0) -> int:
    """Select the RVQ projection kernel (3: clip x split workgroups on the split-bf16 MFMA,
    default; 2: the same on the fp32 MFMA; 1: 48-frame tiles; 0: query). Returns the previous
    variant. 1 and 2 write the same bits (tests/test_gpu_parity.py)."""
    prev = load().vrvq_rvq_project_variant(variant)
    if prev not in (1, 2, 3):
        raise RuntimeError(f"vrvq_rvq_project_variant({variant}) failed ({prev})")
    return prev
