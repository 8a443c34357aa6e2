"""Build libvrvq_hip.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the
repo snapshot to the GPU box)."""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvrvq_hip.so")
ARCH = os.environ.get("VRVQ_OFFLOAD_ARCH", "gfx950")
# -fno-slp-vectorize: the SLP pass packs independent fp32 chains into v_pk_* with extra
# v_mov shuffles and +40 VGPRs in the RVQ kernel; packed math is written explicitly instead.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-slp-vectorize",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [
        os.path.join(REPO, "include", "vrvq.h"), os.path.abspath(__file__)]


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in deps())


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build vrvq_amd)")


def build_library(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return LIB
    tmp = LIB + ".tmp"
    cmd = [hipcc()] + FLAGS + ["-I", os.path.join(REPO, "include"), "-o", tmp] + sources()
    if verbose:
        print("[vrvq_amd] " + " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


def build_stamped(verbose: bool = True) -> str:
    """Diagnostic build with in-kernel s_memtime stamps (tools/rvq_stamps.py)."""
    out = os.path.join(HERE, "libvrvq_hip_stamps.so")
    cmd = [hipcc()] + FLAGS + ["-DVRVQ_STAMPS", "-I", os.path.join(REPO, "include"), "-o", out] + sources()
    if verbose:
        print("[vrvq_amd] " + " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    if "--stamps" in sys.argv:
        build_stamped()
    else:
        build_library(force="--force" in sys.argv)
