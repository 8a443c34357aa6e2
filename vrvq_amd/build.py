"""Build the two in-tree libraries with hipcc for gfx950 (no JIT cache: the .so files travel
with the repo snapshot to the GPU box):

  libvrvq_hip.so    the HIP kernels + the C-ABI of include/vrvq.h (no torch dependency)
  libvrvq_torch.so  TORCH_LIBRARY(vrvq) custom operators (csrc/torch_ops.cpp, host code only)
                    over that C-ABI, loaded with torch.ops.load_library
"""
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
TORCH_LIB = os.path.join(HERE, "libvrvq_torch.so")
TORCH_SRC = os.path.join(CSRC, "torch_ops.cpp")
ARCH = os.environ.get("VRVQ_OFFLOAD_ARCH", "gfx950")
# -fno-slp-vectorize: the SLP pass packs independent fp32 chains into v_pk_* with extra
# v_mov shuffles and +40 VGPRs in the RVQ kernel; packed math is written explicitly instead.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]
OBJ_DIR = os.path.join(HERE, "build")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [
        os.path.join(REPO, "include", "vrvq.h"), os.path.abspath(__file__)]


def _newer(out: str, inputs) -> bool:
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in inputs)


def up_to_date() -> bool:
    return _newer(LIB, deps()) and _newer(TORCH_LIB, [TORCH_SRC, LIB] + deps())


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build vrvq_amd)")


def _compile_and_link(out: str, extra, verbose: bool, tag: str, srcs=None) -> str:
    """One hipcc process per translation unit (they compile in parallel), then one link."""
    os.makedirs(OBJ_DIR, exist_ok=True)
    procs, objs = [], []
    headers = [d for d in deps() if not d.endswith(".hip")]
    for src in (srcs or sources()):
        obj = os.path.join(OBJ_DIR, os.path.basename(src)[:-4] + tag + ".o")
        objs.append(obj)
        if os.path.exists(obj) and all(os.path.getmtime(d) <= os.path.getmtime(obj)
                                       for d in headers + [src]):
            continue  # object newer than its source and every header
        cmd = [hipcc()] + FLAGS + list(extra) + ["-I", os.path.join(REPO, "include"), "-c", src,
                                                 "-o", obj]
        if verbose:
            print("[vrvq_amd] " + " ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd))
    failed = [cmd for p, cmd in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    tmp = out + ".tmp"
    subprocess.run([hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}",
                    f"-Wl,-soname,{os.path.basename(out)}", "-o", tmp] + objs, check=True)
    os.replace(tmp, out)
    return out


def build_torch_ops(verbose: bool = True) -> str:
    """libvrvq_torch.so: the TORCH_LIBRARY registration (host-only C++ against the torch ROCm
    headers), linked to libvrvq_hip.so through an $ORIGIN rpath."""
    from torch.utils import cpp_extension as ce
    import torch

    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    inc = sum((["-I", p] for p in ce.include_paths()), [])
    tlib = ce.library_paths()[0]
    tmp = TORCH_LIB + ".tmp"
    cmd = [hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-variable",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           *inc, "-I", os.path.join(REPO, "include"), TORCH_SRC, "-o", tmp,
           "-L", HERE, "-lvrvq_hip", "-L", tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
           "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{tlib}", "-Wl,-soname,libvrvq_torch.so"]
    if verbose:
        print("[vrvq_amd] " + " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, TORCH_LIB)
    return TORCH_LIB


def _objects_current() -> bool:
    """Every object newer than its source and the headers (a source edited while a build ran
    leaves the library newer than it but its object stale)."""
    headers = [d for d in deps() if not d.endswith(".hip")]
    for src in sources():
        obj = os.path.join(OBJ_DIR, os.path.basename(src)[:-4] + ".o")
        if not _newer(obj, headers + [src]):
            return False
    return True


def build_library(force: bool = False, verbose: bool = True) -> str:
    if not force and _newer(LIB, deps()) and (not os.path.isdir(OBJ_DIR) or _objects_current()):
        pass
    else:
        _compile_and_link(LIB, [], verbose, "")
    if force or not _newer(TORCH_LIB, [TORCH_SRC, LIB] + deps()):
        build_torch_ops(verbose)
    return LIB


def build_stamped(verbose: bool = True) -> str:
    """Diagnostic build with in-kernel s_memtime stamps (tools/rvq_chain_stamps.py): the RVQ
    translation unit only (the stamped kernels and the entry points the tool calls)."""
    return _compile_and_link(os.path.join(HERE, "libvrvq_hip_stamps.so"), ["-DVRVQ_STAMPS"],
                             verbose, "_stamps", srcs=[os.path.join(CSRC, "rvq.hip")])


if __name__ == "__main__":
    if "--stamps" in sys.argv:
        build_stamped()
    else:
        build_library(force="--force" in sys.argv)
