"""Build the MI355X-native extension libraries in-tree.

Two shared objects are produced under ``modelopt_amd/_lib/``:

* ``libmtq_amd.so`` -- the HIP kernels for gfx950 behind the C ABI of ``include/mtq_amd.h``
  (``hipcc --offload-arch=gfx950``).  No torch dependency.
* ``_C.so`` -- the PyTorch-ROCm custom-op registration (``TORCH_LIBRARY(modelopt_amd)``) over that
  C ABI; links ``libmtq_amd.so`` with an ``$ORIGIN`` rpath.

Both are built in-tree (not pip-installed, not in a JIT cache) so they travel with the repository
snapshot to the GPU box.  Rebuilds only when a source is newer than its output.

Usage: ``python tensorrt-model-optimizer_amd/build.py [--force] [-j N]``
"""

from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent
CSRC = HERE / "csrc"
INC = REPO / "include"
OUT = HERE / "modelopt_amd" / "_lib"
OBJ = HERE / "_obj"  # per-source objects (git- and gpurun-ignored)

ARCH = os.environ.get("MTQ_AMD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the MI355X-native build needs ROCm's hipcc")


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_kernels(force: bool = False) -> Path:
    """One object per source (compiled in parallel, each rebuilt only when it or a shared header
    changed), then one link."""
    out = OUT / "libmtq_amd.so"
    srcs = [CSRC / "mtq_kernels.hip", CSRC / "mtq_search.hip", CSRC / "mtq_qlinear.hip", CSRC / "mtq_awq_gemm.hip",
            CSRC / "mtq_awq_scale.hip", CSRC / "mtq_attention.hip", CSRC / "mtq_cpu.cpp"]
    hdrs = [CSRC / "mtq_device.hpp", INC / "mtq_amd.h"]
    OBJ.mkdir(parents=True, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Werror=misleading-indentation", "-Wno-unused-function", f"-I{INC}"]
    objs, jobs = [], []
    for src in srcs:
        obj = OBJ / (src.name + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *hdrs]):
            tmp = obj.with_suffix(".o.tmp")
            cmd = [_hipcc(), *flags, "-c", str(src), "-o", str(tmp)]
            print("+", " ".join(cmd), flush=True)
            jobs.append((subprocess.Popen(cmd), tmp, obj))
    failed = 0
    for proc, tmp, obj in jobs:
        if proc.wait() != 0:
            failed = proc.returncode
        else:
            tmp.replace(obj)
    if failed:
        raise subprocess.CalledProcessError(failed, "hipcc")
    if force or jobs or _stale(out, objs):
        OUT.mkdir(parents=True, exist_ok=True)
        tmp = out.with_suffix(".so.tmp")
        _run([_hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", *[str(o) for o in objs], "-o", str(tmp)])
        tmp.replace(out)
    return out


def _torch_paths() -> tuple[list[str], list[str], bool]:
    import torch  # noqa: PLC0415  (import only for include/lib paths)

    root = Path(torch.__file__).resolve().parent
    incs = [str(root / "include"), str(root / "include" / "torch" / "csrc" / "api" / "include")]
    libs = [str(root / "lib")]
    return incs, libs, bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def build_torch_ops(force: bool = False) -> Path:
    out = OUT / "_C.so"
    kern = OUT / "libmtq_amd.so"
    deps = [CSRC / "torch_ops.cpp", INC / "mtq_amd.h", kern]
    if force or _stale(out, deps):
        incs, libs, cxx11 = _torch_paths()
        py_inc = sysconfig.get_paths()["include"]
        tmp = out.with_suffix(".so.tmp")
        cmd = [
            _hipcc(),
            "-O2",
            "-std=c++17",
            "-fPIC",
            "-shared",
            "-D__HIP_PLATFORM_AMD__=1",
            "-DUSE_ROCM=1",
            f"-D_GLIBCXX_USE_CXX11_ABI={int(cxx11)}",
            f"-I{INC}",
            f"-I{py_inc}",
        ]
        cmd += [f"-I{i}" for i in incs]
        cmd += [str(CSRC / "torch_ops.cpp"), "-o", str(tmp)]
        cmd += [f"-L{l}" for l in libs]
        cmd += [f"-L{OUT}", "-lmtq_amd", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip"]
        cmd += ["-Wl,-rpath,$ORIGIN", "-Wl,--no-as-needed"]
        _run(cmd)
        tmp.replace(out)
    return out


def build(force: bool = False) -> None:
    build_kernels(force)
    build_torch_ops(force)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args()
    try:
        build(args.force)
    except subprocess.CalledProcessError as e:
        sys.exit(e.returncode)
