"""Build the native parts in-tree (gfx950 only).

  gmres_amd/lib/libgmres_hip.so     HIP kernels + C-ABI (include/gmres_hip.h), hipcc
  gmres_amd/lib/libgmres_fhost.so   Fortran host (restart loop, Givens), amdflang
  gmres_amd/lib/test_mfp_hip        Fortran driver mirroring tests/test_poisson_mf.f90
  gmres_amd/lib/sweep_hip           Fortran sweep drivers (utils.f90 table layout)

hipcc cross-compiles gfx950 code objects without a GPU, so this runs in the
build container; the .so files travel to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "lib")
CSRC = os.path.join(PKG, "csrc")
FSRC = os.path.join(PKG, "fortran")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

HIP_SO = os.path.join(LIB, "libgmres_hip.so")
FHOST_SO = os.path.join(LIB, "libgmres_fhost.so")
DRIVER = os.path.join(LIB, "test_mfp_hip")

HIP_SOURCES = [os.path.join(CSRC, "gk_api.hip")]
HIP_DEPS = HIP_SOURCES + [os.path.join(CSRC, "gk_kernels.hpp"), os.path.join(ROOT, "include", "gmres_hip.h")]
F_SOURCES = [os.path.join(FSRC, "gmres_hip.f90")]


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str], cwd: str | None = None) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=cwd)


def hipcc() -> str:
    for c in (os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc") or ""):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def flang() -> str:
    for c in (os.path.join(ROCM, "lib", "llvm", "bin", "flang"), os.path.join(ROCM, "bin", "amdflang"),
              shutil.which("flang") or ""):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("amdflang not found")


def build_hip(force: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    if force or _newer(HIP_SO, HIP_DEPS):
        _run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-ffp-contract=off", "-Wall", *HIP_SOURCES, "-o", HIP_SO, "-lrccl"])
    return HIP_SO


def build_fortran(force: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    moddir = os.path.join(LIB, "mod")
    os.makedirs(moddir, exist_ok=True)
    common = ["-O2", "-ffp-contract=off", "-fPIC", f"-J{moddir}"]
    link = [f"-L{LIB}", "-lgmres_hip", "-Wl,-rpath,$ORIGIN"]
    if force or _newer(FHOST_SO, F_SOURCES + [HIP_SO]):
        _run([flang(), *common, "-shared", *F_SOURCES, "-o", FHOST_SO, *link])
    for name in ("test_mfp_hip", "sweep_hip"):
        src = os.path.join(FSRC, name + ".f90")
        exe = os.path.join(LIB, name)
        if force or _newer(exe, [src, FHOST_SO]):
            _run([flang(), *common, src, "-o", exe, f"-L{LIB}", "-lgmres_fhost", "-lgmres_hip", "-Wl,-rpath,$ORIGIN"])
    return FHOST_SO


def build_variant(name: str, defines: list[str]) -> str:
    """An A/B build: libgmres_hip.so compiled with extra -D macros (kernel
    geometry knobs such as GK_RES_RW / GK_RES_WB) plus a copy of the Fortran
    host beside it (its $ORIGIN rpath then binds that build); select it with
    GK_LIB_DIR=<returned dir>."""
    d = os.path.join(LIB, "variants", name)
    os.makedirs(d, exist_ok=True)
    so = os.path.join(d, "libgmres_hip.so")
    _run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
          *[f"-D{x}" for x in defines], *HIP_SOURCES, "-o", so, "-lrccl"])
    build_fortran()
    shutil.copy2(FHOST_SO, os.path.join(d, "libgmres_fhost.so"))
    return d


def build_all(force: bool = False) -> None:
    build_hip(force)
    build_fortran(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
