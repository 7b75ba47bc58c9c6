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

# Translation units compiled in parallel: the C-ABI + every kernel but the
# Chebyshev pass, and the Chebyshev pass split by level count (its many
# unrolled instantiations dominate the build time).
HIP_SOURCES = [os.path.join(CSRC, "gk_api.hip"), os.path.join(CSRC, "gk_cheb.hip"), os.path.join(CSRC, "gk_blk.hip")]
# (source, extra defines, object name): the Chebyshev pass in GK_CF_PARTS parts
GK_CF_PARTS = 4
HIP_UNITS = ([(HIP_SOURCES[0], [], "gk_api.o")] + [(HIP_SOURCES[1], [f"GK_CF_PART={p}"], f"gk_cheb{p}.o")
                                                    for p in range(GK_CF_PARTS)]
             + [(HIP_SOURCES[2], [], "gk_blk.o")])
HIP_HEADERS = [os.path.join(CSRC, h) for h in ("gk_common.hpp", "gk_kernels.hpp", "gk_cheb.hpp", "gk_res.hpp",
                                                "gk_blk.hpp", "gk_sr.hpp")]
HIP_DEPS = HIP_SOURCES + HIP_HEADERS + [os.path.join(ROOT, "include", "gmres_hip.h")]
HIP_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall"]
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


def _scratch_kernels(remarks: str, name: str) -> list[str]:
    """Kernels named like `name` whose resource-usage remark reports scratch."""
    bad, fn = [], None
    for line in remarks.splitlines():
        if "Function Name:" in line:
            fn = line.split("Function Name:", 1)[1].split()[0]
        elif "ScratchSize [bytes/lane]:" in line and fn and name in fn:
            if int(line.split("ScratchSize [bytes/lane]:", 1)[1].split()[0]) > 0:
                bad.append(fn)
    return bad


def _compile_link(so: str, defines: list[str]) -> None:
    """Compile the HIP translation units in parallel into objects beside `so`,
    then link them into the shared library.  The Chebyshev pass and the resident
    step kernels must not spill registers to scratch (gk_cheb.hip refuses such a
    pass at run time; a spilled resident kernel holds w in scratch memory): the
    build fails here, naming them."""
    objs, procs = [], []
    for src, unit_defs, oname in HIP_UNITS:
        obj = os.path.join(os.path.dirname(so), oname)
        cmd = [hipcc(), *HIP_FLAGS, *[f"-D{x}" for x in defines + unit_defs], "-c", src, "-o", obj,
               "-Rpass-analysis=kernel-resource-usage"]
        print("+", " ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd, stderr=subprocess.PIPE, text=True))
        objs.append(obj)
    bad = []
    for p in procs:
        err = p.communicate()[1]
        sys.stderr.write("".join(l + "\n" for l in err.splitlines() if "warning:" in l or "error" in l))
        for name in ("k_cheb_fused", "k_mgs_wpc", "k_mgs_wres", "k_mgs_res", "k_mgs_blk"):
            bad += _scratch_kernels(err, name)
    if any(p.returncode for p in procs):
        raise subprocess.CalledProcessError(max(p.returncode for p in procs), "hipcc")
    if bad:
        raise RuntimeError(f"kernels built with a register spill to scratch (refused): {bad}")
    _run([hipcc(), "--offload-arch=gfx950", "-fPIC", "-shared", *objs, "-o", so, "-lrccl"])
    for o in objs:
        os.remove(o)


def build_hip(force: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    if force or _newer(HIP_SO, HIP_DEPS):
        _compile_link(HIP_SO, [])
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
    _compile_link(so, defines)
    build_fortran()
    shutil.copy2(FHOST_SO, os.path.join(d, "libgmres_fhost.so"))
    return d


def build_all(force: bool = False) -> None:
    build_hip(force)
    build_fortran(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
