"""Host-side checks that need no GPU: the C-ABI library and the Fortran host
library load and export every declared symbol, argument validation fails
loudly, the slab decomposition is sound."""
import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def built():
    from gmres_amd import build

    build.build_all()
    from gmres_amd import _native

    return _native


def test_cabi_exports_every_header_symbol(built):
    L = built.hip()
    syms = built.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert L.gk_version() >= 1


def test_cabi_signatures_cover_header(built):
    """Every header function has a ctypes signature in _native (and vice versa)."""
    assert sorted(built._SIGS) == built.header_symbols()


def test_fortran_host_exports(built):
    F = built.fhost()
    for s in ("gmres_mgsr_hip_run", "gmres_hh_hip_run"):
        assert hasattr(F, s)
    out = subprocess.run(["nm", "-D", built.FHOST_SO], capture_output=True, text=True).stdout
    # the drop-in module procedures exist (Fortran-mangled)
    for name in ("gmres_mgsr_hip", "gmres_hh_hip", "gmres_hh_prec_hip", "hip_poisson5", "hip_cbpr2"):
        assert name in out, name


def test_cabi_rejects_bad_arguments(built):
    L = built.hip()
    h = ctypes.c_void_p()
    assert L.gk_create(0, 1, 0, 1, 10, ctypes.byref(h)) == -1  # N < 2
    assert b"bad shape" in L.gk_last_error()
    assert L.gk_create(0, 16, 10, 10, 10, ctypes.byref(h)) == -1  # slab beyond the grid
    assert L.gk_mgs_step(None, 1, None) == -1
    assert L.gk_poisson5(1, 1, None, None, None, None, None) == -1


def test_driver_executable_built(built):
    exe = os.path.join(ROOT, "gmres_amd", "lib", "test_mfp_hip")
    assert os.access(exe, os.X_OK)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert "usage" in out.stdout


def test_slab_partition():
    from gmres_amd import slab_partition

    for N in (5, 64, 4096, 8192):
        for R in (1, 2, 3, 4, 7, 8):
            if R > N:
                continue
            parts = slab_partition(N, R)
            assert parts[0][0] == 0
            assert sum(nl for _, nl in parts) == N
            for (a, na), (b, _) in zip(parts, parts[1:]):
                assert a + na == b
            assert max(nl for _, nl in parts) - min(nl for _, nl in parts) <= 1
    with pytest.raises(ValueError):
        slab_partition(4, 5)


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    """The product path refuses to run without the HIP library."""
    from gmres_amd import _native

    monkeypatch.setattr(_native, "HIP_SO", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_native, "_hip", None)
    with pytest.raises(_native.GkError):
        _native.hip()


def test_product_does_not_import_oracle():
    """Only tests/, __graft_entry__.smoke and bench.py's cpu_baseline may use oracle/."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "gmres_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".f90", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                for bad in ("import oracle", "from oracle", "liboracle", "gmres_oracle", "or_gmres", "or_stvec"):
                    assert bad not in txt, (f, bad)


def test_build_refuses_chebyshev_scratch_spills():
    """gmres_amd/build.py parses the resource-usage remarks of the Chebyshev
    translation units and fails the build when any k_cheb_fused instantiation
    spills registers to scratch (gk_cheb.hip refuses such kernels at run time
    too: a spilled build gave wrong results past two unrolled trips)."""
    from gmres_amd import build as b

    remarks = ("gk_cheb.hip:46:1: remark: Function Name: _ZN2gk12k_cheb_fusedILi8ELb1ELb1ELi1ELb0EEEvNS_6CFArgsE\n"
               "gk_cheb.hip:46:1: remark:     ScratchSize [bytes/lane]: 16 [-Rpass-analysis=kernel-resource-usage]\n"
               "gk_cheb.hip:46:1: remark: Function Name: _ZN2gk12k_cheb_fusedILi4ELb1ELb1ELi1ELb0EEEvNS_6CFArgsE\n"
               "gk_cheb.hip:46:1: remark:     ScratchSize [bytes/lane]: 0 [-Rpass-analysis=kernel-resource-usage]\n"
               "gk_api.hip:9:1: remark: Function Name: _ZN2gk6k_projILi0ELb1ELi2EEEvPdPKdS3_\n"
               "gk_api.hip:9:1: remark:     ScratchSize [bytes/lane]: 32 [-Rpass-analysis=kernel-resource-usage]\n")
    assert b._scratch_kernels(remarks, "k_cheb_fused") == ["_ZN2gk12k_cheb_fusedILi8ELb1ELb1ELi1ELb0EEEvNS_6CFArgsE"]
    assert [u[2] for u in b.HIP_UNITS] == (["gk_api.o"] + [f"gk_cheb{p}.o" for p in range(b.GK_CF_PARTS)]
                                           + ["gk_blk.o"])
    # the blocked-projection step's kernels (gk_blk.hip) are held to the same rule
    rb = ("gk_blk.hip:46:1: remark: Function Name: _ZN2gk9k_mgs_blkILi32ELi0ELi2ELi9ELi2ELi4ELi0ELi512EEEvNS_7ResArgsE\n"
          "gk_blk.hip:46:1: remark:     ScratchSize [bytes/lane]: 40 [-Rpass-analysis=kernel-resource-usage]\n")
    assert b._scratch_kernels(rb, "k_mgs_blk") == ["_ZN2gk9k_mgs_blkILi32ELi0ELi2ELi9ELi2ELi4ELi0ELi512EEEvNS_7ResArgsE"]


def test_torch_import_after_native_load_is_refused(built):
    """The product never imports torch; once libgmres_hip.so runs on /opt/rocm's
    HIP runtime in a torch-free process, importing torch (which would map its
    bundled runtime as a second one and abort at exit) fails at the import."""
    code = ("import importlib.util, gmres_amd._native as n; n.hip()\n"
            "print('PROBE', importlib.util.find_spec('torch') is not None)\n"  # probes answered, not refused
            "try:\n    import torch\n    print('IMPORTED')\n"
            "except ImportError as e:\n    print('REFUSED', 'second one' in str(e), 'torch' in __import__('sys').modules)\n")
    env = dict(os.environ)
    env.pop("GK_TORCH_FIRST", None)
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.split() == ["PROBE", "True", "REFUSED", "True", "False"], p.stdout
    # torch first, then the library: torch's runtime serves both (one runtime)
    code2 = "import torch, gmres_amd._native as n; n.hip(); print('OK', 'torch' in n.runtime_paths().get('hip', 'torch'))"
    p = subprocess.run([sys.executable, "-c", code2], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and p.stdout.split()[0] == "OK", (p.stdout, p.stderr[-2000:])
