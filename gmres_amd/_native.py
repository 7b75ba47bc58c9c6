"""ctypes bindings of the in-tree native libraries.

libgmres_hip.so   -- HIP kernels + C-ABI (include/gmres_hip.h)
libgmres_fhost.so -- Fortran host drivers (gmres_amd/fortran/gmres_hip.f90)

There is no fallback: if a library is missing the import of the solver API
raises, so a GPU run can never silently execute anything but the HIP path.
"""
from __future__ import annotations

import ctypes
import os
import sys
import re

PKG = os.path.dirname(os.path.abspath(__file__))
# GK_LIB_DIR: an A/B build of both libraries (gmres_amd/build.py build_variant);
# the default is the in-tree build.
LIB_DIR = os.environ.get("GK_LIB_DIR") or os.path.join(PKG, "lib")
HIP_SO = os.path.join(LIB_DIR, "libgmres_hip.so")
FHOST_SO = os.path.join(LIB_DIR, "libgmres_fhost.so")
HEADER = os.path.join(os.path.dirname(PKG), "include", "gmres_hip.h")

GK_OK = 0
GK_ERR_COMM = -6
GK_TUNE_PROJ_NT = 0
GK_TUNE_STENCIL_BLOCKS = 2
GK_TUNE_SR_BLOCKS = 28
GK_TUNE_SR_TWO_LEVEL = 29
GK_TUNE_XCHG_TIMEOUT_MS = 7
GK_TUNE_RES, GK_TUNE_RES_R2, GK_TUNE_RES_SHARE, GK_TUNE_RES_TIMEOUT_MS = 8, 9, 10, 11
GK_TUNE_VERR_ORDER = 14
GK_TUNE_HH_FUSE = 15
GK_TUNE_CHEB_STEN = 16
GK_TUNE_SPIN_WAIT = 18
GK_TUNE_GRAPH = 19
GK_TUNE_RES_QDEF = 20
GK_TUNE_RES_PC = 21
GK_TUNE_RES_FOLD = 22
GK_TUNE_RES_BLOCK = 23
GK_TUNE_WATCHDOG_MS = 24
GK_TUNE_HH_NORM_ORDER = 25
GK_TUNE_RES_PF = 27
GK_PREC_IDENTITY, GK_PREC_CBPR2, GK_PREC_CHEB = 0, 1, 2
(GK_KID_PROJ, GK_KID_STENCIL, GK_KID_SCALE, GK_KID_UPDATE, GK_KID_COMM, GK_KID_OTHER, GK_KID_RES, GK_KID_PREC,
 GK_KID_HALO, GK_KID_GRAPH) = range(10)
# short-recurrence passes (GK_KID_SR + pass kind, gmres_amd/csrc/gk_sr.hpp)
GK_KID_SR = 10
SR_PASS_NAMES = ["sr_cg_p", "sr_cg_x", "sr_cg_z", "sr_bi_p", "sr_bi_pc", "sr_bi_s", "sr_bi_sc", "sr_st1", "sr_st2",
                 "sr_bi_x", "sr_bi_pe", "sr_bi_se", "sr_dot", "sr_cg_xz", "sr_bi_pz", "sr_bi_sz"]
KID_NAMES = ["proj", "stencil", "scale", "update", "comm", "other", "res", "prec", "halo", "graph"] + SR_PASS_NAMES
GK_SR_PCG, GK_SR_BICGSTAB = 0, 1
COMM_KINDS = {0: None, 1: "rccl", 2: "local-group", 3: "xgmi-device-exchange"}
# resident-step variants (gk_res_info / gk_res_plan_query)
RES_VARIANTS = {0: None, 1: "prefetch", 2: "pairs", 3: "pairs+lds", 4: "w-only", 5: "w+column", 6: "blocked"}
RES_INFO_KEYS = ["variant", "G", "r2", "l2", "pf", "cw", "wo", "nt", "r2e", "l2e", "lds", "nres2", "unused12", "cheb_sten", "wt", "blk"]

c_int, c_double, c_ll, c_vp = ctypes.c_int, ctypes.c_double, ctypes.c_longlong, ctypes.c_void_p
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)

_hip = None
_fhost = None


class GkError(RuntimeError):
    pass


def header_symbols() -> list[str]:
    """Every function the C-ABI header declares."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(gk_\w+)\s*\(", txt, re.M)))


_SIGS = {
    "gk_last_error": (ctypes.c_char_p, []),
    "gk_version": (c_int, []),
    "gk_runtime_info": (c_int, [_ip, _ip, _ip, ctypes.c_char_p, ctypes.c_char_p, c_int]),
    "gk_create": (c_int, [c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_vp)]),
    "gk_destroy": (c_int, [c_vp]),
    "gk_comm_unique_id": (c_int, [ctypes.c_char_p]),
    "gk_comm_init": (c_int, [c_vp, c_int, c_int, c_int, ctypes.c_char_p]),
    "gk_local_size": (c_int, [c_vp, ctypes.POINTER(c_ll)]),
    "gk_comm_info": (c_int, [c_vp, _ip, _ip]),
    "gk_peer_info": (c_int, [c_int, c_int, _ip, _ip, _ip]),
    "gk_comm_latency": (c_int, [c_vp, c_int, _dp, _dp]),
    "gk_group_create": (c_int, [c_int, ctypes.POINTER(c_vp)]),
    "gk_group_destroy": (c_int, [c_vp]),
    "gk_comm_init_local": (c_int, [c_vp, c_vp, c_int, c_int]),
    "gk_comm_init_xgmi": (c_int, [c_vp, c_int, c_int, c_int]),
    "gk_xchg_handle": (c_int, [c_vp, ctypes.c_char_p]),
    "gk_xchg_open": (c_int, [c_vp, ctypes.c_char_p]),
    "gk_xchg_local": (c_int, [c_vp]),
    "gk_xchg_enable": (c_int, [c_vp, c_int]),
    "gk_xchg_selftest": (c_int, [c_vp, c_int]),
    "gk_set_precond": (c_int, [c_vp, c_int, _dp, c_int, c_int]),
    "gk_set_rhs": (c_int, [c_vp, _dp]),
    "gk_set_rhs_ones": (c_int, [c_vp]),
    "gk_rhs_norm": (c_int, [c_vp, _dp]),
    "gk_zero_x": (c_int, [c_vp]),
    "gk_get_x": (c_int, [c_vp, _dp]),
    "gk_get_basis": (c_int, [c_vp, c_int, c_int, _dp]),
    "gk_set_x": (c_int, [c_vp, _dp]),
    "gk_apply": (c_int, [c_vp, c_int, _dp, _dp]),
    "gk_true_residual": (c_int, [c_vp, _dp]),
    "gk_mgs_cycle_start": (c_int, [c_vp, _dp]),
    "gk_mgs_step": (c_int, [c_vp, c_int, _dp]),
    "gk_mgs_step_async": (c_int, [c_vp, c_int]),
    "gk_mgs_step_wait": (c_int, [c_vp, c_int, _dp]),
    "gk_update_x": (c_int, [c_vp, _dp, c_int]),
    "gk_mgs_verr": (c_int, [c_vp, c_int, c_int, _dp]),
    "gk_hh_cycle_start": (c_int, [c_vp, c_int, _dp]),
    "gk_hh_step": (c_int, [c_vp, c_int, c_int, _dp]),
    "gk_hh_step_async": (c_int, [c_vp, c_int, c_int]),
    "gk_hh_step_wait": (c_int, [c_vp, c_int, _dp]),
    "gk_hh_update_x": (c_int, [c_vp, _dp, c_int]),
    "gk_hh_verr": (c_int, [c_vp, c_int, _dp]),
    "gk_profile_enable": (c_int, [c_vp, c_int]),
    "gk_profile_reset": (c_int, [c_vp]),
    "gk_profile_read": (c_int, [c_vp, c_int, _dp, ctypes.POINTER(c_ll)]),
    "gk_sync": (c_int, [c_vp]),
    "gk_debug_hold_stream": (c_int, [c_vp, c_int]),
    "gk_profile_res_wg": (c_int, [c_vp, c_int, _dp, _dp, c_int, _ip]),
    "gk_profile_res_trace": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_int, c_int, _ip, _ip, _dp]),
    "gk_profile_res_split": (c_int, [c_vp, c_int, c_int, _dp, _dp, _dp, ctypes.POINTER(c_ll)]),
    "gk_set_tuning": (c_int, [c_vp, c_int, c_int]),
    "gk_res_plan_query": (c_int, [c_ll, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_ll)]),
    "gk_res_info": (c_int, [c_vp, c_int, ctypes.POINTER(c_ll)]),
    "gk_lanczos_bounds": (c_int, [c_vp, c_int, _dp, _dp]),
    "gk_vec_count": (c_int, [c_vp, _ip]),
    "gk_vec_apply": (c_int, [c_vp, c_int, c_int, c_int]),
    "gk_vec_dot": (c_int, [c_vp, c_int, c_int, _dp]),
    "gk_vec_lincomb": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_double, c_double]),
    "gk_sr_start": (c_int, [c_vp, c_int, c_double, c_int]),
    "gk_sr_iterate": (c_int, [c_vp, c_int]),
    "gk_sr_status": (c_int, [c_vp, c_int, _ip, _ip, _dp]),
    "gk_sr_history": (c_int, [c_vp, _dp, c_int]),
    "gk_poisson5": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gk_precond_apply": (c_int, [c_int, c_int, _dp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "gk_mgs_project": (c_int, [c_ll, c_vp, c_vp, c_vp, c_vp]),
    "gk_dot": (c_int, [c_ll, c_vp, c_vp, c_vp, c_vp]),
}

_FSIGS = {
    "pcg_hip_run": (c_int, [c_vp, c_double, _ip, _dp, c_int, _dp]),
    "pbicgstab_hip_run": (c_int, [c_vp, c_double, _ip, _dp, c_int, _dp]),
    "sr_hip_run_seq": (c_int, [c_vp, c_int, c_double, _ip, _dp, c_int, _dp]),
    "gmres_mgsr_hip_run": (c_int, [c_vp, c_int, c_double, c_int, c_int, _dp, _dp, _dp, _ip, _ip, c_int, c_int,
                                   _dp, _dp, _ip, c_int]),
    "gmres_hh_hip_run": (c_int, [c_vp, c_int, c_double, c_int, c_int, c_int, _dp, _dp, _dp, _ip, _ip, c_int,
                                 c_int, _dp, _dp, _ip, c_int]),
}


class _TorchAfterNative:
    """Import guard, installed once this library runs on /opt/rocm's HIP runtime
    in a process that had not imported torch: torch bundles its own
    libamdhip64 / libhsa-runtime64 / librccl and loads them by path, so
    importing it now would put a second HIP runtime into the process (measured:
    the process aborts at exit, "double free or corruption").  Fail at the
    import instead, with the remedy.  A probe (importlib.util.find_spec) is
    answered as without the guard -- torch's real spec, or None -- and only
    loading the module raises: optional-dependency checks elsewhere keep working."""

    def find_spec(self, name, path=None, target=None):
        if name != "torch":
            return None
        import importlib.machinery
        import importlib.util

        real = importlib.machinery.PathFinder.find_spec(name, path)
        if real is None:
            return None
        return importlib.util.spec_from_loader(name, _RefuseTorchLoader(), origin=real.origin)


class _RefuseTorchLoader:
    def create_module(self, spec):
        raise ImportError("gmres_amd already runs on " + (runtime_paths().get("hip") or "/opt/rocm's HIP runtime")
                          + "; importing torch now would load torch's bundled HIP runtime as a second one. "
                            "Import torch before gmres_amd's first native call (then torch's runtime is "
                            "used), or keep this process torch-free.")

    def exec_module(self, module):  # not reached: create_module raises
        raise ImportError("torch import refused")


def runtime_paths() -> dict:
    """The HIP / RCCL / HSA libraries this process has mapped (/proc/self/maps)."""
    out = {}
    try:
        for line in open("/proc/self/maps"):
            f = line.split()[-1] if len(line.split()) >= 6 else ""
            for key, stem in (("hip", "libamdhip64.so"), ("rccl", "librccl.so"), ("hsa", "libhsa-runtime64.so")):
                if stem in os.path.basename(f):
                    out.setdefault(key, f)
    except OSError:
        pass
    return out


def _one_hip_runtime() -> None:
    """One HIP runtime per process.  The product runs on the runtime it was
    built against (/opt/rocm, the NEEDED entries of libgmres_hip.so) and never
    imports torch.  If the caller imported torch first, torch's bundled
    runtime is already mapped and satisfies this library's sonames (one
    runtime: torch's; gk_runtime_info / runtime_paths() say which).  If not,
    a later `import torch` is refused (_TorchAfterNative).  GK_TORCH_FIRST=1
    restores the rounds-1..3 behaviour: import torch here, before the load."""
    if "torch" in sys.modules:
        return
    if os.environ.get("GK_TORCH_FIRST") == "1":
        try:
            import torch  # noqa: F401
            return
        except ImportError:
            pass
    if not any(isinstance(f, _TorchAfterNative) for f in sys.meta_path):
        sys.meta_path.insert(0, _TorchAfterNative())


def _load(path: str, what: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise GkError(f"{what} not built at {path}: run `python -m gmres_amd.build` "
                      "(or __graft_entry__.build()); there is no CPU fallback")
    _one_hip_runtime()
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def hip() -> ctypes.CDLL:
    global _hip
    if _hip is None:
        L = _load(HIP_SO, "libgmres_hip.so")
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _hip = L
    return _hip


def fhost() -> ctypes.CDLL:
    global _fhost
    if _fhost is None:
        hip()
        L = _load(FHOST_SO, "libgmres_fhost.so")
        for name, (res, args) in _FSIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _fhost = L
    return _fhost


def peer_info(device: int, peer: int) -> dict:
    """gk_peer_info: peer access and the link between two devices of the node."""
    a, t, h = c_int(), c_int(), c_int()
    check(hip().gk_peer_info(int(device), int(peer), ctypes.byref(a), ctypes.byref(t), ctypes.byref(h)),
          "gk_peer_info")
    return {"device": int(device), "peer": int(peer), "can_access_peer": bool(a.value),
            "link_type": {4: "xgmi", 2: "pcie"}.get(t.value, t.value), "hops": h.value}


def runtime_info() -> dict:
    """The runtime the product is running on: HIP runtime / driver and RCCL
    versions (gk_runtime_info) and the library files mapped for them."""
    a, b, c = c_int(), c_int(), c_int()
    hp, rp = ctypes.create_string_buffer(512), ctypes.create_string_buffer(512)
    check(hip().gk_runtime_info(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), hp, rp, 512), "gk_runtime_info")
    maps = runtime_paths()
    return {"hip_runtime_version": a.value, "hip_driver_version": b.value, "rccl_version": c.value,
            "libamdhip64": hp.value.decode() or maps.get("hip"), "librccl": rp.value.decode() or maps.get("rccl"),
            "libhsa_runtime64": maps.get("hsa"), "torch_imported": "torch" in sys.modules}


def last_error() -> str:
    msg = hip().gk_last_error()
    return msg.decode() if msg else ""


def check(status: int, what: str) -> None:
    if status != GK_OK:
        msg = hip().gk_last_error()
        raise GkError(f"{what} failed (status {status}): {msg.decode() if msg else ''}")
