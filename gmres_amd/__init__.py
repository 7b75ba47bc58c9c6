"""gmres_amd -- MI355X-native GMRES(m) inner cycle for matrix-free stencil operators.

Drop-in for the Arnoldi cycle of AlexanderGSC/gmres (src/gmres_mgsr.f90,
src/gmres_hh.f90) behind its stencil_vector / precond plug-in interface
(src/interfaces.f90): HIP kernels for gfx950 (gmres_amd/csrc), a C-ABI
(include/gmres_hip.h), and a Fortran host (gmres_amd/fortran) that keeps the
restart loop and the Givens rotations.
"""
from ._native import GkError, peer_info, runtime_info
from .solver import (MGSR_MF, MGSR_OMP, PREC, Context, LocalGroup, SolveResult, gmres_hh, gmres_mgsr, pbicgstab,
                     SrSolve, pcg, res_plan_query, slab_partition)

__all__ = ["GkError", "Context", "LocalGroup", "SolveResult", "gmres_mgsr", "gmres_hh", "slab_partition", "pcg", "pbicgstab", "MGSR_OMP", "MGSR_MF", "PREC",
           "res_plan_query", "runtime_info", "SrSolve", "peer_info"]
