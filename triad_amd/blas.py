"""Which vendor BLAS serves the plain library GEMMs (backbone projections through torch, the
projection heads' input-side GEMMs).

rocBLAS, not hipBLASLt. hipBLASLt's gfx950 GEMM kernels are stream-K kernels (the "SK3"
solutions, its default choices for the c3 shapes): a workgroup that owns the start of a split
tile spins on a flag (`label_SK_Fixup`: scalar load, compare, branch back) until the workgroups
holding the tile's later k-range publish their partials, and flags are reset with scalar-cache
stores. The step runs the three backbones on concurrent HIP streams; two stream-K GEMMs resident
at once, each spinning for workgroups that cannot be dispatched while the other's spinners hold
the CUs, can deadlock -- the step hung once in ~16 bench runs with hipBLASLt --
and this pool forbids GPU code that writes through the scalar data cache. rocBLAS's gfx950
Tensile kernels contain neither (disassembly of its bf16 libraries: no `label_SK_Fixup`, no
scalar stores; checked with llvm-objdump when this was written).
"""
from __future__ import annotations

import os

import torch

LIBRARY = "rocblas"   # "rocblas" | "hipblaslt"
_configured = None


def configure(warn_if_late: bool = True) -> str:
    """Point PyTorch's BLAS dispatch at LIBRARY (process-wide, idempotent).

    warn_if_late: warn when the HIP runtime is already up (a GEMM MAY have fixed the switches).
    TriadTrainer passes False: a model moved to the GPU has initialised HIP without running a
    GEMM, so the warning would fire on every ordinary construction."""
    global _configured
    if _configured != LIBRARY:
        if warn_if_late and torch.cuda.is_initialized():
            # the two environment switches are read once (first addmm / first rocBLAS handle): a
            # GEMM that ran before this call has fixed them already
            import warnings
            warnings.warn("triad_amd.blas.configure() called after the HIP runtime was initialised: if "
                          "a GEMM already ran, DISABLE_ADDMM_CUDA_LT / ROCBLAS_USE_HIPBLASLT no longer take "
                          "effect in this process (call configure() first)", RuntimeWarning, stacklevel=2)
        torch.backends.cuda.preferred_blas_library("cublas" if LIBRARY == "rocblas" else "cublaslt")
        # addmm with a bias vector (every nn.Linear under autocast) takes PyTorch's Lt path
        # (hipBLASLt gemm_and_bias) whatever the preferred library, unless this is set; PyTorch
        # reads it once, at the first addmm, so it is set at import (before any GEMM runs)
        # and rocBLAS itself forwards gfx950 GEMMs to hipBLASLt unless ROCBLAS_USE_HIPBLASLT=0
        # (read when its first handle is created)
        if LIBRARY == "rocblas":
            os.environ["DISABLE_ADDMM_CUDA_LT"] = "1"
            os.environ["ROCBLAS_USE_HIPBLASLT"] = "0"
        else:
            os.environ.pop("DISABLE_ADDMM_CUDA_LT", None)
            os.environ.pop("ROCBLAS_USE_HIPBLASLT", None)
        _configured = LIBRARY
    return LIBRARY
