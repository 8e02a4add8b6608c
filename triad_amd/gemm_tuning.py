"""Library-GEMM solution choices for the backbone forward / input-gradient GEMMs.

The HuBERT / DINOv2 / DistilBERT projections stay on hipBLASLt / rocBLAS (they run those shapes
at ~1 PFLOP/s). Their default heuristic is not always the fastest solution on
MI355X: PyTorch's TunableOp searched every hipBLASLt and rocBLAS solution for each shape of the
c3 step (tools/tunable_probe.py: 147.1 -> 143.1 ms per step on one box) and the winners are
kept in tuning/tunableop_gfx950_c3.csv. Loading it makes the same library calls pick those
solutions (same math: bf16 operands, fp32 accumulation); shapes outside the file, or a
different PyTorch / hipBLASLt / arch (the file's validator lines), keep the default. No tuning
runs here. TRIAD_TUNABLEOP=0 turns it off.
"""
from __future__ import annotations

import os
import tempfile

import torch

TUNING_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "tunableop_gfx950_c3.csv")
_loaded = False


def load_gemm_tuning(device=None) -> bool:
    """Enable TunableOp in lookup-only mode with the committed gfx950 results (idempotent)."""
    global _loaded
    if _loaded:
        return True
    if os.environ.get("TRIAD_TUNABLEOP", "1") == "0" or not os.path.exists(TUNING_FILE):
        return False
    if not torch.cuda.is_available():
        return False
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda" or "gfx950" not in getattr(torch.cuda.get_device_properties(dev), "gcnArchName", ""):
        return False
    from . import blas
    if blas.configure() == "rocblas":
        # the committed choices are hipBLASLt solution indices (also the "Rocblas" ones: rocBLAS
        # forwarded them to hipBLASLt), i.e. the stream-K kernels triad_amd/blas.py avoids
        return False
    path = TUNING_FILE
    tun = torch.cuda.tunable
    # torch writes its results file at exit: point that at a per-process scratch path so the
    # committed file is never rewritten (and ranks never write one file together)
    tun.set_filename(os.path.join(tempfile.gettempdir(), f"triad_tunableop_{os.getpid()}.csv"))
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    ok = bool(tun.read_file(path))
    if not ok:
        tun.enable(False)
        return False
    _loaded = True
    return True
