"""Backbone projection GEMMs on the HIP GEMM (gemm.hip `triad_gemm_bf16_bias`) instead of a vendor
BLAS: F.linear under autocast (bf16 operands, fp32 accumulation, bias added before the one bf16
rounding) and its input gradient dy . W. Measured on the c3 shapes at 790-940 TFLOP/s against
rocBLAS's 300-790 (tools/gemm_backend_probe.py); hipBLASLt is not used (triad_amd/blas.py).
Shapes the kernel does not tile (rows not a multiple of 128 -- small batches --, widths not a
multiple of 128, contractions not a multiple of 64) go to torch, i.e. rocBLAS."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import call, ptr, stream_ptr

_BF = torch.bfloat16
def _ok(M, N, K):
    return M > 0 and M % 128 == 0 and N % 128 == 0 and K % 64 == 0


def _rows(x):
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(1) != 1 or x2.stride(0) != x2.shape[1]:
        x2 = x2.contiguous()
    return x2


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, meta=None) -> torch.Tensor:
    """bf16 F.linear(x, w, b) with autocast's numerics; x [..., K], w [N][K] -> [..., N]."""
    xb = x if x.dtype == _BF else x.to(_BF)
    wb = w if w.dtype == _BF else w.to(_BF)
    K = xb.shape[-1]
    N = wb.shape[0]
    x2 = _rows(xb)
    M = x2.shape[0]
    if not (x2.is_cuda and _ok(M, N, K)):
        return F.linear(xb, wb, None if b is None else b.to(_BF))
    wc = wb if wb.is_contiguous() else wb.contiguous()
    # the bias as autocast holds it (bf16), read by the epilogue as is: no cast launch when the
    # model's bias already is bf16 (the trainer's shadowed Linear layers, the projection heads)
    bias = None if b is None else b.detach().to(_BF).contiguous()
    out = torch.empty(M, N, dtype=_BF, device=x2.device)
    call("triad_gemm_bf16_bias_bf16", ptr(x2), K, 1, ptr(wc), K, 1, M, N, K, ptr(bias), ptr(out), N,
         stream_ptr(x2.device), meta=meta or dict(backbone=True, flops=2.0 * M * N * K))
    return out.view(*xb.shape[:-1], N)


def mm(a: torch.Tensor, b: torch.Tensor, meta=None) -> torch.Tensor:
    """bf16 a @ b for a [M][K], b [K][N] (the input gradient dy . W of a linear layer)."""
    ab = a if a.dtype == _BF else a.to(_BF)
    bb = b if b.dtype == _BF else b.to(_BF)
    M, K = ab.shape
    N = bb.shape[1]
    if not (ab.is_cuda and _ok(M, N, K)):
        return ab @ bb
    a2 = ab if ab.is_contiguous() else ab.contiguous()
    b2 = bb if bb.is_contiguous() else bb.contiguous()
    out = torch.empty(M, N, dtype=_BF, device=a2.device)
    call("triad_gemm_bf16_bias", ptr(a2), K, 1, ptr(b2), N, 0, M, N, K, None, ptr(out), N, stream_ptr(a2.device),
         meta=meta or dict(backbone=True, flops=2.0 * M * N * K))
    return out
