"""Backbone nn.Linear layers with the weight gradient on the HIP split-K GEMM.

The reference trains HuBERT and DistilBERT end to end after `unfreeze_*_step` (SajayR/TRIAD
train.py:527-548; model.py:29-30, 79-80) under bf16 autocast (model.py:483, 603). Their
weight gradients dW = dy^T x contract over all B*N tokens (50,944 for HuBERT at c3) into a
768 x 768 .. 3,072 x 768 output: too few output tiles for the library GEMM's heuristics, which
reach 230-620 TFLOP/s on these shapes on MI355X (tools/dw_variants.py). The split-K MFMA GEMM of
csrc/gemm.hip (fp32 slabs over token ranges, one bf16 rounding at the end) runs them 1.1-2.4x
faster (c3 step: 1108 -> 1140 triples/s). Forward and dX stay on torch (hipBLASLt runs those shapes at ~1 PFLOP/s).

Numerics equal autocast's F.linear: bf16 operands, fp32 accumulation, bf16 dX / dW / db.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import call, ptr, stream_ptr

MIN_TOKENS = 4096  # DistilBERT at B=256 (8,192 tokens) still gains 1.1-1.8x


def _splits(M, out_f, in_f):
    """Token-range splits: 8 for the 36-144-tile outputs at 50 K tokens, ~2 K tokens per split
    below that (measured, tools/dw_variants.py)."""
    tiles = (out_f // 128) * (in_f // 128)
    return min(8 if tiles <= 160 else 4, max(2, M // 2048))


def weight_grad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """dW = dy2^T x2 (bf16 [O][K]) for dy2 [M][O], x2 [M][K] bf16 row-major, M % 64 == 0."""
    M, O = dy2.shape
    K = x2.shape[1]
    sp = _splits(M, O, K)
    slabs = torch.empty(sp * O * K, dtype=torch.float32, device=dy2.device)
    dw = torch.empty(O, K, dtype=torch.bfloat16, device=dy2.device)
    _lib.META = dict(backbone=True)
    call("triad_gemm_bf16_splitk", ptr(dy2), dy2.stride(0), 0, ptr(x2), x2.stride(0), 0, O, K, M, sp, None,
         ptr(slabs), ptr(dw), 1, stream_ptr(dy2.device))
    return dw


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        xb = x.to(torch.bfloat16)
        wb = w.to(torch.bfloat16)
        bb = None if b is None else b.to(torch.bfloat16)
        ctx.save_for_backward(xb, wb)
        ctx.meta = (x.dtype, w.dtype, None if b is None else b.dtype)
        return F.linear(xb, wb, bb)

    @staticmethod
    def backward(ctx, dy):
        xb, wb = ctx.saved_tensors
        x_dtype, w_dtype, b_dtype = ctx.meta
        O, K = wb.shape
        dy2 = dy.reshape(-1, O).to(torch.bfloat16).contiguous()
        x2 = xb.reshape(-1, K)
        if x2.stride(1) != 1 or x2.stride(0) != K:
            x2 = x2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dy2, wb).view(*xb.shape).to(x_dtype)
        if ctx.needs_input_grad[1]:
            dw = weight_grad(dy2, x2).to(w_dtype)
        if b_dtype is not None and ctx.needs_input_grad[2]:
            from .ops import colsum
            db = colsum(dy2, torch.bfloat16 if b_dtype == torch.bfloat16 else torch.float32).to(b_dtype)
        return dx, dw, db


def _eligible(mod: nn.Linear, x: torch.Tensor) -> bool:
    if not (x.is_cuda and mod.weight.requires_grad and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    M = x.numel() // max(1, x.shape[-1])
    return M >= MIN_TOKENS and M % 64 == 0 and mod.in_features % 128 == 0 and mod.out_features % 128 == 0


class TriadLinear(nn.Linear):
    """nn.Linear whose training-mode weight gradient runs on the HIP split-K GEMM (same
    parameters and state-dict keys; any other case is nn.Linear.forward)."""

    def forward(self, x):
        if _eligible(self, x):
            return _LinearFn.apply(x, self.weight, self.bias)
        return super().forward(x)


def install_fast_linear(root: nn.Module) -> nn.Module:
    """Re-class every nn.Linear under `root` as TriadLinear (in place); returns `root`."""
    for mod in root.modules():
        if type(mod) is nn.Linear:
            mod.__class__ = TriadLinear
    return root
