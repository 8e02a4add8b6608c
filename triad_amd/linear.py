"""Backbone nn.Linear layers with the weight gradient on the HIP split-K GEMM.

The reference trains HuBERT and DistilBERT end to end after `unfreeze_*_step` (SajayR/TRIAD
train.py:527-548; model.py:29-30, 79-80) under bf16 autocast (model.py:483, 603). Their
weight gradients dW = dy^T x contract over all B*N tokens (50,944 for HuBERT at c3) into a
768 x 768 .. 3,072 x 768 output: too few output tiles for the library GEMM's heuristics, which
reach 230-620 TFLOP/s on these shapes on MI355X (round-1 A/B, profiles/r01_dw_gemm_*.log). The split-K MFMA GEMM of
csrc/gemm.hip (fp32 slabs over token ranges, one bf16 rounding at the end) runs them 1.1-2.4x
faster (c3 step: 1108 -> 1140 triples/s). Forward and dX stay on torch (hipBLASLt runs those shapes at ~1 PFLOP/s).

Numerics equal autocast's F.linear: bf16 operands, fp32 accumulation, bf16 dX / dW / db.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import gemm as hipgemm
from ._lib import call, ptr, stream_ptr



# Split-K factors measured per output-tile count on MI355X (round-1 A/B with
# TRIAD_DW_SPLITS, profiles/r01_dw_splits_{50944,8192}.log). The best factor is set by how
# tiles x splits workgroups quantise onto the CUs' slots, not by a smooth rule: e.g. 144 tiles
# run 7 splits (1,008 workgroups) 8-11 % faster than 8 (1,152) at 50,944 tokens, and 3 splits
# (432) 15-26 % faster than 4 (576) at 8,192 tokens.
_SPLITS_LONG = {36: 7, 108: 9, 144: 7}   # M >= 32,768 tokens (HuBERT at c3: 50,944)
_SPLITS_SHORT = {36: 7, 108: 4, 144: 3}  # 4,096 <= M < 16,384 (DistilBERT at c3: 8,192)


def _splits(M, out_f, in_f):
    """Token-range splits for dW: the measured table for the c3 tile counts, else 8 for the
    36-144-tile outputs at 50 K tokens and ~2 K tokens per split below that."""
    tiles = (out_f // 128) * (in_f // 128)
    table = _SPLITS_LONG if M >= 32768 else _SPLITS_SHORT if 4096 <= M < 16384 else {}
    if tiles in table:
        return table[tiles]
    return min(8 if tiles <= 160 else 4, max(2, M // 2048))


# Eight-wave 256 x 256 form for the long-token weight gradients, split counts per 256 x 256 tile
# count (tools/dw_w8_probe.py, profiles/r02_dw_w8_probe.log, 50,944 tokens: 2304 x 768 202 vs 247 us
# on the 128 x 128 table above, 768 x 768 98 vs 101, 3072 x 768 275 vs 298, 768 x 3072 284 vs 315;
# at 8,192 tokens the 128 x 128 table stays faster).
_W8_SPLITS = {27: 8, 9: 24, 36: 12}
# of those, the ones whose workgroups of one split all go to one XCD (gemm.hip tile_split, form
# flag 8; splits % 8 == 0): 768 x 768 at 50,944 tokens 99.6 -> 86.2 us, 2304 x 768 209.6 -> 200.2
# (profiles/r04_dw_xcd_ab.log; 3072 x 768 / 768 x 3072 keep 12 splits, faster than any 8k split)
_W8_XCD = {27, 9}


def _form_splits(M, out_f, in_f):
    tiles8 = (out_f // 256) * (in_f // 256) if out_f % 256 == 0 and in_f % 256 == 0 else 0
    if M >= 32768 and tiles8 in _W8_SPLITS:
        return 4 | (8 if tiles8 in _W8_XCD else 0), _W8_SPLITS[tiles8]
    return 0, _splits(M, out_f, in_f)


def weight_grad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """dW = dy2^T x2 (bf16 [O][K]) for dy2 [M][O], x2 [M][K] bf16 row-major (a token count that is
    not a multiple of the GEMM's 64-deep k step is padded with zero rows, which add nothing)."""
    M, O = dy2.shape
    K = x2.shape[1]
    if M % 64:
        Mp = (M + 63) // 64 * 64
        dy2 = torch.cat([dy2, dy2.new_zeros(Mp - M, O)])
        x2 = torch.cat([x2, x2.new_zeros(Mp - M, K)])
        M = Mp
    form, sp = _form_splits(M, O, K)
    slabs = torch.empty(sp * O * K, dtype=torch.float32, device=dy2.device)
    dw = torch.empty(O, K, dtype=torch.bfloat16, device=dy2.device)
    call("triad_gemm_bf16_splitk_form", ptr(dy2), dy2.stride(0), 0, ptr(x2), x2.stride(0), 0, O, K, M, sp, None,
         ptr(slabs), ptr(dw), 1, form, stream_ptr(dy2.device), meta=dict(backbone=True))
    return dw


# ---- weight gradients on a side stream ------------------------------------------------------
# A layer's dW does not feed the rest of the backward, so it runs on a second stream beside the
# next layers' dX GEMMs and (HBM-bound) elementwise passes. Only for bf16 (mixed-precision
# shadow) weights whose .grad is still empty: autograd then just stores the tensor (no kernel on
# the main stream reads it); the main stream waits for the side stream at the end of the
# backward pass (autograd callback), before anything can read a gradient.
_SIDE = {}
_JOIN_TASK = {}  # device index -> autograd graph task that already has a join callback queued


def _dev_index(dev) -> int:
    """The ordinal of a CUDA device given as torch.device("cuda") (index None: the current
    device) or "cuda:N". Every per-device table here is keyed by it: a trainer built with
    device="cuda" asks for the side stream under index None while the backward nodes ask under
    the tensors' index 0 -- two different streams, and the reducer's fold of a side-stream weight
    gradient then waited on the wrong one (the two-rank Mode G test's audio conv dW,
    profiles/r04_gpu_tests_modeg_nan.log)."""
    dev = torch.device(dev)
    return dev.index if dev.index is not None else torch.cuda.current_device()


def _side_stream(dev):
    i = _dev_index(dev)
    s = _SIDE.get(i)
    if s is None:
        s = _SIDE[i] = torch.cuda.Stream(device=i)
    return s


def _join(dev):
    def cb():
        torch.cuda.current_stream(dev).wait_stream(_side_stream(dev))
    return cb


_CLAIMED = {}  # device index -> (autograd graph task, ids of the weights whose dW went to the side stream)


def side_stream_ok(*ws: torch.Tensor) -> bool:
    """May this backward node compute the dW of `ws` on the side stream? Only for bf16 weights
    whose .grad is empty, inside a backward pass, and only at a weight's FIRST use in the pass:
    a weight used twice in one graph (two chunks through one layer, profiles/r03_audio_reuse_diag.log)
    has its two dW summed by autograd on the main stream as soon as the second arrives, so the
    second node makes the main stream wait for the side stream (which holds the first dW) and
    computes its dW there."""
    task = torch._C._current_graph_task_id()
    if not (SIDE_STREAM_DW and task != -1 and all(w.is_cuda and w.dtype == torch.bfloat16 and w.grad is None
                                                   for w in ws)):
        return False
    dev = ws[0].device
    di = _dev_index(dev)
    t, seen = _CLAIMED.get(di, (None, None))
    if t != task:
        seen = set()
        _CLAIMED[di] = (task, seen)
    if any(id(w) in seen for w in ws):
        if di in _SIDE:
            torch.cuda.current_stream(dev).wait_stream(_SIDE[di])
        seen.update(id(w) for w in ws)
        return False
    seen.update(id(w) for w in ws)
    return True


def on_side_stream(fn, inputs):
    """Run fn() on the device's side stream after the work queued so far; `inputs` (produced on
    the main stream) are kept alive for it, the outputs are recorded for the main stream."""
    dev = inputs[0].device
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        outs = fn()
    for t in inputs:
        t.record_stream(side)
    for o in (outs if isinstance(outs, (list, tuple)) else (outs,)):
        o.record_stream(main)
    task = torch._C._current_graph_task_id()
    if _JOIN_TASK.get(_dev_index(dev)) != task:  # once per backward pass (robust to an aborted one)
        _JOIN_TASK[_dev_index(dev)] = task
        torch.autograd.Variable._execution_engine.queue_callback(_join(dev))
    return outs


# On by default (with the modality streams; model.set_concurrent_streams / TRIAD_SIDE_STREAM_DW=0
# turn it off): safe since every bias sum reads its rows by LDS-DMA (ops.bias_grad).
SIDE_STREAM_DW = os.environ.get("TRIAD_SIDE_STREAM_DW", "1") != "0"


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        xb = x.to(torch.bfloat16)
        wb = w.to(torch.bfloat16)
        bb = None if b is None else b.to(torch.bfloat16)
        ctx.save_for_backward(xb, wb)
        ctx.meta = (x.dtype, w.dtype, None if b is None else b.dtype)
        ctx.w_ref = w
        return hipgemm.linear(xb, wb, bb)

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
            dx = hipgemm.mm(dy2, wb).view(*xb.shape).to(x_dtype)
        if ctx.needs_input_grad[1]:
            if w_dtype == torch.bfloat16 and side_stream_ok(ctx.w_ref):
                dw = on_side_stream(lambda: weight_grad(dy2, x2), (dy2, x2))
            else:
                dw = weight_grad(dy2, x2).to(w_dtype)
        if b_dtype is not None and ctx.needs_input_grad[2]:
            from .ops import bias_grad
            db = bias_grad(dy2, torch.bfloat16 if b_dtype == torch.bfloat16 else torch.float32).to(b_dtype)
        return dx, dw, db


class _QKVFn(torch.autograd.Function):
    """y = x [Wq; Wk; Wv]^T + [bq; bk; bv]: a self-attention's three projections of the same
    input as ONE GEMM each way. Forward: one N = 3E GEMM (columns identical to the three
    autocast F.linear calls: bf16 operands, fp32 accumulation, bf16 out); backward: dX as one
    K = 3E GEMM (autograd would sum three dX products with two extra bf16 adds), dW as one
    split-K GEMM over [3E][K] and db as one column sum, split back per projection."""

    @staticmethod
    def forward(ctx, x, wq, bq, wk, bk, wv, bv):
        xb = x.to(torch.bfloat16)
        wb = torch.cat([wq, wk, wv]).to(torch.bfloat16)  # = cat of the per-weight casts, bit for bit
        bb = None if bq is None else torch.cat([bq, bk, bv]).to(torch.bfloat16)
        ctx.save_for_backward(xb, wb)
        ctx.meta = (x.dtype, wq.dtype, None if bq is None else bq.dtype, (wq.shape[0], wk.shape[0], wv.shape[0]))
        ctx.w_refs = (wq, wk, wv)
        return hipgemm.linear(xb, wb, bb)

    @staticmethod
    def backward(ctx, dy):
        xb, wb = ctx.saved_tensors
        x_dtype, w_dtype, b_dtype, sizes = ctx.meta
        O, K = wb.shape
        dy2 = dy.reshape(-1, O).to(torch.bfloat16).contiguous()
        x2 = xb.reshape(-1, K)
        if x2.stride(1) != 1 or x2.stride(0) != K:
            x2 = x2.contiguous()
        dx = hipgemm.mm(dy2, wb).view(*xb.shape).to(x_dtype) if ctx.needs_input_grad[0] else None
        dws = [None] * 3
        if any(ctx.needs_input_grad[i] for i in (1, 3, 5)):
            if w_dtype == torch.bfloat16 and side_stream_ok(*ctx.w_refs):
                # three tensors over the one buffer's storage that are not autograd views, so
                # autograd stores each as .grad as is (a view might be cloned on the main stream)
                dws = list(on_side_stream(lambda: _split_rows(weight_grad(dy2, x2), sizes), (dy2, x2)))
            else:
                dws = [t.to(w_dtype) for t in weight_grad(dy2, x2).split(sizes)]
        dbs = [None] * 3
        if b_dtype is not None and any(ctx.needs_input_grad[i] for i in (2, 4, 6)):
            from .ops import bias_grad
            db = bias_grad(dy2, torch.bfloat16 if b_dtype == torch.bfloat16 else torch.float32).to(b_dtype)
            dbs = list(db.split(sizes))
        return dx, dws[0], dbs[0], dws[1], dbs[1], dws[2], dbs[2]


def _split_rows(buf: torch.Tensor, sizes):
    """Row blocks of a contiguous [sum(sizes)][K] tensor as separate (non-view) tensors sharing
    its storage."""
    out, r = [], 0
    K = buf.shape[1]
    for n in sizes:
        t = torch.empty((0,), dtype=buf.dtype, device=buf.device)
        t.set_(buf.untyped_storage(), buf.storage_offset() + r * K, (n, K), (K, 1))
        out.append(t)
        r += n
    return out


def qkv_eligible(q: nn.Linear, k: nn.Linear, v: nn.Linear, x: torch.Tensor) -> bool:
    """The fused projection applies where TriadLinear would to each of the three."""
    return (all(_eligible(m, x) for m in (q, k, v)) and q.in_features == k.in_features == v.in_features
            and (q.bias is None) == (k.bias is None) == (v.bias is None))


def qkv_projection(q: nn.Linear, k: nn.Linear, v: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    """[q(x) | k(x) | v(x)] along the last dim (bf16, autocast numerics) via _QKVFn."""
    return _QKVFn.apply(x, q.weight, q.bias, k.weight, k.bias, v.weight, v.bias)


def _eligible(mod: nn.Linear, x: torch.Tensor) -> bool:
    # frozen weights too (the DINOv2 base, backbones before their unfreeze step): forward and dX
    # still run on the HIP GEMM, the weight gradient is simply not requested
    if not (x.is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    # every token count: no bias gradient may fall back to PyTorch's reduction kernels beside another
    # stream's GEMMs (ops.bias_grad takes every shape by LDS-DMA, weight_grad pads the tokens;
    # DESIGN.md §2b). Widths must tile the split-K GEMM (every backbone Linear's do; LoRA's rank-8
    # layers have no bias).
    return x.numel() > 0 and mod.in_features % 128 == 0 and mod.out_features % 128 == 0


class TriadLinear(nn.Linear):
    """nn.Linear under bf16 autocast on HIP GEMMs: forward and dX on the tiled GEMM with the bias
    epilogue (gemm.py), the weight gradient on the split-K GEMM (same parameters and state-dict
    keys; any other case is nn.Linear.forward)."""

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
