"""Backbone self-attention on the HIP kernels of csrc/attention.hip.

The reference's encoders (SajayR/TRIAD model.py:29-30,79-80,218-227: DINOv2, HuBERT,
DistilBERT) run softmax(Q K^T * scale) V over short sequences -- 261 visual tokens, 199 audio
frames, 32 text tokens -- with head dim 64. PyTorch-ROCm's flash-attention kernels are tuned for
long sequences; here each (sample, head) sequence sits in LDS and a wave keeps a whole 32-row
tile of scores in registers (exact softmax, no online rescaling). Used for mask-free attention
with N <= 320 and head dim 64 in bf16, with or without dropout on the attention probabilities
(keep bits from the common.h counter hash, stored as bit words for the backward); anything
else goes to F.scaled_dot_product_attention.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ._lib import call, ptr, stream_ptr

HEAD_DIM = 64
MAX_TOKENS = 320


def supported(x: torch.Tensor, n: int, head_dim: int) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16 and head_dim == HEAD_DIM and 0 < n <= MAX_TOKENS


def _rows(t):
    """(B, N, H, 64) view with the head dim contiguous and heads adjacent -> (sB, sN)."""
    return t.stride(0), t.stride(1)


def _as_bnhd(t):
    if t.stride(3) != 1 or t.stride(2) != HEAD_DIM:
        t = t.contiguous()
    return t


def _dropmask(B, H, N, p, device):
    """Keep bits of the attention-probability dropout in both layouts (triad_attn_dropmask)."""
    nkt = (N + 31) // 32
    wq = torch.empty(B * H * N * nkt, dtype=torch.int32, device=device)
    wk = torch.empty_like(wq)
    call("triad_attn_dropmask", B, H, N, float(p), _SEEDS(), ptr(wq), ptr(wk), stream_ptr(device))
    return wq, wk


def _fwd(q, k, v, scale, drop=None):
    B, N, H, D = q.shape
    out = torch.empty(B, N, H, D, dtype=torch.bfloat16, device=q.device)
    lse = torch.empty(B * H, N, dtype=torch.float32, device=q.device)
    wq, p = (drop[0], drop[2]) if drop is not None else (None, 0.0)
    call("triad_attn_fwd_dropout", ptr(q), *_rows(q), ptr(k), *_rows(k), ptr(v), *_rows(v), B, H, N, D, float(scale),
         ptr(wq), float(p), ptr(out), *_rows(out), ptr(lse), stream_ptr(q.device))
    return out, lse


def _bwd(q, k, v, out, lse, dout, scale, drop=None):
    """-> (B, N, 3, H, 64) buffer holding dq, dk, dv (a fused qkv projection's gradient layout)."""
    B, N, H, D = q.shape
    do = _as_bnhd(dout.to(torch.bfloat16))
    g = torch.empty(B, N, 3, H, D, dtype=torch.bfloat16, device=q.device)
    dq, dk, dv = g[:, :, 0], g[:, :, 1], g[:, :, 2]
    delta = torch.empty(B * H, N, dtype=torch.float32, device=q.device)
    wq, wk, p = drop if drop is not None else (None, None, 0.0)
    call("triad_attn_bwd_dropout", ptr(q), *_rows(q), ptr(k), *_rows(k), ptr(v), *_rows(v), ptr(out), *_rows(out),
         ptr(do), *_rows(do), ptr(lse), B, H, N, D, float(scale), ptr(wq), ptr(wk), float(p), ptr(dq), *_rows(dq),
         ptr(dk), *_rows(dk), ptr(dv), *_rows(dv), ptr(delta), stream_ptr(q.device))
    return g


def _SEEDS():
    """Per-call 32-bit dropout seed drawn from torch's default CPU generator (no device sync):
    torch.manual_seed reproduces the masks, as it does for torch's own dropout kernels."""
    return int(torch.randint(0, 2 ** 32 - 1, (1,)))


class _Attention(torch.autograd.Function):
    """q, k, v: (B, N, H, 64) bf16 views (head dim contiguous, heads adjacent) -> O (B, N, H, 64);
    dropout p > 0 drops attention probabilities (keep bits drawn per call, kept for the backward)."""

    @staticmethod
    def forward(ctx, q, k, v, scale, p=0.0):
        q, k, v = _as_bnhd(q), _as_bnhd(k), _as_bnhd(v)
        drop = None
        if p > 0.0:
            B, N, H, _ = q.shape
            drop = (*_dropmask(B, H, N, p, q.device), float(p))
        out, lse = _fwd(q, k, v, scale, drop)
        ctx.save_for_backward(q, k, v, out, lse, *(drop[:2] if drop else ()))
        ctx.scale = float(scale)
        ctx.p = float(p)
        return out

    @staticmethod
    def backward(ctx, dout):
        saved = ctx.saved_tensors
        q, k, v, out, lse = saved[:5]
        drop = (saved[5], saved[6], ctx.p) if ctx.p > 0.0 else None
        g = _bwd(q, k, v, out, lse, dout, ctx.scale, drop)
        return g[:, :, 0], g[:, :, 1], g[:, :, 2], None, None


class _AttentionQKV(torch.autograd.Function):
    """qkv: (B, N, 3*H*64) bf16 output of a fused projection (q | k | v, heads inside each) ->
    O (B, N, H*64); dropout p > 0 on the probabilities as in _Attention; the backward returns
    d qkv as one tensor (the fused projection's gradient, no per-view scatter)."""

    @staticmethod
    def forward(ctx, qkv, heads, scale, p=0.0):
        B, N, C3 = qkv.shape
        x = qkv.contiguous().view(B, N, 3, heads, HEAD_DIM)
        q, k, v = x[:, :, 0], x[:, :, 1], x[:, :, 2]
        drop = (*_dropmask(B, heads, N, p, qkv.device), float(p)) if p > 0.0 else None
        out, lse = _fwd(q, k, v, scale, drop)
        ctx.save_for_backward(x, out, lse, *(drop[:2] if drop else ()))
        ctx.scale = float(scale)
        ctx.p = float(p)
        return out.view(B, N, heads * HEAD_DIM)

    @staticmethod
    def backward(ctx, dout):
        saved = ctx.saved_tensors
        x, out, lse = saved[:3]
        drop = (saved[3], saved[4], ctx.p) if ctx.p > 0.0 else None
        B, N = x.shape[0], x.shape[1]
        g = _bwd(x[:, :, 0], x[:, :, 1], x[:, :, 2], out, lse, dout.view(out.shape), ctx.scale, drop)
        return g.view(B, N, -1), None, None, None


def attention_qkv(qkv, heads, scale=None, dropout=0.0):
    """Fused-projection attention: qkv (B, N, 3*heads*64) bf16 -> (B, N, heads*64)."""
    if scale is None:
        scale = 1.0 / math.sqrt(HEAD_DIM)
    return _AttentionQKV.apply(qkv, heads, scale, float(dropout))


def attention_bnhd(q, k, v, scale=None, dropout=0.0):
    """dropout(softmax(q k^T * scale)) v over (B, N, H, 64) bf16 views -> (B, N, H, 64)."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return _Attention.apply(q, k, v, scale, float(dropout))


def dropout_keep_dense(B, H, N, p, seed, device):
    """(B, H, N, N) keep mask (bool) of the attention dropout for a given seed, unpacked from both
    stored layouts (tests: the two must agree)."""
    nkt = (N + 31) // 32
    wq = torch.empty(B * H * N * nkt, dtype=torch.int32, device=device)
    wk = torch.empty_like(wq)
    call("triad_attn_dropmask", B, H, N, float(p), seed, ptr(wq), ptr(wk), stream_ptr(device))
    bits = torch.arange(32, device=device, dtype=torch.int32)

    def unpack(w):
        m = ((w.view(B, H, N, nkt, 1) >> bits) & 1).bool().view(B, H, N, nkt * 32)
        return m[..., :N]
    return unpack(wq), unpack(wk).transpose(-1, -2)


def sdpa(q, k, v, scale=None):
    """F.scaled_dot_product_attention(q, k, v) (no mask / dropout) for (B, H, N, d) inputs: the
    HIP kernels when supported, else PyTorch."""
    B, H, N, d = q.shape
    if not supported(q, N, d) or k.shape != q.shape or v.shape != q.shape:
        return F.scaled_dot_product_attention(q, k, v, scale=scale)
    o = attention_bnhd(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale)
    return o.transpose(1, 2)


def hf_attention_forward(module, query, key, value, attention_mask, dropout=0.0, scaling=None, is_causal=None,
                         **kwargs):
    """transformers attention-interface function ("triad"): the HIP kernels for unmasked attention
    over <= 320 tokens (attention dropout included), else the stock sdpa implementation.
    Returns (B, N, H, d) as the interface requires."""
    from transformers.integrations.sdpa_attention import sdpa_attention_forward
    B, H, N, d = query.shape
    p = float(dropout) if module.training else 0.0
    if (attention_mask is not None or kwargs.get("output_attentions") or not 0.0 <= p < 1.0
            or key.shape != query.shape or value.shape != query.shape or not supported(query, N, d)
            or getattr(module, "is_causal", False)):
        return sdpa_attention_forward(module, query, key, value, attention_mask, dropout=dropout, scaling=scaling,
                                      is_causal=is_causal, **kwargs)
    o = attention_bnhd(query.transpose(1, 2), key.transpose(1, 2), value.transpose(1, 2), scaling, dropout=p)
    return o, None
