"""Autograd ops over the HIP kernels of libtriad_hip.so.

`contrastive_head` is the fused replacement of the reference's
`compute_all_similarities_{av,tv}` + `compute_contrastive_loss_{av,tv}` pair
(SajayR/TRIAD src/model.py:370-472 and 490-593): it returns the same scalar
losses and statistics without ever materialising the (B, B, Nq, Nk) token
similarity tensor, and its backward produces d/dq, d/dk and d/dtemperature.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib
from ._lib import TriadError, call, ptr, stream_ptr

D = 512
ROWS_PER_WG = 256
AV, TV = 0, 1
CLAMP_LO = {AV: -60.0, TV: -20.0}  # model.py:417 / 524


def _rup(x, m):
    return (x + m - 1) // m * m


def _check_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise TriadError("triad_amd ops run only on a HIP device (MI355X); got a CPU tensor. "
                             "There is no CPU fallback in the product path.")


@dataclass(frozen=True)
class Geometry:
    Bq: int
    Nq: int
    Bk: int
    Nk_eff: int

    @property
    def R(self):
        return self.Bq * self.Nq

    @property
    def R_pad(self):
        return _rup(max(self.R, 1), ROWS_PER_WG)

    @property
    def Nk_pad(self):
        return _rup(self.Nk_eff, 32)

    @property
    def C_pad(self):
        return self.Bk * self.Nk_pad

    @property
    def C_alloc(self):
        return _rup(self.C_pad, 128)


def pack_queries(q: torch.Tensor, g: Geometry) -> torch.Tensor:
    """(Bq, Nq, 512) -> zero-padded [R_pad][512] bf16 (layout of include/triad_hip.h)."""
    out = torch.empty(g.R_pad, D, dtype=torch.bfloat16, device=q.device)
    out[:g.R].copy_(q.reshape(g.R, D))
    if g.R_pad > g.R:
        out[g.R:].zero_()
    return out


def pack_keys(k: torch.Tensor, g: Geometry) -> torch.Tensor:
    """(Bk, Nk_eff, 512) -> [C_alloc][512] bf16, each sample padded to Nk_pad rows."""
    out = torch.empty(g.C_alloc, D, dtype=torch.bfloat16, device=k.device)
    if g.Nk_pad == g.Nk_eff:
        out[:g.C_pad].copy_(k.reshape(g.C_pad, D))
    else:
        v = out[:g.C_pad].view(g.Bk, g.Nk_pad, D)
        v[:, :g.Nk_eff].copy_(k)
        v[:, g.Nk_eff:].zero_()
    if g.C_alloc > g.C_pad:
        out[g.C_pad:].zero_()
    return out


class _ContrastiveHead(torch.autograd.Function):
    """losses = [total, ce, reg, aux] (aux = 0.01*l_smooth for AV, sparsity for TV), stats[9]."""

    @staticmethod
    def forward(ctx, q, k, temperature, kind, q_mask, thr, w_sparse):
        _check_device(q, k, temperature, q_mask)
        Bq, Nq, dq = q.shape
        Bk, Nk, dk = k.shape
        if dq != D or dk != D:
            raise TriadError(f"feature dim must be {D}")
        if Bq != Bk:
            raise TriadError("local head needs matching batch sizes")
        if Bq < 2:
            # the reference takes max() of the empty off-diagonal set and raises (model.py:447/565)
            raise TriadError("batch size must be >= 2 (no negatives for B == 1)")
        g = Geometry(Bq, Nq, Bk, Nk)
        dev = q.device
        st = stream_ptr(dev)
        Qb = pack_queries(q, g)
        Kb = pack_keys(k, g)
        temp = temperature.detach().reshape(1).to(torch.float32).contiguous()
        nparts = call("triad_pairsim_nparts", g.R_pad, g.Bk)
        rowmax = torch.empty(g.Bk, g.R_pad, dtype=torch.float32, device=dev)
        argmax = torch.empty(g.Bk, g.R_pad, dtype=torch.int32, device=dev)
        nn_part = torch.empty(nparts, dtype=torch.float64, device=dev)
        diagS = torch.empty(g.Bq, g.Nq, g.Nk_pad, dtype=torch.float32, device=dev)
        call("triad_pairsim_fwd", ptr(Qb), ptr(Kb), g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, D,
             ptr(temp), CLAMP_LO[kind], 1, 0, ptr(rowmax), ptr(argmax), ptr(nn_part), ptr(diagS), st)
        clip = torch.empty(g.Bq, g.Bk, dtype=torch.float32, device=dev)
        qw = torch.empty(g.R, dtype=torch.float32, device=dev)
        qm = None if q_mask is None else q_mask.to(torch.float32).contiguous()
        call("triad_clip_reduce", ptr(rowmax), g.R_pad, g.Nq, g.Bq, g.Bk, ptr(qm), ptr(clip), ptr(qw), st)
        dg_part = torch.empty(g.Bq, dtype=torch.float64, device=dev)
        if kind == AV:
            cnt = float(g.Bq * (g.Nq - 1) * g.Nk_eff)
            gdiag = torch.empty_like(diagS)
            call("triad_diag_smooth", ptr(diagS), g.Bq, g.Nq, g.Nk_pad, g.Nk_eff, cnt, ptr(dg_part), ptr(gdiag), st)
        else:
            cnt = float(g.Bq * g.Nk_eff)
            call("triad_diag_sparsity", ptr(diagS), g.Bq, g.Nq, g.Nk_pad, g.Nk_eff, float(thr), cnt,
                 ptr(dg_part), st)
            gdiag = diagS
        out = torch.empty(13, dtype=torch.float32, device=dev)
        dclip = torch.empty(g.Bq, g.Bk, dtype=torch.float32, device=dev)
        lse = torch.empty(2 * g.Bq, dtype=torch.float32, device=dev)
        n_el = float(g.Bq) * g.Bk * g.Nq * g.Nk_eff
        call("triad_losshead", ptr(clip), g.Bq, kind, ptr(temp), ptr(nn_part), nparts, n_el, ptr(dg_part), g.Bq,
             cnt, float(w_sparse), ptr(out), ptr(dclip), ptr(lse), st)

        ctx.save_for_backward(Qb, Kb, argmax, dclip, qw, gdiag, temp)
        ctx.geom, ctx.kind, ctx.n_el, ctx.w_sparse, ctx.nparts = g, kind, n_el, float(w_sparse), nparts
        ctx.q_dtype, ctx.k_dtype, ctx.t_dtype = q.dtype, k.dtype, temperature.dtype
        losses, stats = out[:4].clone(), out[4:].clone()
        ctx.mark_non_differentiable(stats, clip)
        ctx.set_materialize_grads(False)
        return losses, stats, clip

    @staticmethod
    def backward(ctx, g_losses, g_stats, g_clip):
        if g_losses is None:
            return None, None, None, None, None, None, None
        Qb, Kb, argmax, dclip, qw, gdiag, temp = ctx.saved_tensors
        g, kind = ctx.geom, ctx.kind
        dev = Qb.device
        st = stream_ptr(dev)
        gl = g_losses.to(torch.float32)
        c_ce = gl[0] + gl[1]
        c_reg = gl[0] + gl[2]
        c_nn = c_reg * (0.15 * 2.0 / ctx.n_el)
        if kind == AV:
            c_diag = 0.01 * (c_reg + gl[3])   # reg = ... + 0.01*l_smooth; aux = 0.01*l_smooth
            c_cal = 20.0 * c_reg
        else:
            c_diag = ctx.w_sparse * c_reg + gl[3]  # reg = ... + w*sparsity; aux = sparsity
            c_cal = torch.zeros_like(c_reg)
        coef = torch.stack([c_ce, c_nn, c_diag, c_cal]).contiguous()
        dS = torch.empty(g.R_pad, g.C_alloc, dtype=torch.bfloat16, device=dev)
        if g.C_alloc > g.C_pad:
            dS[:, g.C_pad:].zero_()
        dt_part = torch.empty(ctx.nparts, dtype=torch.float64, device=dev)
        call("triad_pairsim_dS", ptr(Qb), ptr(Kb), g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, D, ptr(temp),
             CLAMP_LO[kind], 1, 0, ptr(argmax), ptr(dclip), ptr(qw), ptr(gdiag), ptr(coef), ptr(dS), g.C_alloc,
             ptr(dt_part), st)
        gq = gk = gt = None
        if ctx.needs_input_grad[0]:
            dQ = torch.empty(g.R_pad, D, dtype=torch.bfloat16, device=dev)
            call("triad_gemm_bf16", ptr(dS), g.C_alloc, 1, ptr(Kb), D, 0, g.R_pad, D, g.C_alloc, ptr(temp), ptr(dQ), D,
                 1, st)
            gq = dQ[:g.R].view(g.Bq, g.Nq, D).to(ctx.q_dtype)
        if ctx.needs_input_grad[1]:
            dK = torch.empty(g.C_alloc, D, dtype=torch.bfloat16, device=dev)
            call("triad_gemm_bf16", ptr(dS), g.C_alloc, 0, ptr(Qb), D, 0, g.C_alloc, D, g.R_pad, ptr(temp), ptr(dK), D,
                 1, st)
            gk = dK[:g.C_pad].view(g.Bk, g.Nk_pad, D)[:, :g.Nk_eff].to(ctx.k_dtype)
        if ctx.needs_input_grad[2]:
            dt = torch.empty(1, dtype=torch.float32, device=dev)
            call("triad_dtemp_finalize", ptr(dt_part), ctx.nparts, ptr(temp), ptr(coef), 1 if kind == AV else 0,
                 ptr(dt), st)
            gt = dt.reshape(()).to(ctx.t_dtype)
        return gq, gk, gt, None, None, None, None


def contrastive_head(kind, q, k, temperature, q_mask=None, threshold=0.0, sparsity_weight=0.0):
    """Fused similarity + aggregation + InfoNCE + regularisers.

    kind AV: q = audio feats (B,Na,512), k = visual feats (B,Nv,512) (model.py:470-472)
    kind TV: q = text feats (B,Nt,512) with q_mask (B,Nt), k = visual feats (model.py:593)
    Returns (losses[4], stats[9], clip[B,B]); losses = total, contrastive, reg, aux.
    """
    return _ContrastiveHead.apply(q, k, temperature, kind, q_mask, threshold, sparsity_weight)


def gather_rows(src: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """out[b][t] = src[b][idx[b][t]] (idx -1 -> zero row); src (B, N, D) contiguous."""
    _check_device(src, idx)
    B, N = src.shape[0], src.shape[1]
    M = idx.shape[1]
    row_bytes = src[0, 0].numel() * src.element_size()
    out = torch.empty((B, M) + tuple(src.shape[2:]), dtype=src.dtype, device=src.device)
    call("triad_gather_rows", ptr(src.contiguous()), N, ptr(idx.to(torch.int32).contiguous()), B, M, row_bytes,
         ptr(out), stream_ptr(src.device))
    return out


def l2_normalize(x: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """F.normalize(x, dim=-1) for bf16 rows (model.py:363-364)."""
    _check_device(x)
    xc = x.to(torch.bfloat16).contiguous()
    y = torch.empty_like(xc)
    rows = xc.numel() // xc.shape[-1]
    call("triad_l2norm_rows", ptr(xc), rows, xc.shape[-1], eps, ptr(y), stream_ptr(x.device))
    return y
