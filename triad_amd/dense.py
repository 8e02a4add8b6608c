"""Materialising debug path of the loss head, on the HIP kernels of csrc/dense.hip + gemm.hip.

SURVEY §8b keeps the reference's small-B methods on the drop-in model with their signatures and
return tuples: `compute_all_similarities_{av,tv}` -> (clip, token_sims (B, B, Nq, Nk)),
`compute_temporal_smoothness_loss`, `compute_regularization_losses_{av,tv}` and
`compute_contrastive_loss_{av,tv}` (reference src/model.py:370-472, 490-593). Training never
takes this path (it materialises B^2 Nq Nk fp32 values); `ops.contrastive_head` is the fused form.

Each piece is an autograd Function over HIP kernels, so the reference's composition (written out
in `triad_amd.model.MultiModalModel`) differentiates exactly as the reference's autograd does:
  all_similarities  S = temp <q, k> (bf16 operands, fp32 accumulate, triad_gemm_bf16), first-index
                    max over keys (triad_dense_rowmax), (masked) mean (triad_clip_reduce);
                    backward: one pack of dS = dtok + max routing (triad_sims_bwd_pack), two GEMMs
  nonneg            mean(clamp(S, lo, 0)^2) (triad_nonneg_fwd / _bwd)
  diag_smoothness   mean over the diagonal pairs of the squared step along Nq (triad_diag_smooth)
  diag_sparsity     softmax patch-usage excess on the diagonal pairs (triad_diag_sparsity)
  clip_ce           symmetric InfoNCE + similarity statistics of a (B, B) clip (triad_losshead)

Deliberate deviation (precision): token_sims come back fp32 and clip / max / the regularisers are
computed from fp32 S. In the reference, under autocast, the bf16 einsum result times the 0-dim
fp32 temperature stays bf16 (SURVEY §2 records that promotion as measured), so its token_sims and
everything downstream carry bf16 rounding (~2^-9 relative) and half the memory. These debug
methods keep the fused head's arithmetic (fp32 S from fp32 MFMA accumulation, the same as
`ops.contrastive_head`) so the two paths agree with each other. The golden fixtures were made by
the reference on the CPU without autocast (fp32 throughout, tests/golden/gen_golden.py), and
these methods match them at 1e-4 (`tests/test_dropin_gpu.py`); agreement with the reference's
bf16 autocast values is bf16 rounding and is not pinned by a fixture.
"""
from __future__ import annotations

import torch

from ._lib import TriadError, call, ptr, stream_ptr

D = 512


def _rup(x, m):
    return (x + m - 1) // m * m


def _dev_check(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise TriadError("triad_amd ops run only on a HIP device (MI355X); got a CPU tensor. "
                             "There is no CPU fallback in the product path.")


def _temp32(temperature):
    return temperature.detach().reshape(1).to(torch.float32).contiguous()


class _AllSims(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, temperature, q_mask):
        _dev_check(q, k, temperature)
        Bq, Nq, dq = q.shape
        Bk, Nk, dk = k.shape
        if dq != D or dk != D:
            raise TriadError(f"feature dim must be {D}")
        dev = q.device
        st = stream_ptr(dev)
        R, C = Bq * Nq, Bk * Nk
        Rp, Cp = _rup(R, 128), _rup(C, 128)
        Qf = torch.zeros(Rp, D, dtype=torch.bfloat16, device=dev)
        Qf[:R].copy_(q.reshape(R, D))
        Kf = torch.zeros(Cp, D, dtype=torch.bfloat16, device=dev)
        Kf[:C].copy_(k.reshape(C, D))
        temp = _temp32(temperature)
        flat = torch.empty(Rp, Cp, dtype=torch.float32, device=dev)
        call("triad_gemm_bf16", ptr(Qf), D, 1, ptr(Kf), D, 1, Rp, Cp, D, ptr(temp), ptr(flat), Cp, 0, st)
        S = flat[:R, :C].view(Bq, Nq, Bk, Nk).permute(0, 2, 1, 3).contiguous()   # (Bq, Bk, Nq, Nk)
        rowmax = torch.empty(Bk, R, dtype=torch.float32, device=dev)
        argmax = torch.empty(Bk, R, dtype=torch.int32, device=dev)
        call("triad_dense_rowmax", ptr(S), Bq, Bk, Nq, Nk, R, ptr(rowmax), ptr(argmax), st)
        clip = torch.empty(Bq, Bk, dtype=torch.float32, device=dev)
        qw = torch.empty(R, dtype=torch.float32, device=dev)
        qm = None if q_mask is None else q_mask.to(device=dev, dtype=torch.float32).contiguous()
        call("triad_clip_reduce", ptr(rowmax), R, Nq, Bq, Bk, ptr(qm), ptr(clip), ptr(qw), st)
        ctx.save_for_backward(Qf, Kf, S, argmax, qw, temp)
        ctx.dims = (Bq, Nq, Bk, Nk, R, C, Rp, Cp)
        ctx.dtypes = (q.dtype, k.dtype, temperature.dtype)
        ctx.set_materialize_grads(False)
        return clip, S

    @staticmethod
    def backward(ctx, dclip, dtok):
        Qf, Kf, S, argmax, qw, temp = ctx.saved_tensors
        Bq, Nq, Bk, Nk, R, C, Rp, Cp = ctx.dims
        if dclip is None and dtok is None:
            return None, None, None, None
        dev = S.device
        st = stream_ptr(dev)
        A = torch.zeros(Rp, Cp, dtype=torch.bfloat16, device=dev)
        n = S.numel()
        nparts = call("triad_dense_nparts", n)
        part = torch.empty(nparts, dtype=torch.float64, device=dev)
        dc = None if dclip is None else dclip.to(torch.float32).contiguous()
        dt = None if dtok is None else dtok.to(torch.float32).contiguous()
        call("triad_sims_bwd_pack", ptr(S), ptr(dt), ptr(dc), ptr(qw), ptr(argmax), Bq, Bk, Nq, Nk, R, ptr(temp),
             ptr(A), Cp, ptr(part), st)
        gq = gk = gt = None
        qd, kd, td = ctx.dtypes
        if ctx.needs_input_grad[0]:
            dQ = torch.empty(Rp, D, dtype=torch.float32, device=dev)
            call("triad_gemm_bf16", ptr(A), Cp, 1, ptr(Kf), D, 0, Rp, D, Cp, ptr(temp), ptr(dQ), D, 0, st)
            gq = dQ[:R].view(Bq, Nq, D).to(qd)
        if ctx.needs_input_grad[1]:
            dK = torch.empty(Cp, D, dtype=torch.float32, device=dev)
            call("triad_gemm_bf16", ptr(A), Cp, 0, ptr(Qf), D, 0, Cp, D, Rp, ptr(temp), ptr(dK), D, 0, st)
            gk = dK[:C].view(Bk, Nk, D).to(kd)
        if ctx.needs_input_grad[2]:
            out = torch.empty(1, dtype=torch.float32, device=dev)
            call("triad_sum_parts", ptr(part), nparts, 1.0, ptr(out), st)
            gt = out.reshape(()).to(td)
        return gq, gk, gt, None


def all_similarities(q, k, temperature, q_mask=None):
    """(clip (Bq, Bk), token_sims (Bq, Bk, Nq, Nk) fp32) = model.py:370-392 (q_mask None) /
    490-514 (masked mean over the query tokens)."""
    return _AllSims.apply(q, k, temperature, q_mask)


class _NonNeg(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S, lo):
        _dev_check(S)
        S = S.to(torch.float32).contiguous()
        n = S.numel()
        st = stream_ptr(S.device)
        nparts = call("triad_dense_nparts", n)
        part = torch.empty(nparts, dtype=torch.float64, device=S.device)
        call("triad_nonneg_fwd", ptr(S), n, float(lo), ptr(part), st)
        out = torch.empty(1, dtype=torch.float32, device=S.device)
        call("triad_sum_parts", ptr(part), nparts, 1.0 / n, ptr(out), st)
        ctx.save_for_backward(S)
        ctx.lo = float(lo)
        return out.reshape(())

    @staticmethod
    def backward(ctx, g):
        (S,) = ctx.saved_tensors
        dS = torch.empty_like(S)
        gc = g.reshape(1).to(torch.float32).contiguous()
        call("triad_nonneg_bwd", ptr(S), S.numel(), ctx.lo, 1.0 / S.numel(), ptr(gc), ptr(dS), stream_ptr(S.device))
        return dS, None


def nonneg(S, lo):
    """mean(clamp(S, lo, 0)^2) over every element (model.py:417-418, lo = -60 / 524-525, lo = -20)."""
    return _NonNeg.apply(S, lo)


class _DiagLoss(torch.autograd.Function):
    """Regulariser over the diagonal pairs S[i, i] only (B, Nq, Nk)."""

    @staticmethod
    def forward(ctx, S, sparsity, thr):
        _dev_check(S)
        B, B2, Nq, Nk = S.shape
        if B != B2:
            raise TriadError("token_sims must be (B, B, Nq, Nk)")
        dev = S.device
        st = stream_ptr(dev)
        diag = S.to(torch.float32).diagonal(0, 0, 1).permute(2, 0, 1).contiguous()   # (B, Nq, Nk)
        part = torch.empty(B, dtype=torch.float64, device=dev)
        dtp = torch.empty(B, dtype=torch.float64, device=dev)
        g = torch.empty_like(diag)
        if sparsity:
            cnt = float(B * Nk)
            call("triad_diag_sparsity", ptr(diag), B, Nq, Nk, Nk, float(thr), cnt, ptr(part), ptr(g), ptr(dtp), st)
        else:
            cnt = float(B * (Nq - 1) * Nk)
            call("triad_diag_smooth", ptr(diag), B, Nq, Nk, Nk, cnt, ptr(part), ptr(g), ptr(dtp), st)
        out = torch.empty(1, dtype=torch.float32, device=dev)
        # mean over an empty set (Nq == 1) is NaN in the reference (model.py:407)
        call("triad_sum_parts", ptr(part), B, 1.0 / cnt if cnt > 0 else float("nan"), ptr(out), st)
        ctx.save_for_backward(g)
        ctx.shape = S.shape
        ctx.dtype = S.dtype
        return out.reshape(())

    @staticmethod
    def backward(ctx, gout):
        (g,) = ctx.saved_tensors
        dS = torch.zeros(ctx.shape, dtype=torch.float32, device=g.device)
        dS.diagonal(0, 0, 1).copy_((g * gout.to(torch.float32)).permute(1, 2, 0))
        return dS.to(ctx.dtype), None, None


def diag_smoothness(S):
    """mean((S_ii[1:] - S_ii[:-1])^2) over the diagonal pairs (model.py:394-408)."""
    return _DiagLoss.apply(S, False, 0.0)


def diag_sparsity(S, thr):
    """mean(relu(softmax_k(S_ii).sum(t) / Nt - thr)^2) over the diagonal pairs (model.py:527-540)."""
    return _DiagLoss.apply(S, True, thr)


class _ClipCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, clip):
        _dev_check(clip)
        B = clip.shape[0]
        if clip.dim() != 2 or clip.shape[1] != B:
            raise TriadError("clip must be (B, B)")
        if B < 2:
            # the reference takes max() of the empty off-diagonal set and raises (model.py:447/565)
            raise TriadError("batch size must be >= 2 (no negatives for B == 1)")
        dev = clip.device
        c = clip.to(torch.float32).contiguous()
        out = torch.empty(13, dtype=torch.float32, device=dev)
        dclip = torch.empty(B, B, dtype=torch.float32, device=dev)
        lse = torch.empty(2 * B, dtype=torch.float32, device=dev)
        call("triad_losshead", ptr(c), B, 1, None, None, 0, 1.0, None, 0, 1.0, 0.0, ptr(out), ptr(dclip), ptr(lse),
             stream_ptr(dev))
        ctx.save_for_backward(dclip)
        ctx.dtype = clip.dtype
        stats = out[4:10].clone()
        ctx.mark_non_differentiable(stats)
        return out[1].clone(), stats

    @staticmethod
    def backward(ctx, g, _gs):
        (dclip,) = ctx.saved_tensors
        if g is None:
            return None
        return (dclip * g.to(torch.float32)).to(ctx.dtype)


def clip_ce(clip):
    """(symmetric InfoNCE, stats[6]) of a (B, B) clip matrix (model.py:431-459 / 549-578):
    stats = pos mean, pos std (unbiased), neg mean, neg std, separation, hardest negative."""
    return _ClipCE.apply(clip)
