"""CPU restatement (oracle) of TRIAD's dense tri-modal contrastive hot path.

TEST INFRASTRUCTURE ONLY. This module is the checker for the HIP product path:
only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import it. The product package `triad_amd` never imports it and has no CPU
fallback.

It restates, op for op and in plain PyTorch on the CPU, the reference's
algorithm (reference snapshot SajayR/TRIAD @ 2025-06-14, `src/model.py`):

  similarity_matrix        model.py:355-368  (L2-normalise, bmm, * temperature)
  similarities_av          model.py:370-392  (B x B x Na x Nv token sims, max over Nv, mean over Na)
  temporal_smoothness      model.py:394-408  (diagonal pairs, diff along Na)
  regularization_av        model.py:410-428  (20*l_cal + 0.15*l_nonneg[-60,0] + 0.01*l_smooth)
  contrastive_av           model.py:430-472  (symmetric InfoNCE + stats, unbiased std)
  similarities_tv          model.py:490-514  (masked mean over Nt)
  regularization_tv        model.py:516-542  (0.15*l_nonneg[-20,0] + w*patch sparsity)
  contrastive_tv           model.py:544-593
  patch_dropout            model.py:268-308  (Bernoulli keep mask is an INPUT here, so the
                                              compaction is reproducible across implementations)
  projection_head          model.py:32-34,68 / 81-83,116 / 253-255,326 under bf16 autocast
                           (model.py:483,603): bf16 Linear -> fp32 LayerNorm -> bf16 Linear

Parity pinning: the functions are checked against golden vectors produced by
running the reference's own methods (tests/golden/gen_golden.py, fixtures
tests/golden/*.npz) in tests/test_oracle_golden.py.

All functions take a `dtype` for the arithmetic (float64 by default for a tight
checker; float32 mirrors the reference's CPU arithmetic).
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import torch
import torch.nn.functional as F

AV_STAT_KEYS = ("av_pos_sim_mean", "av_pos_sim_std", "av_neg_sim_mean",
                "av_neg_sim_std", "av_separation", "av_hardest_negative")
TV_STAT_KEYS = tuple("tv_" + k[3:] for k in AV_STAT_KEYS)


def similarity_matrix(f1, f2, temperature, dtype=torch.float64):
    """model.py:355-368: per-sample (B,N1,N2) cosine-similarity map times temperature."""
    a = F.normalize(f1.to(dtype), dim=-1)
    b = F.normalize(f2.to(dtype), dim=-1)
    return torch.bmm(a, b.transpose(1, 2)) * temperature.to(dtype)


def _token_sims(q, v, temperature, dtype):
    # (B,Nq,D) x (B,Nv,D) -> (Bq,Bk,Nq,Nv): every query sample against every key sample
    return torch.einsum("iqd,jvd->ijqv", q.to(dtype), v.to(dtype)) * temperature.to(dtype)


def similarities_av(audio_feats, visual_feats, temperature, dtype=torch.float64):
    """model.py:370-392 -> (clip (B,B), token_sims (B,B,Na,Nv))."""
    s = _token_sims(audio_feats, visual_feats, temperature, dtype)
    return s.max(dim=3).values.mean(dim=2), s


def temporal_smoothness(token_sims):
    """model.py:394-408: mean squared difference of consecutive audio tokens on the diagonal pairs."""
    diag = torch.diagonal(token_sims, dim1=0, dim2=1).permute(2, 0, 1)  # (B,Na,Nv)
    d = diag[:, 1:] - diag[:, :-1]
    return (d * d).mean()


def regularization_av(token_sims, temperature):
    """model.py:410-428 -> (reg, 0.01*l_smooth)."""
    t = temperature.to(token_sims.dtype)
    l_nonneg = token_sims.clamp(min=-60, max=0).pow(2).mean()
    l_cal = (-torch.log(t)).clamp(min=0).pow(2)  # log(1) - log(temp)
    l_smooth = temporal_smoothness(token_sims)
    return 20 * l_cal + 0.15 * l_nonneg + 0.01 * l_smooth, 0.01 * l_smooth


def _symmetric_ce(clip):
    n = clip.shape[0]
    idx = torch.arange(n)
    row = -F.log_softmax(clip, dim=1)[idx, idx]
    col = -F.log_softmax(clip.t(), dim=1)[idx, idx]
    return (row + col).mean() / 2


def _stats(clip, keys):
    n = clip.shape[0]
    pos = torch.diagonal(clip)
    off = ~torch.eye(n, dtype=torch.bool)
    neg = clip[off]
    vals = [pos.mean(), pos.std(), neg.mean(), neg.std()]
    vals = [float(v.detach()) for v in vals]
    hardest = float(neg.max().detach())  # raises on B == 1, as the reference does
    return dict(zip(keys, vals[:4] + [vals[0] - vals[2], hardest]))


def contrastive_av(clip, token_sims, temperature):
    """model.py:430-472 -> (total, contrastive, reg, 0.01*smooth, stats)."""
    stats = _stats(clip, AV_STAT_KEYS)
    ce = _symmetric_ce(clip)
    reg, smooth = regularization_av(token_sims, temperature)
    return ce + reg, ce, reg, smooth, stats


def similarities_tv(text_feats, visual_feats, attention_mask, temperature, dtype=torch.float64):
    """model.py:490-514 -> (clip (B,B), token_sims (B,B,Nt,Nv))."""
    s = _token_sims(text_feats, visual_feats, temperature, dtype)
    mx = s.max(dim=3).values  # (B,B,Nt)
    m = attention_mask.to(dtype)[:, None, :]
    return (mx * m).sum(dim=2) / m.sum(dim=2).clamp(min=1e-7), s


def regularization_tv(token_sims, threshold, weight):
    """model.py:516-542."""
    l_nonneg = token_sims.clamp(min=-20, max=0).pow(2).mean()
    diag = torch.diagonal(token_sims, dim1=0, dim2=1).permute(2, 0, 1)  # (B,Nt,Nv)
    probs = torch.softmax(diag, dim=-1)
    frac = probs.sum(dim=1) / probs.shape[1]
    sparsity = F.relu(frac - threshold).pow(2).mean()
    return 0.15 * l_nonneg + weight * sparsity


def contrastive_tv(clip, token_sims, threshold, weight):
    """model.py:544-593 -> (total, stats)."""
    stats = _stats(clip, TV_STAT_KEYS)
    return _symmetric_ce(clip) + regularization_tv(token_sims, threshold, weight), stats


def patch_dropout(x, keep_mask):
    """model.py:268-308 with the Bernoulli keep mask supplied by the caller.

    Kept tokens of each sample stay in their original order; samples are
    zero-padded to the longest kept length.
    """
    kept = [x[i][keep_mask[i].bool()] for i in range(x.shape[0])]
    n = max(k.shape[0] for k in kept)
    out = x.new_zeros(x.shape[0], n, x.shape[2])
    for i, k in enumerate(kept):
        out[i, :k.shape[0]] = k
    return out


def _bf16(x):
    return x.to(torch.bfloat16).to(torch.float32)


def projection_head(h, w1, b1, gamma, beta, w2, b2, amp=True, eps=1e-5):
    """proj2(LN(proj1(h))) (model.py:68,116,326).

    amp=True emulates CUDA bf16 autocast (model.py:483,603): Linear operands and
    outputs rounded to bf16, LayerNorm computed in fp32 from the bf16 input.
    """
    if not amp:
        y = F.linear(h, w1, b1)
        y = F.layer_norm(y, (y.shape[-1],), gamma, beta, eps)
        return F.linear(y, w2, b2)
    y = _bf16(F.linear(_bf16(h), _bf16(w1), _bf16(b1)))
    y = F.layer_norm(y, (y.shape[-1],), gamma.float(), beta.float(), eps)
    return _bf16(F.linear(_bf16(y), _bf16(w2), _bf16(b2)))


def av_loss(audio_feats, visual_feats, temperature, dtype=torch.float64):
    """forward_audio_visual's loss half (model.py:486-488) on given features."""
    clip, s = similarities_av(audio_feats, visual_feats, temperature, dtype)
    return contrastive_av(clip, s, temperature)


def tv_loss(text_feats, visual_feats, mask, temperature, threshold, weight, dtype=torch.float64):
    """forward_text_visual's loss half (model.py:606-608) on given features."""
    clip, s = similarities_tv(text_feats, visual_feats, mask, temperature, dtype)
    return contrastive_tv(clip, s, threshold, weight)


def loss_mix(phase, av, tv, progress=0.0, av_start=0.8, av_end=0.5):
    """train.py:972-984 curriculum loss mixing."""
    if phase == "av_focus":
        return av
    if phase == "tv_warmup":
        return tv
    if phase == "weighted_joint":
        w = av_start - progress * (av_start - av_end)
        return w * av + (1.0 - w) * tv
    return av + tv


# ---- audio front-end ----------------------------------------------------------------------
def audio_znorm(x, eps=1e-7):
    """AudioEmbedder.forward's processor call (model.py:56-62): the hubert-large-ls960-ft
    Wav2Vec2FeatureExtractor receives the (B, T) tensor as ONE utterance (a tensor is not taken as
    a batch), so one mean and one population variance over all B*T samples:
    (x - mean) / sqrt(var + 1e-7). Pinned by tests/golden/znorm_*.npz."""
    xd = torch.as_tensor(x).double()
    return (xd - xd.mean()) / torch.sqrt(xd.var(unbiased=False) + eps)


# ---- 1000-way retrieval (src/retrieval.py) ---------------------------------------------
def aggregator_a2v(a_feats, v_feats, temperature):
    """retrieval.py:106-109 (and 190-193 for text): mean over query tokens of the max over keys,
    similarities divided by the temperature."""
    s = a_feats.double() @ v_feats.double().t() / temperature
    return float(s.max(dim=1).values.mean())


def aggregator_v2a(a_feats, v_feats, temperature):
    """retrieval.py:111-114 (and 195-198): mean over the visual tokens of the max over audio tokens."""
    s = a_feats.double() @ v_feats.double().t() / temperature
    return float(s.max(dim=0).values.mean())


def retrieval_matrices(q_list, k_list, temperature):
    """(N x N) q->k and k->q aggregation matrices of retrieval.py:161-174 / 255-264."""
    import numpy as np
    n = len(q_list)
    q2k = np.zeros((n, n))
    k2q = np.zeros((n, n))
    for i in range(n):
        for j in range(n):
            q2k[i, j] = aggregator_a2v(q_list[i], k_list[j], temperature)
            k2q[i, j] = aggregator_v2a(q_list[j], k_list[i], temperature)
    return q2k, k2q


def recall_ranks(sim):
    """retrieval.py:124-131: rank of the matching item i in np.argsort(-row) with numpy's DEFAULT
    (unstable) sort, so exact ties are ordered as the reference orders them (pinned by
    tests/golden/retrieval_*_ties.npz, which the reference itself produced)."""
    import numpy as np
    sim = np.asarray(sim, np.float32)   # the reference's np.zeros((N, N), float32) matrices
    return np.array([int(np.where(np.argsort(-sim[i]) == i)[0][0]) for i in range(sim.shape[0])])


def recall_at_k(sim):
    """retrieval.py:117-144."""
    import numpy as np
    ranks = recall_ranks(sim)
    return {f"r{k}": float(np.mean(ranks < k)) for k in (1, 5, 10, 20)}


# ---- chunked form for BASELINE-size parity checks -----------------------------------------
def head_loss_chunked(kind, q, k, temperature, q_mask=None, threshold=0.8, weight=0.01, chunk=8,
                      dtype=torch.float64, grads=True, grad_rows=None):
    """The same values as av_loss (kind "av", model.py:370-472) / tv_loss (kind "tv",
    model.py:490-593), evaluated in chunks of query samples so the (B, B, Nq, Nk) tensor is never
    held whole (c3: 13 GB in fp32). Runs on whatever device the inputs are on (plain torch;
    test infrastructure only).

    Pass 1 builds clip, the l_nonneg sum and the diagonal regulariser sums chunk by chunk; the CE
    and the statistics are evaluated on the full (B, B) clip exactly as _symmetric_ce / _stats.
    Pass 2 (grads=True) re-evaluates each chunk under autograd with the surrogate
        sum(dCE/dclip * clip_chunk) + 0.15 * sum clamp(S)^2 / N_el + w_diag * diag_chunk / cnt,
    whose gradient equals the loss gradient (every term is additive over query samples, and the
    CE enters only through clip). grad_rows=(i0, i1): pass 2 over those query samples only -- dq
    of those rows, and dk / dtemp = the CONTRIBUTION of those rows (what one data-parallel rank
    holding them computes before the reduce-scatter / all-reduce, SURVEY §8e Mode G; the l_cal
    term of dtemp is included). Returns a dict of floats / tensors (fp64)."""
    av = kind == "av"
    B, Nq, _ = q.shape
    Nk = k.shape[1]
    lo = -60.0 if av else -20.0
    Qd, Kd = q.detach().to(dtype), k.detach().to(dtype)
    t = torch.as_tensor(temperature, dtype=dtype, device=q.device).detach()
    m = None if av else q_mask.to(device=q.device, dtype=dtype)

    def chunk_terms(Qc, Kall, tt, i0):
        s = torch.einsum("iqd,jkd->ijqk", Qc, Kall) * tt
        mx = s.max(dim=3).values
        if av:
            clip_c = mx.mean(dim=2)
        else:
            mc = m[i0:i0 + Qc.shape[0]][:, None, :]
            clip_c = (mx * mc).sum(dim=2) / mc.sum(dim=2).clamp(min=1e-7)
        nn_c = s.clamp(min=lo, max=0).pow(2).sum()
        c = Qc.shape[0]
        ar = torch.arange(c, device=q.device)
        diag = s[ar, i0 + ar]   # (c, Nq, Nk)
        if av:
            d = diag[:, 1:] - diag[:, :-1]
            dg_c = (d * d).sum()
        else:
            frac = torch.softmax(diag, dim=-1).sum(dim=1) / Nq
            dg_c = F.relu(frac - threshold).pow(2).sum()
        return clip_c, nn_c, dg_c

    clip = torch.zeros(B, B, dtype=dtype, device=q.device)
    nn_sum = torch.zeros((), dtype=dtype, device=q.device)
    dg_sum = torch.zeros((), dtype=dtype, device=q.device)
    with torch.no_grad():
        for i0 in range(0, B, chunk):
            c_, n_, d_ = chunk_terms(Qd[i0:i0 + chunk], Kd, t, i0)
            clip[i0:i0 + chunk] = c_
            nn_sum += n_
            dg_sum += d_
    n_el = float(B) * B * Nq * Nk
    cnt = float(B * (Nq - 1) * Nk) if av else float(B * Nk)
    l_nonneg = nn_sum / n_el
    l_dg = dg_sum / cnt if cnt > 0 else torch.full((), float("nan"), dtype=dtype, device=q.device)
    l_cal = (-torch.log(t)).clamp(min=0).pow(2)
    if av:
        reg = 20 * l_cal + 0.15 * l_nonneg + 0.01 * l_dg
        aux = 0.01 * l_dg
        w_dg = 0.01
    else:
        reg = 0.15 * l_nonneg + weight * l_dg
        aux = l_dg
        w_dg = weight
    cl = clip.clone().requires_grad_(True)
    ce = _symmetric_ce_dev(cl)
    ce.backward()
    ce = ce.detach()
    dclip = cl.grad.detach()
    keys = AV_STAT_KEYS if av else TV_STAT_KEYS
    stats = _stats(clip.cpu(), keys)
    out = dict(total=float(ce + reg), ce=float(ce), reg=float(reg), aux=float(aux), l_nonneg=float(l_nonneg),
               l_cal=float(l_cal), diag=float(l_dg), stats=stats, clip=clip)
    if not grads:
        return out
    Qg = Qd.clone().requires_grad_(True)
    Kg = Kd.clone().requires_grad_(True)
    tg = t.clone().requires_grad_(True)
    g0, g1 = (0, B) if grad_rows is None else grad_rows
    for i0 in range(g0, g1, chunk):
        c_, n_, d_ = chunk_terms(Qg[i0:min(i0 + chunk, g1)], Kg, tg, i0)
        sur = (dclip[i0:i0 + c_.shape[0]] * c_).sum() + 0.15 * n_ / n_el + (w_dg * d_ / cnt if cnt > 0 else 0.0)
        sur.backward()
    dtemp = tg.grad.detach().clone()
    if av:
        tc = t.clone().requires_grad_(True)
        (20 * (-torch.log(tc)).clamp(min=0).pow(2)).backward()
        dtemp += tc.grad
    out.update(dq=Qg.grad.detach(), dk=Kg.grad.detach(), dtemp=float(dtemp))
    return out


def near_ties(q, k, temperature, rel=8 * 2.0 ** -23, chunk=8, dtype=torch.float64):
    """Where a row max of S = temp * q k^T is decided below fp32 resolution.

    For every (query sample i, key sample j, query token r) the gap between the largest and the
    second-largest S[i, j, r, :] is computed in `dtype`; a gap <= rel * |max| (8 fp32 ulps of the
    max by default) is a near-tie: an fp32 evaluation with another summation order (the MFMA
    kernels) may pick the other key, which moves that row's max gradient (model.py:389 / 507) from
    one key to the other -- both answers are the reference's at fp32 precision. Returns
    (tie_q (Bq, Nq) bool: query rows with a near-tie against any key sample, tie_k (Bk, Nk) bool:
    keys that are the first or second candidate of one, number of near-tie rows)."""
    Bq, Nq, _ = q.shape
    Bk, Nk, _ = k.shape
    Qd, Kd = q.detach().to(dtype), k.detach().to(dtype)
    t = torch.as_tensor(temperature, dtype=dtype, device=q.device)
    tie_q = torch.zeros(Bq, Nq, dtype=torch.bool, device=q.device)
    tie_k = torch.zeros(Bk, Nk, dtype=torch.bool, device=q.device)
    n = 0
    if Nk < 2:
        return tie_q, tie_k, 0
    with torch.no_grad():
        for i0 in range(0, Bq, chunk):
            s = torch.einsum("iqd,jkd->ijqk", Qd[i0:i0 + chunk], Kd) * t
            v, ix = s.topk(2, dim=3)
            near = (v[..., 0] - v[..., 1]) <= rel * v[..., 0].abs()     # (c, Bk, Nq)
            n += int(near.sum())
            tie_q[i0:i0 + chunk] |= near.any(dim=1)
            jj = torch.arange(Bk, device=q.device)[None, :, None].expand_as(near)
            for c in (0, 1):
                tie_k[jj[near], ix[..., c][near]] = True
    return tie_q, tie_k, n


def grad_rel(got, ref, skip_rows=None):
    """Relative L2 error of a (B, N, D) gradient, rows flagged in skip_rows (B, N) left out."""
    g = got.detach().double().reshape(-1, got.shape[-1])
    r = ref.detach().double().to(g.device).reshape(-1, ref.shape[-1])
    if skip_rows is not None:
        keep = ~skip_rows.reshape(-1).to(g.device)
        g, r = g[keep], r[keep]
    return float((g - r).norm() / r.norm().clamp(min=1e-30))


def _symmetric_ce_dev(clip):
    """_symmetric_ce on any device."""
    n = clip.shape[0]
    idx = torch.arange(n, device=clip.device)
    row = -F.log_softmax(clip, dim=1)[idx, idx]
    col = -F.log_softmax(clip.t(), dim=1)[idx, idx]
    return (row + col).mean() / 2
