"""1000-way cross-modal retrieval on the fused similarity kernel.

Reference: src/retrieval.py. It scores N x N (query, item) pairs with a Python double
loop (retrieval.py:161-174, 255-264), one matmul + max + mean + `.item()` per pair
(2 x 10^6 host syncs at N = 1000). Here each direction is ONE launch of the fused
pair-similarity kernel over all N^2 pairs (token lists packed and zero-padded, per-sample
query masks and key lengths so padding never takes part), plus the clip reduction.

  A->V: sim[i][j] = mean_a max_v  <a_i,a , v_j,v> / temp      (retrieval.py:106-109)
  V->A: sim[i][j] = mean_v max_a  <a_j,a , v_i,v> / temp      (retrieval.py:111-114)
  T->V / V->T: same with text tokens trimmed to their attention mask (retrieval.py:243-244);
  AV features are L2-normalised first (retrieval.py:93-94), TV features are not.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch

from . import ops
from ._lib import call, ptr, stream_ptr

D = ops.D


def _pack(feats: Sequence[torch.Tensor], device, rows_multiple: int):
    """list of (n_i, D) -> zero-padded (N, n_max, D) bf16 + lengths."""
    n_max = max(int(f.shape[0]) for f in feats)
    n_pad = ops._rup(n_max, rows_multiple)
    out = torch.zeros(len(feats), n_pad, D, dtype=torch.bfloat16, device=device)
    lens = torch.tensor([int(f.shape[0]) for f in feats], dtype=torch.int32)
    for i, f in enumerate(feats):
        out[i, :f.shape[0]] = f.to(device)
    return out, lens, n_max


def aggregated_similarity(queries: Sequence[torch.Tensor], items: Sequence[torch.Tensor], temperature: float,
                          device="cuda") -> torch.Tensor:
    """(N_q x N_k) matrix of mean over each query's tokens of the max over each item's tokens of
    <q, k> / temperature -- all pairs in one kernel launch."""
    dev = torch.device(device)
    Q, qlen, nq = _pack(queries, dev, 1)
    K, klen, nk = _pack(items, dev, 1)
    Bq, Bk = Q.shape[0], K.shape[0]
    g = ops.Geometry(Bq, nq, Bk, nk)
    Qb = ops.pack_queries(Q[:, :nq], g)
    Kb = ops.pack_keys(K[:, :nk], g)
    qmask = (torch.arange(nq)[None, :] < qlen[:, None]).to(torch.float32).to(dev)
    kl = klen.to(dev)
    inv_t = torch.tensor([1.0 / float(temperature)], dtype=torch.float32, device=dev)
    nparts = call("triad_pairsim_nparts", g.R_pad, g.Bk)
    rowmax = torch.empty(g.Bk, g.R_pad, dtype=torch.float32, device=dev)
    argmax = torch.empty(g.Bk, g.R_pad, dtype=torch.int32, device=dev)
    nn_part = torch.empty(nparts, dtype=torch.float64, device=dev)
    st = stream_ptr(dev)
    call("triad_pairsim_fwd", ptr(Qb), ptr(Kb), g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, D, ptr(inv_t),
         -60.0, 0, 0, ptr(rowmax), ptr(argmax), ptr(nn_part), None, None, 0, None, ptr(kl), st)
    sim = torch.empty(Bq, Bk, dtype=torch.float32, device=dev)
    call("triad_clip_reduce", ptr(rowmax), g.R_pad, g.Nq, g.Bq, g.Bk, ptr(qmask), ptr(sim), None, st)
    return sim


def ranks(sim: torch.Tensor, ties: str = "reference") -> torch.Tensor:
    """Rank of the matching item j = i in each query row (retrieval.py:124-131).

    ties="reference" orders exact ties as the reference does: its ranking is numpy's default
    (unstable) argsort of -row on the host, whose tie order is not an index rule, so the (N x N)
    fp32 matrix -- 4 MB at N = 1000 -- is ranked by that same host call (one batched argsort,
    not N). ties="stable" ranks on the device, ties resolved by item index."""
    if ties == "stable":
        n = sim.shape[0]
        diag = sim.diagonal()[:, None]
        idx = torch.arange(n, device=sim.device)
        ahead = (sim > diag) | ((sim == diag) & (idx[None, :] < idx[:, None]))
        return ahead.sum(1)
    if ties != "reference":
        raise ValueError(f"ties must be 'reference' or 'stable', not {ties!r}")
    import numpy as np
    s = sim.detach().to(torch.float32).cpu().numpy()
    order = np.argsort(-s, axis=1)   # row-wise identical to the reference's per-row np.argsort(-row)
    return torch.from_numpy((order == np.arange(s.shape[0])[:, None]).argmax(1))


def recall_at_k(sim: torch.Tensor, ks=(1, 5, 10, 20), ties: str = "reference") -> Dict[str, float]:
    """compute_recall_at_k (retrieval.py:117-144): fraction of queries whose match ranks < k."""
    r = ranks(sim, ties)
    return {f"r{k}": float((r < k).double().mean()) for k in ks}


def av_retrieval_metrics(audio_feats: List[torch.Tensor], video_feats: List[torch.Tensor], temperature: float,
                         device="cuda") -> Dict[str, float]:
    """compute_av_retrieval_metrics (retrieval.py:146-198) from embedded subsets
    (already L2-normalised as embed_av_subset does, retrieval.py:93-94)."""
    a2v = aggregated_similarity(audio_feats, video_feats, temperature, device)
    v2a = aggregated_similarity(video_feats, audio_feats, temperature, device)
    ra, rv = recall_at_k(a2v), recall_at_k(v2a)
    return {**{f"A->V_{k}": v for k, v in ra.items()}, **{f"V->A_{k}": v for k, v in rv.items()}}


def tv_retrieval_metrics(text_feats: List[torch.Tensor], image_feats: List[torch.Tensor], temperature: float,
                         device="cuda") -> Dict[str, float]:
    """compute_tv_retrieval_metrics (retrieval.py:250-292) from embedded subsets (text trimmed
    to its attention mask, no normalisation)."""
    t2v = aggregated_similarity(text_feats, image_feats, temperature, device)
    v2t = aggregated_similarity(image_feats, text_feats, temperature, device)
    rt, rv = recall_at_k(t2v), recall_at_k(v2t)
    return {**{f"T->V_{k}": v for k, v in rt.items()}, **{f"V->T_{k}": v for k, v in rv.items()}}
