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

Model-level entry points with the reference's names, arguments and return values:
`select_subset_indices`, `embed_av_subset`, `embed_tv_subset`, `compute_av_retrieval_metrics`,
`compute_tv_retrieval_metrics` (retrieval.py:9-104, 146-188, 200-292). The dataset side (the
reference's DataLoader over its video / CC3M datasets) is the caller's: any map-style dataset
with the reference's item format works. Precision: with `model.use_amp` (the default) the
embedders run under the model's bf16 autocast and the pairs are scored on the bf16 MFMA kernel,
multiplying by 1 / temperature in fp32 where the reference divides (the product path); with
`model.use_amp = False` the drop-in matches the reference's arithmetic -- fp32 embeddings, fp32
normalisation (triad_l2norm_rows_f32) and the fp32 scorer (triad_retrieval_maxmean_f32: the
reference's division by the temperature, max, mean), so matrices agree to fp32 evaluation order.
"""
from __future__ import annotations

import json
import os
import random
from typing import Dict, List, Sequence

import numpy as np
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


def _feature_width(*lists) -> int:
    """The common feature width of every (n_i, D) tensor in `lists`; the fp32 scorer takes any
    D that is a multiple of 32 (its 32-wide k step)."""
    widths = {int(f.shape[-1]) for feats in lists for f in feats}
    if len(widths) != 1:
        raise ops.TriadError(f"retrieval features must share one width, got {sorted(widths)}")
    (d,) = widths
    if d <= 0 or d % 32:
        raise ops.TriadError(f"the fp32 retrieval scorer needs a feature width that is a multiple of 32, got {d}")
    return d


def _pack_f32(feats: Sequence[torch.Tensor], device, d: int):
    """list of (n_i, d) -> zero-padded (N, n_pad, d) fp32 (n_pad a multiple of 64) + device lengths."""
    n_pad = ops._rup(max(int(f.shape[0]) for f in feats), 64)
    out = torch.zeros(len(feats), n_pad, d, dtype=torch.float32, device=device)
    for i, f in enumerate(feats):
        out[i, :f.shape[0]] = f.to(device, torch.float32)
    lens = torch.tensor([int(f.shape[0]) for f in feats], dtype=torch.int32).to(device)
    return out, lens, n_pad


def aggregated_similarity_f32(queries: Sequence[torch.Tensor], items: Sequence[torch.Tensor], temperature: float,
                              device="cuda") -> torch.Tensor:
    """aggregated_similarity in the reference's fp32 arithmetic (retrieval.py:106-114: fp32 matmul,
    division by the temperature, max, mean) -- all pairs in one triad_retrieval_maxmean_f32 launch."""
    dev = torch.device(device)
    d = _feature_width(queries, items)
    Q, qlen, nq_pad = _pack_f32(queries, dev, d)
    K, klen, nk_pad = _pack_f32(items, dev, d)
    sim = torch.empty(len(queries), len(items), dtype=torch.float32, device=dev)
    call("triad_retrieval_maxmean_f32", ptr(Q), ptr(qlen), len(queries), nq_pad, ptr(K), ptr(klen), len(items),
         nk_pad, d, float(temperature), ptr(sim), stream_ptr(dev))
    return sim


# ---- the reference's per-pair aggregators and recall (retrieval.py:106-144, 190-198) -----------
# Same names, arguments and return types (a Python float / a dict of r1..r20). Each pair is one
# launch of the fp32 scorer -- the reference's arithmetic (fp32 products, division by the
# temperature, max, mean) -- so a caller looping over pairs as retrieval.py does gets its numbers;
# the all-pairs matrices of compute_*_retrieval_metrics take one launch per direction instead.
def _pair_maxmean(q_feats, k_feats, temperature) -> float:
    dev = q_feats.device if q_feats.is_cuda else k_feats.device
    return float(aggregated_similarity_f32([q_feats], [k_feats], float(temperature), dev)[0, 0])


def aggregator_av_a2v(a_feats, v_feats, temperature):
    """retrieval.py:106-110: mean over audio tokens of the max over visual tokens of a.v / temp."""
    return _pair_maxmean(a_feats, v_feats, temperature)


def aggregator_av_v2a(a_feats, v_feats, temperature):
    """retrieval.py:112-115: mean over visual tokens of the max over audio tokens of a.v / temp."""
    return _pair_maxmean(v_feats, a_feats, temperature)


def aggregator_tv_t2v(t_feats, v_feats, temperature):
    """retrieval.py:190-193: mean over text tokens of the max over visual tokens of t.v / temp."""
    return _pair_maxmean(t_feats, v_feats, temperature)


def aggregator_tv_v2t(t_feats, v_feats, temperature):
    """retrieval.py:195-198: mean over visual tokens of the max over text tokens of t.v / temp."""
    return _pair_maxmean(v_feats, t_feats, temperature)


def compute_recall_at_k(sim_matrix):
    """retrieval.py:117-144: R@1/5/10/20 of an N x N matrix (numpy or torch), the match at j = i,
    ranks with the reference's own tie order (per-row numpy argsort of -row)."""
    sim = sim_matrix if isinstance(sim_matrix, torch.Tensor) else torch.from_numpy(
        np.asarray(sim_matrix, dtype=np.float32))
    return recall_at_k(sim, ks=(1, 5, 10, 20), ties="reference")


def aggregated_similarity(queries: Sequence[torch.Tensor], items: Sequence[torch.Tensor], temperature: float,
                          device="cuda", precision: str = "bf16") -> torch.Tensor:
    """(N_q x N_k) matrix of mean over each query's tokens of the max over each item's tokens of
    <q, k> / temperature -- all pairs in one kernel launch. precision "bf16": the product path
    (bf16 operands on the MFMA pair kernel); "fp32": aggregated_similarity_f32."""
    if precision == "fp32":
        return aggregated_similarity_f32(queries, items, temperature, device)
    if precision != "bf16":
        raise ValueError(f"precision must be 'bf16' or 'fp32', not {precision!r}")
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
    s = sim.detach().to(torch.float32).cpu().numpy()
    order = np.argsort(-s, axis=1)   # row-wise identical to the reference's per-row np.argsort(-row)
    return torch.from_numpy((order == np.arange(s.shape[0])[:, None]).argmax(1))


def recall_at_k(sim: torch.Tensor, ks=(1, 5, 10, 20), ties: str = "reference") -> Dict[str, float]:
    """compute_recall_at_k (retrieval.py:117-144): fraction of queries whose match ranks < k."""
    r = ranks(sim, ties)
    return {f"r{k}": float((r < k).double().mean()) for k in ks}


def av_retrieval_metrics(audio_feats: List[torch.Tensor], video_feats: List[torch.Tensor], temperature: float,
                         device="cuda", precision: str = "bf16") -> Dict[str, float]:
    """compute_av_retrieval_metrics (retrieval.py:146-198) from embedded subsets
    (already L2-normalised as embed_av_subset does, retrieval.py:93-94)."""
    a2v = aggregated_similarity(audio_feats, video_feats, temperature, device, precision)
    v2a = aggregated_similarity(video_feats, audio_feats, temperature, device, precision)
    ra, rv = recall_at_k(a2v), recall_at_k(v2a)
    return {**{f"A->V_{k}": v for k, v in ra.items()}, **{f"V->A_{k}": v for k, v in rv.items()}}


def tv_retrieval_metrics(text_feats: List[torch.Tensor], image_feats: List[torch.Tensor], temperature: float,
                         device="cuda", precision: str = "bf16") -> Dict[str, float]:
    """compute_tv_retrieval_metrics (retrieval.py:250-292) from embedded subsets (text trimmed
    to its attention mask, no normalisation)."""
    t2v = aggregated_similarity(text_feats, image_feats, temperature, device, precision)
    v2t = aggregated_similarity(image_feats, text_feats, temperature, device, precision)
    rt, rv = recall_at_k(t2v), recall_at_k(v2t)
    return {**{f"T->V_{k}": v for k, v in rt.items()}, **{f"V->T_{k}": v for k, v in rv.items()}}


# ---- model-level drop-in (retrieval.py:9-104, 146-188, 200-292) ------------------------------
def select_subset_indices(dataset, subset_file, subset_size=1000):
    """retrieval.py:9-30: the indices stored in `subset_file` (JSON list) if it exists, else a
    random subset (python `random.shuffle` of range(len(dataset)), first `subset_size`), written
    there -- the same draw as the reference from the same `random` state."""
    if os.path.exists(subset_file):
        with open(subset_file, "r") as f:
            indices = json.load(f)
        print(f"Loaded {len(indices)} subset indices from {subset_file}")
        return indices
    all_indices = list(range(len(dataset)))
    random.shuffle(all_indices)
    subset = all_indices[:subset_size]
    with open(subset_file, "w") as f:
        json.dump(subset, f)
    print(f"Created new subset of size {subset_size} and wrote to {subset_file}")
    return subset


class _Subset(torch.utils.data.Dataset):
    def __init__(self, base, indices, av):
        self.base, self.indices, self.av = base, indices, av

    def __len__(self):
        return len(self.indices)

    def __getitem__(self, i):
        if self.av:   # the AV dataset's evaluation item (no augmentation), retrieval.py:75
            return self.base.__getitem__(self.indices[i], apply_augmentation=False)
        return self.base.__getitem__(self.indices[i])


def _collate_av(batch):
    """retrieval.py:46-64: stack frames, zero-pad the waveforms to the batch's longest."""
    audios = [item["audio"] for item in batch]
    n = max(a.shape[0] for a in audios)
    audio = torch.zeros(len(audios), n)
    for i, a in enumerate(audios):
        audio[i, :a.shape[0]] = a
    return {"frames": torch.stack([item["video_frames"] for item in batch]), "audio": audio,
            "paths": [item["video_path"] for item in batch]}


def _collate_tv(batch):
    images, captions = zip(*batch)
    return torch.stack(images), list(captions)


def _amp(model):
    return torch.autocast("cuda", dtype=getattr(model, "amp_dtype", torch.bfloat16), enabled=_uses_amp(model))


def _uses_amp(model) -> bool:
    """bf16 product path unless the model was built with use_amp=False (then the reference's fp32)."""
    return bool(getattr(model, "use_amp", True))


def embed_av_subset(model, dataset, subset_indices, device="cuda", batch_size=8, num_workers=4,
                    out_device="cpu"):
    """retrieval.py:32-104: (audio_feats_list, video_feats_list, video_paths_list), one
    L2-normalised (N_i, 512) tensor per item (the HIP row normalisation, F.normalize's eps).
    Like the reference this leaves the model in eval mode (no patch dropout). `out_device`:
    where the per-item tensors go ("cpu" as the reference; the device keeps them resident for
    compute_av_retrieval_metrics)."""
    model.eval()
    N = len(subset_indices)
    a_list, v_list, p_list = [None] * N, [None] * N, [None] * N
    loader = torch.utils.data.DataLoader(_Subset(dataset, subset_indices, True), batch_size=batch_size,
                                         shuffle=False, num_workers=num_workers, collate_fn=_collate_av,
                                         drop_last=False)
    off = 0
    with torch.no_grad():
        for batch in loader:
            frames = batch["frames"].to(device)
            audio = batch["audio"].to(device)
            with _amp(model):
                vfeats = model.visual_embedder(frames)
                afeats = model.audio_embedder(audio)
            norm = ops.l2_normalize if _uses_amp(model) else ops.l2_normalize_f32
            vfeats, afeats = norm(vfeats), norm(afeats)
            for b in range(vfeats.shape[0]):
                a_list[off + b] = afeats[b].to(out_device)
                v_list[off + b] = vfeats[b].to(out_device)
                p_list[off + b] = batch["paths"][b]
            off += vfeats.shape[0]
    return a_list, v_list, p_list


def embed_tv_subset(model, dataset, subset_indices, device="cuda", batch_size=8, num_workers=4, out_device="cpu"):
    """retrieval.py:200-248: (text_feats_list, image_feats_list); each caption's features trimmed
    to its attention mask's token count (retrieval.py:243-244), no normalisation."""
    model.eval()
    N = len(subset_indices)
    t_list, i_list = [None] * N, [None] * N
    loader = torch.utils.data.DataLoader(_Subset(dataset, subset_indices, False), batch_size=batch_size,
                                         shuffle=False, num_workers=num_workers, collate_fn=_collate_tv)
    off = 0
    with torch.no_grad():
        for images, captions in loader:
            images = images.to(device)
            with _amp(model):
                vfeats = model.visual_embedder(images)
                tfeats, mask = model.text_embedder(captions)
            n_tok = mask.sum(1).tolist()   # host list (one small copy per batch)
            for b in range(vfeats.shape[0]):
                t_list[off + b] = tfeats[b, :int(n_tok[b])].to(out_device)
                i_list[off + b] = vfeats[b].to(out_device)
            off += vfeats.shape[0]
    return t_list, i_list


def compute_av_retrieval_metrics(model, dataset, subset_file, device="cuda", subset_size=1000, batch_size=8,
                                 num_workers=4):
    """retrieval.py:146-188: subset -> embed -> A->V and V->A matrices (one fused-kernel launch
    each instead of the reference's N^2 per-pair loop) -> R@1/5/10/20 with the reference's keys."""
    indices = select_subset_indices(dataset, subset_file, subset_size=subset_size)
    a, v, _ = embed_av_subset(model, dataset, indices, device=device, batch_size=batch_size,
                              num_workers=num_workers, out_device=device)
    return av_retrieval_metrics(a, v, model.temperature.item(), device, "bf16" if _uses_amp(model) else "fp32")


def compute_tv_retrieval_metrics(model, dataset, subset_file, device="cuda", subset_size=1000, batch_size=8,
                                 num_workers=4):
    """retrieval.py:250-292, as compute_av_retrieval_metrics with T->V / V->T keys."""
    indices = select_subset_indices(dataset, subset_file, subset_size=subset_size)
    t, im = embed_tv_subset(model, dataset, indices, device=device, batch_size=batch_size,
                            num_workers=num_workers, out_device=device)
    return tv_retrieval_metrics(t, im, model.temperature.item(), device, "bf16" if _uses_amp(model) else "fp32")
