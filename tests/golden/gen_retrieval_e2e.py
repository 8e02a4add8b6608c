"""Freeze the reference's MODEL-LEVEL retrieval on deterministic stand-ins (the fixture of
tests/test_retrieval_gpu.py::test_model_level_retrieval_matches_reference).

Runs ONLY in the build container: it imports /root/reference/src/retrieval.py (json, numpy,
torch, tqdm) and calls its own select_subset_indices, embed_av_subset, embed_tv_subset,
compute_av_retrieval_metrics and compute_tv_retrieval_metrics (retrieval.py:9-292) on the
stub model / datasets of tests/retrieval_stub.py, on the CPU, with python's `random` seeded
before each subset draw. Saves the subset indices, the embedded per-item features, the
reference's own N x N matrices and its result dicts. No reference source is copied.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_retrieval_e2e.py
"""
import os
import random
import sys
import tempfile

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(OUT))          # tests/ (retrieval_stub)
sys.path.insert(0, "/root/reference/src")
import retrieval as ref  # noqa: E402  (the reference module)
from retrieval_stub import AVStubDataset, StubModel, TVStubDataset  # noqa: E402

N_DATA, N_SUB, SEED = 24, 16, 7


def _flat(lst):
    lens = np.array([t.shape[0] for t in lst], dtype=np.int32)
    return np.concatenate([t.numpy() for t in lst]).astype(np.float16), lens   # compared at the bf16 bar


def _matrix(fn, q, k, temp):
    """The reference's double loop (retrieval.py:161-174 / 265-278) on the CPU."""
    n = len(q)
    s = np.zeros((n, n), dtype=np.float32)
    for i in range(n):
        for j in range(n):
            s[i, j] = fn(q[i], k[j], temp)
    return s


def main():
    torch.manual_seed(0)
    model = StubModel()
    temp = model.temperature.item()
    out = {"kind": "retrieval_e2e", "n_data": N_DATA, "n_sub": N_SUB, "seed": SEED, "temp": np.float32(temp)}
    with tempfile.TemporaryDirectory() as d:
        # AV
        av = AVStubDataset(N_DATA)
        random.seed(SEED)
        out["av_idx_sub"] = np.array(ref.select_subset_indices(av, os.path.join(d, "av1.json"), subset_size=N_SUB))
        random.seed(SEED)
        idx = ref.select_subset_indices(av, os.path.join(d, "av2.json"), subset_size=1000)
        a, v, paths = ref.embed_av_subset(model, av, idx, device="cpu", batch_size=8)
        random.seed(SEED)
        res_av = _compute(ref.compute_av_retrieval_metrics, model, av, os.path.join(d, "av3.json"))
        out["av_idx"] = np.array(idx, dtype=np.int64)
        out["av_a"], out["av_a_len"] = _flat(a)
        out["av_v"], out["av_v_len"] = _flat(v)
        out["av_a2v"] = _matrix(lambda x, y, t: ref.aggregator_av_a2v(x, y, t), a, v, temp)
        out["av_v2a"] = _matrix(lambda x, y, t: ref.aggregator_av_v2a(y, x, t), v, a, temp)
        out["av_keys"] = np.array(list(res_av.keys()))
        out["av_vals"] = np.array([float(x) for x in res_av.values()], dtype=np.float64)
        # TV
        tv = TVStubDataset(N_DATA)
        random.seed(SEED + 1)
        out["tv_idx_sub"] = np.array(ref.select_subset_indices(tv, os.path.join(d, "tv1.json"), subset_size=N_SUB))
        random.seed(SEED + 1)
        idx = ref.select_subset_indices(tv, os.path.join(d, "tv2.json"), subset_size=1000)
        t, im = ref.embed_tv_subset(model, tv, idx, device="cpu", batch_size=8)
        random.seed(SEED + 1)
        res_tv = _compute(ref.compute_tv_retrieval_metrics, model, tv, os.path.join(d, "tv3.json"))
        out["tv_idx"] = np.array(idx, dtype=np.int64)
        out["tv_t"], out["tv_t_len"] = _flat(t)
        out["tv_i"], out["tv_i_len"] = _flat(im)
        out["tv_t2v"] = _matrix(lambda x, y, tt: ref.aggregator_tv_t2v(x, y, tt), t, im, temp)
        out["tv_v2t"] = _matrix(lambda x, y, tt: ref.aggregator_tv_v2t(y, x, tt), im, t, temp)
        out["tv_keys"] = np.array(list(res_tv.keys()))
        out["tv_vals"] = np.array([float(x) for x in res_tv.values()], dtype=np.float64)
    out["av_paths"] = np.array(paths)
    np.savez_compressed(os.path.join(OUT, "retrieval_e2e_n24.npz"), **out)
    for k in ("av", "tv"):
        print(k, dict(zip(out[k + "_keys"], out[k + "_vals"])))


def _compute(fn, model, ds, path):
    """compute_*_retrieval_metrics draws a subset of 1000 (retrieval.py:154 / 258); the stand-in
    dataset holds N_DATA < 1000 items, so its subset is all of them, shuffled (select_subset_
    indices's own behaviour) -- the order the embed_* call and the matrices above use, from the
    same `random` seed. An N_SUB-item draw is recorded for the subset rule itself."""
    return fn(model, ds, path, device="cpu")


if __name__ == "__main__":
    main()
