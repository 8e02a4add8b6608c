"""Generate golden fixtures for the dense tri-modal contrastive hot path.

Runs ONLY in the build container (it needs /root/reference). It imports the
reference's own `src/model.py` and calls its hot-path methods on seeded inputs,
then freezes inputs, outputs and autograd gradients as small .npz fixtures in
this directory. The fixtures are data; no reference source is copied.

Import recipe:
  * `transformers` is imported first (it probes `torchvision.__spec__`);
  * `torchvision`, `torchvision.transforms` and `peft` are absent from the image.
    They are only used by the reference's embedder constructors and by
    `MultiModalModel.forward` (model.py:13,17-21,235-248,616-622), never by the
    hot-path methods called here, so empty placeholder modules satisfy the
    module-level imports;
  * `MultiModalModel` is built without `__init__` (its __init__ fetches
    pretrained weights by name), and only the attributes the hot-path methods
    read are set: `temperature`, `patch_sparsity_threshold`,
    `patch_sparsity_weight` (model.py:348-351).

Methods exercised (file:line in /root/reference/src/model.py):
  compute_similarity_matrix            355-368
  compute_all_similarities_av          370-392
  compute_contrastive_loss_av          430-472 (-> 394-428)
  compute_all_similarities_tv          490-514
  compute_contrastive_loss_tv          544-593 (-> 516-542)
  ViTLoRAEmbedder.patch_dropout        268-308
and from /root/reference/src/retrieval.py: aggregator_av_a2v / _v2a (106-114),
compute_recall_at_k (117-144), aggregator_tv_t2v / _v2t (236-244); plus the
audio z-norm of AudioEmbedder.forward (model.py:56-62) through transformers'
Wav2Vec2FeatureExtractor.

Inputs are bf16-representable fp32 values (SURVEY §7 "hard parts": the parity
target is the fp32 computation on bf16-rounded inputs). Gradients are taken
w.r.t. the features and the temperature of the scalar `total` output.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

OUT = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
D = 512


def _import_reference():
    import transformers  # noqa: F401  (must precede the placeholders)
    for name in ("torchvision", "torchvision.transforms", "peft"):
        if name not in sys.modules:
            sys.modules[name] = types.ModuleType(name)
    sys.modules["peft"].LoraConfig = object
    sys.modules["peft"].get_peft_model = None
    sys.modules["peft"].TaskType = types.SimpleNamespace(FEATURE_EXTRACTION=None)
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.path.insert(0, REF_SRC)
    import model as ref_model  # the reference module
    return ref_model


def _make_model(ref_model, temperature, thr=0.80, w=0.01):
    m = ref_model.MultiModalModel.__new__(ref_model.MultiModalModel)
    nn.Module.__init__(m)
    m.temperature = nn.Parameter(torch.tensor(float(temperature)))
    m.patch_sparsity_threshold = thr
    m.patch_sparsity_weight = w
    return m


def _bf16(x):
    return x.to(torch.bfloat16).to(torch.float32)


def _feats(g, shape, scale=0.58):
    # LN->Linear(512,512)-like magnitudes (SURVEY §8d kernel microbench inputs)
    return _bf16(torch.randn(*shape, generator=g) * scale)


def _u16(x):
    """bf16-exact fp32 -> uint16 bit pattern (lossless for bf16 values)."""
    a = x.detach().to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    return a


def gen_av(ref_model, name, B, Na, Nv, temp, seed, nv_len=None):
    g = torch.Generator().manual_seed(seed)
    A = _feats(g, (B, Na, D))
    V = _feats(g, (B, Nv, D))
    if nv_len is not None:  # emulate patch-dropout zero padding: rows >= len are 0
        for j in range(B):
            V[j, nv_len[j]:] = 0
    m = _make_model(ref_model, temp)
    A.requires_grad_(True)
    V.requires_grad_(True)
    clip, tok = m.compute_all_similarities_av(A, V)
    total, ce, reg, smooth, stats = m.compute_contrastive_loss_av(clip, tok)
    total.backward()
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"),
        kind="av", A=_u16(A), V=_u16(V),
        nv_len=np.array(nv_len if nv_len is not None else [Nv] * B, np.int32),
        temp=np.float32(temp),
        clip=clip.detach().numpy().astype(np.float32),
        total=np.float64(total.item()), ce=np.float64(ce.item()),
        reg=np.float64(reg.item()), smooth=np.float64(smooth.item()),
        stats=np.array([stats[k] for k in (
            "av_pos_sim_mean", "av_pos_sim_std", "av_neg_sim_mean",
            "av_neg_sim_std", "av_separation", "av_hardest_negative")], np.float64),
        dA=A.grad.numpy().astype(np.float32), dV=V.grad.numpy().astype(np.float32),
        dtemp=np.float64(m.temperature.grad.item()),
    )
    print(name, "total", total.item(), "ce", ce.item())


def gen_tv(ref_model, name, B, Nt, Nv, temp, seed, lens, thr=0.80, w=0.01, nv_len=None):
    g = torch.Generator().manual_seed(seed)
    T = _feats(g, (B, Nt, D))
    V = _feats(g, (B, Nv, D))
    if nv_len is not None:
        for j in range(B):
            V[j, nv_len[j]:] = 0
    mask = torch.zeros(B, Nt, dtype=torch.long)
    for i, L in enumerate(lens):
        mask[i, :L] = 1
    m = _make_model(ref_model, temp, thr, w)
    T.requires_grad_(True)
    V.requires_grad_(True)
    clip, tok = m.compute_all_similarities_tv(T, V, mask)
    total, stats = m.compute_contrastive_loss_tv(clip, tok)
    total.backward()
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"),
        kind="tv", T=_u16(T), V=_u16(V), mask=mask.numpy().astype(np.int64),
        nv_len=np.array(nv_len if nv_len is not None else [Nv] * B, np.int32),
        temp=np.float32(temp), thr=np.float64(thr), w=np.float64(w),
        clip=clip.detach().numpy().astype(np.float32),
        total=np.float64(total.item()),
        stats=np.array([stats[k] for k in (
            "tv_pos_sim_mean", "tv_pos_sim_std", "tv_neg_sim_mean",
            "tv_neg_sim_std", "tv_separation", "tv_hardest_negative")], np.float64),
        dT=T.grad.numpy().astype(np.float32), dV=V.grad.numpy().astype(np.float32),
        dtemp=np.float64(m.temperature.grad.item()),
    )
    print(name, "total", total.item())


def gen_simmat(ref_model, name, B, N1, N2, temp, seed):
    g = torch.Generator().manual_seed(seed)
    f1 = _feats(g, (B, N1, D))
    f2 = _feats(g, (B, N2, D))
    m = _make_model(ref_model, temp)
    sim = m.compute_similarity_matrix(f1, f2)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), kind="simmat",
                        f1=_u16(f1), f2=_u16(f2), temp=np.float32(temp),
                        sim=sim.detach().numpy().astype(np.float32))
    print(name, sim.shape)


def gen_dropout(ref_model, name, B, N, drop, seed):
    emb = ref_model.ViTLoRAEmbedder.__new__(ref_model.ViTLoRAEmbedder)
    nn.Module.__init__(emb)
    emb.train()
    g = torch.Generator().manual_seed(seed)
    x = _feats(g, (B, N, D))
    torch.manual_seed(seed)
    out = emb.patch_dropout(x, drop)  # draws its own Bernoulli mask (model.py:282-284)
    # Re-draw the identical mask from the same global RNG state (same call shape and dtype).
    torch.manual_seed(seed)
    keep = torch.bernoulli(torch.ones(B, N, dtype=x.dtype) * (1 - drop)).bool()
    np.savez_compressed(os.path.join(OUT, name + ".npz"), kind="dropout",
                        x=_u16(x), keep=keep.numpy(), drop=np.float64(drop),
                        out=_u16(out))
    print(name, tuple(out.shape), keep.sum(1).tolist())


def _import_retrieval():
    sys.path.insert(0, REF_SRC)
    import retrieval as ref_retrieval  # the reference module (json/numpy/torch/tqdm only)
    return ref_retrieval


def _token_lists(g, n, lo, hi, normalize):
    out = []
    for _ in range(n):
        L = int(torch.randint(lo, hi + 1, (1,), generator=g))
        x = torch.randn(L, D, generator=g)
        if normalize:  # embed_av_subset L2-normalises (retrieval.py:93-94)
            x = torch.nn.functional.normalize(x, dim=-1)
        out.append(_bf16(x))
    return out


def gen_retrieval(ref_retrieval, name, kind, N, q_lens, k_lens, temp, seed, dup_items=(), zero_queries=()):
    """The reference's per-pair aggregators (retrieval.py:106-114 / 236-244) in its own double
    loop (retrieval.py:161-174, 255-264) and compute_recall_at_k (retrieval.py:117-144) on both
    N x N matrices. `dup_items` makes those item token lists identical (exact ties in every row);
    `zero_queries` zeroes those queries (a whole row of exact ties): both exercise the reference's
    unstable np.argsort tie order."""
    g = torch.Generator().manual_seed(seed)
    q = _token_lists(g, N, q_lens[0], q_lens[1], kind == "av")
    k = _token_lists(g, N, k_lens[0], k_lens[1], kind == "av")
    for i in range(N):  # matching pairs share content so recall is informative
        n = min(len(q[i]), len(k[i]))
        k[i][:n] = _bf16(k[i][:n] + 0.5 * q[i][:n])
    for j in dup_items[1:]:
        k[j] = k[dup_items[0]].clone()
    for i in zero_queries:
        q[i] = torch.zeros_like(q[i])
    f_qk = ref_retrieval.aggregator_av_a2v if kind == "av" else ref_retrieval.aggregator_tv_t2v
    f_kq = ref_retrieval.aggregator_av_v2a if kind == "av" else ref_retrieval.aggregator_tv_v2t
    s_qk = np.zeros((N, N), dtype=np.float32)
    s_kq = np.zeros((N, N), dtype=np.float32)
    for i in range(N):
        for j in range(N):
            s_qk[i, j] = f_qk(q[i], k[j], temp)      # query i (audio/text) vs item j (video)
            s_kq[i, j] = f_kq(q[j], k[i], temp)      # video i vs audio/text j (retrieval.py:171-174)
    r_qk = ref_retrieval.compute_recall_at_k(s_qk)
    r_kq = ref_retrieval.compute_recall_at_k(s_kq)
    ranks = lambda s: np.array([int(np.where(np.argsort(-s[i]) == i)[0][0]) for i in range(N)], np.int32)
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"), kind="retrieval_" + kind, temp=np.float32(temp),
        q=_u16(torch.cat(q)), q_len=np.array([len(x) for x in q], np.int32),
        k=_u16(torch.cat(k)), k_len=np.array([len(x) for x in k], np.int32),
        sim_qk=s_qk, sim_kq=s_kq, ranks_qk=ranks(s_qk), ranks_kq=ranks(s_kq),
        recall_qk=np.array([r_qk[x] for x in ("r1", "r5", "r10", "r20")], np.float64),
        recall_kq=np.array([r_kq[x] for x in ("r1", "r5", "r10", "r20")], np.float64))
    print(name, r_qk, r_kq)


def gen_znorm(name, B, T, seed, offset=0.0, scale=0.1):
    """The reference's audio z-norm: AutoProcessor("facebook/hubert-large-ls960-ft") called on the
    (B, T) waveform tensor (model.py:56-62). That checkpoint's processor is a
    Wav2Vec2FeatureExtractor(feature_size=1, sampling_rate=16000, padding_value=0.0,
    do_normalize=True, return_attention_mask=True) (its preprocessor_config.json); built here from
    those values because the hub is unreachable. A torch tensor is not recognised as a batch, so
    the whole (B, T) array is one utterance: ONE mean / variance over all B*T samples."""
    from transformers import Wav2Vec2FeatureExtractor
    fe = Wav2Vec2FeatureExtractor(feature_size=1, sampling_rate=16000, padding_value=0.0, do_normalize=True,
                                  return_attention_mask=True)
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, T, generator=g) * scale + offset
    y = fe(x, return_tensors="pt", sampling_rate=16000, padding=True,
           return_attention_mask=True).input_values.squeeze(0)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), kind="znorm", x=x.numpy().astype(np.float32),
                        y=y.numpy().astype(np.float32))
    print(name, tuple(y.shape), float(y.mean()), float(y.std()))


def main():
    torch.set_num_threads(8)
    ref = _import_reference()
    gen_av(ref, "av_b2_na7_nv16", 2, 7, 16, 1.5, 1)
    gen_av(ref, "av_b3_na49_nv32_t07", 3, 49, 32, 0.7, 2)          # l_cal branch (temp < 1)
    gen_av(ref, "av_b4_na1_nv16", 4, 1, 16, 1.5, 3)                # Na=1: smoothness over empty set
    gen_av(ref, "av_b5_na33_nv40_pad", 5, 33, 40, 1.5, 4, nv_len=[40, 31, 35, 27, 38])
    gen_av(ref, "av_b4_na199_nv64", 4, 199, 64, 1.5, 5, nv_len=[64, 50, 57, 61])
    gen_av(ref, "av_b8_na20_nv1", 8, 20, 1, 1.2, 6)                # Nv=1
    gen_tv(ref, "tv_b2_nt16_nv16", 2, 16, 16, 1.5, 11, lens=[16, 9])
    gen_tv(ref, "tv_b4_nt32_nv48", 4, 32, 48, 1.5, 12, lens=[32, 17, 1, 25])
    gen_tv(ref, "tv_b3_nt1_nv24", 3, 1, 24, 1.5, 13, lens=[1, 1, 1])
    gen_tv(ref, "tv_b4_nt8_nv20_sparse", 4, 8, 20, 0.9, 14, lens=[8, 3, 6, 5],
           thr=0.02, w=0.5, nv_len=[20, 14, 17, 19])                # sparsity term active
    gen_tv(ref, "tv_b3_nt5_nv12_zeromask", 3, 5, 12, 1.5, 15, lens=[5, 0, 2])  # empty caption
    gen_simmat(ref, "simmat_b2_n7_n16", 2, 7, 16, 1.5, 21)
    gen_dropout(ref, "dropout_b4_n64", 4, 64, 0.25, 31)
    gen_dropout(ref, "dropout_b3_n256", 3, 256, 0.25, 32)
    rr = _import_retrieval()
    gen_retrieval(rr, "retrieval_av_n40", "av", 40, (6, 24), (10, 30), 1.5, 41)
    gen_retrieval(rr, "retrieval_av_n24_ties", "av", 24, (4, 12), (5, 16), 0.9, 42, dup_items=(3, 7, 12, 20))
    gen_retrieval(rr, "retrieval_tv_n32_ties", "tv", 32, (1, 12), (8, 20), 1.5, 43, dup_items=(5, 9),
                  zero_queries=(2, 17))
    gen_znorm("znorm_b3_t8000", 3, 8000, 51)
    gen_znorm("znorm_b2_t4000_offset", 2, 4000, 52, offset=0.3, scale=0.02)
    gen_znorm("znorm_b1_t16000", 1, 16000, 53, scale=0.5)


if __name__ == "__main__":
    main()
