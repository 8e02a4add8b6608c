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


if __name__ == "__main__":
    main()
