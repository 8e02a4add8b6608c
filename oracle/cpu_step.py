"""CPU port of the TRIAD full_joint training step -- the `cpu_baseline` of bench.py.

TEST / BASELINE INFRASTRUCTURE ONLY (see oracle/ref_cpu.py header). It runs the
reference's step on the host in fp32, exactly as src/train.py:954-1041 would on a
machine without a GPU (torch.cuda.amp.autocast is a no-op there):
  backbones (same architectures as the product: transformers HuBERT-base,
  DistilBERT-base, DINOv2-B/14-reg + LoRA) -> projection heads (ref_cpu) ->
  patch dropout (ref_cpu) -> AV / TV losses (ref_cpu, which materialises the
  (B,B,Nq,Nv) tensors like model.py) -> backward -> grad norms / clip ->
  four torch.optim.AdamW steps.
"""
from __future__ import annotations

import time

import torch
import torch.nn as nn

from . import ref_cpu


class _Head(nn.Module):
    def __init__(self, h):
        super().__init__()
        self.projection1 = nn.Linear(h, 512)
        self.layer_norm = nn.LayerNorm(512)
        self.projection2 = nn.Linear(512, 512)

    def forward(self, x):
        return ref_cpu.projection_head(x, self.projection1.weight, self.projection1.bias, self.layer_norm.weight,
                                       self.layer_norm.bias, self.projection2.weight, self.projection2.bias,
                                       amp=False)


class CPUTriad(nn.Module):
    def __init__(self, vit_arch="dinov2_vitb14_reg"):
        super().__init__()
        import transformers
        from triad_amd.vit import DinoVisionTransformer, apply_lora
        self.hubert = transformers.HubertModel(transformers.HubertConfig())
        self.encoder = transformers.DistilBertModel(transformers.DistilBertConfig())
        self.vit = apply_lora(DinoVisionTransformer(vit_arch))
        self.ha, self.ht, self.hv = _Head(768), _Head(768), _Head(self.vit.embed_dim)
        self.temperature = nn.Parameter(torch.tensor(1.5))


def make_batch(B, seed=1234, T=64000, Nt=32, px=224):
    g = torch.Generator().manual_seed(seed)
    frames = torch.randn(B, 3, px, px, generator=g)
    audio = torch.randn(B, T, generator=g) * 0.1
    ids = torch.randint(1000, 30522, (B, Nt), generator=g)
    mask = torch.ones(B, Nt, dtype=torch.long)
    return frames, audio, ids, mask


def time_steps(B=4, steps=2, warmup=1, threads=None, seed=1234):
    """Seconds per full_joint step of the CPU port at batch B."""
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    m = CPUTriad()
    m.train()
    opts = [torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-4)]
    frames, audio, ids, mask = make_batch(B, seed)
    gk = torch.Generator().manual_seed(seed + 1)

    def step():
        x = (audio - audio.mean()) / torch.sqrt(audio.var(unbiased=False) + 1e-7)
        a = m.ha(m.hubert(x).last_hidden_state)
        t = m.ht(m.encoder(input_ids=ids, attention_mask=mask).last_hidden_state)
        v = m.hv(m.vit.get_intermediate_layers(frames, n=1)[0])
        keep_av = torch.bernoulli(torch.full(v.shape[:2], 0.75), generator=gk)
        keep_tv = torch.bernoulli(torch.full(v.shape[:2], 0.75), generator=gk)
        v_av = ref_cpu.patch_dropout(v, keep_av)
        v_tv = ref_cpu.patch_dropout(v, keep_tv)
        av = ref_cpu.av_loss(a, v_av, m.temperature, dtype=torch.float32)[0]
        tv = ref_cpu.tv_loss(t, v_tv, mask, m.temperature, 0.80, 0.01, dtype=torch.float32)[0]
        loss = av + tv
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(m.hubert.parameters()) + list(m.ha.parameters()), 10.0)
        torch.nn.utils.clip_grad_norm_(list(m.encoder.parameters()) + list(m.ht.parameters()), 10.0)
        for o in opts:
            o.step()
            o.zero_grad()
        return float(loss.detach())

    for _ in range(warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    return (time.perf_counter() - t0) / steps


def time_head(B=8, Na=199, Nv=205, Nt=32, steps=3, warmup=1, threads=None, seed=1234):
    """Seconds per hot-path step of the CPU port at batch B: the AV + TV losses of the reference
    (materialising (B,B,Nq,Nv) fp32 tensors, model.py:370-593) forward + backward on random
    head-output features. Its pairwise part grows as B^2 (bench.py extrapolates to B = 256)."""
    if threads:
        torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(seed)
    a = (torch.randn(B, Na, 512, generator=g) * 0.58).requires_grad_(True)
    t = (torch.randn(B, Nt, 512, generator=g) * 0.58).requires_grad_(True)
    v = (torch.randn(B, Nv, 512, generator=g) * 0.58).requires_grad_(True)
    mask = torch.ones(B, Nt, dtype=torch.long)
    temp = torch.tensor(1.5, requires_grad=True)

    def step():
        av = ref_cpu.av_loss(a, v, temp, dtype=torch.float32)[0]
        tv = ref_cpu.tv_loss(t, v, mask, temp, 0.80, 0.01, dtype=torch.float32)[0]
        (av + tv).backward()

    for _ in range(warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    return (time.perf_counter() - t0) / steps
