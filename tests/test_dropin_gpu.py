"""The drop-in model API of the reference (reference src/model.py:370-608) on the HIP
path: the materialising debug methods (compute_all_similarities_* -> compute_contrastive_loss_*,
compute_regularization_losses_*, compute_temporal_smoothness_loss) against the golden fixtures
the reference itself produced, and forward_audio_visual / forward_text_visual with injected
embedder outputs (the backbones are stubs returning the fixture features).

Tolerances (north star): losses / clip / statistics 1e-4 relative (fp32 arithmetic on
bf16-exact inputs); feature gradients the bf16 bar (relative L2 < 1e-2; the token-similarity
gradient is a bf16 GEMM operand); d/dtemp 1e-3 relative.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import ref_cpu
from tests import golden_io as G

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _close(a, b, rtol=1e-4, atol=1e-5):
    if math.isnan(b):
        return math.isnan(a)
    return abs(a - b) <= atol + rtol * abs(b)


def _grad_ok(got, ref, bar=1e-2):
    got = got.detach().float().cpu().numpy()
    assert _rel(got, ref) < bar, _rel(got, ref)


def light_model(temp, thr=0.80, w=0.01):
    """A MultiModalModel with only what the loss-head methods read (the embedders are attached
    by the caller): the same construction the golden generator used on the reference."""
    from triad_amd.model import MultiModalModel
    m = MultiModalModel.__new__(MultiModalModel)
    nn.Module.__init__(m)
    m.temperature = nn.Parameter(torch.tensor(float(temp), device=dev))
    m.patch_sparsity_threshold = thr
    m.patch_sparsity_weight = w
    m.use_amp = True
    m.amp_dtype = torch.bfloat16
    m.negatives_group = None
    return m


class _Stub(nn.Module):
    """Embedder stand-in: returns fixed features (and a mask for text) as bf16, like autocast."""

    def __init__(self, feats, mask=None):
        super().__init__()
        self.feats = feats
        self.mask = mask

    def forward(self, _x):
        f = self.feats.to(torch.bfloat16)
        return f if self.mask is None else (f, self.mask)


@pytest.mark.parametrize("name", G.names("av"))
def test_debug_path_av_matches_golden(name):
    f = G.load(name)
    m = light_model(f["temp"])
    A = G.bf16(f["A"]).to(dev).requires_grad_(True)
    V = G.bf16(f["V"]).to(dev).requires_grad_(True)
    clip, tok = m.compute_all_similarities_av(A, V)
    assert tok.shape == (A.shape[0], V.shape[0], A.shape[1], V.shape[1]) and tok.dtype == torch.float32
    total, ce, reg, smooth, stats = m.compute_contrastive_loss_av(clip, tok)
    total.backward()
    np.testing.assert_allclose(clip.detach().cpu().numpy(), f["clip"], rtol=1e-4, atol=1e-4)
    for got, key in ((total, "total"), (ce, "ce"), (reg, "reg"), (smooth, "smooth")):
        assert _close(float(got), float(f[key])), (key, float(got), float(f[key]))
    keys = ("av_pos_sim_mean", "av_pos_sim_std", "av_neg_sim_mean", "av_neg_sim_std", "av_separation",
            "av_hardest_negative")
    assert list(stats) == list(keys)
    for k, want in zip(keys, f["stats"]):
        assert isinstance(stats[k], float) and _close(stats[k], float(want), 1e-4, 1e-4)
    _grad_ok(A.grad, f["dA"])
    _grad_ok(V.grad, f["dV"])
    assert _close(float(m.temperature.grad), float(f["dtemp"]), 1e-3, 1e-5)


@pytest.mark.parametrize("name", G.names("tv"))
def test_debug_path_tv_matches_golden(name):
    f = G.load(name)
    m = light_model(f["temp"], float(f["thr"]), float(f["w"]))
    T = G.bf16(f["T"]).to(dev).requires_grad_(True)
    V = G.bf16(f["V"]).to(dev).requires_grad_(True)
    mask = torch.from_numpy(f["mask"]).to(dev)
    clip, tok = m.compute_all_similarities_tv(T, V, mask)
    total, stats = m.compute_contrastive_loss_tv(clip, tok)
    total.backward()
    np.testing.assert_allclose(clip.detach().cpu().numpy(), f["clip"], rtol=1e-4, atol=1e-4)
    assert _close(float(total), float(f["total"]))
    for k, want in zip(stats, f["stats"]):
        assert _close(stats[k], float(want), 1e-4, 1e-4)
    _grad_ok(T.grad, f["dT"])
    _grad_ok(V.grad, f["dV"])
    assert _close(float(m.temperature.grad), float(f["dtemp"]), 1e-3, 1e-5)


@pytest.mark.parametrize("Nq", [1, 7])
def test_regularisers_on_given_token_sims_vs_oracle(Nq):
    """compute_temporal_smoothness_loss / compute_regularization_losses_{av,tv} on a token_sims
    leaf tensor (fp32, no bf16 rounding anywhere): values and d/d token_sims to fp32 precision;
    Nq = 1 gives the reference's mean-of-empty NaN smoothness."""
    g = torch.Generator().manual_seed(9)
    B, Nk = 4, 19
    S = (torch.randn(B, B, Nq, Nk, generator=g) * 30).float()
    m = light_model(0.8, thr=0.05, w=0.4)
    t = torch.tensor(0.8, dtype=torch.float64, requires_grad=True)
    for kind in ("av", "tv"):
        Sg = S.to(dev).requires_grad_(True)
        Sr = S.double().requires_grad_(True)
        if kind == "av":
            sm = m.compute_temporal_smoothness_loss(Sg)
            sm_ref = ref_cpu.temporal_smoothness(Sr)
            assert _close(float(sm), float(sm_ref), 1e-5, 1e-6)
            reg, sm1 = m.compute_regularization_losses_av(Sg)
            reg_ref, sm1_ref = ref_cpu.regularization_av(Sr, t)
            assert _close(float(sm1), float(sm1_ref), 1e-5, 1e-6)
        else:
            reg = m.compute_regularization_losses_tv(Sg)
            reg_ref = ref_cpu.regularization_tv(Sr, 0.05, 0.4)
        assert _close(float(reg), float(reg_ref), 1e-5, 1e-6), (kind, float(reg), float(reg_ref))
        if Nq == 1 and kind == "av":
            continue   # NaN smoothness: its gradient is NaN in both
        reg.backward()
        reg_ref.backward()
        np.testing.assert_allclose(Sg.grad.cpu().numpy(), Sr.grad.numpy(), rtol=1e-4,
                                   atol=1e-6 * float(Sr.grad.abs().max()))


def _attach_stubs(m, a_or_t, V, mask=None):
    m.visual_embedder = _Stub(V)
    if mask is None:
        m.audio_embedder = _Stub(a_or_t)
    else:
        m.text_embedder = _Stub(a_or_t, mask)


@pytest.mark.parametrize("name", G.names("av"))
def test_forward_audio_visual_injected_matches_golden(name):
    """forward_audio_visual (fused HIP head) on injected embedder outputs: the reference's return
    tuple (total, contrastive, reg, 0.01 smooth, stats) and the gradients that reach the
    embedder outputs."""
    f = G.load(name)
    m = light_model(f["temp"])
    A = G.bf16(f["A"]).to(dev).requires_grad_(True)
    V = G.bf16(f["V"]).to(dev).requires_grad_(True)
    _attach_stubs(m, A, V)
    out = m.forward_audio_visual(torch.zeros(1, device=dev), torch.zeros(1, device=dev))
    assert len(out) == 5
    total, ce, reg, smooth, stats = out
    total.backward()
    for got, key in ((total, "total"), (ce, "ce"), (reg, "reg"), (smooth, "smooth")):
        assert _close(float(got), float(f[key])), key
    for k, want in zip(stats, f["stats"]):
        assert _close(stats[k], float(want), 1e-4, 1e-4)
    _grad_ok(A.grad, f["dA"])
    _grad_ok(V.grad, f["dV"])
    assert _close(float(m.temperature.grad), float(f["dtemp"]), 1e-3, 1e-5)


@pytest.mark.parametrize("name", G.names("tv"))
def test_forward_text_visual_injected_matches_golden(name):
    f = G.load(name)
    m = light_model(f["temp"], float(f["thr"]), float(f["w"]))
    T = G.bf16(f["T"]).to(dev).requires_grad_(True)
    V = G.bf16(f["V"]).to(dev).requires_grad_(True)
    _attach_stubs(m, T, V, torch.from_numpy(f["mask"]).to(dev))
    out = m.forward_text_visual(torch.zeros(1, device=dev), ["x"])
    assert len(out) == 2
    total, stats = out
    total.backward()
    assert _close(float(total), float(f["total"]))
    for k, want in zip(stats, f["stats"]):
        assert _close(stats[k], float(want), 1e-4, 1e-4)
    _grad_ok(T.grad, f["dT"])
    _grad_ok(V.grad, f["dV"])
    assert _close(float(m.temperature.grad), float(f["dtemp"]), 1e-3, 1e-5)


def test_debug_and_fused_paths_agree():
    """The materialising debug path and the fused training head give the same losses, stats and
    gradients on one random AV case with zero-padded keys."""
    from triad_amd import ops
    g = torch.Generator().manual_seed(77)
    B, Na, Nv = 6, 33, 45
    A = (torch.randn(B, Na, 512, generator=g) * 0.58).to(torch.bfloat16)
    V = (torch.randn(B, Nv, 512, generator=g) * 0.58).to(torch.bfloat16)
    V[3, 30:] = 0
    m = light_model(1.5)
    Ad, Vd = A.to(dev).float().requires_grad_(True), V.to(dev).float().requires_grad_(True)
    clip, tok = m.compute_all_similarities_av(Ad, Vd)
    res = m.compute_contrastive_loss_av(clip, tok)
    res[0].backward()
    A2, V2 = A.to(dev).requires_grad_(True), V.to(dev).requires_grad_(True)
    t2 = torch.tensor(1.5, device=dev, requires_grad=True)
    losses, st, clip2 = ops.contrastive_head(ops.AV, A2, V2, t2)
    losses[0].backward()
    np.testing.assert_allclose(clip.detach().cpu().numpy(), clip2.cpu().numpy(), rtol=1e-5, atol=1e-5)
    for a, b in zip(res[:4], losses):
        assert _close(float(a), float(b), 1e-5, 1e-6)
    assert _rel(Ad.grad.cpu(), A2.grad.float().cpu()) < 1e-2
    assert _rel(Vd.grad.cpu(), V2.grad.float().cpu()) < 1e-2
    assert _close(float(m.temperature.grad), float(t2.grad), 1e-3, 1e-6)


@pytest.mark.parametrize("name", G.names("dropout"))
def test_vit_embedder_patch_dropout_matches_reference(name):
    """ViTEmbedder (model.py:120-205; the non-LoRA visual embedder) drops patches with the same
    algorithm as ViTLoRAEmbedder (model.py:143-183 == 268-308): against the reference's own
    patch_dropout outputs (the golden fixtures) with the fixture's keep mask injected."""
    from triad_amd.model import ViTEmbedder
    f = G.load(name)
    emb = ViTEmbedder(arch="dinov2_vits14").to(dev).train()
    x = G.bf16(f["x"]).to(dev, torch.bfloat16)
    out = emb.patch_dropout(x, 0.25, torch.from_numpy(f["keep"]))
    np.testing.assert_array_equal(out.float().cpu().numpy(), G.bf16(f["out"]).numpy())
    emb.eval()
    assert emb.patch_dropout(x, 0.25) is x   # eval / drop 0: unchanged (model.py:150-151)


def test_vit_embedder_forward_is_backbone_head_dropout():
    """ViTEmbedder.forward = DINOv2 patch tokens (get_intermediate_layers(x, n=1)[0]) -> projection
    head (HIP) -> patch dropout (HIP gather), every parameter trainable: against the same steps
    composed by hand (the head through the oracle's bf16-autocast emulation), and gradients reach
    the backbone (no frozen base, model.py:136-141)."""
    from triad_amd.model import ViTEmbedder
    torch.manual_seed(3)
    emb = ViTEmbedder(arch="dinov2_vits14", dropout_prob=0.25).to(dev).train()
    x = torch.randn(3, 3, 224, 224, device=dev)
    keep = torch.rand(3, 256, generator=torch.Generator().manual_seed(4)) > 0.25
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = emb(x, keep_mask=keep)
        patches = emb.model.get_intermediate_layers(x, n=1)[0]
    assert patches.shape == (3, 256, 384)
    w = [p.detach() for m in (emb.projection1, emb.layer_norm, emb.projection2) for p in m.parameters()]
    head = ref_cpu.projection_head(patches.detach().float(), *w, amp=True)
    ref = torch.zeros(3, int(keep.sum(1).max()), 512, device=dev)
    for b in range(3):
        kept = keep[b].nonzero().flatten().to(dev)
        ref[b, :len(kept)] = head[b, kept]
    assert out.shape == ref.shape and out.dtype == torch.bfloat16
    np.testing.assert_allclose(out.detach().float().cpu().numpy(), ref.cpu().numpy(), rtol=1.6e-2, atol=2e-2)
    out.float().sum().backward()
    assert all(p.requires_grad for p in emb.parameters())
    assert emb.model.blocks[0].attn.qkv.weight.grad is not None
    assert float(emb.model.patch_embed.proj.weight.grad.abs().sum()) > 0
