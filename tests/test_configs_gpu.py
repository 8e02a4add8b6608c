"""Parity at the BASELINE.json configurations, through the drop-in model on the HIP path.

Each test runs the product path at the configuration's real shapes (real random-init backbones,
real patch-dropout padding), captures the embedder outputs that reach the fused loss heads, and
checks the head's losses, statistics and every gradient that leaves it against the fp64 oracle
evaluated chunk by chunk on the device (oracle.ref_cpu.head_loss_chunked: the materialising
reference restatement, never holding the (B, B, Nq, Nk) tensor whole; pinned to the
materialising oracle in tests/test_oracle_golden.py, which is pinned to the reference's own
outputs).

  c1  image-text, DINOv2-S/14-reg + DistilBERT, B=2, 16-token captions   forward_text_visual
  c2  image-audio, DINOv2-B/14-reg + HuBERT-base, B=128, 4 s audio       forward_audio_visual
  c3  tri-modal, B=256 (AV Na=199, Nk_eff ~ 215; TV Nt=32)             forward_triad (bench step)
  c5  DINOv2-L/14-reg + HuBERT-large, 518 px, 10 s, per-rank B=32        forward_triad
  (c4 -- 8-GPU global negatives -- is the multi-rank form of c3: tests/test_dist_*.py.)

Tolerances (north star): losses / clip / statistics 1e-4 relative (the kernels do exact fp32
arithmetic on the bf16 features; the oracle is fp64 on the same values); feature gradients the
bf16 bar, relative L2 < 1e-2 (dS is a bf16 MFMA operand; measured 1.8e-3 - 3.0e-3 at every
configuration, profiles/r02_config_grad_errors.log) over the rows no fp32 near-tie of a row max
touches (oracle.ref_cpu.near_ties; those rows are counted, < 3 %); d/dtemp 1e-3 relative.
"""
import math

import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu
dev = "cuda"


def _log(msg):
    """Progress on stderr (shown with -s): the large configurations take tens of seconds."""
    import sys
    import time
    print(f"[configs {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


def _close(a, b, rtol=1e-4, atol=1e-5):
    if math.isnan(b):
        return math.isnan(a)
    return abs(a - b) <= atol + rtol * abs(b)


class Capture:
    """Records the tensors that enter the loss heads (and keeps their gradients)."""

    def __init__(self, model):
        self.v, self.a, self.t, self.mask = [], None, None, None
        ve = model.visual_embedder
        inner = ve.patch_dropout

        def patch_dropout(x, rate, keep=None):
            out = inner(x, rate, keep)
            out.retain_grad()
            self.v.append(out)
            return out
        ve.patch_dropout = patch_dropout
        model.audio_embedder.register_forward_hook(self._audio)
        model.text_embedder.register_forward_hook(self._text)

    def _audio(self, mod, inp, out):
        out.retain_grad()
        self.a = out

    def _text(self, mod, inp, out):
        out[0].retain_grad()
        self.t, self.mask = out


def _check_feature_grads(kind, q, k, temp, o, grad_bar, mask=None):
    """Feature gradients at the bf16 bar, with the rows an fp32 near-tie of a row max touches left
    out (oracle.ref_cpu.near_ties: there the kernels may legitimately take the other key's
    gradient); the near-tied rows are counted and must stay a small minority. No seed picking: any
    input passes or fails on the same rule."""
    tq, tk, n = ref_cpu.near_ties(q.detach().float(), k.detach().float(), float(temp.detach()))
    eq = ref_cpu.grad_rel(q.grad, o["dq"], tq)
    ek = ref_cpu.grad_rel(k.grad, o["dk"], tk)
    _log(f"{kind} feature-gradient relative L2 (near-tie rows excluded: {int(tq.sum())} query / {int(tk.sum())} "
         f"key rows, {n} tied row maxima): dq {eq:.3e}  dk {ek:.3e}; all rows dq {_rel(q.grad, o['dq']):.3e} "
         f"dk {_rel(k.grad, o['dk']):.3e}")
    assert float(tq.float().mean()) < 0.03 and float(tk.float().mean()) < 0.03, (int(tq.sum()), int(tk.sum()))
    assert eq < grad_bar, eq
    assert ek < grad_bar, ek


def _check_head(kind, losses, stats, q, k, temp, temp_grad, mask=None, thr=0.8, w=0.01, grad_bar=1e-2):
    o = ref_cpu.head_loss_chunked(kind, q.detach().float(), k.detach().float(), float(temp.detach()), q_mask=mask,
                                  threshold=thr, weight=w, chunk=8)
    names = ("total", "ce", "reg", "aux")
    for got, key in zip(losses, names):
        assert _close(float(got), o[key]), (kind, key, float(got), o[key])
    for key, want in o["stats"].items():
        assert _close(stats[key], want, 1e-4, 1e-4), (key, stats[key], want)
    _check_feature_grads(kind, q, k, temp, o, grad_bar, mask)
    if temp_grad is not None:
        return o["dtemp"]
    return None


def _model(**kw):
    from triad_amd.model import MultiModalModel
    torch.manual_seed(1234)
    _log(f"building model {kw}")
    m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.80, patch_sparsity_weight=0.01,
                        visual_dropout_prob=0.25, use_amp=True, **kw).to(dev)
    m.train()
    _log("model on device")
    return m


def _inputs(B, px, secs, ntok):
    g = torch.Generator(device=dev).manual_seed(4321)
    frames = torch.randn(B, 3, px, px, generator=g, device=dev)
    audio = torch.randn(B, 16000 * secs, generator=g, device=dev) * 0.1
    ids = torch.randint(1000, 30522, (B, ntok), generator=torch.Generator().manual_seed(5))
    lens = torch.randint(ntok // 2, ntok + 1, (B,), generator=torch.Generator().manual_seed(6))
    lens[0] = ntok
    mask = (torch.arange(ntok)[None] < lens[:, None]).long()
    return frames, audio, {"input_ids": ids, "attention_mask": mask}


@pytest.fixture(scope="module")
def base_model():
    """DINOv2-B/14-reg + HuBERT-base + DistilBERT (c2 / c3)."""
    return _model()


def _triad_step_check(m, B, px, secs, ntok, grad_bar=1e-2, np_seed=0):
    if np_seed is not None:
        np.random.seed(np_seed)  # HuBERT's SpecAugment masks are drawn from numpy (transformers)
    cap = Capture(m)
    frames, audio, text = _inputs(B, px, secs, ntok)
    (av_total, av_ce, av_reg, av_sm, av_st), (tv_total, tv_st) = m.forward_triad(frames, audio, text)
    _log("forward done")
    (av_total + tv_total).backward()   # full_joint (train.py:983-984)
    torch.cuda.synchronize()
    _log("backward done; oracle AV")
    v_av, v_tv = cap.v
    dt_av = _check_head("av", (av_total, av_ce, av_reg, av_sm), av_st, cap.a, v_av, m.temperature, True,
                        grad_bar=grad_bar)
    # TV: the returned tuple is (total, stats); compare total only and the gradients
    _log("oracle TV")
    o = ref_cpu.head_loss_chunked("tv", cap.t.detach().float(), v_tv.detach().float(), float(m.temperature.detach()),
                                  q_mask=cap.mask, threshold=0.8, weight=0.01, chunk=8)
    assert _close(float(tv_total), o["total"]), (float(tv_total), o["total"])
    for key, want in o["stats"].items():
        assert _close(tv_st[key], want, 1e-4, 1e-4), key
    _check_feature_grads("tv", cap.t, v_tv, m.temperature, o, grad_bar)
    # the temperature gets both heads' gradients (plus nothing else)
    assert _close(float(m.temperature.grad), dt_av + o["dtemp"], 1e-3, 1e-6), \
        (float(m.temperature.grad), dt_av + o["dtemp"])
    return cap, v_av, v_tv


def test_c3_triad_step_b256(base_model):
    """c3: the bench's tri-modal step at B=256 (Na=199, 32-token captions, ragged masks),
    both heads and d/dtemp against the chunked fp64 oracle; real patch-dropout padding."""
    m = base_model
    m.zero_grad(set_to_none=True)
    cap, v_av, v_tv = _triad_step_check(m, 256, 224, 4, 32)
    assert cap.a.shape == (256, 199, 512)
    assert 190 < v_av.shape[1] <= 256 and 190 < v_tv.shape[1] <= 256   # Nk_eff = max kept of 256 patches


def test_c2_forward_audio_visual_b128(base_model):
    """c2: forward_audio_visual at B=128 with 4 s audio (the reference's AV step, train.py:954)."""
    m = base_model
    m.zero_grad(set_to_none=True)
    cap = Capture(m)
    frames, audio, _ = _inputs(128, 224, 4, 32)
    total, ce, reg, sm, st = m.forward_audio_visual(frames, audio)
    total.backward()
    (v,) = cap.v
    dt = _check_head("av", (total, ce, reg, sm), st, cap.a, v, m.temperature, True)
    assert _close(float(m.temperature.grad), dt, 1e-3, 1e-6)


def test_c1_forward_text_visual_b2():
    """c1: image-text with DINOv2-S/14-reg + DistilBERT, B=2, 16-token captions."""
    m = _model(vit_arch="dinov2_vits14_reg")
    cap = Capture(m)
    words = "a dog runs across the wet grass while two children laugh near an old red barn today".split()
    captions = [" ".join(words[:16]), " ".join(words[3:14])]
    frames = torch.randn(2, 3, 224, 224, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    total, st = m.forward_text_visual(frames, captions)
    total.backward()
    (v,) = cap.v
    assert cap.t.shape == (2, 16, 512) and int(cap.mask.sum()) == 16 + 11
    o = ref_cpu.head_loss_chunked("tv", cap.t.detach().float(), v.detach().float(),
                                  float(m.temperature.detach()), q_mask=cap.mask, threshold=0.8, weight=0.01)
    assert _close(float(total), o["total"])
    for key, want in o["stats"].items():
        assert _close(st[key], want, 1e-4, 1e-4), key
    _check_feature_grads("tv", cap.t, v, m.temperature, o, 1e-2)
    assert _close(float(m.temperature.grad), o["dtemp"], 1e-3, 1e-6)


def test_c5_large_backbones_per_rank_b32():
    """c5 per rank: DINOv2-L/14-reg on 518 px frames (1369 patches), HuBERT-large on 10 s audio
    (Na = 499), DistilBERT captions, B=32, the tri-modal step."""
    m = _model(audio_model_name="facebook/hubert-large-ls960-ft", vit_arch="dinov2_vitl14_reg")
    assert m.audio_embedder.hubert.config.hidden_size == 1024 and m.visual_embedder.model.embed_dim == 1024
    # SpecAugment's numpy draws are NOT seeded here: near-tied row maxima (which once moved an
    # unseeded run to 1.012e-2, profiles/r02_gpu_tests_c5.log) are excluded by rule, not by input
    cap, v_av, v_tv = _triad_step_check(m, 32, 518, 10, 32, np_seed=None)
    assert cap.a.shape == (32, 499, 512)
    assert 1000 < v_av.shape[1] <= 1369
