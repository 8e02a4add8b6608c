"""GPU parity of the fused HuBERT post-LN passes (triad_amd.postln, csrc/postln.hip) against
torch on the SAME dropout masks (the kernels' keep bits exposed by triad_dropout_keep), and of
the fused encoder against the stock transformers encoder with dropout off."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("M,D,p", [(1000, 768, 0.1), (333, 1024, 0.1), (64, 768, 0.0), (5, 256, 0.3)])
def test_drop_add_ln_matches_torch_on_same_mask(M, D, p):
    from triad_amd import postln
    g = torch.Generator(device=dev).manual_seed(M + D)
    res = torch.randn(M, D, device=dev, generator=g)
    y = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    w = 1 + 0.1 * torch.randn(D, device=dev, generator=g)
    b = 0.1 * torch.randn(D, device=dev, generator=g)
    norm = torch.nn.LayerNorm(D, eps=1e-5).to(dev)
    with torch.no_grad():
        norm.weight.copy_(w)
        norm.bias.copy_(b)
    seed = 12345 + M
    keep = postln.dropout_keep(M * D, p, seed, dev).view(M, D).float()
    dh = torch.randn(M, D, device=dev, generator=g)
    dhb = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)

    rr = res.clone().requires_grad_(True)
    yr = y.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yd = (yr.float() * keep * (1.0 / (1.0 - p))).to(torch.bfloat16)
    hr = F.layer_norm(rr + yd.float(), (D,), wr, br, 1e-5)
    hbr = hr.to(torch.bfloat16)
    ((hr * dh).sum() + (hbr.float() * dhb.float()).sum()).backward()

    rf = res.clone().requires_grad_(True)
    yf = y.clone().requires_grad_(True)
    h, hb = postln.drop_add_ln(rf, yf, norm, p, seed)
    ((h * dh).sum() + (hb.float() * dhb.float()).sum()).backward()
    assert _rel(h, hr) < 1e-5
    assert (hb.float() - hbr.float()).abs().max() <= 2 ** -7 * hbr.float().abs().max()
    assert _rel(rf.grad, rr.grad) < 1e-4
    assert _rel(yf.grad, yr.grad) < 1e-2
    assert _rel(norm.weight.grad, wr.grad) < 1e-4
    assert _rel(norm.bias.grad, br.grad) < 1e-4


@pytest.mark.parametrize("n,p", [(256 * 199 * 48, 0.1), (4096, 0.5), (8, 0.0)])
def test_gelu_drop_matches_torch_on_same_mask(n, p):
    from triad_amd import postln
    g = torch.Generator(device=dev).manual_seed(n)
    u = (2 * torch.randn(n, device=dev, generator=g)).to(torch.bfloat16)
    dv = torch.randn(n, device=dev, generator=g).to(torch.bfloat16)
    seed = 777
    keep = postln.dropout_keep(n, p, seed, dev).float()
    ur = u.clone().requires_grad_(True)
    vr = (F.gelu(ur).float() * keep * (1.0 / (1.0 - p))).to(torch.bfloat16)
    vr.backward(dv)
    uf = u.clone().requires_grad_(True)
    vf = postln.gelu_drop(uf, p, seed)
    vf.backward(dv)
    assert _rel(vf, vr) < 1e-3
    assert _rel(uf.grad, ur.grad) < 1e-2


def test_dropout_keep_bits_statistics():
    from triad_amd import postln
    n = 1 << 22
    k1 = postln.dropout_keep(n, 0.1, 1, dev).float()
    k2 = postln.dropout_keep(n, 0.1, 2, dev).float()
    for k in (k1, k2):
        assert abs(float(k.mean()) - 0.9) < 2e-3
        a, b = k[:-1] - 0.9, k[1:] - 0.9  # neighbouring elements (same / adjacent hash pairs)
        assert abs(float((a * b).mean()) / 0.09) < 5e-3
    assert abs(float(((k1 - 0.9) * (k2 - 0.9)).mean()) / 0.09) < 5e-3  # seeds decorrelate
    assert float(postln.dropout_keep(n, 0.0, 3, dev).float().mean()) == 1.0


def test_fused_hubert_encoder_matches_stock_without_dropout():
    """Fused encoder vs the stock HubertEncoder (transformers) with every dropout and LayerDrop
    off: same last_hidden_state and parameter gradients to bf16 tolerance."""
    from triad_amd import model as Mdl
    torch.manual_seed(0)
    over = dict(hidden_size=768, num_hidden_layers=2, num_attention_heads=12, intermediate_size=3072,
                hidden_dropout=0.0, activation_dropout=0.0, attention_dropout=0.0, layerdrop=0.0,
                feat_proj_dropout=0.0, mask_time_prob=0.0)  # SpecAugment draws fresh masks per call
    hub = Mdl.hubert_execution_tweaks(Mdl._hf_model("HubertModel", "none/none", over)).to(dev)
    hub.train()
    enc = hub.encoder
    assert hasattr(enc, "_triad_stock_forward")
    x = 0.1 * torch.randn(2, 16000, device=dev)

    def run(fwd):
        hub.zero_grad(set_to_none=True)
        enc.forward = fwd
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = hub(x).last_hidden_state
        gy = torch.linspace(-1, 1, out.numel(), device=dev).view_as(out)
        (out.float() * gy).sum().backward()
        return out.detach().float(), {n: q.grad.float().clone() for n, q in hub.named_parameters()
                                      if q.grad is not None}

    fused_fwd = enc.forward
    try:
        o_f, g_f = run(fused_fwd)
        o_s, g_s = run(enc._triad_stock_forward)
    finally:
        enc.forward = fused_fwd
    assert o_f.shape == o_s.shape and o_f.dtype == o_s.dtype == torch.float32
    assert _rel(o_f, o_s) < 1e-2
    assert set(g_f) == set(g_s)
    for n in g_s:
        if n.endswith("k_proj.bias"):  # exactly 0 in exact arithmetic (softmax shift invariance): noise
            assert float(g_f[n].norm()) < 1e-3 * float(g_s[n.replace("bias", "weight")].norm()) + 1e-6
            continue
        assert _rel(g_f[n], g_s[n]) < 3e-2, (n, _rel(g_f[n], g_s[n]))


def test_fused_distilbert_matches_stock_without_dropout():
    """Fused DistilBERT transformer (postln passes) vs the stock one with dropout off: same
    last_hidden_state and parameter gradients to bf16 tolerance."""
    from triad_amd import model as Mdl
    from triad_amd import postln
    torch.manual_seed(0)
    enc = Mdl._hf_model("DistilBertModel", "none/none", dict(n_layers=2, dropout=0.0, attention_dropout=0.0))
    enc = postln.install_fused_distilbert(enc).to(dev).train()
    tr = enc.transformer
    ids = torch.randint(1000, 30000, (4, 32), device=dev)

    def run(fwd):
        enc.zero_grad(set_to_none=True)
        tr.forward = fwd
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = enc(input_ids=ids).last_hidden_state
        gy = torch.linspace(-1, 1, out.numel(), device=dev).view_as(out)
        (out.float() * gy).sum().backward()
        return out.detach().float(), {n: q.grad.float().clone() for n, q in enc.named_parameters() if q.grad is not None}

    fused_fwd = tr.forward
    try:
        o_f, g_f = run(fused_fwd)
        o_s, g_s = run(tr._triad_stock_forward)
    finally:
        tr.forward = fused_fwd
    assert o_f.shape == o_s.shape
    assert _rel(o_f, o_s) < 1e-2
    assert set(g_f) == set(g_s)
    for n in g_s:
        if n.endswith("k_lin.bias"):  # exactly 0 in exact arithmetic: noise
            continue
        assert _rel(g_f[n], g_s[n]) < 3e-2, (n, _rel(g_f[n], g_s[n]))


@pytest.mark.parametrize("shape", [(66 * 261, 3072), (3, 7, 8), (1 << 20,)])
def test_gelu_matches_aten_bit_exact(shape):
    """postln.gelu (geludrop kernels at p = 0, used for the ViT MLP, the HuBERT conv stack and the
    positional conv) against aten gelu / gelu_backward on bf16: identical values and gradients."""
    from triad_amd.postln import gelu
    g = torch.Generator(device=dev).manual_seed(len(shape))
    u = (torch.randn(shape, device=dev, generator=g) * 3).to(torch.bfloat16)
    dv = torch.randn(shape, device=dev, generator=g).to(torch.bfloat16)
    ud = u.clone().requires_grad_(True)
    v = gelu(ud)
    assert v.grad_fn is not None and "GeluDrop" in type(v.grad_fn).__name__
    torch.testing.assert_close(v, torch.nn.functional.gelu(u), rtol=0, atol=0)
    v.backward(dv)
    torch.testing.assert_close(ud.grad, torch.ops.aten.gelu_backward(dv, u), rtol=0, atol=0)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gelu_table_every_bf16_pattern(p):
    """The table-driven GELU passes (triad_gelu_table: |x| in [2^-40, 2^6) from the table, every
    other pattern by the formula) over ALL 65536 bf16 bit patterns, against aten gelu /
    gelu_backward on the same dropout mask: identical values (NaN where aten gives NaN)."""
    from triad_amd import postln
    bits = torch.arange(65536, dtype=torch.int32, device=dev).to(torch.int16)
    u = bits.view(torch.bfloat16).repeat(2)  # 131072 elements: every pattern at even and odd positions
    u = torch.cat([u[1:], u[:1]])
    g = torch.Generator(device=dev).manual_seed(7)
    dv = torch.randn(u.shape, device=dev, generator=g).to(torch.bfloat16)
    keep = postln.dropout_keep(u.numel(), p, 1234, dev).bool()
    ud = u.clone().requires_grad_(True)
    v = postln.gelu_drop(ud, p, 1234)
    s = 1.0 / (1.0 - p)
    ref = torch.where(keep, (torch.nn.functional.gelu(u).float() * s).to(torch.bfloat16), torch.zeros_like(u))
    torch.testing.assert_close(v, ref, rtol=0, atol=0, equal_nan=True)
    v.backward(dv)
    dg = torch.where(keep, (dv.float() * s).to(torch.bfloat16), torch.zeros_like(dv))
    torch.testing.assert_close(ud.grad, torch.ops.aten.gelu_backward(dg, u), rtol=0, atol=0, equal_nan=True)


@pytest.mark.parametrize("family", ["hubert", "distilbert"])
def test_fused_qkv_self_attention_matches_module(family):
    """postln.self_attention (q / k / v as one projection GEMM, linear._QKVFn, and the fused-qkv
    HIP attention with dropout) against the HubertAttention / DistilBertSelfAttention module
    itself (three projections, the same HIP attention kernels via the 'triad' interface) on the
    same dropout masks: values and gradients of the input and of every projection parameter."""
    from triad_amd import model as Mdl, postln
    torch.manual_seed(0)
    if family == "hubert":
        over = dict(hidden_size=768, num_hidden_layers=1, num_attention_heads=12, intermediate_size=3072,
                    attention_dropout=0.1, mask_time_prob=0.0)
        hub = Mdl.hubert_execution_tweaks(Mdl._hf_model("HubertModel", "none/none", over)).to(dev)
        attn = hub.encoder.layers[0].attention.train()
    else:
        enc = Mdl._hf_model("DistilBertModel", "none/none", dict(n_layers=1, attention_dropout=0.1)).to(dev)
        attn = enc.transformer.layer[0].attention.train()
    x0 = (torch.randn(64, 128, 768, device=dev)).to(torch.bfloat16)
    gy = torch.randn(64, 128, 768, device=dev)

    def run(fn):
        attn.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        torch.manual_seed(5)  # attention-dropout seeds come from torch's generator
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = fn(x)
        (y.float() * gy).sum().backward()
        return y.detach().float(), x.grad.float(), {n: p.grad.float().clone() for n, p in attn.named_parameters()}

    y_m, gx_m, g_m = run(lambda x: attn(x)[0])
    y_f, gx_f, g_f = run(lambda x: postln.self_attention(attn, x))
    assert _rel(y_f, y_m) < 1e-2
    assert _rel(gx_f, gx_m) < 2e-2
    assert set(g_f) == set(g_m) and len(g_m) == 8
    for n in g_m:
        if n in ("k_proj.bias", "k_lin.bias"):  # softmax shift invariance: exactly 0 up to rounding noise
            continue
        assert _rel(g_f[n], g_m[n]) < 2e-2, (n, _rel(g_f[n], g_m[n]))
