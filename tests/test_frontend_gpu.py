"""GPU parity of the backbone front-ends (triad_amd.frontend): the fused channels-last
GroupNorm(C groups) + GELU HIP kernels against torch fp32 (values, dx, dgamma, dbeta), and the
whole HuBERT conv feature encoder in GEMM form against the transformers modules it replaces,
both under bf16 autocast on the device."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("B,T,C", [(3, 1000, 512), (2, 12799, 512), (4, 77, 64), (1, 5, 512)])
def test_channel_group_norm_gelu(B, T, C):
    from triad_amd import frontend
    g = torch.Generator(device=dev).manual_seed(T)
    x = (torch.randn(B, T, C, device=dev, generator=g) * 2.0 + 0.5).to(torch.bfloat16)
    gamma = (torch.rand(C, device=dev, generator=g) + 0.5).requires_grad_(True)
    beta = (torch.randn(C, device=dev, generator=g) * 0.2).requires_grad_(True)
    xr = x.float().requires_grad_(True)
    gr = gamma.detach().clone().requires_grad_(True)
    br = beta.detach().clone().requires_grad_(True)
    ref = F.gelu(F.group_norm(xr.transpose(1, 2), C, gr, br, 1e-5)).transpose(1, 2)
    xd = x.clone().requires_grad_(True)
    y = frontend.channel_group_norm_gelu(xd, gamma, beta, 1e-5)
    assert y.dtype == torch.bfloat16 and y.shape == x.shape
    # bf16 output of fp32 arithmetic: within one bf16 rounding of the fp32 reference
    torch.testing.assert_close(y.float(), ref.detach(), rtol=8e-3, atol=8e-3)
    dy = (torch.randn(B, T, C, device=dev, generator=g)).to(torch.bfloat16)
    ref.backward(dy.float())
    y.backward(dy)
    assert xd.grad.dtype == torch.bfloat16
    assert _rel(xd.grad.float(), xr.grad) < 8e-3
    assert _rel(gamma.grad, gr.grad) < 1e-4
    assert _rel(beta.grad, br.grad) < 1e-4


@pytest.mark.parametrize("B,L", [(3, 16000), (4, 16000), (8, 64000), (2, 16400)])
def test_hubert_feature_encoder_gemm_matches_transformers(B, L):
    """Padded-frame conv stack (HIP overlapping-row GEMMs where the row counts allow, the same
    products through torch otherwise) and, for lengths whose frame chain turns odd (16400), the
    im2col path -- against transformers' nn.Conv1d stack under autocast."""
    import transformers
    from triad_amd import frontend
    torch.manual_seed(0)
    ref_m = transformers.HubertModel(transformers.HubertConfig()).to(dev).train()
    m = transformers.HubertModel(transformers.HubertConfig()).to(dev).train()
    m.load_state_dict(ref_m.state_dict())
    frontend.install_hubert_frontend(m)
    x = torch.randn(B, L, device=dev) * 0.5
    assert (frontend._frame_stack_plan(m.feature_extractor, x.to(torch.bfloat16)) is None) == (L == 16400)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = ref_m.feature_extractor(x)
        got = m.feature_extractor(x)
    assert got.shape == ref.shape
    assert _rel(got.float(), ref.float()) < 2e-2
    gy = torch.randn_like(ref.float())
    (ref.float() * gy).sum().backward()
    (got.float() * gy).sum().backward()
    for (n, p), (_, q) in zip(m.feature_extractor.named_parameters(), ref_m.feature_extractor.named_parameters()):
        assert _rel(p.grad, q.grad) < 5e-2, n


@pytest.mark.parametrize("C,G,T", [(768, 16, 199), (768, 16, 37), (1024, 16, 499), (768, 16, 1)])
def test_hubert_pos_conv_matches_transformers(C, G, T):
    """Implicit-GEMM positional conv (forward + input grad) + HIP weight grad (triad_posconv_dw at
    48 channels per group, the overlapping-row GEMM at 64) vs the transformers module
    (conv -> SamePad -> GELU) under bf16 autocast."""
    import transformers
    from transformers.models.hubert.modeling_hubert import HubertPositionalConvEmbedding
    from triad_amd import frontend
    cfg = transformers.HubertConfig(hidden_size=C, num_conv_pos_embedding_groups=G)
    torch.manual_seed(T)
    ref_m = HubertPositionalConvEmbedding(cfg).to(dev)
    m = HubertPositionalConvEmbedding(cfg).to(dev)
    m.load_state_dict(ref_m.state_dict())
    m._triad_hf_forward = m.forward
    import types
    m.forward = types.MethodType(frontend._hubert_pos_conv_forward, m)
    x = torch.randn(3, T, C, device=dev)
    xr = x.clone().requires_grad_(True)
    xd = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        xr_b = xr.to(torch.bfloat16)
        xd_b = xd.to(torch.bfloat16)
        ref = ref_m(xr_b)
        got = m(xd_b)
    assert got.shape == ref.shape == (3, T, C)
    assert _rel(got.float(), ref.float()) < 1e-2
    gy = torch.randn_like(ref.float())
    (ref.float() * gy).sum().backward()
    (got.float() * gy).sum().backward()
    assert _rel(xd.grad, xr.grad) < 2e-2
    for (n, p), (_, q) in zip(m.named_parameters(), ref_m.named_parameters()):
        assert _rel(p.grad, q.grad) < 3e-2, n


@pytest.mark.parametrize("M,K,O", [(66 * 261, 768, 2304), (5 * 37, 768, 768), (3, 384, 1152), (1001, 1024, 3072),
                                   (33, 768, 768), (256 * 261, 768, 2304)])
def test_lora_linear_matches_reference_chain(M, K, O):
    """ViT LoRA (triad_amd.vit._LoRALinear: rows_nt / lora_update / lora_tn HIP kernels + one base GEMM and an
    in-place rank-8 update) against the reference chain base(x) + B(A(x)) * s under bf16 autocast."""
    from triad_amd.vit import LoRALinear
    torch.manual_seed(M)
    base = torch.nn.Linear(K, O).to(dev)
    base.weight.data = base.weight.data.to(torch.bfloat16)
    base.bias.data = base.bias.data.to(torch.bfloat16)
    for p in base.parameters():
        p.requires_grad = False
    m = LoRALinear(base, 8, 16).to(dev)
    with torch.no_grad():
        m.lora_B.normal_(0, 0.05)
    x = torch.randn(M, K, device=dev)
    xr = x.clone().requires_grad_(True)
    xd = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = base(xr) + torch.nn.functional.linear(torch.nn.functional.linear(xr, m.lora_A), m.lora_B) * m.scaling
        got = m(xd)
    assert got.dtype == torch.bfloat16 and got.shape == ref.shape
    assert _rel(got.float(), ref.float()) < 1e-2
    gy = torch.randn(M, O, device=dev)
    rx, gA, gB = torch.autograd.grad((ref.float() * gy).sum(), (xr, m.lora_A, m.lora_B))
    dx, dA, dB = torch.autograd.grad((got.float() * gy).sum(), (xd, m.lora_A, m.lora_B))
    assert _rel(dx, rx) < 2e-2
    assert _rel(dA, gA) < 2e-2
    assert _rel(dB, gB) < 2e-2


def test_vit_fused_residual_ln_matches_unfused(monkeypatch):
    """DINOv2-B/14-reg + LoRA blocks with the fused residual + LayerScale + LayerNorm passes
    (vit._AddScaleLN, csrc/resid_ln.hip) against the unfused autocast chain: same features and
    LoRA gradients to bf16 tolerance."""
    from triad_amd import vit as V
    torch.manual_seed(0)
    m = V.apply_lora(V.DinoVisionTransformer("dinov2_vitb14_reg"), 8, 16).to(dev)
    V.store_frozen_base_bf16(m)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.02)
        for blk in m.blocks:  # LayerScale 1e-5 would make every block near-identity
            blk.ls1.gamma.fill_(0.3)
            blk.ls2.gamma.fill_(0.3)
    x = torch.randn(2, 3, 98, 98, device=dev)
    gy = torch.randn(2, 49, 768, device=dev)

    def run(fused):
        monkeypatch.setattr(V.DinoVisionTransformer, "_fused_ok",
                            (lambda self, t, n, norm: True) if fused else (lambda self, t, n, norm: False))
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m.get_intermediate_layers(x, n=1)[0]
        (out.float() * gy).sum().backward()
        return out.detach().float(), {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}

    o_ref, g_ref = run(False)
    o_fus, g_fus = run(True)
    assert o_fus.shape == o_ref.shape == (2, 49, 768) and o_fus.dtype == o_ref.dtype
    assert _rel(o_fus, o_ref) < 1e-2
    assert set(g_fus) == set(g_ref) and len(g_ref) == 48
    for n in g_ref:
        assert _rel(g_fus[n], g_ref[n]) < 3e-2, n


@pytest.mark.parametrize("B,T,splits", [(5, 199, 2), (3, 300, 3), (2, 37, 1)])
def test_posconv_weight_grad_vs_fp32(B, T, splits):
    """triad_posconv_dw (groups of 48 channels, 128 taps, padding 64, first T outputs) against the
    fp32 grouped-conv weight gradient of the same bf16 operands (fp32 accumulation both ways)."""
    from triad_amd._lib import call, ptr, stream_ptr
    C, G, K, pad = 768, 16, 128, 64
    g = torch.Generator(device=dev).manual_seed(T)
    x = torch.randn(B, T, C, device=dev, generator=g).to(torch.bfloat16)
    dy = torch.randn(B, T, C, device=dev, generator=g).to(torch.bfloat16)
    part = torch.empty(int(call("triad_posconv_dw_part_bytes", C, G, splits)) // 4, device=dev)
    call("triad_posconv_dw", ptr(x), ptr(dy), B, T, C, G, pad, splits, ptr(part), stream_ptr(x.device))
    dw = part.view(splits, -1).sum(0).view(G, K, 48, 48).permute(0, 2, 3, 1).reshape(C, 48, K)
    # full conv output has T + 1 steps; the dropped last one gets zero gradient
    dy_full = torch.cat([dy.float(), torch.zeros(B, 1, C, device=dev)], 1).transpose(1, 2)
    ref = torch.nn.grad.conv1d_weight(x.float().transpose(1, 2), (C, 48, K), dy_full, padding=pad, groups=G)
    assert _rel(dw, ref) < 1e-5


@pytest.mark.parametrize("B,T,C,G", [(3, 499, 1024, 16), (2, 37, 256, 4), (2, 60, 512, 4)])
def test_posconv_weight_grad_gemm_vs_fp32(B, T, C, G):
    """frontend._posconv_dw_gemm (channels per group dividing 128: HuBERT-large's 64; one split-K
    GEMM per 128-channel block with overlapping B rows) against the fp32 grouped-conv weight
    gradient of the same bf16 operands."""
    from triad_amd import frontend
    K, pad = 128, 64
    g = torch.Generator(device=dev).manual_seed(T + C)
    x = torch.randn(B, T, C, device=dev, generator=g).to(torch.bfloat16)
    dy = torch.randn(B, T, C, device=dev, generator=g).to(torch.bfloat16)
    dw = frontend._posconv_dw_gemm(x, dy, G, pad, K)
    dy_full = torch.cat([dy.float(), torch.zeros(B, 1, C, device=dev)], 1).transpose(1, 2)
    ref = torch.nn.grad.conv1d_weight(x.float().transpose(1, 2), (C, C // G, K), dy_full, padding=pad, groups=G)
    assert dw.shape == ref.shape
    assert _rel(dw, ref) < 1e-5


def test_feature_encoder_side_stream_weight_grads_bit_identical():
    """Conv-stack weight gradients of bf16 (shadow) conv weights on the side stream
    (frontend._FrameConvS2, queued before the input-gradient GEMMs) equal the in-stream ones
    bit for bit."""
    import transformers
    from triad_amd import frontend, linear as L
    torch.manual_seed(0)
    m = transformers.HubertModel(transformers.HubertConfig()).to(dev).train()
    frontend.install_hubert_frontend(m)
    fe = m.feature_extractor
    for layer in fe.conv_layers:
        layer.conv.weight.data = layer.conv.weight.data.to(torch.bfloat16)
    x = torch.randn(4, 16000, device=dev) * 0.5

    def run(side):
        L.SIDE_STREAM_DW = side
        fe.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = fe(x)
        (y.float() ** 2).mean().backward()
        return [layer.conv.weight.grad.clone() for layer in fe.conv_layers]

    prev = L.SIDE_STREAM_DW
    try:
        g_main = run(False)
        g_side = run(True)
    finally:
        L.SIDE_STREAM_DW = prev
    for a, b in zip(g_side, g_main):
        assert a.dtype == torch.bfloat16 and a.is_contiguous()
        assert torch.equal(a, b)
