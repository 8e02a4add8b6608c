"""Backbone front-ends in GEMM form (triad_amd.frontend) against the convolutions they
replace: CPU float64 parity of the im2col + GEMM conv1d (HuBERT feature encoder layers,
values and all three gradients) and of the patch-embedding GEMM (DINOv2 PatchEmbed)."""
import pytest
import torch
import torch.nn.functional as F

from triad_amd import frontend


@pytest.mark.parametrize("C,O,k,s,T", [(1, 16, 10, 5, 203), (8, 16, 3, 2, 101), (8, 16, 3, 2, 100),
                                       (8, 16, 2, 2, 50), (8, 8, 2, 2, 51), (4, 8, 3, 2, 3)])
@pytest.mark.parametrize("bias", [False, True])
def test_conv1d_gemm_matches_conv1d(C, O, k, s, T, bias):
    g = torch.Generator().manual_seed(C * 1000 + T)
    x = torch.randn(2, T, C, dtype=torch.float64, generator=g, requires_grad=True)
    w = torch.randn(O, C, k, dtype=torch.float64, generator=g, requires_grad=True)
    b = torch.randn(O, dtype=torch.float64, generator=g, requires_grad=True) if bias else None
    y = frontend.conv1d_gemm(x, w, b, s)
    yr = F.conv1d(x.transpose(1, 2), w, b, stride=s).transpose(1, 2)
    assert y.shape == yr.shape
    torch.testing.assert_close(y, yr, rtol=1e-12, atol=1e-12)
    gy = torch.randn(yr.shape, dtype=torch.float64, generator=g)
    ins = (x, w) + ((b,) if bias else ())
    got = torch.autograd.grad((y * gy).sum(), ins)
    ref = torch.autograd.grad((yr * gy).sum(), ins)
    for a, r in zip(got, ref):
        torch.testing.assert_close(a, r, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("px,patch", [(224, 14), (70, 14), (32, 8)])
def test_patch_embed_gemm_matches_conv2d(px, patch):
    g = torch.Generator().manual_seed(px)
    conv = torch.nn.Conv2d(3, 24, patch, patch).double()
    x = torch.randn(2, 3, px, px, dtype=torch.float64, generator=g)
    ref = conv(x).flatten(2).transpose(1, 2)
    got = frontend.patch_embed(x, conv.weight, conv.bias, patch)
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12)


def test_hubert_feature_encoder_cpu_path_is_the_original():
    """On CPU tensors the installed encoder falls through to the transformers forward."""
    import transformers
    cfg = transformers.HubertConfig(conv_dim=(16, 16, 16), conv_kernel=(10, 3, 2), conv_stride=(5, 2, 2),
                                    hidden_size=32, num_hidden_layers=1, num_attention_heads=2, intermediate_size=64,
                                    num_conv_pos_embeddings=16, num_conv_pos_embedding_groups=2)
    torch.manual_seed(0)
    m = transformers.HubertModel(cfg).eval()
    x = torch.randn(2, 800)
    with torch.no_grad():
        ref = m.feature_extractor(x)
        frontend.install_hubert_frontend(m)
        got = m.feature_extractor(x)
    torch.testing.assert_close(got, ref)
