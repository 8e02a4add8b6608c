"""Projection head (reference model.py:32-34,68 / 81-83,116 / 253-255,326) at the
row counts the training step runs, through both forms: "passes" (tiled GEMMs + LayerNorm row
passes) and "rows" (row-panel GEMMs with the LayerNorm and its backward in the epilogues):

  65,536 x 768   visual head, B=256 x 256 patches (before patch dropout)   c3
  50,944 x 768   audio head, B=256 x 199 frames                            c3
   8,192 x 768   text head, B=256 x 32 tokens                              c3
  43,808 x 1024  visual head of DINOv2-L at 518 px, B=32 x 1369 patches    c5

At these sizes the forward GEMMs take the eight-wave 256 x 256 tile form (M >= 32,768) or the
256 x 128 ring, and the weight gradients the split-K GEMM with 16+ splits -- code paths the
small-row test in test_ops_gpu.py does not reach. Forward against the oracle's bf16-autocast
emulation (oracle.ref_cpu.projection_head(amp=True)), all seven gradients against fp64 autograd of
the unrounded head, both evaluated on the device in row chunks (plain torch; test infrastructure).
Bars: forward |d| <= 2e-2 + 1.6e-2 |ref| elementwise (an y1 rounding flip moves a few bf16 ulps through
LN and GEMM2) and 4e-3 relative L2; gradients 1e-2 relative L2 (bf16 operands, fp32 accumulation)."""
import pytest
import torch
import torch.nn as nn

from oracle import ref_cpu

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a = a.detach().double()
    b = b.detach().double().to(a.device)
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


@pytest.mark.parametrize("form", ["passes", "rows"])
@pytest.mark.parametrize("rows,H", [(65536, 768), (50944, 768), (8192, 768), (43808, 1024)])
def test_projection_head_at_step_rows(rows, H, form):
    from triad_amd import ops
    torch.manual_seed(rows + H)
    p1, ln, p2 = nn.Linear(H, 512), nn.LayerNorm(512), nn.Linear(512, 512)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    mods = [m.to(dev) for m in (p1, ln, p2)]
    g = torch.Generator(device=dev).manual_seed(rows)
    h = torch.randn(rows, H, device=dev, generator=g)
    gy = torch.randn(rows, 512, device=dev, generator=g) * 0.01
    # product path
    hd = h.clone().requires_grad_(True)
    y = ops.projection_head(hd.view(1, rows, H), *mods, form=form)
    assert y.dtype == torch.bfloat16 and y.shape == (1, rows, 512)
    y.float().view(rows, 512).backward(gy)
    got = [hd.grad] + [p.grad.detach().clone() for m in mods for p in m.parameters()]
    # the weight gradients' split-K plans: 32 / 40 splits, one XCD per split, at the long token lists;
    # one round of 16 128 x 128 splits for the 8,192-row text head
    Mp = (rows + 127) // 128 * 128
    if Mp >= 32768:
        assert ops._dw_plan(Mp, 512) == (1 | 8, 32) and ops._dw_plan(Mp, H) == (4 | 8, 40 if H == 768 else 32)
    else:
        assert ops._dw_plan(Mp, 512) == (0, 16)
    # oracle forward (bf16 autocast emulation), chunked over rows
    w = [p.detach() for m in mods for p in m.parameters()]
    yf = y.detach().float().view(rows, 512)
    worst, num, den = 0.0, 0.0, 0.0
    for r0 in range(0, rows, 16384):
        ref = ref_cpu.projection_head(h[r0:r0 + 16384], *w, amp=True)
        d = (yf[r0:r0 + 16384] - ref).abs()
        worst = max(worst, float((d - 1.6e-2 * ref.abs()).max()))
        num += float((d.double() ** 2).sum())
        den += float((ref.double() ** 2).sum())
    assert worst <= 2e-2, worst   # |d| <= 2e-2 + 1.6e-2 |ref| (the small-row test's bar, test_ops_gpu.py)
    assert (num / den) ** 0.5 < 4e-3, (num / den) ** 0.5
    # fp64 autograd of the unrounded head (the gradients' reference), chunked over rows
    wd = [x.double().requires_grad_(True) for x in w]
    ref_dh = torch.empty(rows, H, dtype=torch.float64, device=dev)
    for r0 in range(0, rows, 16384):
        hc = h[r0:r0 + 16384].double().requires_grad_(True)
        yc = nn.functional.linear(hc, wd[0], wd[1])
        yc = nn.functional.layer_norm(yc, (512,), wd[2], wd[3], 1e-5)
        yc = nn.functional.linear(yc, wd[4], wd[5])
        yc.backward(gy[r0:r0 + 16384].double())
        ref_dh[r0:r0 + 16384] = hc.grad
    refs = [ref_dh] + [x.grad for x in wd]
    names = ["dh", "dW1", "db1", "dgamma", "dbeta", "dW2", "db2"]
    errs = {n: _rel(a, b) for n, a, b in zip(names, got, refs)}
    print(f"projection head {rows} x {H}: gradient relative L2 {errs}")
    for n, e in errs.items():
        assert e < 1e-2, (n, e)


@pytest.mark.parametrize("form", [1, 4])
def test_splitk_xcd_placement_bit_identical(form):
    """Form flag 8 (each split's workgroups on one XCD, gemm.hip tile_split) moves workgroups, not
    arithmetic: bit-identical to the default placement at the same form / splits, and refused
    (TRIAD_EINVAL) when the split count is not a multiple of 8."""
    from triad_amd._lib import TriadError, call, ptr, stream_ptr
    M, O, K, sp = 16384, 512, 768, 16
    g = torch.Generator(device=dev).manual_seed(form)
    dy = (torch.randn(M, O, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    outs = []
    for f in (form, form | 8):
        slabs = torch.empty(sp * O * K, device=dev)
        dw = torch.empty(O, K, device=dev)
        call("triad_gemm_bf16_splitk_form", ptr(dy), O, 0, ptr(x), K, 0, O, K, M, sp, None, ptr(slabs), ptr(dw), 0, f,
             stream_ptr())
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = dy.float().t() @ x.float()
    assert float((outs[1] - ref).norm() / ref.norm()) < 1e-4
    with pytest.raises(TriadError):
        call("triad_gemm_bf16_splitk_form", ptr(dy), O, 0, ptr(x), K, 0, O, K, M, 12, None, ptr(slabs), ptr(dw), 0,
             form | 8, stream_ptr())


def test_rows_form_reads_a_strided_view_in_place():
    """The row-panel head reads the ViT's patch tokens as they lie -- a strided view of
    (B, 5 + N, H) behind the CLS / register tokens, model.py:325 -- with two-level row addressing
    (no packing copy): outputs and every gradient equal, bit for bit, to the same head on a
    contiguous copy of the view, the gradient landing in the view's rows only."""
    from triad_amd import ops
    torch.manual_seed(5)
    B, N, H = 24, 256, 768
    p1, ln, p2 = (m.to(dev) for m in (nn.Linear(H, 512), nn.LayerNorm(512), nn.Linear(512, 512)))
    full = torch.randn(B, 5 + N, H, device=dev).to(torch.bfloat16).requires_grad_(True)
    gy = (torch.randn(B, N, 512, device=dev) * 0.01).to(torch.bfloat16)
    y = ops.projection_head(full[:, 5:], p1, ln, p2, form="rows")
    y.backward(gy)
    got = [y.detach(), full.grad[:, 5:].clone()] + [p.grad.clone() for m in (p1, ln, p2) for p in m.parameters()]
    assert float(full.grad[:, :5].abs().max()) == 0.0
    for m in (p1, ln, p2):
        for p in m.parameters():
            p.grad = None
    hc = full.detach()[:, 5:].contiguous().requires_grad_(True)
    y2 = ops.projection_head(hc, p1, ln, p2, form="rows")
    y2.backward(gy)
    ref = [y2.detach(), hc.grad] + [p.grad for m in (p1, ln, p2) for p in m.parameters()]
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,H", [(8192, 768), (300, 1024), (1, 768), (50944, 768)])
def test_fused_forward_equals_its_two_halves(M, H):
    """triad_projhead_fwd (projection1 + LayerNorm + projection2 in one kernel, the LN'd panel kept in
    LDS) is bit-identical in y1 / ln / mean / rstd / y to triad_projhead_ln_fwd followed by
    triad_rowgemm_bias over the stored ln (ragged last panel, one row, a step shape)."""
    from triad_amd._lib import call, ptr, stream_ptr
    g = torch.Generator(device=dev).manual_seed(M + H)
    bf = torch.bfloat16
    h = torch.randn(M, H, device=dev, generator=g).to(bf)
    w1 = (torch.randn(512, H, device=dev, generator=g) / H ** 0.5).to(bf)
    w2 = (torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5).to(bf)
    b1, b2 = (torch.randn(512, device=dev, generator=g) * 0.1).to(bf), (torch.randn(512, device=dev, generator=g) * 0.1).to(bf)
    gam = torch.rand(512, device=dev, generator=g) + 0.5
    bet = torch.randn(512, device=dev, generator=g) * 0.1
    P = call("triad_rowpanel_count", M)
    Mp = P * 128
    w1p, w2p = torch.empty(H * 512, dtype=bf, device=dev), torch.empty(512 * 512, dtype=bf, device=dev)
    st = stream_ptr()
    call("triad_wpack2", ptr(w1), H, ptr(w1p), ptr(w2), 512, ptr(w2p), st)
    outs = []
    for fused in (True, False):
        y1, ln, y = (torch.full((Mp, 512), 7.0, dtype=bf, device=dev) for _ in range(3))
        mean, rstd = torch.full((Mp,), 7.0, device=dev), torch.full((Mp,), 7.0, device=dev)
        if fused:
            call("triad_projhead_fwd", ptr(h), M, H, H, M, 0, ptr(w1p), ptr(b1), ptr(gam), ptr(bet), 1e-5, ptr(w2p),
                 ptr(b2), ptr(y1), ptr(ln), ptr(mean), ptr(rstd), ptr(y), st)
        else:
            call("triad_projhead_ln_fwd", ptr(h), M, H, H, M, 0, ptr(w1p), ptr(b1), ptr(gam), ptr(bet), 1e-5, ptr(y1),
                 ptr(ln), ptr(mean), ptr(rstd), st)
            call("triad_rowgemm_bias", ptr(ln), M, 512, 512, ptr(w2p), ptr(b2), ptr(y), st)
        outs.append((y1, ln, mean, rstd, y))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert float(outs[0][4][M:].float().abs().max() if Mp > M else 0.0) == 0.0   # pad rows written as zeros
    ref = torch.nn.functional.linear(outs[0][1][:M].float(), w2.float(), b2.float())
    assert float((outs[0][4][:M].float() - ref).abs().max()) <= 2e-2 * float(ref.abs().max())
