"""GPU parity of the fused contrastive head (HIP) against the golden fixtures
and the CPU oracle. Tolerances: forward losses/statistics 1e-4 relative (the
kernels compute the fp32 arithmetic exactly on bf16 inputs); feature gradients
bf16 tolerance (dS is rounded to bf16 before the MFMA GEMMs): relative L2 error
< 1e-2 and elementwise within 3e-2 * max|g|.
"""
import math

import numpy as np
import pytest
import torch

from oracle import ref_cpu
from tests import golden_io as G

pytestmark = pytest.mark.gpu

dev = "cuda"


def _ops():
    from triad_amd import ops
    return ops


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _check_grad(got, ref, skip=None):
    """bf16 bar on a (B, N, 512) feature gradient. skip (B, N) bool: rows whose oracle row max is a
    near-tie (ref_cpu.near_ties) are left out -- there the fp32 kernels may legitimately take the
    other key's gradient -- and must stay a small minority."""
    got = got.detach().float().cpu().numpy()
    ref = np.asarray(ref)
    if skip is not None:
        keep = ~skip.cpu().numpy().reshape(-1)
        assert keep.mean() > 0.97, f"{(~keep).sum()} of {keep.size} rows near-tied"
        got = got.reshape(-1, got.shape[-1])[keep]
        ref = ref.reshape(-1, ref.shape[-1])[keep]
    assert _rel(got, ref) < 1e-2, _rel(got, ref)
    np.testing.assert_allclose(got, ref, rtol=0, atol=3e-2 * float(np.abs(ref).max()) + 1e-12)


def _ties(q, k, temp):
    """(query rows, key rows) touched by an fp32 near-tie of a row max (oracle.ref_cpu.near_ties)."""
    tq, tk, _ = ref_cpu.near_ties(q.double(), k.double(), float(temp))
    return tq, tk


def _scalar_close(a, b, rtol=1e-4, atol=1e-5):
    if math.isnan(b):
        return math.isnan(a)
    return abs(a - b) <= atol + rtol * abs(b)


@pytest.mark.parametrize("name", G.names("av"))
def test_av_head_matches_golden(name):
    ops = _ops()
    f = G.load(name)
    A = G.bf16(f["A"]).to(dev, torch.bfloat16).requires_grad_(True)
    V = G.bf16(f["V"]).to(dev, torch.bfloat16).requires_grad_(True)
    t = torch.tensor(float(f["temp"]), device=dev, requires_grad=True)
    losses, stats, clip = ops.contrastive_head(ops.AV, A, V, t)
    losses[0].backward()
    np.testing.assert_allclose(clip.cpu().numpy(), f["clip"], rtol=1e-4, atol=1e-4)
    lv = torch.stack([x.detach() for x in losses]).cpu().double().numpy()
    for got, key in zip(lv, ("total", "ce", "reg", "smooth")):
        assert _scalar_close(float(got), float(f[key])), (key, got, f[key])
    sv = stats.cpu().double().numpy()
    for got, want in zip(sv[:6], f["stats"]):
        assert _scalar_close(float(got), float(want), 1e-4, 1e-4)
    _check_grad(A.grad, f["dA"])
    _check_grad(V.grad, f["dV"])
    assert _scalar_close(float(t.grad), float(f["dtemp"]), 1e-3, 1e-5), (float(t.grad), float(f["dtemp"]))


@pytest.mark.parametrize("name", G.names("tv"))
def test_tv_head_matches_golden(name):
    ops = _ops()
    f = G.load(name)
    T = G.bf16(f["T"]).to(dev, torch.bfloat16).requires_grad_(True)
    V = G.bf16(f["V"]).to(dev, torch.bfloat16).requires_grad_(True)
    mask = torch.from_numpy(f["mask"]).to(dev)
    t = torch.tensor(float(f["temp"]), device=dev, requires_grad=True)
    losses, stats, clip = ops.contrastive_head(ops.TV, T, V, t, q_mask=mask, threshold=float(f["thr"]),
                                               sparsity_weight=float(f["w"]))
    losses[0].backward()
    np.testing.assert_allclose(clip.cpu().numpy(), f["clip"], rtol=1e-4, atol=1e-4)
    assert _scalar_close(float(losses[0]), float(f["total"]))
    sv = stats.cpu().double().numpy()
    for got, want in zip(sv[:6], f["stats"]):
        assert _scalar_close(float(got), float(want), 1e-4, 1e-4)
    _check_grad(T.grad, f["dT"])
    _check_grad(V.grad, f["dV"])
    assert _scalar_close(float(t.grad), float(f["dtemp"]), 1e-3, 1e-5), (float(t.grad), float(f["dtemp"]))


def _rand_feats(g, shape):
    return (torch.randn(*shape, generator=g) * 0.58).to(torch.bfloat16).float()


@pytest.mark.parametrize("B,Na,Nv,pad,mix", [(8, 199, 256, False, False), (6, 199, 200, True, False),
                                             (16, 50, 96, True, False), (6, 40, 70, True, True),
                                             (5, 499, 1369, True, False)])  # c5: 10 s audio, 518 px
def test_av_head_vs_oracle_random(B, Na, Nv, pad, mix):
    ops = _ops()
    g = torch.Generator().manual_seed(100 + B)
    A = _rand_feats(g, (B, Na, 512))
    V = _rand_feats(g, (B, Nv, 512))
    if pad:
        lens = torch.randint(Nv // 2, Nv + 1, (B,), generator=g)
        lens[0] = Nv
        for j in range(B):
            V[j, lens[j]:] = 0
    temp = 1.5
    Ar, Vr = A.double().requires_grad_(True), V.double().requires_grad_(True)
    tr = torch.tensor(temp, dtype=torch.float64, requires_grad=True)
    total, ce, reg, sm, stats = ref_cpu.av_loss(Ar, Vr, tr)
    # mix: a general combination of the four outputs (exercises the recompute backward)
    obj = (0.5 * total + 1.5 * ce - 0.7 * reg + 3.0 * sm) if mix else total
    obj.backward()
    Ag = A.to(dev, torch.bfloat16).requires_grad_(True)
    Vg = V.to(dev, torch.bfloat16).requires_grad_(True)
    tg = torch.tensor(temp, device=dev, requires_grad=True)
    losses, st, clip = ops.contrastive_head(ops.AV, Ag, Vg, tg)
    (0.5 * losses[0] + 1.5 * losses[1] - 0.7 * losses[2] + 3.0 * losses[3] if mix else losses[0]).backward()
    lv = torch.stack([x.detach() for x in losses]).cpu().double().numpy()
    for got, want in zip(lv, (total, ce, reg, sm)):
        assert _scalar_close(float(got), float(want)), (got, float(want))
    tq, tk = _ties(A, V, temp)
    _check_grad(Ag.grad, Ar.grad.numpy(), tq)
    _check_grad(Vg.grad, Vr.grad.numpy(), tk)
    assert _scalar_close(float(tg.grad), float(tr.grad), 1e-3, 1e-5), (float(tg.grad), float(tr.grad))


@pytest.mark.parametrize("B,Nt,Nv,mix", [(16, 32, 205, False), (12, 16, 64, False), (8, 12, 40, True),
                                         (5, 32, 1369, False)])  # c5: 518 px frames
def test_tv_head_vs_oracle_random(B, Nt, Nv, mix):
    ops = _ops()
    g = torch.Generator().manual_seed(200 + B)
    T = _rand_feats(g, (B, Nt, 512))
    V = _rand_feats(g, (B, Nv, 512))
    mask = (torch.arange(Nt)[None, :] < torch.randint(1, Nt + 1, (B, 1), generator=g)).long()
    temp, thr, w = 1.5, 0.005, 0.3
    Tr, Vr = T.double().requires_grad_(True), V.double().requires_grad_(True)
    tr = torch.tensor(temp, dtype=torch.float64, requires_grad=True)
    total, stats = ref_cpu.tv_loss(Tr, Vr, mask, tr, thr, w)
    (2.0 * total).backward() if mix else total.backward()
    Tg = T.to(dev, torch.bfloat16).requires_grad_(True)
    Vg = V.to(dev, torch.bfloat16).requires_grad_(True)
    tg = torch.tensor(temp, device=dev, requires_grad=True)
    losses, st, clip = ops.contrastive_head(ops.TV, Tg, Vg, tg, q_mask=mask.to(dev), threshold=thr,
                                            sparsity_weight=w)
    if mix:  # total = ce + reg: route the same gradient through the components (recompute backward)
        (losses[0] + losses[1] + losses[2]).backward()
    else:
        losses[0].backward()
    assert _scalar_close(float(losses[0]), float(total))
    tq, tk = _ties(T, V, temp)
    _check_grad(Tg.grad, Tr.grad.numpy(), tq)
    _check_grad(Vg.grad, Vr.grad.numpy(), tk)
    assert _scalar_close(float(tg.grad), float(tr.grad), 1e-3, 1e-5), (float(tg.grad), float(tr.grad))


@pytest.mark.parametrize("kind,B,Nq,Nv", [(0, 10, 61, 90), (1, 9, 24, 70), (0, 4, 33, 40)])
def test_memory_bounded_recompute_backward(kind, B, Nq, Nv):
    """ds_budget below the tiled dS size: the forward writes no dS and the backward recomputes S in
    chunks of 4 key samples (last chunk ragged; one chunk when B = 4), dQ summed over the chunks'
    fp32 partials. Same losses as the materialising head, gradients and d/dtemp against the fp64
    oracle at the bf16 bar, and against the materialising head."""
    ops = _ops()
    g = torch.Generator().manual_seed(300 + B)
    Q = _rand_feats(g, (B, Nq, 512))
    V = _rand_feats(g, (B, Nv, 512))
    lens = torch.randint(Nv // 2, Nv + 1, (B,), generator=g)
    lens[0] = Nv
    for j in range(B):
        V[j, lens[j]:] = 0
    mask = (torch.arange(Nq)[None, :] < torch.randint(1, Nq + 1, (B, 1), generator=g)).long()
    temp, thr, w = 1.3, 0.005, 0.3
    Qr, Vr = Q.double().requires_grad_(True), V.double().requires_grad_(True)
    tr = torch.tensor(temp, dtype=torch.float64, requires_grad=True)
    if kind == 0:
        total = ref_cpu.av_loss(Qr, Vr, tr)[0]
    else:
        total = ref_cpu.tv_loss(Qr, Vr, mask, tr, thr, w)[0]
    total.backward()
    tq, tk = _ties(Q, V, temp)
    geo = ops.Geometry(B, Nq, B, ((Nv + 31) // 32) * 32)
    per_sample = (geo.R_pad // 32) * (geo.Nk_pad // 32) * 2048
    res = []
    for budget in (None, 4 * per_sample):
        Qg = Q.to(dev, torch.bfloat16).requires_grad_(True)
        Vg = V.to(dev, torch.bfloat16).requires_grad_(True)
        tg = torch.tensor(temp, device=dev, requires_grad=True)
        kw = dict(q_mask=mask.to(dev), threshold=thr, sparsity_weight=w) if kind == 1 else {}
        losses, st, clip = ops.contrastive_head(kind, Qg, Vg, tg, ds_budget=budget, **kw)
        losses[0].backward()
        assert _scalar_close(float(losses[0]), float(total))
        _check_grad(Qg.grad, Qr.grad.numpy(), tq)
        _check_grad(Vg.grad, Vr.grad.numpy(), tk)
        assert _scalar_close(float(tg.grad), float(tr.grad), 1e-3, 1e-5), (float(tg.grad), float(tr.grad))
        res.append((Qg.grad.float().cpu(), Vg.grad.float().cpu(), float(tg.grad)))
    assert ops.ds_chunk_samples(geo, 4 * per_sample) == (4 if B > 4 else B)
    (q0, v0, t0), (q1, v1, t1) = res
    assert float((q0 - q1).norm() / q0.norm()) < 1e-2
    assert float((v0 - v1).norm() / v0.norm()) < 1e-2
    assert _scalar_close(t1, t0, 1e-3, 1e-6)


@pytest.mark.parametrize("form", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("kcontig,bk", [(1, 0), (0, 0), (1, 1), (0, 1)])
def test_gemm_layouts_vs_torch(kcontig, bk, form):
    """triad_gemm_bf16_form in each tile form (per-call argument: size policy, 128 x 128, 256 x 128
    ring, 256 x 256 four-wave / eight-wave) against a plain fp32 torch matmul of the same bf16 operands."""
    from triad_amd._lib import call, ptr, stream_ptr
    g = torch.Generator().manual_seed(7)
    M, N, K = 512, 768, 384
    A = torch.randn(M, K, generator=g).to(torch.bfloat16)
    B = torch.randn(K, N, generator=g).to(torch.bfloat16)
    ref = 0.7 * (A.float() @ B.float())
    Ad = (A if kcontig else A.t().contiguous()).to(dev)
    Bd = (B.t().contiguous() if bk else B).to(dev)
    alpha = torch.tensor([0.7], device=dev)
    C = torch.empty(M, N, device=dev)
    call("triad_gemm_bf16_form", ptr(Ad), K if kcontig else M, kcontig, ptr(Bd), K if bk else N, bk, M, N, K,
         ptr(alpha), ptr(C), N, 0, form, stream_ptr())
    torch.cuda.synchronize()
    np.testing.assert_allclose(C.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("temp", [-0.8, 0.35])
def test_tv_head_any_temperature_sign(temp):
    """The forward folds sgn(temp) into the query fragments and works on |temp|-scaled values
    (pairsim_fwd.hip): negative temperatures turn max into min of the raw dot products."""
    ops = _ops()
    g = torch.Generator().manual_seed(300)
    B, Nt, Nv = 8, 16, 40
    T = _rand_feats(g, (B, Nt, 512))
    V = _rand_feats(g, (B, Nv, 512))
    mask = (torch.arange(Nt)[None, :] < torch.randint(1, Nt + 1, (B, 1), generator=g)).long()
    thr, w = 0.005, 0.3
    Tr, Vr = T.double().requires_grad_(True), V.double().requires_grad_(True)
    tr = torch.tensor(temp, dtype=torch.float64, requires_grad=True)
    total, stats = ref_cpu.tv_loss(Tr, Vr, mask, tr, thr, w)
    total.backward()
    Tg = T.to(dev, torch.bfloat16).requires_grad_(True)
    Vg = V.to(dev, torch.bfloat16).requires_grad_(True)
    tg = torch.tensor(temp, device=dev, requires_grad=True)
    losses, st, clip = ops.contrastive_head(ops.TV, Tg, Vg, tg, q_mask=mask.to(dev), threshold=thr,
                                            sparsity_weight=w)
    losses[0].backward()
    assert _scalar_close(float(losses[0]), float(total))
    tq, tk = _ties(T, V, temp)
    _check_grad(Tg.grad, Tr.grad.numpy(), tq)
    _check_grad(Vg.grad, Vr.grad.numpy(), tk)
    assert _scalar_close(float(tg.grad), float(tr.grad), 1e-3, 1e-5), (float(tg.grad), float(tr.grad))


def test_av_head_below_clamp_window():
    """Large features: many S < -60, so the forward's fast unit-gradient form is corrected on
    most tiles (epi_fixup) -- losses, gradients and d/dtemp still match the oracle."""
    ops = _ops()
    g = torch.Generator().manual_seed(400)
    B, Na, Nv = 6, 49, 64
    A = (torch.randn(B, Na, 512, generator=g) * 1.4).to(torch.bfloat16).float()
    V = (torch.randn(B, Nv, 512, generator=g) * 1.4).to(torch.bfloat16).float()
    Ar, Vr = A.double().requires_grad_(True), V.double().requires_grad_(True)
    tr = torch.tensor(1.5, dtype=torch.float64, requires_grad=True)
    total, ce, reg, sm, stats = ref_cpu.av_loss(Ar, Vr, tr)
    total.backward()
    Ag = A.to(dev, torch.bfloat16).requires_grad_(True)
    Vg = V.to(dev, torch.bfloat16).requires_grad_(True)
    tg = torch.tensor(1.5, device=dev, requires_grad=True)
    losses, st, clip = ops.contrastive_head(ops.AV, Ag, Vg, tg)
    losses[0].backward()
    lv = torch.stack([x.detach() for x in losses]).cpu().double().numpy()
    for got, want in zip(lv, (total, ce, reg, sm)):
        assert _scalar_close(float(got), float(want)), (got, float(want))
    tq, tk = _ties(A, V, 1.5)
    _check_grad(Ag.grad, Ar.grad.numpy(), tq)
    _check_grad(Vg.grad, Vr.grad.numpy(), tk)
    assert _scalar_close(float(tg.grad), float(tr.grad), 1e-3, 1e-5), (float(tg.grad), float(tr.grad))


def _untile_dS(dS, R_pad, CT):
    """Tiled dS ([R_pad/32][CT][1024], lane L = query L&31 / half L>>5, value v = key
    (v&3) + 8(v>>2) + 4(L>>5), the 32x32x16 accumulator order; lane L's 16-byte chunks v>>3 = s
    stored at chunk 64 s + L, common.h ds_chunk) -> dense [R_pad][CT*32] fp32."""
    t = dS.float().view(R_pad // 32, CT, 2, 2, 32, 2, 4)  # rt, ct, s, hh, q, w2, w1 (v = 8s + 4w2 + w1)
    t = t.permute(0, 4, 1, 2, 5, 3, 6)                     # rt, q, ct, s, w2, hh, w1 -> key 16s+8w2+4hh+w1
    return t.reshape(R_pad, CT * 32)


@pytest.mark.parametrize("panels,ct", [(16, 64), (7, 36), (400, 24), (3, 4)])
def test_tile_gemm_vs_torch(panels, ct):
    """triad_tile_gemm (ring kernel, split-K slabs where chosen) against fp32 torch matmuls of the
    untiled dS: dQ = alpha dS K, dK = alpha dS^T Q."""
    from triad_amd._lib import stream_ptr
    ops = _ops()
    g = torch.Generator(device=dev).manual_seed(panels * 100 + ct)
    R_pad, CT = panels * 128, ct
    dS = (torch.randn(R_pad // 32 * CT * 1024, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    K = torch.randn(CT * 32, 512, device=dev, generator=g).to(torch.bfloat16)
    Q = torch.randn(R_pad, 512, device=dev, generator=g).to(torch.bfloat16)
    alpha = torch.tensor([0.75], device=dev)
    dense = _untile_dS(dS, R_pad, CT)
    dQ = torch.empty(R_pad, 512, dtype=torch.bfloat16, device=dev)
    ops.tile_gemm(dS, CT, 0, K, R_pad, CT, alpha, dQ, stream_ptr())
    dK = torch.empty(CT * 32, 512, dtype=torch.bfloat16, device=dev)
    if CT % 4 == 0:
        ops.tile_gemm(dS, CT, 1, Q, CT * 32, R_pad // 32, alpha, dK, stream_ptr())
    torch.cuda.synchronize()
    refQ = 0.75 * dense @ K.float()
    assert _rel(dQ.float().cpu(), refQ.cpu()) < 5e-3
    if CT % 4 == 0:
        refK = 0.75 * dense.t() @ Q.float()
        assert _rel(dK.float().cpu(), refK.cpu()) < 5e-3


@pytest.mark.parametrize("panels,ct,splits", [(2, 4, 1), (3, 7, 1), (4, 8, 3), (2, 8, 5), (7, 36, 1),
                                               (7, 36, 3), (16, 64, 4), (5, 12, 2), (3, 9, 1), (8, 28, 4),
                                               (3, 13, 2), (2, 5, 4)])
def test_tile_gemm_mfma16_matches_ring(panels, ct, splits):
    """dQ and dK on v_mfma_f32_16x16x32_bf16 (triad_bfrag_pack16 + triad_tile_gemm_packed16 /
    _packed16_slabs) against the 32x32x16 ring form (bit-identical: the same fp32 sums, in an
    order the two MFMA shapes share -- measured, not assumed) and against an fp64 product over the
    untiled dS, split-K slabs included. The k ranges per split cover every remainder of the
    direct-B loop's four-stage groups (0-3 trailing stages, no whole group, empty last splits)."""
    from triad_amd._lib import call, ptr, stream_ptr
    g = torch.Generator(device=dev).manual_seed(7 * panels + ct + splits)
    R_pad, CT = panels * 128, ct
    dS = (torch.randn(R_pad // 32 * CT * 1024, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    K = torch.randn(CT * 32, 512, device=dev, generator=g).to(torch.bfloat16)
    Q = torch.randn(R_pad, 512, device=dev, generator=g).to(torch.bfloat16)
    alpha = torch.tensor([0.75], device=dev)
    st = stream_ptr()
    dense = _untile_dS(dS, R_pad, CT).double()
    cases = [(0, K, R_pad, CT, dense @ K.double())]
    if CT % 4 == 0:
        cases.append((1, Q, CT * 32, R_pad // 32, dense.t() @ Q.double()))
    for dk, Bm, M, nkt, prod in cases:
        Bp16 = torch.empty(nkt * 32 * 512, dtype=torch.bfloat16, device=dev)
        call("triad_bfrag_pack16", ptr(Bm), nkt, dk, ptr(Bp16), st)
        slabs = torch.empty(splits * M * 512, device=dev) if splits > 1 else None
        slabs2 = torch.empty(splits * M * 512, device=dev) if splits > 1 else None
        out16 = torch.empty(M, 512, dtype=torch.bfloat16, device=dev)
        ring = torch.empty_like(out16)
        call("triad_tile_gemm_packed16", ptr(dS), CT, dk, ptr(Bp16), M, nkt, ptr(alpha), splits, ptr(slabs), ptr(out16),
             st)
        call("triad_tile_gemm", ptr(dS), CT, dk, ptr(Bm), M, nkt, ptr(alpha), splits, ptr(slabs2), ptr(ring), st)
        torch.cuda.synchronize()
        ref = 0.75 * prod
        err = float((out16.double() - ref).abs().max() / ref.abs().max())
        assert err < 8e-3, (dk, err)
        assert torch.equal(out16, ring), (dk, M, nkt, splits)
        if splits > 1:
            assert torch.equal(slabs, slabs2), (dk, "slabs")
            call("triad_tile_gemm_packed16_slabs", ptr(dS), CT, dk, ptr(Bp16), M, nkt, splits, ptr(slabs), st)
            call("triad_tile_gemm_slabs", ptr(dS), CT, dk, ptr(Bm), M, nkt, splits, ptr(slabs2), st)
            torch.cuda.synchronize()
            assert torch.equal(slabs, slabs2), (dk, "slabs only")


@pytest.mark.parametrize("B,Na,Nt,Nv,budget", [(6, 49, 16, 70, None), (16, 199, 32, 205, None),
                                               (5, 300, 8, 40, "mixed"), (3, 2, 1, 33, None)])
def test_pair_launch_matches_two_heads(B, Na, Nt, Nv, budget):
    """contrastive_heads_av_tv (ONE similarity-forward launch over the AV and TV heads,
    triad_pairsim_fwd_multi) against the two single-head launches on the same inputs: losses,
    statistics, clip matrices and every gradient bit-identical (each workgroup runs the same code
    on the same tiles); and against the fp64 oracle. budget "mixed": one dS budget for the pair
    (ADVICE r2), AV's dS within it, TV's over what AV leaves (mixed modes -> two launches, chunked
    recompute backward for TV)."""
    ops = _ops()
    # (seed 500 + B: the (5, 300) case has two keys 2.8e-6 apart at S = 13.28, below fp32
    # resolution -- the MFMA sum order may pick either; _check_grad leaves near-tied rows out)
    g = torch.Generator().manual_seed(500 + B)
    A = _rand_feats(g, (B, Na, 512))
    T = _rand_feats(g, (B, Nt, 512))
    Va = _rand_feats(g, (B, Nv, 512))
    Vt = _rand_feats(g, (B, Nv - 3, 512))
    for V in (Va, Vt):
        lens = torch.randint(V.shape[1] // 2, V.shape[1] + 1, (B,), generator=g)
        lens[0] = V.shape[1]
        for j in range(B):
            V[j, lens[j]:] = 0
    mask = (torch.arange(Nt)[None, :] < torch.randint(1, Nt + 1, (B, 1), generator=g)).long()
    thr, w = 0.005, 0.3

    def leaves():
        return [x.to(dev, torch.bfloat16).requires_grad_(True) for x in (A, Va, T, Vt)]

    ds_budget = bud_av = bud_tv = None
    if budget == "mixed":
        # ONE budget for the pair: AV's whole dS fits, TV gets what AV leaves (half its dS), so TV's
        # backward recomputes in chunks -- mixed modes -> two forward launches
        ga = ops.Geometry(B, Na, B, Va.shape[1])
        gt = ops.Geometry(B, Nt, B, Vt.shape[1])
        ds_budget = bud_av = ops.ds_bytes(ga) + ops.ds_bytes(gt) // 2
        bud_tv = ds_budget - ops.ds_working_bytes(ga, B)
        assert ops.ds_chunk_samples(ga, bud_av) == B and ops.ds_bytes(gt) > bud_tv
    # pair
    a1, va1, t1, vt1 = leaves()
    tg1 = torch.tensor(1.4, device=dev, requires_grad=True)
    (la, sa, ca), (lt, st, ct) = ops.contrastive_heads_av_tv(a1, va1, t1, vt1, tg1, mask.to(dev), threshold=thr,
                                                             sparsity_weight=w, ds_budget=ds_budget)
    (la[0] + lt[0]).backward()
    # two single heads, each with the share of the budget the pair gave it
    a2, va2, t2, vt2 = leaves()
    tg2 = torch.tensor(1.4, device=dev, requires_grad=True)
    la2, sa2, ca2 = ops.contrastive_head(ops.AV, a2, va2, tg2, ds_budget=bud_av)
    lt2, st2, ct2 = ops.contrastive_head(ops.TV, t2, vt2, tg2, q_mask=mask.to(dev), threshold=thr, sparsity_weight=w,
                                         ds_budget=bud_tv)
    (la2[0] + lt2[0]).backward()
    for x, y in [(torch.stack(la), torch.stack(la2)), (torch.stack(lt), torch.stack(lt2)), (sa, sa2), (st, st2),
                 (ca, ca2), (ct, ct2), (a1.grad, a2.grad), (va1.grad, va2.grad), (t1.grad, t2.grad),
                 (vt1.grad, vt2.grad)]:
        assert torch.equal(x, y)
    assert float(tg1.grad) == float(tg2.grad)
    # and the oracle
    Ar, Var, Tr, Vtr = [x.double().requires_grad_(True) for x in (A, Va, T, Vt)]
    tr = torch.tensor(1.4, dtype=torch.float64, requires_grad=True)
    tot_a = ref_cpu.av_loss(Ar, Var, tr)[0]
    tot_t = ref_cpu.tv_loss(Tr, Vtr, mask, tr, thr, w)[0]
    (tot_a + tot_t).backward()
    assert _scalar_close(float(la[0]), float(tot_a)) and _scalar_close(float(lt[0]), float(tot_t))
    ta, tva = _ties(A, Va, 1.4)
    tt, tvt = _ties(T, Vt, 1.4)
    for gg, rr, sk in ((a1.grad, Ar.grad, ta), (va1.grad, Var.grad, tva), (t1.grad, Tr.grad, tt),
                       (vt1.grad, Vtr.grad, tvt)):
        _check_grad(gg, rr.numpy(), sk)
    assert _scalar_close(float(tg1.grad), float(tr.grad), 1e-3, 1e-5), (float(tg1.grad), float(tr.grad))


@pytest.mark.parametrize("counts", [[210, 150, 192, 193, 100, 205, 160, 180],
                                    [210, 0, 1, 32, 33, 192, 64, 150]])   # + empty / one-key samples
def test_pair_launch_compact_key_tiles(counts):
    """Keys straight from patch_dropout carry their kept count per sample (ops.KEPT_ROWS_ATTR):
    the training pair forward then leaves every sample's all-zero last 32-key tile out of K and of
    the tiled dS (kept <= 192 of Nk_pad = 224 here; ops._compact) and applies its S == 0 in closed
    form; the dS patch, dQ and dK run over the stored tiles. Against the same inputs with the
    attribute removed (every tile stored and multiplied): losses, statistics, clip matrices and the
    temperature gradient bit-identical (the forward's sums and the patch partials see the same
    values in the same order); the feature gradients within bf16 rounding (dQ / dK sum the same
    nonzero products, split over the CUs differently). One (audio, visual) pair has only negative
    real similarities, so its row maxima are the zero of the first left-out key."""
    ops = _ops()
    g = torch.Generator().manual_seed(4242)
    B, N, Na, Nt = 8, 256, 40, 16
    A = _rand_feats(g, (B, Na, 512))
    T = _rand_feats(g, (B, Nt, 512))
    X = _rand_feats(g, (B, N, 512))
    e = torch.randn(512, generator=g)
    e = e / e.norm()
    A[0] = (e * 2.0 + 0.01 * torch.randn(Na, 512, generator=g)).to(torch.bfloat16).float()
    X[2] = (-e * 1.5 + 0.01 * torch.randn(N, 512, generator=g)).to(torch.bfloat16).float()
    keep_av = torch.zeros(B, N, dtype=torch.bool)
    keep_tv = torch.zeros(B, N, dtype=torch.bool)
    for j, c in enumerate(counts):
        keep_av[j, torch.randperm(N, generator=g)[:c]] = True
        keep_tv[j, torch.randperm(N, generator=g)[:max(1, c - 7)]] = True
    mask = (torch.arange(Nt)[None, :] < torch.randint(1, Nt + 1, (B, 1), generator=g)).long()
    compacted = []
    orig = ops._compact

    def spy(h):
        orig(h)
        compacted.append(h.Kc is not None)

    outs = []
    try:
        ops._compact = spy
        for strip in (False, True):
            a = A.to(dev, torch.bfloat16).requires_grad_(True)
            t = T.to(dev, torch.bfloat16).requires_grad_(True)
            x = X.to(dev, torch.bfloat16).requires_grad_(True)
            tg = torch.tensor(1.3, device=dev, requires_grad=True)
            va = ops.patch_dropout(x, keep_av)
            vt = ops.patch_dropout(x, keep_tv)
            assert va.shape[1] == max(counts) and hasattr(va, ops.KEPT_ROWS_ATTR)
            if strip:
                delattr(va, ops.KEPT_ROWS_ATTR)
                delattr(vt, ops.KEPT_ROWS_ATTR)
            (la, sa, ca), (lt, st, ct) = ops.contrastive_heads_av_tv(a, va, t, vt, tg, mask.to(dev),
                                                                     threshold=0.005, sparsity_weight=0.3)
            (la[0] + lt[0]).backward()
            outs.append(([torch.stack(la), torch.stack(lt), sa, st, ca, ct, tg.grad], [a.grad, t.grad, x.grad]))
    finally:
        ops._compact = orig
    assert compacted == [True, True, False, False]
    # the crafted pair: every real similarity of (audio 0, visual 2) is negative -> clip = mean of 0
    assert float(outs[0][0][4][0, 2]) == 0.0
    for got, want in zip(outs[0][0], outs[1][0]):
        assert torch.equal(got, want)
    for got, want in zip(outs[0][1], outs[1][1]):
        gf, wf = got.float(), want.float()
        assert float((gf - wf).norm() / wf.norm()) < 2e-3
        assert float((gf - wf).abs().max()) <= 2 ** -6 * float(wf.abs().max())


@pytest.mark.parametrize("bk", [0, 1])
def test_gemm_wide_bf16_nontemporal(bk):
    """Eight-wave form with a wide bf16 output (2304 columns, B k-contiguous or not)
    against an fp32 torch matmul of the same bf16 operands."""
    from triad_amd._lib import call, ptr, stream_ptr
    g = torch.Generator().manual_seed(11 + bk)
    M, N, K = 512, 2304, 384
    A = torch.randn(M, K, generator=g).to(torch.bfloat16)
    B = torch.randn(K, N, generator=g).to(torch.bfloat16)
    ref = A.float() @ B.float()
    Ad = A.to(dev)
    Bd = (B.t().contiguous() if bk else B).to(dev)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    call("triad_gemm_bf16_form", ptr(Ad), K, 1, ptr(Bd), K if bk else N, bk, M, N, K, None, ptr(C), N, 1, 4,
         stream_ptr())
    torch.cuda.synchronize()
    assert float((C.float().cpu() - ref).norm() / ref.norm()) < 4e-3


def test_pair_launch_eval_mode_matches_two_heads():
    """Validation / inference (no gradient): the pair launch's eval instantiation (no dS stream)
    gives the same losses, statistics and clip matrices as the two single-head launches."""
    ops = _ops()
    g = torch.Generator().manual_seed(77)
    B, Na, Nt, Nv = 8, 99, 20, 150
    A, T = _rand_feats(g, (B, Na, 512)), _rand_feats(g, (B, Nt, 512))
    Va, Vt = _rand_feats(g, (B, Nv, 512)), _rand_feats(g, (B, Nv - 7, 512))
    mask = (torch.arange(Nt)[None, :] < torch.randint(1, Nt + 1, (B, 1), generator=g)).long().to(dev)
    xs = [x.to(dev, torch.bfloat16) for x in (A, Va, T, Vt)]
    t = torch.tensor(1.3, device=dev)
    with torch.no_grad():
        (la, sa, ca), (lt, st, ct) = ops.contrastive_heads_av_tv(xs[0], xs[1], xs[2], xs[3], t, mask, threshold=0.01,
                                                                 sparsity_weight=0.2)
        la2, sa2, ca2 = ops.contrastive_head(ops.AV, xs[0], xs[1], t)
        lt2, st2, ct2 = ops.contrastive_head(ops.TV, xs[2], xs[3], t, q_mask=mask, threshold=0.01, sparsity_weight=0.2)
    for x, y in [(torch.stack(la), torch.stack(la2)), (torch.stack(lt), torch.stack(lt2)), (sa, sa2), (st, st2),
                 (ca, ca2), (ct, ct2)]:
        assert torch.equal(x, y)
    total = ref_cpu.av_loss(A.double(), Va.double(), torch.tensor(1.3, dtype=torch.float64))[0]
    assert _scalar_close(float(la[0]), float(total))


def test_pair_head_compact_c3_repeats_bit_stable():
    """The c3-shaped training pair head (B = 256, Na = 199, Nt = 32, keys from patch_dropout so the
    key tiles are compacted) run six times on identical inputs: every gradient bit-identical across
    the repeats. Before the direct-B GEMMs' tail stages drained vmcnt, AV dK --
    3 splits of 534 stages, a 2-stage tail -- differed in 3 of 7 such repeats."""
    ops = _ops()
    g = torch.Generator().manual_seed(7)
    B, N, Na, Nt = 256, 256, 199, 32
    A = (torch.randn(B, Na, 512, generator=g) * 0.58).to(torch.bfloat16).to(dev)
    T = (torch.randn(B, Nt, 512, generator=g) * 0.58).to(torch.bfloat16).to(dev)
    X = (torch.randn(B, N, 512, generator=g) * 0.58).to(torch.bfloat16).to(dev)
    keep_av = torch.rand(B, N, generator=g) < 0.75
    keep_tv = torch.rand(B, N, generator=g) < 0.75
    mask = torch.ones(B, Nt, dtype=torch.long, device=dev)
    first = None
    for _ in range(6):
        a, t, x = (v.clone().requires_grad_(True) for v in (A, T, X))
        tg = torch.tensor(1.5, device=dev, requires_grad=True)
        (la, _, _), (lt, _, _) = ops.contrastive_heads_av_tv(a, ops.patch_dropout(x, keep_av), t,
                                                             ops.patch_dropout(x, keep_tv), tg, mask,
                                                             threshold=0.8, sparsity_weight=0.01)
        (la[0] + lt[0]).backward()
        cur = [a.grad, t.grad, x.grad, tg.grad]
        if first is None:
            first = cur
        else:
            for got, want in zip(cur, first):
                assert torch.equal(got, want)


@pytest.mark.parametrize("kind", [0, 1])
def test_forward_epilogue_forms_agree(kind, monkeypatch):
    """The training forward's two epilogues (pairsim_fwd.hip: the fast form with the per-tile slow
    redo, and the exact per-element form; chosen per head by its clamp window, forced here by
    TRIAD_FWD_EXACT) on both heads, with features large enough that many tiles hold S below the
    window: losses and feature gradients bit-identical between the forms (same unit dS, same
    sum of clamp^2), d/dtemp within fp32 summation order, both against the fp64 oracle."""
    ops = _ops()
    g = torch.Generator().manual_seed(410 + kind)
    B, Nq, Nv = 6, (49 if kind == 0 else 16), 70
    Q = (torch.randn(B, Nq, 512, generator=g) * (1.4 if kind == 0 else 0.58)).to(torch.bfloat16).float()
    V = (torch.randn(B, Nv, 512, generator=g) * (1.4 if kind == 0 else 0.58)).to(torch.bfloat16).float()
    mask = (torch.arange(Nq)[None, :] < torch.randint(1, Nq + 1, (B, 1), generator=g)).long()
    temp, thr, w = 1.5, 0.005, 0.3
    Qr, Vr = Q.double().requires_grad_(True), V.double().requires_grad_(True)
    tr = torch.tensor(temp, dtype=torch.float64, requires_grad=True)
    total = (ref_cpu.av_loss(Qr, Vr, tr) if kind == 0 else ref_cpu.tv_loss(Qr, Vr, mask, tr, thr, w))[0]
    total.backward()
    tq, tk = _ties(Q, V, temp)
    got = []
    for form in ("0", "1"):
        monkeypatch.setenv("TRIAD_FWD_EXACT", form)
        Qg = Q.to(dev, torch.bfloat16).requires_grad_(True)
        Vg = V.to(dev, torch.bfloat16).requires_grad_(True)
        tg = torch.tensor(temp, device=dev, requires_grad=True)
        kw = dict(q_mask=mask.to(dev), threshold=thr, sparsity_weight=w) if kind == 1 else {}
        losses, st, clip = ops.contrastive_head(kind, Qg, Vg, tg, **kw)
        losses[0].backward()
        assert _scalar_close(float(losses[0]), float(total))
        _check_grad(Qg.grad, Qr.grad.numpy(), tq)
        _check_grad(Vg.grad, Vr.grad.numpy(), tk)
        assert _scalar_close(float(tg.grad), float(tr.grad), 1e-3, 1e-5), (float(tg.grad), float(tr.grad))
        got.append((torch.stack([x.detach() for x in losses]).cpu(), Qg.grad.cpu(), Vg.grad.cpu(), float(tg.grad)))
    (l0, q0, v0, t0), (l1, q1, v1, t1) = got
    assert torch.equal(l0, l1) and torch.equal(q0, q1) and torch.equal(v0, v1)
    assert abs(t0 - t1) <= 1e-5 * max(abs(t0), 1e-6), (t0, t1)
