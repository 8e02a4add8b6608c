"""Pin the CPU oracle (oracle/ref_cpu.py) to the reference's own outputs.

The fixtures were produced by running /root/reference/src/model.py's hot-path
methods (tests/golden/gen_golden.py). fp32 reference vs float64 oracle.
"""
import math

import numpy as np
import pytest
import torch

from oracle import ref_cpu
from tests import golden_io as G


def _close(a, b, rtol=1e-4, atol=1e-5):
    if isinstance(a, float) and math.isnan(a):
        return math.isnan(b)
    return abs(a - b) <= atol + rtol * abs(b)


@pytest.mark.parametrize("name", G.names("av"))
def test_av_matches_reference(name):
    f = G.load(name)
    A = G.bf16(f["A"]).double().requires_grad_(True)
    V = G.bf16(f["V"]).double().requires_grad_(True)
    t = torch.tensor(float(f["temp"]), dtype=torch.float64, requires_grad=True)
    clip, s = ref_cpu.similarities_av(A, V, t)
    total, ce, reg, smooth, stats = ref_cpu.contrastive_av(clip, s, t)
    np.testing.assert_allclose(clip.detach().numpy(), f["clip"], rtol=1e-4, atol=1e-4)
    assert _close(float(ce), float(f["ce"]))
    assert _close(float(reg), float(f["reg"]))
    assert _close(float(smooth), float(f["smooth"]))
    assert _close(float(total), float(f["total"]))
    for k, v in zip(ref_cpu.AV_STAT_KEYS, f["stats"]):
        assert _close(stats[k], float(v), rtol=1e-4, atol=1e-4), k
    # Na == 1: the smoothness mean is over an empty set, so `total` is NaN in the
    # reference while its gradients stay finite (the empty term contributes none).
    total.backward()
    np.testing.assert_allclose(A.grad.numpy(), f["dA"], rtol=2e-3, atol=1e-7)
    np.testing.assert_allclose(V.grad.numpy(), f["dV"], rtol=2e-3, atol=1e-7)
    assert _close(float(t.grad), float(f["dtemp"]), rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("name", G.names("tv"))
def test_tv_matches_reference(name):
    f = G.load(name)
    T = G.bf16(f["T"]).double().requires_grad_(True)
    V = G.bf16(f["V"]).double().requires_grad_(True)
    mask = torch.from_numpy(f["mask"])
    t = torch.tensor(float(f["temp"]), dtype=torch.float64, requires_grad=True)
    clip, s = ref_cpu.similarities_tv(T, V, mask, t)
    total, stats = ref_cpu.contrastive_tv(clip, s, float(f["thr"]), float(f["w"]))
    np.testing.assert_allclose(clip.detach().numpy(), f["clip"], rtol=1e-4, atol=1e-4)
    assert _close(float(total), float(f["total"]))
    for k, v in zip(ref_cpu.TV_STAT_KEYS, f["stats"]):
        assert _close(stats[k], float(v), rtol=1e-4, atol=1e-4), k
    total.backward()
    np.testing.assert_allclose(T.grad.numpy(), f["dT"], rtol=2e-3, atol=1e-7)
    np.testing.assert_allclose(V.grad.numpy(), f["dV"], rtol=2e-3, atol=1e-7)
    assert _close(float(t.grad), float(f["dtemp"]), rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("name", G.names("simmat"))
def test_similarity_matrix_matches_reference(name):
    f = G.load(name)
    sim = ref_cpu.similarity_matrix(G.bf16(f["f1"]), G.bf16(f["f2"]),
                                    torch.tensor(float(f["temp"])))
    np.testing.assert_allclose(sim.numpy(), f["sim"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", G.names("dropout"))
def test_patch_dropout_matches_reference(name):
    f = G.load(name)
    out = ref_cpu.patch_dropout(G.bf16(f["x"]), torch.from_numpy(f["keep"]))
    np.testing.assert_array_equal(out.numpy(), G.bf16(f["out"]).numpy())


@pytest.mark.parametrize("kind", ["av", "tv"])
def test_chunked_oracle_equals_materialising_oracle(kind):
    """ref_cpu.head_loss_chunked (used for the BASELINE-size GPU parity tests) reproduces the
    materialising restatement -- losses, statistics and all gradients -- with zero-padded keys,
    a ragged text mask, and chunks that do not divide B."""
    g = torch.Generator().manual_seed(0)
    B, Nq, Nk = 7, 9, 13
    q = torch.randn(B, Nq, 512, generator=g, dtype=torch.float64) * 0.58
    k = torch.randn(B, Nk, 512, generator=g, dtype=torch.float64) * 0.58
    k[2, 9:] = 0
    mask = (torch.arange(Nq)[None] < torch.randint(1, Nq + 1, (B, 1), generator=g)).long()
    t = torch.tensor(0.9, dtype=torch.float64, requires_grad=True)
    qr, kr = q.clone().requires_grad_(True), k.clone().requires_grad_(True)
    if kind == "av":
        tot, ce, reg, sm, st = ref_cpu.av_loss(qr, kr, t)
    else:
        tot, st = ref_cpu.tv_loss(qr, kr, mask, t, 0.1, 0.3)
    tot.backward()
    o = ref_cpu.head_loss_chunked(kind, q, k, 0.9, q_mask=mask, threshold=0.1, weight=0.3, chunk=3)
    assert abs(o["total"] - float(tot)) < 1e-12 * abs(float(tot))
    for key in st:
        assert abs(o["stats"][key] - st[key]) < 1e-12 * max(1.0, abs(st[key]))
    assert torch.allclose(o["dq"], qr.grad, rtol=0, atol=1e-14)
    assert torch.allclose(o["dk"], kr.grad, rtol=0, atol=1e-14)
    assert abs(o["dtemp"] - float(t.grad)) < 1e-12 * abs(float(t.grad))


def _token_lists(flat, lens):
    x = G.bf16(flat)
    return list(torch.split(x, [int(n) for n in lens]))


@pytest.mark.parametrize("name", G.names("retrieval_av") + G.names("retrieval_tv"))
def test_retrieval_oracle_matches_reference(name):
    """The oracle's aggregators (fp64) and recall against the reference's retrieval.py run on the
    same token lists: both N x N matrices, the per-query ranks (exact ties included) and R@k."""
    f = G.load(name)
    q = _token_lists(f["q"], f["q_len"])
    k = _token_lists(f["k"], f["k_len"])
    q2k, k2q = ref_cpu.retrieval_matrices(q, k, float(f["temp"]))
    np.testing.assert_allclose(q2k, f["sim_qk"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(k2q, f["sim_kq"], rtol=1e-5, atol=1e-6)
    for key in ("qk", "kq"):
        np.testing.assert_array_equal(ref_cpu.recall_ranks(f["sim_" + key]), f["ranks_" + key])
        r = ref_cpu.recall_at_k(f["sim_" + key])
        assert [r[x] for x in ("r1", "r5", "r10", "r20")] == list(f["recall_" + key])


@pytest.mark.parametrize("name", G.names("retrieval_av") + G.names("retrieval_tv"))
def test_retrieval_recall_host_ranking_matches_reference(name):
    """triad_amd.retrieval.recall_at_k (ties="reference") on the reference's own matrices gives
    its ranks and R@k exactly; the stable order differs on the tie fixtures."""
    from triad_amd import retrieval
    f = G.load(name)
    for key in ("qk", "kq"):
        s = torch.from_numpy(f["sim_" + key])
        np.testing.assert_array_equal(retrieval.ranks(s).numpy(), f["ranks_" + key])
        r = retrieval.recall_at_k(s)
        assert [r[x] for x in ("r1", "r5", "r10", "r20")] == list(f["recall_" + key])
    if name.endswith("_ties"):
        assert not np.array_equal(retrieval.ranks(torch.from_numpy(f["sim_qk"]), ties="stable").numpy(),
                                  f["ranks_qk"])


@pytest.mark.parametrize("name", G.names("znorm"))
def test_audio_znorm_oracle_matches_feature_extractor(name):
    f = G.load(name)
    y = ref_cpu.audio_znorm(torch.from_numpy(f["x"]))
    np.testing.assert_allclose(y.numpy(), f["y"], rtol=1e-5, atol=2e-5)


def test_near_ties_flags_exact_and_close_row_maxima():
    """oracle.ref_cpu.near_ties (the parity tests' tie rule): an exactly duplicated key and a key
    within a few fp32 ulps of the row max are flagged -- the query row and both candidate keys --,
    a clear winner is not, and random features leave almost every row unflagged."""
    g = torch.Generator().manual_seed(3)
    q = torch.randn(2, 4, 512, generator=g, dtype=torch.float64)
    k = torch.randn(2, 6, 512, generator=g, dtype=torch.float64) * 0.01
    k[0, 1] = q[0, 2] * 0.5                   # clear max of row (0, 2) against sample 0 ...
    k[0, 4] = k[0, 1]                         # ... duplicated: exact tie
    k[1, 0] = q[1, 3] * 0.5
    k[1, 5] = k[1, 0] * (1 + 2e-7)            # 0.2 ppm apart: below 8 fp32 ulps of the max
    tq, tk, n = ref_cpu.near_ties(q, k, 1.5)
    assert bool(tq[0, 2]) and bool(tk[0, 1]) and bool(tk[0, 4])
    assert bool(tq[1, 3]) and bool(tk[1, 0]) and bool(tk[1, 5])
    assert n >= 2 and int(tk.sum()) == 4
    k[1, 5] = k[1, 0] * (1 - 1e-3)            # a clear second: no longer a tie
    tq2, tk2, _ = ref_cpu.near_ties(q, k, 1.5)
    assert not bool(tk2[1, 5])
    qr = (torch.randn(4, 50, 512, generator=g) * 0.58).double()
    kr = (torch.randn(4, 60, 512, generator=g) * 0.58).double()
    tq3, tk3, _ = ref_cpu.near_ties(qr, kr, 1.5)
    assert float(tq3.float().mean()) < 0.02
