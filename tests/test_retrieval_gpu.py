"""1000-way retrieval scorer (HIP, one launch per direction): against the reference's own
retrieval.py outputs (tests/golden/retrieval_*.npz: its aggregators' N x N matrices, ranks with
its unstable-argsort tie order, R@k) and against the oracle's restatement on ragged lists."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu
from tests import golden_io as G

pytestmark = pytest.mark.gpu


def _lists(n, lo, hi, seed, normalize):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        L = int(torch.randint(lo, hi + 1, (1,), generator=g))
        x = torch.randn(L, 512, generator=g)
        if normalize:
            x = torch.nn.functional.normalize(x, dim=-1)
        out.append(x.to(torch.bfloat16).float())
    return out


@pytest.mark.parametrize("normalize,qlo,qhi,klo,khi", [(True, 30, 60, 40, 64), (False, 1, 12, 20, 33)])
def test_retrieval_matrices_and_recall(normalize, qlo, qhi, klo, khi):
    from triad_amd import retrieval
    N, temp = 24, 1.7
    q = _lists(N, qlo, qhi, 1, normalize)
    k = _lists(N, klo, khi, 2, normalize)
    # make the matching pairs similar so recall is informative
    for i in range(N):
        k[i][: min(len(q[i]), len(k[i]))] += 0.5 * q[i][: min(len(q[i]), len(k[i]))]
        k[i] = k[i].to(torch.bfloat16).float()
    q2k, k2q = ref_cpu.retrieval_matrices(q, k, temp)
    s1 = retrieval.aggregated_similarity(q, k, temp).cpu().double().numpy()
    s2 = retrieval.aggregated_similarity(k, q, temp).cpu().double().numpy()
    np.testing.assert_allclose(s1, q2k, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(s2, k2q, rtol=1e-4, atol=1e-5)
    r_ref = ref_cpu.recall_at_k(q2k)
    r = retrieval.recall_at_k(torch.from_numpy(s1))
    assert r == r_ref


@pytest.mark.parametrize("name", G.names("retrieval_av") + G.names("retrieval_tv"))
def test_retrieval_matches_reference_fixtures(name):
    """Both directions' matrices within fp32 rounding of the reference's (it divides by the
    temperature, the kernel multiplies by its inverse); ranks and R@k EXACT -- the duplicated
    items and all-zero queries of the *_ties fixtures produce exact ties in the HIP matrices too,
    ordered as the reference's np.argsort orders them."""
    from triad_amd import retrieval
    f = G.load(name)
    q = list(torch.split(G.bf16(f["q"]), [int(n) for n in f["q_len"]]))
    k = list(torch.split(G.bf16(f["k"]), [int(n) for n in f["k_len"]]))
    temp = float(f["temp"])
    s_qk = retrieval.aggregated_similarity(q, k, temp)
    s_kq = retrieval.aggregated_similarity(k, q, temp)
    for s, key in ((s_qk, "qk"), (s_kq, "kq")):
        np.testing.assert_allclose(s.cpu().numpy(), f["sim_" + key], rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(retrieval.ranks(s).numpy(), f["ranks_" + key])
        r = retrieval.recall_at_k(s)
        assert [r[x] for x in ("r1", "r5", "r10", "r20")] == list(f["recall_" + key])
    kind = str(f["kind"])
    metrics = (retrieval.av_retrieval_metrics if kind == "retrieval_av" else retrieval.tv_retrieval_metrics)(q, k, temp)
    pre = ("A->V", "V->A") if kind == "retrieval_av" else ("T->V", "V->T")
    assert [metrics[f"{pre[0]}_r{x}"] for x in (1, 5, 10, 20)] == list(f["recall_qk"])
    assert [metrics[f"{pre[1]}_r{x}"] for x in (1, 5, 10, 20)] == list(f["recall_kq"])
