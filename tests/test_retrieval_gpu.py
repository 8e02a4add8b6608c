"""1000-way retrieval scorer (HIP, one launch per direction) vs the oracle's restatement of
retrieval.py's per-pair aggregators, on ragged token lists."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu

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
