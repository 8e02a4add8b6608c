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


@pytest.mark.parametrize("normalize,qlo,qhi,klo,khi", [(True, 30, 70, 40, 130), (False, 1, 12, 20, 65)])
def test_fp32_scorer_matches_fp64_restatement(normalize, qlo, qhi, klo, khi):
    """triad_retrieval_maxmean_f32 (the reference-precision mode, retrieval.py:106-114 in fp32) on
    fp32 token lists that are NOT bf16-representable, ragged across the kernel's 64-token tiles:
    both directions within fp32 evaluation order of the fp64 oracle (1e-6 of the matrix scale),
    ranks and R@k exact, one launch per direction; and triad_l2norm_rows_f32 against F.normalize."""
    from triad_amd import _lib, ops, retrieval
    N, temp = 24, 0.07
    g = torch.Generator().manual_seed(5)
    q = [torch.randn(int(torch.randint(qlo, qhi + 1, (1,), generator=g)), 512, generator=g) for _ in range(N)]
    k = [torch.randn(int(torch.randint(klo, khi + 1, (1,), generator=g)), 512, generator=g) for _ in range(N)]
    for i in range(N):
        m = min(len(q[i]), len(k[i]))
        k[i][:m] += 0.3 * q[i][:m]
    if normalize:
        for lst in (q, k):
            for i, x in enumerate(lst):
                got = ops.l2_normalize_f32(x.cuda()).cpu()
                want = torch.nn.functional.normalize(x, dim=-1)
                assert got.dtype == torch.float32 and float((got - want).abs().max()) <= 1e-6
                lst[i] = got
    q2k, k2q = ref_cpu.retrieval_matrices(q, k, temp)
    _lib.TIMERS = {"triad_retrieval_maxmean_f32": []}
    try:
        s1 = retrieval.aggregated_similarity(q, k, temp, precision="fp32").cpu().double().numpy()
        s2 = retrieval.aggregated_similarity(k, q, temp, precision="fp32").cpu().double().numpy()
    finally:
        launches, _lib.TIMERS = len(_lib.TIMERS["triad_retrieval_maxmean_f32"]), None
    assert launches == 2
    for got, ref in ((s1, q2k), (s2, k2q)):
        assert np.abs(got - ref).max() <= 1e-6 * np.abs(ref).max(), np.abs(got - ref).max()
        np.testing.assert_array_equal(retrieval.ranks(torch.from_numpy(got)).numpy(), ref_cpu.recall_ranks(ref))
        assert retrieval.recall_at_k(torch.from_numpy(got)) == ref_cpu.recall_at_k(ref)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
@pytest.mark.parametrize("name", G.names("retrieval_av") + G.names("retrieval_tv"))
def test_retrieval_matches_reference_fixtures(name, precision):
    """Both directions' matrices within fp32 rounding of the reference's (it divides by the
    temperature, the kernel multiplies by its inverse); ranks and R@k EXACT -- the duplicated
    items and all-zero queries of the *_ties fixtures produce exact ties in the HIP matrices too,
    ordered as the reference's np.argsort orders them."""
    from triad_amd import retrieval
    f = G.load(name)
    q = list(torch.split(G.bf16(f["q"]), [int(n) for n in f["q_len"]]))
    k = list(torch.split(G.bf16(f["k"]), [int(n) for n in f["k_len"]]))
    temp = float(f["temp"])
    s_qk = retrieval.aggregated_similarity(q, k, temp, precision=precision)
    s_kq = retrieval.aggregated_similarity(k, q, temp, precision=precision)
    for s, key in ((s_qk, "qk"), (s_kq, "kq")):
        np.testing.assert_allclose(s.cpu().numpy(), f["sim_" + key], rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(retrieval.ranks(s).numpy(), f["ranks_" + key])
        r = retrieval.recall_at_k(s)
        assert [r[x] for x in ("r1", "r5", "r10", "r20")] == list(f["recall_" + key])
    kind = str(f["kind"])
    metrics = (retrieval.av_retrieval_metrics if kind == "retrieval_av" else retrieval.tv_retrieval_metrics)(
        q, k, temp, precision=precision)
    pre = ("A->V", "V->A") if kind == "retrieval_av" else ("T->V", "V->T")
    assert [metrics[f"{pre[0]}_r{x}"] for x in (1, 5, 10, 20)] == list(f["recall_qk"])
    assert [metrics[f"{pre[1]}_r{x}"] for x in (1, 5, 10, 20)] == list(f["recall_kq"])


@pytest.mark.parametrize("name", G.names("retrieval_av") + G.names("retrieval_tv"))
def test_per_pair_aggregators_match_reference_fixtures(name):
    """The reference's per-pair functions by name (aggregator_av_a2v / _v2a, aggregator_tv_t2v /
    _v2t, retrieval.py:106-115, 190-198): Python floats equal to the fixture matrices' entries
    within fp32 evaluation order, for a sample of pairs including the diagonal; and
    compute_recall_at_k (retrieval.py:117-144) on the fixture's matrices returns its R@k."""
    from triad_amd import retrieval
    f = G.load(name)
    q = [x.cuda() for x in torch.split(G.bf16(f["q"]), [int(n) for n in f["q_len"]])]
    k = [x.cuda() for x in torch.split(G.bf16(f["k"]), [int(n) for n in f["k_len"]])]
    temp = float(f["temp"])
    av = str(f["kind"]) == "retrieval_av"
    fwd = retrieval.aggregator_av_a2v if av else retrieval.aggregator_tv_t2v
    bwd = retrieval.aggregator_av_v2a if av else retrieval.aggregator_tv_v2t
    n = len(q)
    scale = max(np.abs(f["sim_qk"]).max(), np.abs(f["sim_kq"]).max())
    for i, j in [(0, 0), (1, 2), (n - 1, 0), (n // 2, n // 2), (3, n - 1)]:
        a = fwd(q[i], k[j], temp)
        b = bwd(q[j], k[i], temp)            # (a_feats, v_feats): V->A of video i against audio j
        assert isinstance(a, float) and isinstance(b, float)
        assert abs(a - f["sim_qk"][i, j]) <= 1e-5 * scale, (i, j, a, f["sim_qk"][i, j])
        assert abs(b - f["sim_kq"][i, j]) <= 1e-5 * scale, (i, j, b, f["sim_kq"][i, j])
    for key in ("qk", "kq"):
        r = retrieval.compute_recall_at_k(f["sim_" + key])
        assert [r[x] for x in ("r1", "r5", "r10", "r20")] == list(f["recall_" + key])


def _near_tie_rows(ref, got):
    """Rows whose reference rank could move under the observed matrix error (the near-tie rule of
    DESIGN §2): some competitor j sits within twice the row's max |got - ref| of the diagonal."""
    err = np.abs(got - ref).max(1)
    n = ref.shape[0]
    return [i for i in range(n) if np.abs(np.delete(ref[i], i) - ref[i, i]).min() <= 2 * err[i]]


@pytest.mark.parametrize("use_amp", [True, False])
@pytest.mark.parametrize("kind", ["av", "tv"])
def test_model_level_retrieval_matches_reference(kind, use_amp, tmp_path):
    """The model-level drop-in (select_subset_indices, embed_av_subset / embed_tv_subset,
    compute_{av,tv}_retrieval_metrics -- retrieval.py:9-104, 146-188, 200-292) against the
    reference's own functions run on the same stand-in model and datasets
    (tests/golden/retrieval_e2e_n24.npz, made by gen_retrieval_e2e.py): subset indices exact
    (same python `random` draw, file written and re-read); embedded per-item features with the
    reference's padding / L2-normalisation (AV) and mask trimming (TV) -- lengths exact, values at
    the bf16 bar; both N x N matrices within 1e-2 of the row scale; ranks exact on every row
    without a near-tie (at most a quarter of the rows may be near-ties: the stand-in features are
    built so that retrieval is hard, i.e. close competitors are common); the result dicts' keys
    exact and R@k equal up to the near-tie rows. With model.use_amp = False (the reference's fp32
    arithmetic: fp32 normalisation and the fp32 scorer) the matrices agree to 1e-5 of the row
    scale, no row is a near-tie and ranks and R@k are exact."""
    import random
    from tests.retrieval_stub import AVStubDataset, StubModel, TVStubDataset
    from triad_amd import retrieval as R
    f = G.load("retrieval_e2e_n24")
    n, n_sub = int(f["n_data"]), int(f["n_sub"])
    seed = int(f["seed"]) + (0 if kind == "av" else 1)
    model = StubModel().cuda()
    model.use_amp = use_amp
    ds = AVStubDataset(n) if kind == "av" else TVStubDataset(n)
    random.seed(seed)
    sub = R.select_subset_indices(ds, str(tmp_path / "s1.json"), subset_size=n_sub)
    assert sub == [int(x) for x in f[kind + "_idx_sub"]]
    assert R.select_subset_indices(ds, str(tmp_path / "s1.json"), subset_size=n_sub) == sub   # re-read
    random.seed(seed)
    idx = R.select_subset_indices(ds, str(tmp_path / "s2.json"), subset_size=1000)
    assert idx == [int(x) for x in f[kind + "_idx"]]
    if kind == "av":
        q, k, paths = R.embed_av_subset(model, ds, idx, device="cuda", num_workers=0)
        assert paths == [str(x) for x in f["av_paths"]]
        keys, fq, fk, m_qk, m_kq, tol = ("a", "v"), f["av_a"], f["av_v"], f["av_a2v"], f["av_v2a"], 8e-3
    else:
        q, k = R.embed_tv_subset(model, ds, idx, device="cuda", num_workers=0)
        keys, fq, fk, m_qk, m_kq, tol = ("t", "i"), f["tv_t"], f["tv_i"], f["tv_t2v"], f["tv_v2t"], 4e-3
    assert model.training is False   # as the reference, the embed leaves the model in eval mode
    for lst, ref, key in ((q, fq, keys[0]), (k, fk, keys[1])):
        assert [int(t.shape[0]) for t in lst] == [int(x) for x in f[f"{kind}_{key}_len"]]
        got = torch.cat([t.float().cpu() for t in lst]).numpy()
        ref = ref.astype(np.float32)
        assert np.abs(got - ref).max() <= tol * max(1.0, np.abs(ref).max()), (key, np.abs(got - ref).max())
    temp = float(f["temp"])
    prec = "bf16" if use_amp else "fp32"
    if not use_amp:
        assert all(t.dtype == torch.float32 for t in q + k)
    s_qk = R.aggregated_similarity(q, k, temp, precision=prec).cpu().double().numpy()
    s_kq = R.aggregated_similarity(k, q, temp, precision=prec).cpu().double().numpy()
    ties = set()
    for got, ref in ((s_qk, m_qk), (s_kq, m_kq)):
        ref = ref.astype(np.float64)
        assert np.abs(got - ref).max() <= (1e-2 if use_amp else 1e-5) * np.abs(ref).max(), np.abs(got - ref).max()
        tied = _near_tie_rows(ref, got)
        # bf16 features (the scorer's MFMA operands) against the reference's fp32 ones: a row whose
        # diagonal has a competitor within twice the row's observed error may rank either way;
        # in the fp32 mode none may
        assert len(tied) <= (len(idx) // 4 if use_amp else 0), tied
        ties.add(len(tied))
        r_ref = ref_cpu.recall_ranks(ref)
        r_got = R.ranks(torch.from_numpy(got)).numpy()
        ok = [i for i in range(len(idx)) if i not in tied]
        np.testing.assert_array_equal(r_got[ok], np.asarray(r_ref)[ok])
    random.seed(seed)
    fn = R.compute_av_retrieval_metrics if kind == "av" else R.compute_tv_retrieval_metrics
    res = fn(model, ds, str(tmp_path / "s3.json"), device="cuda", num_workers=0)
    ref_res = dict(zip([str(x) for x in f[kind + "_keys"]], [float(x) for x in f[kind + "_vals"]]))
    assert list(res) == list(ref_res)
    slack = max(ties) / len(idx) + 1e-12
    for key in ref_res:
        assert abs(res[key] - ref_res[key]) <= slack, (key, res[key], ref_res[key])
    print(f"{kind}: near-tie rows {sorted(ties)}; recall {res}")
