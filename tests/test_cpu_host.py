"""CPU-only tests: the C-ABI library loads and exports every declared symbol, host-side
logic (dropout plan, parameter grouping, loss mix, tokenizer), and the CPU port of the
full step (configs[0]-style plumbing run)."""
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "triad_hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|long long)\s+(triad_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from triad_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.SIGNATURES, f"{n} missing from the ctypes signature table"
    assert set(_lib.SIGNATURES) == set(names)


def test_ops_refuse_cpu_tensors():
    from triad_amd import ops
    from triad_amd._lib import TriadError
    with pytest.raises(TriadError):
        ops.contrastive_head(ops.AV, torch.zeros(2, 3, 512), torch.zeros(2, 4, 512), torch.tensor(1.5))


def test_dropout_plan_matches_oracle_compaction():
    from oracle import ref_cpu
    from triad_amd.ops import dropout_indices
    g = torch.Generator().manual_seed(3)
    keep = torch.rand(5, 37, generator=g) < 0.7
    keep[2] = False
    keep[2, 5] = True
    idx, inv, n_out = dropout_indices(keep)
    x = torch.randn(5, 37, 8)
    out = ref_cpu.patch_dropout(x, keep)
    assert n_out == out.shape[1]
    gathered = torch.zeros_like(out)
    for b in range(5):
        for t in range(n_out):
            if idx[b, t] >= 0:
                gathered[b, t] = x[b, idx[b, t]]
    assert torch.equal(gathered, out)
    for b in range(5):
        for n in range(37):
            assert (inv[b, n] >= 0) == bool(keep[b, n])
            if keep[b, n]:
                assert idx[b, inv[b, n]] == n


def test_param_groups_and_loss_mix():
    from oracle import ref_cpu
    from triad_amd.train import TriadTrainer, split_param_groups

    class Fake(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.audio_embedder = torch.nn.Module()
            self.audio_embedder.hubert = torch.nn.Linear(2, 2)
            self.audio_embedder.projection1 = torch.nn.Linear(2, 2)
            self.text_embedder = torch.nn.Module()
            self.text_embedder.encoder = torch.nn.Linear(2, 2)
            self.visual_embedder = torch.nn.Module()
            self.visual_embedder.model = torch.nn.Module()
            self.visual_embedder.model.blk = torch.nn.Linear(2, 2)
            self.visual_embedder.model.lora_A = torch.nn.Parameter(torch.zeros(2))
            self.temperature = torch.nn.Parameter(torch.tensor(1.5))

    g = split_param_groups(Fake())
    assert [len(g[k]) for k in ("audio", "text", "vit_lora", "vit", "others")] == [2, 2, 1, 2, 3]
    tr = TriadTrainer.__new__(TriadTrainer)
    tr.av_weight_start, tr.av_weight_end = 0.8, 0.5
    for phase, prog in (("av_focus", 0), ("tv_warmup", 0), ("weighted_joint", 0.5), ("full_joint", 0)):
        assert abs(tr._loss_mix(phase, 2.0, 3.0, prog) - ref_cpu.loss_mix(phase, 2.0, 3.0, prog)) < 1e-12
    assert abs(tr._loss_mix("weighted_joint", 2.0, 3.0, 0.5) - (0.65 * 2 + 0.35 * 3)) < 1e-12


def test_hash_tokenizer_shapes():
    from triad_amd.model import HashTokenizer
    t = HashTokenizer()(["A man, riding.", "cat"], max_length=3)
    assert t["input_ids"].shape == (2, 3)
    assert t["attention_mask"].tolist() == [[1, 1, 1], [1, 0, 0]]
    assert int(t["input_ids"].min()) == 0 and int(t["input_ids"][:, 0].min()) >= 1000


@pytest.mark.slow
def test_cpu_port_step_runs():
    """configs[0]-style CPU plumbing: the CPU port of the full step at B=2."""
    from oracle import cpu_step
    sec = cpu_step.time_steps(B=2, steps=1, warmup=0, threads=8)
    assert sec > 0


def test_reference_compile_line_leaves_the_step_methods_eager():
    """The reference wraps the model in torch.compile(mode="max-autotune") (train.py:378) but its
    step calls model.forward_audio_visual / forward_text_visual (train.py:954, 969), which the
    compiled wrapper delegates to the original module: the HIP head (ctypes entry points inside
    autograd Functions) runs exactly as without the compile line -- no graph breaks, no tracing.
    (Why the head is not a torch.library op: DESIGN.md §1b.)"""
    import torch.nn as nn
    from triad_amd.model import MultiModalModel
    m = MultiModalModel.__new__(MultiModalModel)
    nn.Module.__init__(m)
    cm = torch.compile(m, mode="max-autotune")
    assert cm._orig_mod is m
    for name in ("forward_audio_visual", "forward_text_visual", "forward_triad", "compute_contrastive_loss_av"):
        bound = getattr(cm, name)
        assert bound.__self__ is m and bound.__func__ is getattr(MultiModalModel, name)


def test_pairsim_fwd_multi_rejects_bad_arguments():
    """triad_pairsim_fwd_multi validates every problem before it launches anything (no GPU needed):
    problem count outside 1..2, a missing array, a bad geometry, or one head writing dS while the
    other does not -> TRIAD_EINVAL (1001)."""
    import ctypes as C
    from triad_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    lib = _lib.load()
    fake = 4096  # never dereferenced: validation fails first

    def prob(R_pad=256, dS=None, st_part=None):
        return _lib.PairsimProblem(fake, fake, 200, R_pad, 50, 4, 4, 64, 60, fake, -60.0, 1, 0, fake, fake, fake,
                                   fake, dS, 8, st_part)
    f = lib.triad_pairsim_fwd_multi
    two = (_lib.PairsimProblem * 2)(prob(), prob())
    assert f(None, 1, None) == 1001
    assert f(two, 0, None) == 1001
    assert f(two, 3, None) == 1001
    assert f((_lib.PairsimProblem * 1)(prob(R_pad=250)), 1, None) == 1001        # R_pad % 256
    assert f((_lib.PairsimProblem * 1)(prob(dS=fake)), 1, None) == 1001          # dS without st_part
    mixed = (_lib.PairsimProblem * 2)(prob(dS=fake, st_part=fake), prob())
    assert f(mixed, 2, None) == 1001                                            # train + eval in one launch
    nul = prob()
    nul.rowmax = None
    assert f((_lib.PairsimProblem * 1)(nul), 1, None) == 1001
    assert C.sizeof(_lib.PairsimProblem) == 136   # include/triad_hip.h layout, k_tiles last
    assert _lib.PairsimProblem.k_tiles.offset == 128


def test_packed_tile_gemm_and_patch_reject_bad_arguments():
    """The direct-B GEMM entry points, the dS patch and the loss head validate their shapes before
    launching anything (no GPU needed) -> TRIAD_EINVAL (1001)."""
    from triad_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    lib = _lib.load()
    fake = 4096  # never dereferenced: validation fails first
    assert lib.triad_bfrag_pack16(fake, 0, 0, fake, None) == 1001                   # no k tiles
    assert lib.triad_bfrag_pack16(None, 4, 0, fake, None) == 1001                   # no B
    assert lib.triad_tile_gemm_packed16(fake, 8, 0, fake, 200, 8, fake, 1, None, fake, None) == 1001  # M % 128
    assert lib.triad_tile_gemm_packed16(fake, 8, 0, fake, 256, 8, fake, 2, None, fake, None) == 1001  # no slabs
    assert lib.triad_tile_gemm_packed16_slabs(fake, 8, 1, fake, 256, 0, 1, fake, None) == 1001      # nkt = 0
    # dS patch: CT too small for Bk samples of Nk_pad keys; Bk * R past 2^31 (32-bit index math)
    assert lib.triad_dS_patch(fake, 4, 256, 256, 32, 8, 8, 64, 60, 0, fake, fake, fake, fake, 1.0, None, 0.0,
                              fake, 1024, fake, None) == 1001
    assert lib.triad_dS_patch(fake, 1 << 40, 1 << 20, 1 << 20, 32, 8, 4096, 64, 60, 0, fake, fake, fake, fake, 1.0,
                              None, 0.0, fake, 1024, fake, None) == 1001
    # ... and the temperature the tiles are scaled by is required
    assert lib.triad_dS_patch(fake, 1 << 20, 256, 256, 32, 8, 8, 64, 60, 0, fake, fake, fake, fake, 1.0, None, 0.0,
                              fake, 1024, None, None) == 1001
    # loss head: B * B must fit an int
    assert lib.triad_losshead(fake, 50000, 0, fake, fake, 1, 1.0, fake, 1, 1.0, 0.0, fake, fake, fake, None) == 1001


def test_round4_entry_points_reject_bad_arguments():
    """The 16 x 16 x 32 tile GEMM forms and the split-K XCD placement flag validate before any
    launch (no GPU needed) -> TRIAD_EINVAL (1001)."""
    from triad_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    lib = _lib.load()
    fake = 4096
    assert lib.triad_bfrag_pack16(fake, 0, 1, fake, None) == 1001                   # no k tiles
    assert lib.triad_tile_gemm_packed16(fake, 8, 0, fake, 200, 8, fake, 1, None, fake, None) == 1001  # M % 128
    assert lib.triad_tile_gemm_packed16(fake, 8, 1, fake, 256, 8, fake, 2, None, fake, None) == 1001  # no slabs
    assert lib.triad_tile_gemm_packed16_slabs(fake, 8, 0, fake, 256, 8, 1, None, None) == 1001       # no slabs
    # split-K with the XCD placement flag (form | 8) needs splits % 8 == 0; forms beyond 4 refused
    assert lib.triad_gemm_bf16_splitk_form(fake, 512, 0, fake, 768, 0, 512, 768, 65536, 12, None, fake, fake, 0,
                                           1 | 8, None) == 1001
    assert lib.triad_gemm_bf16_splitk_form(fake, 512, 0, fake, 768, 0, 512, 768, 65536, 16, None, fake, fake, 0,
                                           5, None) == 1001
    # LDS-DMA column sums: cols % 8, a 16-byte aligned X, ld >= cols and scratch required
    assert lib.triad_colsum_dma(fake, 1024, 644, 648, fake, 1.0, 0, fake, None) == 1001   # cols % 8
    assert lib.triad_colsum_dma(fake + 2, 1024, 640, 640, fake, 1.0, 0, fake, None) == 1001   # misaligned
    assert lib.triad_colsum_dma(fake, 1024, 640, 632, fake, 1.0, 0, fake, None) == 1001   # ld < cols
    assert lib.triad_colsum_dma(fake, 1024, 768, 768, None, 1.0, 0, fake, None) == 1001
    assert lib.triad_colsum_dma_splits(50944, 768) == 171 and lib.triad_colsum_dma_splits(256, 768) == 4
    assert lib.triad_colsum_dma_splits(50944, 640) == 171 and lib.triad_colsum_dma_splits(50944, 12) == 0
    # fp32 retrieval scorer: padded token counts multiples of 64, D % 32, 16-byte aligned lists
    ok = (fake, fake, 24, 64, fake, fake, 24, 128, 512, 0.07, fake, None)
    assert lib.triad_retrieval_maxmean_f32(*ok[:3], 100, *ok[4:]) == 1001                   # nq_pad % 64
    assert lib.triad_retrieval_maxmean_f32(*ok[:7], 96, *ok[8:]) == 1001                    # nk_pad % 64
    assert lib.triad_retrieval_maxmean_f32(*ok[:8], 500, *ok[9:]) == 1001                   # D % 32
    assert lib.triad_retrieval_maxmean_f32(fake + 4, *ok[1:]) == 1001                       # misaligned
    assert lib.triad_retrieval_maxmean_f32(*ok[:10], None, None) == 1001                    # no output
    assert lib.triad_l2norm_rows_f32(fake, 10, 510, 1e-12, fake, None) == 1001              # D % 4
    assert lib.triad_l2norm_rows_f32(fake + 8, 10, 512, 1e-12, fake, None) == 1001          # misaligned


def test_side_stream_tables_key_by_device_ordinal():
    """linear._dev_index: "cuda:N" -> N without touching a GPU (index None -> the current device,
    GPU-tested in test_ops_gpu.py::test_side_stream_is_one_stream_per_device)."""
    from triad_amd.linear import _dev_index
    assert _dev_index("cuda:3") == 3 and _dev_index(torch.device("cuda", 1)) == 1


def test_weight_gradient_plans():
    """Split-K plans of the projection-head (ops._dw_plan) and backbone (linear._form_splits)
    weight gradients: long token lists on the XCD-per-split placement with a split count that is a
    multiple of 8; the 8,192-row text head and the 3072-wide backbone shapes keep the default."""
    from triad_amd import linear, ops
    for Mp in (65536, 50944, 43904):
        f2, s2 = ops._dw_plan(Mp, 512)
        f1, s1 = ops._dw_plan(Mp, 768)
        assert (f2, s2) == (1 | 8, 32) and (f1, s1) == (4 | 8, 40)   # 40 x 6 tiles: 240 workgroups
    assert ops._dw_plan(43808, 1024) == (4 | 8, 32)
    assert ops._dw_plan(8192, 512) == (0, 16) and ops._dw_plan(8192, 768)[0] == 0
    for O, K, xcd in ((768, 768, True), (2304, 768, True), (3072, 768, False), (768, 3072, False)):
        form, sp = linear._form_splits(50944, O, K)
        assert form & 7 == 4 and bool(form & 8) == xcd
        assert not xcd or sp % 8 == 0
    assert linear._form_splits(8192, 768, 768)[0] == 0
    # HuBERT conv stack (frontend._conv_dw_plan): eight-wave tiles, one round of <= 256 workgroups
    from triad_amd.frontend import _conv_dw_plan
    for M, N in ((1638400, 1536), (204800, 1536), (102400, 1024), (51200, 1024), (4096, 1536)):
        form, sp = _conv_dw_plan(M, 512, N)
        assert form & 7 == 4 and 1 <= sp and sp * (512 // 256) * (N // 256) <= 256 and M // sp >= 2048
        assert not form & 8 or sp % 8 == 0
    assert _conv_dw_plan(1638400, 512, 1536) == (4, 21) and _conv_dw_plan(102400, 512, 1024) == (12, 32)
    assert _conv_dw_plan(65536, 512, 384) == (0, 8)


def test_select_subset_indices_draws_writes_and_rereads(tmp_path):
    """retrieval.select_subset_indices (retrieval.py:9-30): python `random.shuffle` of
    range(len(dataset)), the first `subset_size`, written as JSON; an existing file is read back
    as is. Pinned to the reference's own draw by tests/golden/retrieval_e2e_n24.npz."""
    import json
    import random
    from tests import golden_io as G
    from triad_amd.retrieval import select_subset_indices
    f = G.load("retrieval_e2e_n24")
    ds = list(range(int(f["n_data"])))
    random.seed(int(f["seed"]))
    p = tmp_path / "sub.json"
    got = select_subset_indices(ds, str(p), subset_size=int(f["n_sub"]))
    assert got == [int(x) for x in f["av_idx_sub"]]
    assert json.loads(p.read_text()) == got
    random.seed(12345)   # a different state: the file wins
    assert select_subset_indices(ds, str(p), subset_size=3) == got


@pytest.mark.parametrize("rows,cols,view", [(50944, 768, None), (8192, 3072, None), (37, 520, None),
                                            (200, 776, None), (63, 13, None), (5, 1000, None),
                                            (100, 768, "wide"), (100, 768, "shifted"), (0, 64, None)])
def test_bias_grad_takes_only_the_lds_dma_form(rows, cols, view, monkeypatch):
    """every column sum of the step goes to triad_colsum_dma -- no shape falls back
    to triad_colsum or a PyTorch reduction (the measured victims of DESIGN.md §2b). Host routing
    only (the C-ABI calls are recorded, nothing runs): the DMA entry point gets an aligned,
    row-stride % 8 == 0, cols % 8 == 0 operand; other shapes are first copied into one."""
    from triad_amd import ops
    seen = []

    def fake_call(name, *args, **kw):
        seen.append((name, args))
        return 2 if name.endswith("_splits") else 0

    monkeypatch.setattr(ops, "call", fake_call)
    monkeypatch.setattr(ops, "stream_ptr", lambda *a: None)
    base = torch.zeros(rows, cols + 16, dtype=torch.bfloat16)
    x = {"wide": base[:, :cols], "shifted": base[:, 1:cols + 1]}.get(view, base[:, :cols].contiguous())
    out = ops.bias_grad(x, torch.float32)
    assert out.shape == (cols,)
    names = {n for n, _ in seen}
    assert names <= {"triad_colsum_dma_splits", "triad_colsum_dma"}, names
    if rows:
        (_, (xp, r, c, ld, *_)), = [s for s in seen if s[0] == "triad_colsum_dma"]
        assert r == rows and c % 8 == 0 and ld % 8 == 0 and (xp.value or 0) % 16 == 0


def test_triad_linear_takes_every_token_count():
    """No backbone Linear falls back to nn.Linear (whose bias gradient is PyTorch's reduction) for
    a token count: only widths the split-K GEMM does not tile do (no backbone Linear with a bias)."""
    from triad_amd import linear

    class _X:   # what _eligible reads of the input
        is_cuda = True

        def __init__(self, n, k):
            self.shape = (n, k)

        def numel(self):
            return self.shape[0] * self.shape[1]

    lin = torch.nn.Linear(768, 768)
    orig = torch.is_autocast_enabled, torch.get_autocast_dtype
    try:
        torch.is_autocast_enabled = lambda *a: True
        torch.get_autocast_dtype = lambda *a: torch.bfloat16
        for n in (1, 63, 100, 4095, 8192, 50944):
            assert linear._eligible(lin, _X(n, 768)), n
        assert not linear._eligible(torch.nn.Linear(768, 8), _X(100, 768))
    finally:
        torch.is_autocast_enabled, torch.get_autocast_dtype = orig


def test_vit_embedder_mirrors_the_reference_surface():
    """`from model import ViTEmbedder` (model.py:120-205): the constructor's arguments, the
    attributes the reference reads (model, projection1, layer_norm, projection2,
    patch_dropout_rate), every parameter trainable, no LoRA, no register tokens by default;
    patch_dropout leaves the input alone in eval mode / at rate 0 (no GPU needed)."""
    import inspect
    import warnings
    from triad_amd.model import ViTEmbedder
    sig = inspect.signature(ViTEmbedder.__init__)
    assert list(sig.parameters)[1:] == ["model_name", "arch", "embedding_dim", "dropout_prob"]
    assert sig.parameters["arch"].default == "dinov2_vitb14" and sig.parameters["dropout_prob"].default == 0.1
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        emb = ViTEmbedder(arch="dinov2_vits14", embedding_dim=512)
    names = [n for n, _ in emb.named_parameters()]
    assert not any("lora" in n for n in names)
    assert {n.split(".")[0] for n in names} == {"model", "projection1", "layer_norm", "projection2"}
    assert all(p.requires_grad for p in emb.parameters())
    assert emb.model.num_register_tokens == 0 and emb.projection1.in_features == 384
    assert emb.patch_dropout_rate == 0.1
    x = torch.zeros(2, 5, 512)
    assert emb.eval().patch_dropout(x, 0.1) is x and emb.train().patch_dropout(x, 0) is x


def test_param_sumsq_is_a_segmented_sum_per_parameter(monkeypatch):
    """optim.FlatParamSpace.param_sumsq: the per-chunk partials of triad_grad_sumsq (emulated here
    from the chunk table) are summed per parameter by torch.segment_reduce over the table's
    parameter order -- equal to the per-parameter sums of squares for any id order / repeats, with
    zero for the parameters not asked for (no index_add_ atomics, so the clip coefficient does not
    depend on the order the atomics land in)."""
    from triad_amd import optim as fo
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(n)) for n in (5, fo.CHUNK * 2 + 7, 1, fo.CHUNK, 300)]
    sp = fo.FlatParamSpace(ps, "cpu")
    sp.flat_g.copy_(torch.randn(sp.numel))

    def fake_call(name, *args, **kw):
        assert name == "triad_grad_sumsq"
        g = sp.flat_g.double()
        table = np.frombuffer(args[1].numpy().tobytes(), dtype=fo._CHUNK_DT)
        out = args[3]
        for k, r in enumerate(table[:args[2]]):
            out[k] = float((g[int(r["off"]):int(r["off"]) + int(r["n"])] ** 2).sum())
    monkeypatch.setattr(fo, "call", fake_call)
    monkeypatch.setattr(fo, "ptr", lambda t: t)
    monkeypatch.setattr(fo, "stream_ptr", lambda d: None)
    for ids in ([0, 1, 2, 3, 4], [3, 1, 1], [4], [2, 0]):
        got = sp.param_sumsq(ids)
        want = torch.zeros(len(ps), dtype=torch.float64)
        for i in set(ids):
            o = sp.offsets[i]
            want[i] = (sp.flat_g[o:o + ps[i].numel()].double() ** 2).sum()
        torch.testing.assert_close(got, want, rtol=1e-12, atol=0)



def test_compact_key_tile_tables_match_a_loop_restatement():
    """ops.compact_tables (the compact key-tile layout the training pair forward / backward walk)
    against a per-sample loop: every sample keeps its tiles up to its last non-zero one; a sample
    whose kept count fits in nkb - 1 tiles leaves the last (all-zero) tile out."""
    from triad_amd import ops
    rng = np.random.default_rng(5)
    for Bk, nkb in ((1, 2), (7, 3), (64, 7), (300, 7)):
        Nk = 32 * nkb - int(rng.integers(0, 20))
        kept = rng.integers(0, Nk + 1, size=Bk).astype(np.int32)
        kept[0] = Nk                                # the batch's longest sample sets Nk
        if Bk > 1:
            kept[1] = 32 * (nkb - 1)                # boundary: exactly nkb - 1 full tiles
        tabs = ops.compact_tables(kept, nkb, Nk)
        cb_ref, tidx_ref, kmap_ref = [0], [], np.full((Bk, Nk), -1, dtype=np.int32)
        for j in range(Bk):
            nt = nkb - 1 if kept[j] <= 32 * (nkb - 1) else nkb
            for kb in range(nt):
                for k in range(32 * kb, min(32 * kb + 32, Nk)):
                    kmap_ref[j, k] = 32 * (cb_ref[-1] + kb) + (k - 32 * kb)
                tidx_ref.append(j * nkb + kb)
            cb_ref.append(cb_ref[-1] + nt)
        if cb_ref[-1] == Bk * nkb:
            assert tabs is None
            continue
        cb, tidx, kmap = tabs
        assert cb.dtype == np.int32 and kmap.dtype == np.int32
        np.testing.assert_array_equal(cb, cb_ref)
        np.testing.assert_array_equal(tidx, tidx_ref)
        np.testing.assert_array_equal(kmap, kmap_ref)
    assert ops.compact_tables(np.full(5, 70, np.int32), 3, 70) is None   # every sample needs all tiles


def test_compute_recall_at_k_matches_reference_fixtures():
    """retrieval.compute_recall_at_k (retrieval.py:117-144, by name) on the reference's own N x N
    matrices: its R@k exactly, ties included (host-only arithmetic)."""
    from tests import golden_io as G
    from triad_amd import retrieval
    for name in G.names("retrieval_av") + G.names("retrieval_tv"):
        f = G.load(name)
        for key in ("qk", "kq"):
            r = retrieval.compute_recall_at_k(f["sim_" + key])
            assert [r[x] for x in ("r1", "r5", "r10", "r20")] == list(f["recall_" + key]), (name, key)


def test_retrieval_fp32_width_checked():
    """The fp32 scorer's packing takes the features' own width: mixed widths and widths
    that are not a multiple of 32 raise TriadError before any device work."""
    import torch
    from triad_amd import _lib, retrieval
    with pytest.raises(_lib.TriadError):
        retrieval._feature_width([torch.zeros(3, 512)], [torch.zeros(4, 256)])
    with pytest.raises(_lib.TriadError):
        retrieval._feature_width([torch.zeros(3, 48)], [torch.zeros(4, 48)])
    assert retrieval._feature_width([torch.zeros(3, 256)], [torch.zeros(4, 256)]) == 256


def test_bench_tracks_every_hot_path_entry_point():
    """bench.py times every hot-path launch (VERDICT r5 #3a): its tracked set is derived from the C
    ABI table, and every entry point a head / trainer module calls is in it. Backbone-only entry
    points (never timed) are called only from the backbone modules."""
    import glob
    import bench
    from triad_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    backbone_mods = {"frontend.py", "postln.py", "vit.py", "attention.py", "linear.py"}
    called = {}
    for f in glob.glob(os.path.join(root, "triad_amd", "*.py")):
        mod = os.path.basename(f)
        if mod == "_lib.py":
            continue
        for name in re.findall(r'call\(\s*"(triad_[A-Za-z0-9_]+)"', open(f).read()):
            called.setdefault(name, set()).add(mod)
    assert called, "no entry-point calls found"
    for name, mods in called.items():
        assert name in _lib.SIGNATURES, f"{name} called from {mods} but not declared in _lib.SIGNATURES"
        if name in _lib.RESTYPES:
            continue
        if mods - backbone_mods:
            assert name in bench.TRACKED, f"hot-path entry point {name} (from {sorted(mods)}) is not timed"
        if name in _lib.BACKBONE_ENTRY_POINTS:
            assert mods <= backbone_mods, f"backbone-only {name} is called from {sorted(mods - backbone_mods)}"
    # the round-5 omission: the compact-tile dS patch is the backward's product form
    assert "triad_dS_patch_tiles" in bench.TRACKED and "triad_pairsim_fwd_multi" in bench.TRACKED
    assert not set(bench.TRACKED) & _lib.BACKBONE_ENTRY_POINTS
