"""Global negatives (Mode G) through the HIP kernels: 2 ranks on the box's single GPU,
collectives over gloo (RCCL refuses two ranks on one device). The sharded fused head
must equal the single-process fused head at B_g."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(kind, Bg=6, Nq=33, Nv=40, seed=9):
    g = torch.Generator().manual_seed(seed)
    q = (torch.randn(Bg, Nq, 512, generator=g) * 0.58).to(torch.bfloat16)
    k = (torch.randn(Bg, Nv, 512, generator=g) * 0.58).to(torch.bfloat16)
    k[2, 31:] = 0
    mask = (torch.arange(Nq)[None] < torch.randint(1, Nq + 1, (Bg, 1), generator=g)).long()
    return q, k, mask


def _worker(rank, world, port, kind, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from triad_amd import ops
        q, k, mask = _inputs(kind)
        Bl = q.shape[0] // world
        sl = slice(rank * Bl, (rank + 1) * Bl)
        qd = q[sl].cuda().requires_grad_(True)
        kd = k[sl].cuda().requires_grad_(True)
        t = torch.tensor(1.5, device="cuda", requires_grad=True)
        losses, stats, clip = ops.contrastive_head(kind, qd, kd, t, q_mask=mask[sl].cuda() if kind else None,
                                                   threshold=0.01, sparsity_weight=0.2, group=dist.group.WORLD)
        losses[0].backward()
        q_out.put((rank, torch.stack([x.detach() for x in losses]).cpu().numpy(), stats.cpu().numpy(), qd.grad.float().cpu().numpy(),
                   kd.grad.float().cpu().numpy(), float(t.grad)))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q_out.put((rank, "error", traceback.format_exc(), None, None, None))


@pytest.mark.parametrize("kind", [0, 1])
def test_global_negatives_two_ranks_match_single_process(kind):
    from triad_amd import ops
    world = 2
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, qo)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([qo.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[2]
    q, k, mask = _inputs(kind)
    qd, kd = q.cuda().requires_grad_(True), k.cuda().requires_grad_(True)
    t = torch.tensor(1.5, device="cuda", requires_grad=True)
    losses, stats, clip = ops.contrastive_head(kind, qd, kd, t, q_mask=mask.cuda() if kind else None,
                                               threshold=0.01, sparsity_weight=0.2)
    losses[0].backward()
    L = torch.stack([x.detach() for x in losses]).cpu().numpy()
    Bl = q.shape[0] // world
    dt = 0.0
    for rank, l, st, gq, gk, gt in res:
        np.testing.assert_allclose(l, L, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(st, stats.cpu().numpy(), rtol=1e-5, atol=1e-5)
        ref_q = qd.grad.float().cpu().numpy()[rank * Bl:(rank + 1) * Bl]
        ref_k = kd.grad.float().cpu().numpy()[rank * Bl:(rank + 1) * Bl]
        np.testing.assert_allclose(gq, ref_q, rtol=0, atol=2e-2 * np.abs(ref_q).max())
        np.testing.assert_allclose(gk, ref_k, rtol=0, atol=2e-2 * np.abs(ref_k).max())
        # same features -> same S and argmax bit for bit; what remains is the bf16 rounding of the
        # per-rank dK partials before their reduce-scatter (~2^-9)
        rq = float(np.linalg.norm(gq - ref_q) / np.linalg.norm(ref_q))
        rk = float(np.linalg.norm(gk - ref_k) / np.linalg.norm(ref_k))
        print(f"mode G head kind {kind} rank {rank}: dq rel {rq:.2e} dk rel {rk:.2e}")
        assert rq < 5e-3 and rk < 5e-3, (rq, rk)
        dt += gt
    assert abs(dt - float(t.grad)) <= 1e-3 * abs(float(t.grad)) + 1e-6


def _pair_worker(rank, world, port, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        q_out.put((rank,) + _pair_run(rank, world, dist.group.WORLD))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q_out.put((rank, "error", traceback.format_exc(), None, None))


def _pair_run(rank, world, group):
    """Both heads through ONE similarity-forward launch (ops.contrastive_heads_av_tv) on this rank's
    slice; world = 1: the whole batch in one process."""
    from triad_amd import ops
    qa, ka, _ = _inputs(0, seed=21)
    qt, kt, mask = _inputs(1, Nq=12, Nv=37, seed=22)
    Bl = qa.shape[0] // world
    sl = slice(rank * Bl, (rank + 1) * Bl)
    xs = [x[sl].cuda().requires_grad_(True) for x in (qa, ka, qt, kt)]
    t = torch.tensor(1.4, device="cuda", requires_grad=True)
    (la, sa, _), (lt, st, _) = ops.contrastive_heads_av_tv(xs[0], xs[1], xs[2], xs[3], t, mask[sl].cuda(),
                                                           threshold=0.01, sparsity_weight=0.2, group=group)
    (la[0] + lt[0]).backward()
    losses = torch.stack([x.detach() for x in list(la) + list(lt)]).cpu().numpy()
    return losses, [x.grad.float().cpu().numpy() for x in xs], float(t.grad)


def test_global_negatives_pair_launch_two_ranks_match_single_process():
    """Mode G with the tri-modal step's pair launch (keys of both heads all-gathered before the one
    launch, each head's clip rows gathered after it): 2 ranks vs the single process at B_g."""
    world = 2
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_pair_worker, args=(r, world, port, qo)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([qo.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[2]
    L, G, T = _pair_run(0, 1, None)
    Bl = G[0].shape[0] // world
    dt = 0.0
    for rank, l, grads, gt in res:
        np.testing.assert_allclose(l, L, rtol=1e-5, atol=1e-6)
        for got, ref in zip(grads, G):
            ref = ref[rank * Bl:(rank + 1) * Bl]
            np.testing.assert_allclose(got, ref, rtol=0, atol=2e-2 * np.abs(ref).max())
            r = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
            print(f"mode G pair rank {rank}: feature-gradient rel {r:.2e}")
            assert r < 5e-3, r
        dt += gt
    assert abs(dt - T) <= 1e-3 * abs(T) + 1e-6


# ---- c4 (Mode G at the per-rank batch of the 8-GPU config) against the fp64 oracle ---------
C4_BL, C4_NA, C4_NV, C4_NT = 256, 199, 212, 32


def _c4_inputs(world):
    """Head features of a B_g = world x 256 tri-modal batch at the c3 / c4 token counts (199 audio
    tokens, 212 visual tokens after patch dropout, 32 caption tokens with ragged masks)."""
    Bg = world * C4_BL
    g = torch.Generator().manual_seed(4242)
    qa = (torch.randn(Bg, C4_NA, 512, generator=g) * 0.58).to(torch.bfloat16)
    ka = (torch.randn(Bg, C4_NV, 512, generator=g) * 0.58).to(torch.bfloat16)
    qt = (torch.randn(Bg, C4_NT, 512, generator=g) * 0.58).to(torch.bfloat16)
    kt = (torch.randn(Bg, C4_NV, 512, generator=g) * 0.58).to(torch.bfloat16)
    lens = torch.randint(C4_NT // 4, C4_NT + 1, (Bg,), generator=g)
    mask = (torch.arange(C4_NT)[None] < lens[:, None]).long()
    return qa, ka, qt, kt, mask


def _c4_worker(rank, world, port, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from triad_amd import ops
        qa, ka, qt, kt, mask = _c4_inputs(world)
        sl = slice(rank * C4_BL, (rank + 1) * C4_BL)
        xs = [x[sl].cuda().requires_grad_(True) for x in (qa, ka, qt, kt)]
        t = torch.tensor(1.5, device="cuda", requires_grad=True)
        (la, sa, _), (lt, st, _) = ops.contrastive_heads_av_tv(xs[0], xs[1], xs[2], xs[3], t, mask[sl].cuda(),
                                                               threshold=0.8, sparsity_weight=0.01,
                                                               group=dist.group.WORLD)
        (la[0] + lt[0]).backward()
        # numpy (bf16 bits as int16), not tensors: a tensor in the queue is an fd of this process
        q_out.put((rank, [float(x.detach()) for x in la], [float(x.detach()) for x in lt], sa.cpu().numpy(),
                   st.cpu().numpy(), [x.grad.view(torch.int16).cpu().numpy() for x in xs], float(t.grad)))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q_out.put((rank, "error", traceback.format_exc(), None, None, None, None))


def test_c4_mode_g_per_rank_batch_vs_oracle():
    """BASELINE c4 (tri-modal B = 256 per GPU, RCCL key all-gather for global negatives) at the
    per-rank batch it runs: two ranks of 256 triples each (gloo on the box's one GPU; c4 has eight,
    i.e. 2,048 key samples per rank instead of 512 here), every rank through the tri-modal pair
    launch with the keys of both heads all-gathered, clip rows gathered, key gradients
    reduce-scattered -- against the chunked fp64 ORACLE of the reference loss at B_g = 512
    (model.py:370-472 / 490-593): both heads' losses at 1e-4, each rank's feature gradients at the
    bf16 bar with the near-tie rule, d/dtemp (sum over ranks) at 1e-3."""
    from oracle import ref_cpu
    world = 2
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, qo)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([qo.get(timeout=600) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[2]
    qa, ka, qt, kt, mask = _c4_inputs(world)
    temp = 1.5
    dt_ref = 0.0
    names = ("total", "ce", "reg", "aux")
    for kind, q, k, m, li, gq_i, gk_i in (("av", qa, ka, None, 1, 0, 1), ("tv", qt, kt, mask, 2, 2, 3)):
        qd, kd = q.cuda().float(), k.cuda().float()
        o = ref_cpu.head_loss_chunked(kind, qd, kd, temp, q_mask=None if m is None else m.cuda(), threshold=0.8,
                                      weight=0.01, chunk=4)
        tq, tk, n = ref_cpu.near_ties(qd, kd, temp)
        assert float(tq.float().mean()) < 0.03 and float(tk.float().mean()) < 0.03, (int(tq.sum()), int(tk.sum()))
        dt_ref += float(o["dtemp"])
        for rank, la, lt, sa, st, grads, gt in res:
            losses = la if kind == "av" else lt
            for got, key in zip(losses, names):
                assert abs(got - o[key]) <= 1e-5 + 1e-4 * abs(o[key]), (kind, rank, key, got, o[key])
            stats = sa if kind == "av" else st   # the statistics of the GLOBAL clip matrix on every rank
            for got, (key, want) in zip(np.asarray(stats, dtype=np.float64).ravel()[:6], o["stats"].items()):
                assert abs(got - want) <= 1e-4 + 1e-4 * abs(want), (kind, rank, key, got, want)
            sl = slice(rank * C4_BL, (rank + 1) * C4_BL)
            gq = torch.from_numpy(grads[gq_i]).view(torch.bfloat16).cuda()
            gk = torch.from_numpy(grads[gk_i]).view(torch.bfloat16).cuda()
            eq = ref_cpu.grad_rel(gq, o["dq"][sl], tq[sl])
            ek = ref_cpu.grad_rel(gk, o["dk"][sl], tk[sl])
            print(f"c4 per-rank {kind} rank {rank}: feature-gradient rel dq {eq:.3e} dk {ek:.3e} "
                  f"(near-tie rows left out: {int(tq[sl].sum())} query / {int(tk[sl].sum())} key, {n} ties in all)")
            assert eq < 1e-2 and ek < 1e-2, (kind, rank, eq, ek)
        del o
        torch.cuda.empty_cache()
    dt = sum(r[6] for r in res)
    assert abs(dt - dt_ref) <= 1e-3 * abs(dt_ref) + 1e-6, (dt, dt_ref)


# ---- Mode R: TriadTrainer itself at world size 2 ---------------------------------------
def _mode_r_model():
    """ViT-S/14-reg + HuBERT-base + DistilBERT (c1-sized backbones), every dropout / LayerDrop /
    SpecAugment mask off so two processes and one process draw nothing random
    (tools/grad_determinism.py: with them on, two identical single-process steps differ)."""
    from triad_amd.model import MultiModalModel
    torch.manual_seed(1234)
    m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.80, patch_sparsity_weight=0.01,
                        visual_dropout_prob=0.25, use_amp=True, vit_arch="dinov2_vits14_reg").cuda()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        if isinstance(getattr(mod, "dropout", None), float):
            mod.dropout = 0.0
        cfg = getattr(mod, "config", None)
        if cfg is not None and hasattr(cfg, "layerdrop"):
            cfg.layerdrop = 0.0
        if cfg is not None and hasattr(cfg, "apply_spec_augment"):
            cfg.apply_spec_augment = False   # HuBERT's training-mode time masks come from numpy's RNG
    m.train()
    return m


def _mode_r_batch(step, rank, B=2):
    g = torch.Generator().manual_seed(1000 * step + rank)
    frames = torch.randn(B, 3, 224, 224, generator=g).cuda()
    audio = (torch.randn(B, 32000, generator=g) * 0.1).cuda()
    words = "a dog runs across the wet grass while two children laugh near an old red barn".split()
    text = [" ".join(words[(3 * i + step + rank) % 5:][:10]) for i in range(B)]
    av_keep = torch.rand(B, 256, generator=g) < 0.75
    tv_keep = torch.rand(B, 256, generator=g) < 0.75
    return frames, audio, text, av_keep, tv_keep


def _trainer(model, accum, group=None, wire="fp32"):
    """TriadTrainer whose reduced gradient buffer is snapshotted at each optimizer step (after the
    all-reduce, before clipping) in `tr.reduced`."""
    from triad_amd.train import TriadTrainer
    tr = TriadTrainer(model, learning_rate=1e-4, total_updates=50, gradient_accumulation_steps=accum,
                      unfreeze_audio_step=0, unfreeze_text_step=0, process_group=group, bucket_mb=16.0,
                      grad_wire=wire)
    tr.reduced = []
    inner = tr._allreduce_grads

    def snap():
        inner()
        tr.reduced.append(tr.space.flat_g.clone())
    tr._allreduce_grads = snap
    return tr


def _group_rel(tr, a, b):
    out = {}
    sp = tr.space
    for name, ps in tr.groups.items():
        ids = sp.param_ids(ps)
        if not ids:
            continue
        x = np.concatenate([a[sp.offsets[i]:sp.offsets[i] + sp.params[i].numel()] for i in ids])
        y = np.concatenate([b[sp.offsets[i]:sp.offsets[i] + sp.params[i].numel()] for i in ids])
        out[name] = float(np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30))
    return out


def _worst_params(model, tr, a, b, among=None, k=6):
    """The k parameters (of `among`, default all) whose reduced gradients differ most (relative L2),
    with their gradient norms."""
    names = {id(p): n for n, p in model.named_parameters()}
    keep = None if among is None else {id(p) for p in among}
    sp, rows = tr.space, []
    for i, p in enumerate(sp.params):
        if keep is not None and id(p) not in keep:
            continue
        x = a[sp.offsets[i]:sp.offsets[i] + p.numel()]
        y = b[sp.offsets[i]:sp.offsets[i] + p.numel()]
        ny = float(np.linalg.norm(y))
        rows.append((float(np.linalg.norm(x - y)) / max(ny, 1e-30), ny, names[id(p)]))
    rows.sort(reverse=True)
    return [(f"{r:.2e}", f"{n:.2e}", nm) for r, n, nm in rows[:k]]


def _mode_r_worker(rank, world, port, wire, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        m = _mode_r_model()
        tr = _trainer(m, 1, dist.group.WORLD, wire)
        launched = []
        for step in range(2):
            f, a, t, ak, tk = _mode_r_batch(step, rank)
            tr.step(f, a, t, phase="full_joint", av_keep=ak, tv_keep=tk)
            launched.append(tr.reducer.launched_in_backward)
        torch.cuda.synchronize()
        q_out.put((rank, tr.reduced[0].cpu().numpy(), tr.space.flat_p.cpu().numpy(), launched,
                   len(tr.reducer.buckets)))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q_out.put((rank, "error", traceback.format_exc(), None, None))


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_mode_r_trainer_two_ranks_match_accumulated_single_process(wire):
    """TriadTrainer at world size 2 (Mode R, gradients all-reduced by the overlapped bucket
    reducer; gloo over device tensors -- RCCL refuses two ranks on one GPU). The reduced gradient
    of the first step equals ONE process accumulating the same two micro-batches
    (gradient_accumulation_steps=2, i.e. the average of the ranks' gradients), per parameter
    group; both ranks hold identical parameters after two optimizer steps; from the second step
    on, buckets leave during backward. (Updates are not compared with the single process: AdamW's
    first steps are ~lr * sign(g), so run-to-run noise in near-zero gradients -- which two
    single-process runs show too -- flips whole elements.)"""
    world = 2
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_mode_r_worker, args=(r, world, port, wire, qo)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([qo.get(timeout=600) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[2]
    (_, g0, p0, l0, nb), (_, g1, p1, l1, _) = res
    assert nb >= 4
    np.testing.assert_array_equal(g0, g1)          # one all-reduced gradient on both ranks
    np.testing.assert_array_equal(p0, p1)          # -> identical updates
    assert l0[0] == 0 and l0[1] >= 1 and l1[1] >= 1
    m = _mode_r_model()
    tr = _trainer(m, 2)
    for rank in range(world):
        f, a, t, ak, tk = _mode_r_batch(0, rank)
        tr.step(f, a, t, phase="full_joint", av_keep=ak, tv_keep=tk)
    rel = _group_rel(tr, g0, tr.reduced[0].cpu().numpy())
    print(f"mode R {wire}: reduced-gradient rel error per group {rel}")
    bar = 1e-2 if wire == "fp32" else 2e-2
    for name, r in rel.items():
        assert r < bar, (name, r)


# ---- Mode G through TriadTrainer: overlapped reducer on its own communicator, unfreeze flip ----
def _mode_g_trainer(model, group, unfreeze_audio=1):
    from triad_amd.train import TriadTrainer
    tr = TriadTrainer(model, learning_rate=1e-4, total_updates=50, gradient_accumulation_steps=1,
                      unfreeze_audio_step=unfreeze_audio, unfreeze_text_step=0, process_group=group, bucket_mb=16.0,
                      global_negatives=group is not None)
    tr.reduced = []
    inner = tr._allreduce_grads

    def snap():
        inner()
        tr.reduced.append(tr.space.flat_g.clone())
    tr._allreduce_grads = snap
    return tr


def _no_znorm(audio):
    """The HuBERT processor z-normalises over the WHOLE batch it is given (model.py:56-62), so a
    rank's B_l half and the single process's B_g batch see different statistics -- a property of
    sharding the reference's input pipeline, not of the head; this test compares the head and the
    reducer, so the audio goes in unnormalised on both sides."""
    return audio.float()


def _embed_in_chunks(m, n):
    """Run the embedders over n samples at a time (features concatenated): the backbones' vendor
    GEMMs pick their kernels by row count, so a B_g batch and two B_l halves differ at rounding
    level, which is enough to flip near-tied row maxima in the head (one flip moves ~1/sqrt(B^2 Nq)
    of the max-term gradient: ~2.5 % at B_g = 4). Chunked like the ranks, the single process
    feeds the head bit-identical features and the comparison isolates Mode G and the reducer."""
    import types
    ve, ae, te = m.visual_embedder, m.audio_embedder, m.text_embedder
    enc, afwd, tfwd = ve.encode_patches, ae.forward, te.forward

    def enc_c(self, x):
        return torch.cat([enc(x[i:i + n]) for i in range(0, x.shape[0], n)])

    def a_c(self, audio):
        return torch.cat([afwd(audio[i:i + n]) for i in range(0, audio.shape[0], n)])

    def t_c(self, texts):
        outs = [tfwd(texts[i:i + n]) for i in range(0, len(texts), n)]
        return torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs])
    ve.encode_patches = types.MethodType(enc_c, ve)
    ae.forward = types.MethodType(a_c, ae)
    te.forward = types.MethodType(t_c, te)


@torch.no_grad()
def _load_flat_params(tr, flat):
    """Set every optimizer-owned parameter to the fp32 values `flat` (a FlatParamSpace.flat_p
    snapshot): the flat master buffer in place (plain parameters are views of it, so their
    version counters move) and each bf16 model weight to its master's rounding."""
    sp = tr.space
    sp.flat_p.copy_(torch.from_numpy(flat).to(sp.flat_p.device))
    for i in np.nonzero(sp.shadowed)[0]:
        p = sp.params[int(i)]
        p.data.copy_(sp.master(int(i)).view(p.shape).to(p.dtype))


def _mode_g_trainer_worker(rank, world, port, q_out, unfreeze_audio=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        m = _mode_r_model()
        m.audio_embedder.normalize = _no_znorm
        tr = _mode_g_trainer(m, dist.group.WORLD, unfreeze_audio)
        assert tr.reducer is not None and tr.reducer.group is not dist.group.WORLD
        losses, launched, params = [], [], []
        for step in range(2):
            f, a, t, _, _ = _mode_r_batch(step, rank)
            out = tr.step(f, a, t, phase="full_joint")
            losses.append(float(out["loss"]))
            launched.append(tr.reducer.launched_in_backward)
            params.append(tr.space.flat_p.cpu().numpy())
        torch.cuda.synchronize()
        q_out.put((rank, [g.cpu().numpy() for g in tr.reduced], params, losses, tr.space.touched.copy()))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q_out.put((rank, "error", traceback.format_exc(), None, None))


@pytest.mark.late
def test_mode_g_trainer_two_ranks_with_unfreeze_flip():
    """TriadTrainer(global_negatives=True) at world size 2 (gloo on the box's one GPU): the head's
    key all-gather / clip-row gather / dK reduce-scatter run on the model's group while the
    overlapped bucket reducer (its own communicator) SUM-reduces the parameter
    gradients; two steps, HuBERT unfrozen at the second (train.py:527-548), which also re-derives
    the reducer's launch order. Both ranks compute the identical global loss and hold identical
    parameters; the reduced gradient of each step equals ONE process running the same B_g = 4
    batch (same global patch-dropout masks; embedders run over the ranks' halves, see
    _embed_in_chunks), per parameter group at the bf16 bar. The second step starts the single
    process from the ranks' parameters after the first (_load_flat_params): AdamW's first update
    is ~lr * sign(g), so rounding-level gradient differences flip whole elements and the two runs'
    parameters part by ~2 lr there -- which would make step 1 compare different models."""
    world = 2
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_mode_g_trainer_worker, args=(r, world, port, qo)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([qo.get(timeout=600) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[2]
    (_, g0, p0, l0, t0), (_, g1, p1, l1, t1) = res
    assert l0 == l1                                 # the one global loss on both ranks
    for a, b in zip(g0, g1):
        np.testing.assert_array_equal(a, b)         # one reduced gradient on both ranks
    for a, b in zip(p0, p1):
        np.testing.assert_array_equal(a, b)         # identical parameters after each step
    np.testing.assert_array_equal(t0, t1)
    # single process at B_g = 4: rank-major concatenation of the two ranks' batches, masks from the
    # same shared seed
    def single():
        m = _mode_r_model()
        m.audio_embedder.normalize = _no_znorm
        m.visual_embedder.set_global_mask(1, 0)
        _embed_in_chunks(m, 2)
        tr = _mode_g_trainer(m, None)
        losses = []
        for step in range(2):
            if step:
                _load_flat_params(tr, p0[step - 1])
            b0, b1 = _mode_r_batch(step, 0), _mode_r_batch(step, 1)
            out = tr.step(torch.cat([b0[0], b1[0]]), torch.cat([b0[1], b1[1]]), list(b0[2]) + list(b1[2]),
                          phase="full_joint")
            losses.append(float(out["loss"]))
        return m, tr, losses, [g.cpu().numpy() for g in tr.reduced]

    m, tr, ls, gs = single()
    bad = []
    for step in range(2):
        assert abs(ls[step] - l0[step]) <= 1e-4 * abs(l0[step]), (step, ls[step], l0[step])
        rel = _group_rel(tr, g0[step], gs[step])
        print(f"mode G step {step}: reduced-gradient rel error per group {rel}")
        print(f"mode G step {step}: worst parameters {_worst_params(m, tr, g0[step], gs[step], tr.groups['others'])}")
        bad += [(step, name, r, _worst_params(m, tr, g0[step], gs[step], tr.groups[name], k=4))
                for name, r in rel.items() if not r < 1e-2]
    if bad:
        # diagnosis only (the test has failed): is the single process reproducible, i.e. which of
        # the two sides is the odd one out?
        _, _, ls2, gs2 = single()
        same = all(np.array_equal(a, b) for a, b in zip(gs, gs2)) and ls == ls2
        rel2 = [_group_rel(tr, g0[s], gs2[s]) for s in range(2)]
        raise AssertionError(f"Mode G vs single process beyond the bf16 bar: {bad}; a second single-process run "
                             f"equals the first: {same}, its errors vs the ranks per step: {rel2}")
