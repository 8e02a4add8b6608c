"""Checkpoint format compatibility (reference train.py:397-525), on CPU.

No reference checkpoint exists offline (the reference ships none), so the format is pinned
by construction: the model keys are the peft / transformers names train.py would write, and
the optimizer states are exactly torch.optim.AdamW's (they load into torch.optim.AdamW and
torch's load into ours)."""
import warnings

import numpy as np
import pytest
import torch

from triad_amd import checkpoint as ck


@pytest.fixture(scope="module")
def trainer_pair():
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer

    def make(seed):
        torch.manual_seed(seed)
        m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.8, patch_sparsity_weight=0.01,
                            visual_dropout_prob=0.25)
        return TriadTrainer(m, total_updates=100, unfreeze_audio_step=0, unfreeze_text_step=0, unfreeze_vit_step=0,
                            device="cpu")
    return make(0), make(1)


def _fake_optimizer_progress(tr, seed):
    """Give every optimizer some AdamW state and advance the schedulers (no HIP calls)."""
    g = torch.Generator().manual_seed(seed)
    sp = tr.space
    for i, p in enumerate(sp.params):
        o, n = sp.offsets[i], p.numel()
        sp.steps[i] = 3 + i % 2
        sp.exp_avg[o:o + n] = torch.randn(n, generator=g) * 1e-3
        sp.exp_avg_sq[o:o + n] = torch.rand(n, generator=g) * 1e-6
    for name in ("others", "audio", "text", "vit"):
        with warnings.catch_warnings():  # schedulers stepped without an optimizer step on purpose
            warnings.simplefilter("ignore")
            for _ in range(3):
                getattr(tr, f"sched_{name}").step()
        setattr(tr, f"step_{name}", 3)
    tr.global_step = 7


def test_key_mapping_roundtrip(trainer_pair):
    tr, _ = trainer_pair
    keys = list(tr.model.state_dict())
    ref = [ck.to_reference_key(k) for k in keys]
    assert "visual_embedder.model.base_model.model.blocks.0.attn.qkv.lora_A.default.weight" in ref
    assert "visual_embedder.model.base_model.model.blocks.0.attn.proj.base_layer.weight" in ref
    assert "visual_embedder.model.base_model.model.patch_embed.proj.weight" in ref
    assert "audio_embedder.hubert.feature_extractor.conv_layers.0.conv.weight" in ref
    assert "text_embedder.encoder.embeddings.word_embeddings.weight" in ref
    assert [ck.from_reference_key(k) for k in ref] == keys
    assert [ck.from_reference_key("_orig_mod." + k) for k in ref] == keys  # train.py:443-452


def test_fused_adamw_state_is_torch_adamw_format(trainer_pair):
    tr, _ = trainer_pair
    _fake_optimizer_progress(tr, 0)
    for name in ("others", "audio", "text", "vit"):
        opt = getattr(tr, f"opt_{name}")
        sd = opt.state_dict()
        params = opt.param_groups[0]["params"]
        ref = torch.optim.AdamW([torch.nn.Parameter(p.detach().clone()) for p in params], lr=1e-4)
        ref.load_state_dict(sd)  # torch accepts it as its own
        rsd = ref.state_dict()
        assert rsd["param_groups"][0].keys() == sd["param_groups"][0].keys()
        assert rsd["state"].keys() == sd["state"].keys()
        for k, st in sd["state"].items():
            assert float(rsd["state"][k]["step"]) == float(st["step"])
            assert torch.equal(rsd["state"][k]["exp_avg"], st["exp_avg"])
            assert torch.equal(rsd["state"][k]["exp_avg_sq"], st["exp_avg_sq"])
        # and back: torch's state_dict loads into the flat buffers unchanged
        opt.load_state_dict(rsd)
        sd2 = opt.state_dict()
        for k, st in sd["state"].items():
            assert torch.equal(sd2["state"][k]["exp_avg"], st["exp_avg"])
            assert float(sd2["state"][k]["step"]) == float(st["step"])


def test_checkpoint_save_load_roundtrip(trainer_pair, tmp_path):
    a, b = trainer_pair
    _fake_optimizer_progress(a, 1)
    path = tmp_path / "checkpoint_epoch0_step7.pt"
    ck.save_checkpoint(a, path, epoch=0, step=7, best_loss=3.5, config={"av_focus_epochs": 1})
    raw = ck.load_file(path)
    for key in ("epoch", "step", "current_batch_idx", "current_segment", "rng_state", "model_state_dict",
                "opt_others_state", "opt_audio_state", "opt_text_state", "opt_vit_state", "sched_others_state",
                "sched_audio_state", "sched_text_state", "sched_vit_state", "sched_step_others", "sched_step_audio",
                "sched_step_text", "sched_step_vit", "best_loss", "config", "vis_samples_av", "vis_samples_tv"):
        assert key in raw, key  # train.py:406-428
    # a torch.compile'd reference model saves `_orig_mod.` keys (train.py:412); both load
    raw["model_state_dict"] = {"_orig_mod." + k: v for k, v in raw["model_state_dict"].items()}
    ck.load_checkpoint(b, raw)
    for (n, pa), (_, pb) in zip(a.model.named_parameters(), b.model.named_parameters()):
        assert torch.equal(pa.detach().float(), pb.detach().float()), n
    assert b.global_step == 7 and b.step_audio == 3
    for name in ("others", "audio", "text", "vit"):
        sa, sb = getattr(a, f"opt_{name}").state_dict(), getattr(b, f"opt_{name}").state_dict()
        assert sa["state"].keys() == sb["state"].keys()
        for k in sa["state"]:
            assert torch.equal(sa["state"][k]["exp_avg_sq"], sb["state"][k]["exp_avg_sq"])
        assert getattr(a, f"sched_{name}").last_epoch == getattr(b, f"sched_{name}").last_epoch
        assert sa["param_groups"][0]["lr"] == sb["param_groups"][0]["lr"]
    # flat-buffer aliasing survives the load: parameters are still views of the flat space
    p0 = b.space.params[0]
    assert p0.data_ptr() == b.space.flat_p[b.space.offsets[0]:].data_ptr()
    assert np.all(b.space.steps >= 3)


def _reference_shaped_state_dict(model, seed):
    """A `model_state_dict` as the reference's train.py:413 would write it, built WITHOUT the
    mirror's key mapping: HuBERT / DistilBERT keys from the stock `transformers` classes (no
    execution tweaks installed), the ViT under peft's wrapper names, all fp32, with the
    `_orig_mod.` prefix of a torch.compile'd model (train.py:412)."""
    import transformers
    g = torch.Generator().manual_seed(seed)
    sd = {}
    hub = transformers.HubertModel(transformers.HubertConfig()).state_dict()
    dbert = transformers.DistilBertModel(transformers.DistilBertConfig()).state_dict()
    for prefix, part in (("audio_embedder.hubert.", hub), ("text_embedder.encoder.", dbert)):
        for k, v in part.items():
            sd[prefix + k] = v
    ours = model.state_dict()
    for k, v in ours.items():
        if k.startswith(ck.VIT):
            rest = k[len(ck.VIT):]
            if rest.endswith(".base.weight") or rest.endswith(".base.bias"):
                rest = rest.replace(".base.", ".base_layer.")
            elif rest.endswith(".lora_A") or rest.endswith(".lora_B"):
                rest += ".default.weight"
            sd[ck.PEFT + rest] = v
        elif not (k.startswith("audio_embedder.hubert.") or k.startswith("text_embedder.encoder.")):
            sd[k] = v  # projection heads, temperature
    out = {}
    for k, v in sd.items():
        if v.is_floating_point():
            v = torch.randn(v.shape, generator=g, dtype=torch.float32) * 0.02
        out["_orig_mod." + k] = v.clone()
    return out


def test_reference_shaped_checkpoint_loads_and_saves_bit_exact(trainer_pair):
    """A reference-layout fp32 state dict loads strictly (every stock transformers / peft key is
    matched, none left over) and saves back bit-exact -- including the frozen ViT base, which
    executes from bf16 copies (vit.store_frozen_base_bf16) but is kept and saved in fp32."""
    _, b = trainer_pair
    sd = _reference_shaped_state_dict(b.model, 5)
    missing, unexpected = ck.load_reference_state_dict(b.model, sd, strict=True, space=b.space)
    assert not missing and not unexpected
    back = ck.reference_state_dict(b.model, b.space)
    assert set(back) == {k[len("_orig_mod."):] for k in sd}
    frozen_bf16 = 0
    for k, v in back.items():
        want = sd["_orig_mod." + k]
        assert v.dtype == want.dtype, k
        assert torch.equal(v, want), k
    for n, p in b.model.named_parameters():
        frozen_bf16 += int(p.dtype == torch.bfloat16 and not p.requires_grad)
    assert frozen_bf16 > 0  # the bf16 execution copies exist and did not leak into the save


def test_state_load_refreshes_positional_embedding_cache():
    """The ViT caches its interpolated positional embedding for frozen weights; a state load
    after a forward must invalidate it (the cache is keyed on the tensor version, and the
    loader copies in place under no_grad, which bumps it; refresh_frozen_copies clears it)."""
    from triad_amd.vit import DinoVisionTransformer, apply_lora
    torch.manual_seed(0)
    vit = apply_lora(DinoVisionTransformer("dinov2_vits14_reg"))
    x = torch.randn(1, 3, 56, 70)   # 4 x 5 patches: the 16 x 16 table is interpolated
    with torch.no_grad():
        y0 = vit.get_intermediate_layers(x, n=1)[0].clone()
        sd = {ck.VIT + k: v.clone() for k, v in vit.state_dict().items()}
        sd[ck.VIT + "pos_embed"] = torch.randn_like(sd[ck.VIT + "pos_embed"])

        class Holder(torch.nn.Module):
            pass
        h = Holder()
        h.visual_embedder = torch.nn.Module()
        h.visual_embedder.model = vit
        ck.load_reference_state_dict(h, sd)
        y1 = vit.get_intermediate_layers(x, n=1)[0]
        fresh = apply_lora(DinoVisionTransformer("dinov2_vits14_reg"))
        fresh.load_state_dict({k[len(ck.VIT):]: v for k, v in sd.items()})
        y2 = fresh.get_intermediate_layers(x, n=1)[0]
    assert not torch.equal(y0, y1)
    assert torch.equal(y1, y2)


class _MaskOwner:
    """The patch-mask generator interface of ViTLoRAEmbedder (mask_generator), without a ViT."""

    def __init__(self, seed):
        self.gen = torch.Generator()
        self.gen.manual_seed(seed)

    def mask_generator(self):
        return self.gen


def _mask_ckpt_worker(rank, world, port, q, path):
    import os
    import types
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from triad_amd import checkpoint as ck
        ve = _MaskOwner(100 + rank)
        tr = types.SimpleNamespace(world=world, pg=None, global_negatives=False,
                                   model=types.SimpleNamespace(visual_embedder=ve))
        torch.rand(5, generator=ve.gen)                       # some draws before the save
        saved = ck.gather_mask_states(tr)                     # collective
        # save_checkpoint: every rank calls it (the gather inside is a collective), rank 0 writes
        real = ck.trainer_checkpoint
        ck.trainer_checkpoint = lambda t, e, st, **kw: {"writer": rank, "mask": ck.gather_mask_states(t)}
        try:
            ck.save_checkpoint(tr, path, 1, 2)
        finally:
            ck.trainer_checkpoint = real
        want = torch.rand(8, generator=ve.gen)                # what an uninterrupted run draws next
        fresh = _MaskOwner(0)
        ck._restore_mask_generator(tr, fresh, saved)
        got = torch.rand(8, generator=fresh.gen)
        single = _MaskOwner(0)                                # an old single-state checkpoint
        ck._restore_mask_generator(tr, single, saved[0])
        q.put((rank, len(saved), bool(torch.equal(got, want)), torch.rand(8, generator=single.gen).tolist()))
    finally:
        dist.destroy_process_group()


def test_patch_mask_generator_state_per_rank(tmp_path):
    """a Mode R checkpoint keeps every rank's patch-mask generator (gathered, indexed by
    rank) and each rank resumes its own sequence; a single saved state restored on several ranks
    re-mixes the rank in, so replicas never draw identical masks. ADVICE r3: save_checkpoint is
    called on every rank and only rank 0 writes the file (with both ranks' states)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "ck.pt")
    procs = [ctx.Process(target=_mask_ckpt_worker, args=(r, 2, port, q, path)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)])
    for p in procs:
        p.join(timeout=30)
    (_, n0, ok0, s0), (_, n1, ok1, s1) = res
    assert n0 == n1 == 2 and ok0 and ok1
    assert s0 != s1
    from triad_amd import checkpoint as ck
    saved = ck.load_file(path)
    assert saved["writer"] == 0 and len(saved["mask"]) == 2
