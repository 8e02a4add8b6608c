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
