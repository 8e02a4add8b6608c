"""The TRIAD training step on MI355X (mirror of SajayR/TRIAD src/train.py:932-1041).

`TriadTrainer` keeps the reference's step semantics:
  * parameter groups by name (train.py:251-261): audio_embedder.hubert -> audio,
    text_embedder.encoder -> text, visual_embedder.model + lora -> vit LoRA,
    visual_embedder.model (frozen base, no optimizer), everything else -> others;
  * staged unfreezing of HuBERT / DistilBERT by global step (train.py:527-548);
  * curriculum loss mixing by phase (train.py:972-984) and 1/grad_accum scaling
    (train.py:986-987);
  * per-group grad norms, clip_grad_norm_(audio_embedder / text_embedder, 10)
    and the four AdamW + OneCycleLR steps gated by the unfreeze steps
    (train.py:990-1041).
Differences by design: the optimizer state is a flat fp32 buffer with a
fused HIP AdamW (`optimizer="fused"`, default; `"torch"` keeps torch.optim.AdamW for
parity tests); stats/grad norms stay on the device (no per-step `.item()`), and
`torch.cuda.empty_cache()` is not called every step.

Data parallel (one process per GPU, RCCL over xGMI): the flat gradient buffer is
averaged with bucketed all-reduces launched from gradient hooks while backward is still
running (triad_amd.dist.GradBucketReducer; fp32 or bf16 on the wire) -- the reference
has no distributed code; this is SURVEY §8e Mode R. `global_negatives=True` is Mode G
(triad_amd.dist).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.distributed as dist

from . import dist as tdist
from . import optim as fo


def split_param_groups(model):
    """train.py:251-261 name-based grouping."""
    groups = {"audio": [], "text": [], "vit_lora": [], "vit": [], "others": []}
    for name, p in model.named_parameters():
        if "audio_embedder.hubert" in name:
            groups["audio"].append(p)
        elif "text_embedder.encoder" in name:
            groups["text"].append(p)
        elif "visual_embedder.model" in name and "lora" in name:
            groups["vit_lora"].append(p)
        elif "visual_embedder.model" in name:
            groups["vit"].append(p)
        else:
            groups["others"].append(p)
    return groups


def bf16_weight_params(model):
    """Weights autocast feeds to bf16 matmuls/convs exactly once per forward: every nn.Linear /
    nn.Conv1d parameter of HuBERT and DistilBERT (model.py:29-30,79-80), except weight-normalised
    convolutions (HuBERT's positional conv computes its weight from g, v in fp32 before the cast),
    and the three projection heads' Linear layers (model.py:32-34, 81-83, 253-255; the LayerNorm
    between them stays fp32, as autocast runs it). These can live as bf16 model weights over fp32
    masters: the forward sees what autocast's cast would produce, and the gradients arrive in
    bf16 as autocast's backward produces them."""
    out = []
    for root in (model.audio_embedder.hubert, model.text_embedder.encoder):
        for mod in root.modules():
            if isinstance(mod, (torch.nn.Linear, torch.nn.Conv1d)) and not hasattr(mod, "parametrizations") \
                    and not hasattr(mod, "weight_g"):
                out.extend(p for p in mod.parameters(recurse=False) if p.dtype == torch.float32)
    for emb in (model.audio_embedder, model.text_embedder, model.visual_embedder):
        for mod in (emb.projection1, emb.projection2):
            out.extend(p for p in mod.parameters(recurse=False) if p.dtype == torch.float32)
    return out


def _one_cycle(opt, max_lr, total):
    return torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=max_lr, total_steps=max(1, total), pct_start=0.1,
                                               div_factor=10, final_div_factor=1e4, anneal_strategy="cos")


class TriadTrainer:
    def __init__(self, model, learning_rate=1e-4, total_updates=10000, gradient_accumulation_steps=1,
                 unfreeze_audio_step=5000, unfreeze_text_step=5000, unfreeze_vit_step=5000,
                 optimizer="fused", device="cuda", process_group=None, bucket_mb=64.0,
                 av_weight_start=0.8, av_weight_end=0.5, global_negatives=False, bf16_weights=None,
                 overlap_grad_reduce=True, grad_wire="fp32"):
        self.model = model
        self.device = torch.device(device)
        if self.device.type == "cuda":  # library GEMMs on rocBLAS, not hipBLASLt (explicit opt-in, blas.py)
            from . import blas
            blas.configure(warn_if_late=False)
        self.grad_accum = gradient_accumulation_steps
        self.unfreeze = dict(audio=unfreeze_audio_step, text=unfreeze_text_step, vit=unfreeze_vit_step)
        self.av_weight_start, self.av_weight_end = av_weight_start, av_weight_end
        self.groups = split_param_groups(model)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        self.bucket_elems = int(bucket_mb * (1 << 20) / 4)
        self.global_negatives = global_negatives and self.world > 1
        if self.global_negatives:
            model.enable_global_negatives(process_group)
        opt_params = self.groups["others"] + self.groups["audio"] + self.groups["text"] + self.groups["vit_lora"]
        self.kind = optimizer
        if optimizer == "fused":
            # mixed-precision model weights for the autocast backbones (default: when the
            # model runs under bf16 autocast on the GPU); see optim.FlatParamSpace
            if bf16_weights is None:
                bf16_weights = bool(getattr(model, "use_amp", False)) and self.device.type == "cuda"
            shadow = bf16_weight_params(model) if bf16_weights else []
            self.space = fo.FlatParamSpace(opt_params, self.device, shadow=shadow)
            mk = lambda ps: fo.FusedAdamW(self.space, ps, lr=learning_rate)  # noqa: E731
        elif optimizer == "torch":
            self.space = None
            mk = lambda ps: torch.optim.AdamW(ps, lr=learning_rate)  # noqa: E731
        else:
            raise ValueError(optimizer)
        # train.py:272-287 + the freezing block at 289-296
        self.opt_others = mk(self.groups["others"])
        self.opt_audio = mk(self.groups["audio"])
        self.opt_text = mk(self.groups["text"])
        self.opt_vit = mk(self.groups["vit_lora"])
        for p in self.groups["audio"] + self.groups["text"] + self.groups["vit"]:
            p.requires_grad = False
        for p in self.groups["vit_lora"]:
            p.requires_grad = True
        # data parallel: bucketed gradient all-reduce overlapped with backward (fused optimizer).
        # NOTE: dist.new_group is collective over the default group -- every rank of the job must
        # construct its TriadTrainer (the usual one-trainer-per-rank script does).
        self.reducer = None
        self.mask_group = None
        if self.world > 1:
            # the touched-set OR after each reduction (dist.agree_touched) runs on the host: a gloo
            # group beside an RCCL job, so it never waits for the GPU
            ranks = (dist.get_process_group_ranks(process_group) if process_group is not None
                     else list(range(self.world)))
            self.mask_group = (process_group if dist.get_backend(process_group) == "gloo"
                               else dist.new_group(ranks=ranks, backend="gloo"))
        if self.world > 1 and self.space is not None and overlap_grad_reduce:
            # its own communicator: the bucket all-reduces are issued from gradient hooks during
            # backward, while Mode G's head issues its reduce-scatter / all-gathers inside the same
            # backward on the model's group -- on separate communicators the two sequences can
            # never interleave differently on different ranks
            ranks = (dist.get_process_group_ranks(process_group) if process_group is not None
                     else list(range(self.world)))
            self.reducer_group = dist.new_group(ranks=ranks)
            self.reducer = tdist.GradBucketReducer(self.space, bucket_mb, grad_wire,
                                                   average=not self.global_negatives, group=self.reducer_group,
                                                   mask_group=self.mask_group)
        self.total_updates = total_updates
        self.sched_others = _one_cycle(self.opt_others, learning_rate, total_updates)
        self.sched_audio = _one_cycle(self.opt_audio, learning_rate * 0.25, total_updates - unfreeze_audio_step)
        self.sched_text = _one_cycle(self.opt_text, learning_rate * 0.75, total_updates - unfreeze_text_step)
        self.sched_vit = _one_cycle(self.opt_vit, learning_rate * 0.5, total_updates - unfreeze_vit_step)
        self.step_others = self.step_audio = self.step_text = self.step_vit = 0
        self.global_step = 0
        self.accumulation_counter = 0

    # train.py:527-548
    def _update_frozen_params(self, step):
        m = self.model
        for p in m.audio_embedder.hubert.parameters():
            p.requires_grad = step >= self.unfreeze["audio"]
        for p in m.text_embedder.encoder.parameters():
            p.requires_grad = step >= self.unfreeze["text"]

    def _loss_mix(self, phase, av, tv, progress):
        """train.py:972-984."""
        if phase == "av_focus":
            return av
        if phase == "tv_warmup":
            return tv
        if phase == "weighted_joint":
            w = self.av_weight_start - progress * (self.av_weight_start - self.av_weight_end)
            return w * av + (1.0 - w) * tv
        return av + tv

    def _allreduce_grads(self):
        """Data-parallel gradient reduction over the flat gradient buffer (bucketed RCCL
        all-reduce). Mode R averages (replicas of the reference loss); Mode G sums (every rank
        holds its share of the one global loss's gradient). A parameter then has a gradient iff some
        rank produced one (dist.agree_touched: an OR over ranks on the host)."""
        if self.world <= 1:
            return
        if self.reducer is not None:   # launched during backward; wait for the reductions
            self.reducer.finish()
            return
        avg = not self.global_negatives
        if self.space is None:
            for p in self.model.parameters():
                if p.grad is not None:
                    tdist.allreduce_grads(p.grad.view(-1), p.grad.numel(), avg, self.pg)
            return
        tdist.allreduce_grads(self.space.flat_g, self.bucket_elems, avg, self.pg)
        # every rank now holds the same reduced gradient; a parameter counts as having one iff
        # some rank produced it (dist.agree_touched)
        tdist.agree_touched(self.space, self.mask_group)

    def step(self, frames, audio, text, phase="full_joint", progress=0.0, av_keep=None, tv_keep=None,
             shared_frames=True, frames_tv=None):
        """One training step (forward + backward [+ optimizer at the accumulation boundary]).
        Returns a dict of device tensors (nothing is synchronised)."""
        self._update_frozen_params(self.global_step)
        if self.space is not None:
            self.space.release_held_grads()
        m = self.model
        out: Dict[str, torch.Tensor] = {}
        av = tv = None
        if phase == "full_joint" and shared_frames and frames_tv is None:
            av, tv = m.forward_triad(frames, audio, text, av_keep=av_keep, tv_keep=tv_keep)
        else:
            if phase != "tv_warmup":
                av = m.forward_audio_visual(frames, audio)
            if phase != "av_focus":
                tv = m.forward_text_visual(frames if frames_tv is None else frames_tv, text)
        av_loss = av[0] if av is not None else None
        tv_loss = tv[0] if tv is not None else None
        loss_total = self._loss_mix(phase, av_loss, tv_loss, progress)
        if self.space is not None:
            self.space.release_held_grads()
        if self.reducer is not None and (self.accumulation_counter + 1) % self.grad_accum == 0:
            self.reducer.begin(accumulate=self.accumulation_counter % self.grad_accum != 0)
        (loss_total / self.grad_accum).backward()
        if self.space is not None:  # bf16 weight grads -> flat fp32 grads (accumulating micro-steps)
            self.space.gather_shadow_grads(accumulate=self.accumulation_counter % self.grad_accum != 0)
        self.accumulation_counter += 1
        out["loss"] = loss_total.detach()
        if av is not None:
            out.update(loss_av=av[0].detach(), av_contrastive=av[1].detach(), av_reg=av[2].detach(),
                       av_smooth=av[3].detach())
            out["av_stats"] = av[4]
        if tv is not None:
            out["loss_tv"] = tv[0].detach()
            out["tv_stats"] = tv[1]
        if self.accumulation_counter % self.grad_accum == 0:
            out.update(self._optimizer_step())
        self.global_step += 1
        return out

    def _optimizer_step(self):
        self._allreduce_grads()
        res = {}
        m = self.model
        if self.space is not None:
            norms, sq = fo.grad_norms(self.space, {k: self.groups[k] for k in
                                                   ("others", "audio", "vit", "vit_lora", "text")})
            res.update({f"grad_norm_{k}": v for k, v in norms.items()})
            fo.clip_grad_norm_(self.space, list(m.audio_embedder.parameters()), 10.0, sq)
            fo.clip_grad_norm_(self.space, list(m.text_embedder.parameters()), 10.0, sq)
        else:
            for k in ("others", "audio", "vit", "vit_lora", "text"):
                gs = [p.grad.norm() for p in self.groups[k] if p.grad is not None]
                res[f"grad_norm_{k}"] = torch.norm(torch.stack(gs)) if gs else torch.zeros((), device=self.device)
            torch.nn.utils.clip_grad_norm_(m.audio_embedder.parameters(), 10.0)
            torch.nn.utils.clip_grad_norm_(m.text_embedder.parameters(), 10.0)
        # train.py:1010-1040
        self.opt_others.step()
        self.opt_others.zero_grad()
        if self.step_others < self.total_updates:
            self.sched_others.step()
            self.step_others += 1
        if self.global_step >= self.unfreeze["audio"]:
            self.opt_audio.step()
            self.opt_audio.zero_grad()
            if self.step_audio < self.total_updates - self.unfreeze["audio"]:
                self.sched_audio.step()
                self.step_audio += 1
        else:
            self.opt_audio.zero_grad()
        if self.global_step >= self.unfreeze["text"]:
            self.opt_text.step()
            self.opt_text.zero_grad()
            if self.step_text < self.total_updates - self.unfreeze["text"]:
                self.sched_text.step()
                self.step_text += 1
        else:
            self.opt_text.zero_grad()
        self.opt_vit.step()
        self.opt_vit.zero_grad()
        if self.step_vit < self.total_updates - self.unfreeze["vit"]:
            self.sched_vit.step()
            self.step_vit += 1
        return res
