"""Checkpoint format compatibility with SajayR/TRIAD.

Reference: src/train.py:397-437 (save_checkpoint) and 439-525 (load_checkpoint). A checkpoint
is one `torch.save`d dict with `model_state_dict` (the uncompiled module's state_dict; a
`_orig_mod.` prefix from torch.compile is stripped on load), four AdamW states
(`opt_{others,audio,text,vit}_state`), four OneCycleLR states (`sched_*_state`), the
per-scheduler step counters (`sched_step_*`), `epoch`, `step`, `best_loss`, `config` and
bookkeeping fields of the data pipeline.

Two name spaces differ between the reference model and this mirror, and are mapped here:
  * the DINOv2 backbone is wrapped by peft in the reference (model.py:232-245):
      visual_embedder.model.base_model.model.<hub name>            (frozen weights)
      ...attn.qkv.base_layer.{weight,bias}                          (the wrapped Linear)
      ...attn.qkv.lora_A.default.weight  (r, in)  / lora_B.default.weight (out, r)
    here: visual_embedder.model.<hub name>, ...attn.qkv.base.{weight,bias},
    ...attn.qkv.lora_A (r, in) / lora_B (out, r) -- same shapes, same layout;
  * HuBERT / DistilBERT keys are the transformers classes' own on both sides.
Optimizer states use torch.optim.AdamW's format on both sides (FusedAdamW.state_dict).
"""
from __future__ import annotations

import random
from collections import OrderedDict
from typing import Dict

import numpy as np
import torch

VIT = "visual_embedder.model."
PEFT = "visual_embedder.model.base_model.model."


def to_reference_key(k: str) -> str:
    if not k.startswith(VIT):
        return k
    rest = k[len(VIT):]
    for ours, theirs in ((".base.weight", ".base_layer.weight"), (".base.bias", ".base_layer.bias")):
        if rest.endswith(ours):
            rest = rest[: -len(ours)] + theirs
    if rest.endswith(".lora_A") or rest.endswith(".lora_B"):
        rest = rest + ".default.weight"
    return PEFT + rest


def from_reference_key(k: str) -> str:
    if k.startswith("_orig_mod."):  # train.py:443-452
        k = k[len("_orig_mod."):]
    if not k.startswith(PEFT):
        return k
    rest = k[len(PEFT):]
    for theirs, ours in ((".base_layer.weight", ".base.weight"), (".base_layer.bias", ".base.bias"),
                         (".lora_A.default.weight", ".lora_A"), (".lora_B.default.weight", ".lora_B")):
        if rest.endswith(theirs):
            rest = rest[: -len(theirs)] + ours
    return VIT + rest


def _masters(model, space):
    """{state_dict key: fp32 master} for parameters held as bf16 model weights: trainable ones
    by the optimizer's flat `space`, frozen ones (the ViT base, vit.store_frozen_base_bf16) by
    the module's `frozen_fp32` dict."""
    out = {}
    for mname, mod in model.named_modules():
        for k, v in getattr(mod, "frozen_fp32", {}).items():
            out[f"{mname}.{k}" if mname else k] = v
    if space is None or not getattr(space, "shadowed", np.zeros(0, bool)).any():
        return out
    by_id = {id(p): k for k, p in model.named_parameters()}
    out.update({by_id[id(space.params[i])]: space.master(i) for i in np.nonzero(space.shadowed)[0]
                if id(space.params[i]) in by_id})
    return out


def reference_state_dict(model: torch.nn.Module, space=None) -> "OrderedDict[str, torch.Tensor]":
    """The mirror's parameters and buffers under the reference model's state_dict names
    (fp32, as the reference keeps them: bf16 model weights are replaced by their fp32 masters
    from the optimizer's flat space; frozen bf16 copies are an execution detail)."""
    masters = _masters(model, space)
    out = OrderedDict()
    for k, v in model.state_dict().items():
        v = masters.get(k, v)
        out[to_reference_key(k)] = v.detach().float().clone() if v.is_floating_point() else v.detach().clone()
    return out


@torch.no_grad()
def load_reference_state_dict(model: torch.nn.Module, sd: Dict[str, torch.Tensor], strict: bool = True,
                              space=None):
    """Load a reference `model_state_dict` (with or without `_orig_mod.`) into the mirror.
    Copies in place, so flat optimizer buffers that alias the parameters stay valid; bf16
    model weights get the fp32 value in their master and its bf16 rounding."""
    mapped = {from_reference_key(k): v for k, v in sd.items()}
    for k, m in _masters(model, space).items():
        if k in mapped:
            m.copy_(mapped[k].to(device=m.device, dtype=m.dtype))
    own = model.state_dict(keep_vars=True)
    missing = [k for k in own if k not in mapped]
    unexpected = [k for k in mapped if k not in own]
    if strict and (missing or unexpected):
        raise KeyError(f"state_dict mismatch: missing {missing[:5]}..., unexpected {unexpected[:5]}...")
    for k, t in own.items():
        if k in mapped:
            src = mapped[k]
            if tuple(src.shape) != tuple(t.shape):
                raise ValueError(f"{k}: shape {tuple(src.shape)} vs {tuple(t.shape)}")
            # an in-place copy under no_grad bumps the tensor version (caches keyed on it see the
            # new values) and keeps flat optimizer buffers that alias the parameter valid
            t.copy_(src.to(device=t.device, dtype=t.dtype))
    for mod in model.modules():
        if hasattr(mod, "refresh_frozen_copies"):
            mod.refresh_frozen_copies()
    return missing, unexpected


_OPTS = ("others", "audio", "text", "vit")


def trainer_checkpoint(trainer, epoch: int, step: int, best_loss: float = float("inf"), config=None,
                       current_batch_idx: int = 0, current_segment: int = 0, vis_samples_av=None,
                       vis_samples_tv=None, mask_states=None) -> dict:
    """The dict train.py:406-428 saves, built from a TriadTrainer.

    Data parallel (Mode R, world > 1): the patch-mask generator states of all ranks go into the
    dict, which takes a collective. Either call this on EVERY rank, or have every rank call
    `gather_mask_states(trainer)` and pass its result as `mask_states` to a call made on one rank
    only (e.g. rank 0, inside `if rank == 0:`)."""
    rng_state = {"torch": torch.get_rng_state(),
                 "cuda": torch.cuda.get_rng_state_all() if torch.cuda.is_available() else [],
                 "numpy": np.random.get_state(), "python": random.getstate()}
    ve = getattr(trainer.model, "visual_embedder", None)
    if ve is not None and hasattr(ve, "mask_generator"):
        # extra key (the reference ignores it): the host generator of the patch-dropout masks, so a
        # resumed run draws the masks an uninterrupted one would
        rng_state["triad_patch_mask"] = mask_states if mask_states is not None else gather_mask_states(trainer)
    ck = {"epoch": epoch, "step": step, "current_batch_idx": current_batch_idx, "current_segment": current_segment,
          "rng_state": rng_state, "model_state_dict": reference_state_dict(trainer.model, trainer.space)}
    for n in _OPTS:
        ck[f"opt_{n}_state"] = getattr(trainer, f"opt_{n}").state_dict()
    for n in _OPTS:
        ck[f"sched_{n}_state"] = getattr(trainer, f"sched_{n}").state_dict()
    for n in _OPTS:
        ck[f"sched_step_{n}"] = getattr(trainer, f"step_{n}")
    ck.update(best_loss=best_loss, config=config or {}, vis_samples_av=vis_samples_av, vis_samples_tv=vis_samples_tv)
    return ck


def gather_mask_states(trainer):
    """The patch-mask generator state(s) a checkpoint stores. Data parallel (Mode R): every rank's
    own state, gathered into a list indexed by rank -- a COLLECTIVE, every rank must call it;
    one process or Mode G (ranks share one state): the state itself."""
    ve = getattr(trainer.model, "visual_embedder", None)
    if ve is None or not hasattr(ve, "mask_generator"):
        return None
    st = ve.mask_generator().get_state()
    world = getattr(trainer, "world", 1)
    if world > 1 and not getattr(trainer, "global_negatives", False):
        import torch.distributed as dist
        states = [None] * world
        dist.all_gather_object(states, st, group=getattr(trainer, "pg", None))
        return [torch.as_tensor(x) for x in states]
    return st


def _restore_mask_generator(trainer, ve, saved):
    """Per-rank patch-mask generator state: a list (one state per rank) restores this rank's; a
    single state (a one-process checkpoint, or Mode G's shared state) restores it, and in Mode R
    with several ranks then re-mixes the rank in -- from a seed drawn from the restored state, so
    the result is reproducible -- instead of letting every replica draw the same masks."""
    import torch.distributed as dist
    gen = ve.mask_generator()
    world = getattr(trainer, "world", 1)
    rank = dist.get_rank(getattr(trainer, "pg", None)) if world > 1 else 0
    if isinstance(saved, (list, tuple)):
        st = saved[rank] if len(saved) == world else saved[0]
        gen.set_state(torch.as_tensor(st, dtype=torch.uint8).cpu())
        if len(saved) == world:
            return
    else:
        gen.set_state(torch.as_tensor(saved, dtype=torch.uint8).cpu())
    if world > 1 and not getattr(trainer, "global_negatives", False):
        seed = int(torch.randint(0, 2 ** 62, (1,), generator=gen))
        gen.manual_seed((seed + 0x9E3779B1 * rank) % (2 ** 63))


def save_checkpoint(trainer, path, epoch: int, step: int, **kw):
    """train.py:398-437. Data parallel: call it on EVERY rank (the per-rank mask states are
    gathered, a collective); only rank 0 writes `path` (the model / optimizer state is identical
    on every rank after the reduced step). Returns the checkpoint dict on every rank."""
    ck = trainer_checkpoint(trainer, epoch, step, **kw)
    import torch.distributed as dist
    rank = dist.get_rank(getattr(trainer, "pg", None)) if getattr(trainer, "world", 1) > 1 else 0
    if rank == 0:
        torch.save(ck, path)
    return ck


def _numpy_array_globals():
    """The weights_only unpickler's allowlist additions for numpy arrays (the RNG state of
    np.random.get_state(), train.py:402): ndarray / dtype reconstruction only."""
    out = [np.ndarray, np.dtype, type(np.dtype(np.uint32))]
    try:
        from numpy._core.multiarray import _reconstruct
    except ImportError:  # numpy < 2
        from numpy.core.multiarray import _reconstruct
    out.append(_reconstruct)
    return out


def load_file(path, device="cpu") -> dict:
    """torch.load with weights_only=True (never unpickles code), numpy arrays allowed."""
    with torch.serialization.safe_globals(_numpy_array_globals()):
        return torch.load(path, map_location=device, weights_only=True)


def load_checkpoint(trainer, path_or_dict, restore_rng: bool = True) -> dict:
    """train.py:439-525 on a TriadTrainer: model, optimizers, schedulers, counters, RNG.
    Returns the checkpoint dict (epoch, best_loss, config, ... for the caller's loop).
    Loaded with weights_only=True (tensors, numbers, strings and the RNG tuples only)."""
    if isinstance(path_or_dict, dict):
        ck = path_or_dict
    else:
        ck = load_file(path_or_dict, trainer.device)
    load_reference_state_dict(trainer.model, ck["model_state_dict"], space=trainer.space)
    for n in _OPTS:
        getattr(trainer, f"opt_{n}").load_state_dict(ck[f"opt_{n}_state"])
    for n in _OPTS:
        getattr(trainer, f"sched_{n}").load_state_dict(ck[f"sched_{n}_state"])
    for n in _OPTS:
        setattr(trainer, f"step_{n}", ck.get(f"sched_step_{n}", 0))
    trainer.global_step = ck["step"]
    if restore_rng and ck.get("rng_state") is not None:
        rs = ck["rng_state"]
        torch.set_rng_state(torch.as_tensor(rs["torch"], dtype=torch.uint8).cpu())
        if torch.cuda.is_available():
            for i, s in enumerate(rs["cuda"]):
                torch.cuda.set_rng_state(torch.as_tensor(s, dtype=torch.uint8).cpu(), device=i)
        np.random.set_state(rs["numpy"])
        random.setstate(rs["python"])
        ve = getattr(trainer.model, "visual_embedder", None)
        if rs.get("triad_patch_mask") is not None and ve is not None and hasattr(ve, "mask_generator"):
            _restore_mask_generator(trainer, ve, rs["triad_patch_mask"])
    trainer._update_frozen_params(trainer.global_step)
    return ck
