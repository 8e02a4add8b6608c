"""Flat-buffer fused AdamW + grad-norm / clip for the TRIAD train step.

Reference semantics (SajayR/TRIAD src/train.py):
  * four torch.optim.AdamW optimizers with defaults (betas (0.9, 0.999), eps 1e-8,
    weight_decay 1e-2) over name-based parameter groups (train.py:251-287);
  * OneCycleLR per optimizer (train.py:289-343) -- it also cycles beta1
    (cycle_momentum=True), which this implementation honours per step;
  * per-group gradient norms (train.py:992-1002) and clip_grad_norm_(..., 10.0)
    on the audio and text embedders (train.py:1004-1006);
  * optimizers step only once their group is unfrozen (train.py:1016-1040).

MI355X design: every optimised parameter lives in ONE contiguous fp32 buffer
(`FlatParamSpace.params`), its gradient in another (`.grads`) and the AdamW
moments in two more; each nn.Parameter's `.data` and `.grad` are re-pointed at
views, so autograd accumulates straight into the flat gradient buffer, the
data-parallel all-reduce is one collective over it, and a whole optimizer step
is one HIP launch (triad_adamw_step) after one norm launch (triad_grad_sumsq).
Clipping is deferred into the AdamW launch as a per-parameter scale, so the
gradients are never rewritten in HBM.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import TriadError, call, ptr, stream_ptr

CHUNK = 16384
ALIGN = 64  # elements (256 B) per parameter slot
_CHUNK_DT = np.dtype([("off", "<i8"), ("n", "<i4"), ("param", "<i4")])
_PIECE_DT = np.dtype([("src", "<u8"), ("dst", "<i8"), ("n", "<i4"), ("f32", "<i4")])


class FlatParamSpace:
    """Owns the flat param / grad / exp_avg / exp_avg_sq buffers for a list of parameters.

    `shadow`: parameters to hold as bf16 MODEL weights backed by the fp32 master in the flat
    buffer (mixed precision for the bf16-autocast backbones): the nn.Parameter's .data becomes
    bf16 (what autocast would cast it to on every forward), autograd leaves its bf16 gradient
    in .grad (what autocast's backward produces before casting to fp32), `gather_shadow_grads`
    moves those into the flat fp32 gradient buffer in one launch, and the AdamW launch writes
    the new bf16 weight. Only for weights consumed exactly as autocast consumes them (Linear /
    Conv inputs), used once per backward (a second use would accumulate in bf16).

    On a GPU the fp32 parameters' gradients take the same route (`gathered`): .grad stays empty
    through backward, autograd stores each gradient as it comes (no kernel), and the same one
    gather launch adds them into the flat buffer -- instead of one PyTorch add kernel per fp32
    parameter (biases, LayerNorm affines: ~400 launches per tri-modal step) that .grad views of
    the flat buffer would cost. TRIAD_GATHER_FP32_GRADS=0: the views."""

    def __init__(self, params: Sequence[torch.nn.Parameter], device, shadow: Sequence[torch.nn.Parameter] = ()):
        self.device = torch.device(device)
        self.params: List[torch.nn.Parameter] = list(params)
        self.index = {id(p): i for i, p in enumerate(self.params)}
        shadow_ids = {id(p) for p in shadow}
        self.shadowed = np.array([id(p) in shadow_ids for p in self.params], dtype=bool)
        gather_fp32 = self.device.type == "cuda" and os.environ.get("TRIAD_GATHER_FP32_GRADS", "1") != "0"
        self.gathered = self.shadowed | gather_fp32   # .grad empty through backward, gathered after
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.offsets = offs
        self.numel = max(o, ALIGN)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.flat_p = torch.zeros(self.numel, **f32)
        self.flat_g = torch.zeros(self.numel, **f32)
        self.exp_avg = torch.zeros(self.numel, **f32)
        self.exp_avg_sq = torch.zeros(self.numel, **f32)
        self.touched = np.zeros(len(self.params), dtype=bool)
        self.steps = np.zeros(len(self.params), dtype=np.int64)
        self.scale = torch.ones(len(self.params), **f32)
        self._hooks = []
        shadow_base = np.zeros(len(self.params), dtype=np.uint64)
        with torch.no_grad():
            for i, p in enumerate(self.params):
                if p.dtype != torch.float32:
                    raise TriadError("flat AdamW expects fp32 master parameters")
                v = self.flat_p[offs[i]:offs[i] + p.numel()].view_as(p)
                v.copy_(p.data)
                if self.shadowed[i]:
                    p.data = v.to(torch.bfloat16)
                    p.grad = None
                    shadow_base[i] = (p.data_ptr() - 2 * offs[i]) % (1 << 64)
                else:
                    p.data = v
                    if self.gathered[i]:
                        p.grad = None
                    else:
                        p.grad = self.flat_g[offs[i]:offs[i] + p.numel()].view_as(p)
                        self._hooks.append(p.register_post_accumulate_grad_hook(self._mark(i)))
        self.shadow_base = (torch.from_numpy(shadow_base.view(np.int64)).to(self.device)
                            if self.shadowed.any() else None)
        # where each shadowed bf16 model weight lived when shadow_base was taken: the AdamW
        # kernel writes there, so check_shadows() refuses to launch if one has moved
        self._shadow_ptrs = {int(i): self.params[i].data_ptr() for i in np.nonzero(self.shadowed)[0]}
        self._chunk_cache: Dict[tuple, tuple] = {}
        self._index_cache: Dict[tuple, torch.Tensor] = {}
        # persistent pinned staging slots for the per-step host->device tables (gather pieces, AdamW
        # scalars): a fresh pinned allocation per call, whenever the caching host allocator had no
        # free block, could synchronise the device -- the bench trace showed the GPU idle for up to
        # 7.6 ms in the optimizer phase (profiles/r05_bench_kernel_trace_summary.csv)
        self._stage = [(None, None)] * 8
        self._stage_next = 0
        self._held = None   # (.grad tensors read by the last gather launch, its completion event)

    def check_shadows(self, ids: Sequence[int]):
        """Raise if a shadowed parameter's bf16 storage was reallocated (model.to(), p.data = ...)
        since the flat space was built: the step would otherwise write into freed memory."""
        for i in ids:
            want = self._shadow_ptrs.get(int(i))
            if want is not None and self.params[i].data_ptr() != want:
                raise TriadError(f"parameter {i} ({tuple(self.params[i].shape)}) was reallocated after the "
                                 "optimizer was built; rebuild the trainer (FlatParamSpace) after moving the model")

    def _mark(self, i):
        def hook(_p):
            self.touched[i] = True
        return hook

    def param_ids(self, params: Iterable[torch.nn.Parameter]):
        return [self.index[id(p)] for p in params if id(p) in self.index]

    def chunks(self, ids: Sequence[int]):
        """Device chunk table for the given parameter indices (cached)."""
        key = tuple(ids)
        hit = self._chunk_cache.get(key)
        if hit is not None:
            return hit
        rows = []
        for i in ids:
            n = self.params[i].numel()
            for s in range(0, n, CHUNK):
                rows.append((self.offsets[i] + s, min(CHUNK, n - s), i))
        arr = np.array(rows, dtype=_CHUNK_DT) if rows else np.zeros(0, dtype=_CHUNK_DT)
        dev = _lib.h2d(torch.from_numpy(arr.view(np.uint8).copy()), self.device) if rows else None
        owner = _lib.h2d(torch.tensor([r[2] for r in rows], dtype=torch.long), self.device) if rows else None
        out = (dev, len(rows), owner)
        if len(self._chunk_cache) > 64:
            self._chunk_cache.clear()
        self._chunk_cache[key] = out
        return out

    def index_tensor(self, ids: Sequence[int]) -> torch.Tensor:
        """Device int64 tensor of parameter ids (cached: the same few id sets recur every step,
        and each fresh host->device copy would be a host sync)."""
        key = tuple(ids)
        t = self._index_cache.get(key)
        if t is None:
            if len(self._index_cache) > 64:
                self._index_cache.clear()
            t = _lib.h2d(torch.tensor(list(key), dtype=torch.long), self.device)
            self._index_cache[key] = t
        return t

    def touched_ids(self, ids: Sequence[int]):
        return [i for i in ids if self.touched[i]]

    def param_sumsq(self, ids: Sequence[int]) -> torch.Tensor:
        """Per-parameter sum of squared gradients (float64, indexed by parameter id). The per-chunk
        partials are summed per parameter by a segmented reduction over the chunk table (ordered by
        parameter), not index_add_'s atomics: the clip coefficient is then the same every run."""
        ids = sorted(set(int(i) for i in ids))
        table, n, owner = self.chunks(ids)
        if not n:
            return torch.zeros(len(self.params), dtype=torch.float64, device=self.device)
        part = torch.empty(n, dtype=torch.float64, device=self.device)
        call("triad_grad_sumsq", ptr(self.flat_g), ptr(table), n, ptr(part), stream_ptr(self.device))
        return torch.segment_reduce(part, "sum", lengths=self._segment_lengths(ids), unsafe=True)

    def _segment_lengths(self, ids: Sequence[int]) -> torch.Tensor:
        """Chunks per parameter id (0 for the ids not in `ids`) as a device int64 tensor (cached)."""
        key = ("seg",) + tuple(ids)
        t = self._index_cache.get(key)
        if t is None:
            lens = [0] * len(self.params)
            for i in ids:
                lens[i] = (self.params[i].numel() + CHUNK - 1) // CHUNK
            if len(self._index_cache) > 64:
                self._index_cache.clear()
            t = _lib.h2d(torch.tensor(lens, dtype=torch.long), self.device)
            self._index_cache[key] = t
        return t

    def master(self, i: int) -> torch.Tensor:
        """fp32 master of parameter i (a view of the flat buffer)."""
        p = self.params[i]
        return self.flat_p[self.offsets[i]:self.offsets[i] + p.numel()].view(p.shape)

    def _h2d(self, raw: np.ndarray) -> torch.Tensor:
        """Host bytes -> a fresh device uint8 tensor, copied on the current stream through the ring
        of pinned staging slots (a slot is rewritten only after the copy that last used it has
        completed -- several launches, i.e. about a step, earlier)."""
        raw = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
        if self.device.type != "cuda":
            return torch.from_numpy(raw.copy())
        n = raw.nbytes
        slot = self._stage_next
        self._stage_next = (slot + 1) % len(self._stage)
        buf, ev = self._stage[slot]
        if ev is not None:
            ev.synchronize()
        if buf is None or buf.numel() < n:
            buf = torch.empty(max(2 * n, 1 << 16), dtype=torch.uint8, pin_memory=True)
        buf[:n].numpy()[:] = raw
        out = torch.empty(n, dtype=torch.uint8, device=self.device)
        out.copy_(buf[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._stage[slot] = (buf, ev)
        return out

    @torch.no_grad()
    def gather_shadow_grads(self, accumulate: bool):
        """.grad of the gathered parameters (bf16 for the shadowed ones, fp32 for the rest) ->
        flat fp32 gradient buffer (one launch); the .grad tensors are released (stream-ordered
        reuse by the caching allocator)."""
        if not self.gathered.any():
            return
        if self._held is not None:   # the previous gather has read its .grad tensors: release them
            self._held[1].synchronize()
            self._held = None
        self._gather_launch(accumulate)

    def release_held_grads(self):
        """Drop the .grad tensors the last gather read as soon as its launch has run (a non-blocking
        event query; TriadTrainer.step polls it at the step's start and before backward), so the
        caching allocator can reuse them during the step instead of only at the next gather."""
        if self._held is not None and self._held[1].query():
            self._held = None

    def _gather_launch(self, accumulate: bool):
        src, dst, cnt, f32s, ids, grads = [], [], [], [], [], []
        for i in np.nonzero(self.gathered)[0]:
            p = self.params[i]
            gr = p.grad
            if gr is None:
                continue
            dt = torch.bfloat16 if self.shadowed[i] else torch.float32
            if gr.dtype != dt or not gr.is_contiguous():
                gr = gr.to(dt).contiguous()
            n, f32 = gr.numel(), int(dt == torch.float32)
            s0 = np.arange(0, n, CHUNK, dtype=np.int64)
            src.append(gr.data_ptr() + (2 + 2 * f32) * s0)
            dst.append(self.offsets[i] + s0)
            cnt.append(np.minimum(CHUNK, n - s0))
            f32s.append(np.full(len(s0), f32, dtype=np.int32))
            ids.append(int(i))
            grads.append(gr)
        if not ids:
            return
        arr = np.empty(sum(len(a) for a in src), dtype=_PIECE_DT)
        arr["src"] = np.concatenate(src).astype(np.uint64)
        arr["dst"] = np.concatenate(dst)
        arr["n"] = np.concatenate(cnt)
        arr["f32"] = np.concatenate(f32s)
        table = self._h2d(arr)
        call("triad_gather_grads", ptr(table), len(arr), ptr(self.flat_g), int(accumulate and True),
             stream_ptr(self.device))
        if self.device.type == "cuda":
            # gradients made on other streams (side-stream dW, modality streams) stay referenced
            # until this launch has read them (instead of one record_stream per parameter)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._held = (grads, ev)
        for i in ids:
            self.params[i].grad = None
        self.touched[ids] = True

    def zero_grad(self, ids: Sequence[int]):
        """Zero the gradient slots of these parameters (contiguous runs -> few memsets)."""
        ids = sorted(ids)
        s = 0
        while s < len(ids):
            e = s
            while e + 1 < len(ids) and ids[e + 1] == ids[e] + 1:
                e += 1
            a = self.offsets[ids[s]]
            b = self.offsets[ids[e]] + self.params[ids[e]].numel()
            self.flat_g[a:b].zero_()
            s = e + 1
        if ids:
            self.touched[ids] = False
            self.scale.index_fill_(0, self.index_tensor(ids), 1.0)
            for i in ids:
                if self.gathered[i]:
                    self.params[i].grad = None


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW-compatible facade over a FlatParamSpace (one per reference optimizer),
    so torch's LR schedulers (OneCycleLR, incl. beta1 cycling) drive it unchanged."""

    def __init__(self, space: FlatParamSpace, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        params = list(params)
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.space = space
        self.ids = space.param_ids(params)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        sp = self.space
        ids = sp.touched_ids(self.ids)  # torch skips parameters whose .grad is None
        if not ids:
            return loss
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
        # per-parameter {lr / bc1, 1 / sqrt(bc2), 1 - lr wd} (float64 on the host, as torch computes
        # them), staged through the space's pinned ring
        idx = np.asarray(ids, dtype=np.int64)
        sp.steps[idx] += 1
        t = sp.steps[idx].astype(np.float64)
        pp = np.zeros((len(sp.params), 3), dtype=np.float32)
        pp[idx, 0] = lr / (1.0 - b1 ** t)
        pp[idx, 1] = 1.0 / np.sqrt(1.0 - b2 ** t)
        pp[idx, 2] = 1.0 - lr * wd
        pp_dev = sp._h2d(pp).view(torch.float32)
        sp.check_shadows(ids)
        table, n, _ = sp.chunks(ids)
        call("triad_adamw_step", ptr(sp.flat_p), ptr(sp.flat_g), ptr(sp.exp_avg), ptr(sp.exp_avg_sq), ptr(table), n,
             ptr(pp_dev), ptr(sp.scale), float(b1), float(b2), float(1.0 - b1), float(1.0 - b2), float(eps),
             ptr(sp.shadow_base),
             stream_ptr(sp.device))
        return loss

    def zero_grad(self, set_to_none: bool = False):
        self.space.zero_grad(self.ids)

    # torch.optim.AdamW's state_dict format, so reference checkpoints (train.py:412-415,
    # 460-463) load here and ours load into torch: per-parameter {"step" (CPU f32 tensor),
    # "exp_avg", "exp_avg_sq"} keyed by position, one param group with AdamW's keys.
    def state_dict(self):
        sp = self.space
        state = {}
        for k, i in enumerate(self.ids):
            if sp.steps[i] > 0:
                p, o = sp.params[i], sp.offsets[i]
                n = p.numel()
                state[k] = {"step": torch.tensor(float(sp.steps[i])),
                            "exp_avg": sp.exp_avg[o:o + n].view_as(p).clone(),
                            "exp_avg_sq": sp.exp_avg_sq[o:o + n].view_as(p).clone()}
        groups = []
        for g in self.param_groups:
            d = dict(_ADAMW_GROUP_DEFAULTS)
            d.update({k: v for k, v in g.items() if k != "params"})
            d["params"] = list(range(len(self.ids)))
            groups.append(d)
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, sd):
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self.ids):
            raise ValueError("optimizer state does not match this parameter group")
        for k, v in groups[0].items():
            if k != "params" and k in self.param_groups[0] or k in ("initial_lr", "max_lr", "min_lr",
                                                                     "max_momentum", "base_momentum"):
                self.param_groups[0][k] = tuple(v) if k == "betas" else v
        sp = self.space
        for k, i in enumerate(self.ids):
            st = sd["state"].get(k, sd["state"].get(str(k)))
            o, p = sp.offsets[i], sp.params[i]
            n = p.numel()
            if st is None:
                sp.steps[i] = 0
                sp.exp_avg[o:o + n].zero_()
                sp.exp_avg_sq[o:o + n].zero_()
                continue
            sp.steps[i] = int(float(st["step"]))
            sp.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1).to(sp.exp_avg))
            sp.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1).to(sp.exp_avg_sq))


def _adamw_group_defaults():
    d = torch.optim.AdamW([torch.zeros(1, requires_grad=True)]).param_groups[0]
    return {k: v for k, v in d.items() if k != "params"}


_ADAMW_GROUP_DEFAULTS = _adamw_group_defaults()


def grad_norms(space: FlatParamSpace, groups: Dict[str, Sequence[torch.nn.Parameter]]):
    """{name: ||grad||_2} per group as device scalars (no host sync), train.py:992-1002."""
    ids_all = space.touched_ids(range(len(space.params)))
    sq = space.param_sumsq(ids_all)
    out = {}
    for name, params in groups.items():
        ids = [i for i in space.param_ids(params) if space.touched[i]]
        if ids:
            out[name] = sq[space.index_tensor(ids)].sum().sqrt().float()
        else:
            out[name] = torch.zeros((), device=space.device)
    return out, sq


def clip_grad_norm_(space: FlatParamSpace, params, max_norm: float, sq: torch.Tensor = None):
    """torch.nn.utils.clip_grad_norm_ semantics (2-norm, clip_coef = max_norm/(norm+1e-6)
    clamped to 1), applied lazily as the per-parameter scale of the next AdamW launch.
    Returns the total norm (device scalar)."""
    ids = [i for i in space.param_ids(params) if space.touched[i]]
    if not ids:
        return torch.zeros((), device=space.device)
    if sq is None:
        sq = space.param_sumsq(ids)
    idx = space.index_tensor(ids)
    total = sq[idx].sum().sqrt().float()
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    space.scale[idx] = space.scale[idx] * coef
    return total
