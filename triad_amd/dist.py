"""Collectives of the data-parallel hot path (one process per GPU, RCCL over xGMI).

The reference has no distributed code (no DDP / NCCL call sites). Two
modes are provided:

  Mode R (replicas, local negatives): every rank runs the reference loss on its own
    B_l triples; the trainer averages the flat gradient buffer (bucketed all-reduce,
    triad_amd.train.TriadTrainer._allreduce_grads).

  Mode G (global negatives, B_g = W * B_l): the projected visual key tokens are
    all-gathered (`gather_keys`), each rank computes its B_l query rows of the
    (B_g x B_g) clip matrix against every key, the clip row blocks are all-gathered
    (`gather_rows`) so every rank evaluates the identical loss head, the l_nonneg /
    diagonal partial sums are all-reduced (`allreduce_sum`), and in backward the key
    gradients of all B_g samples are reduce-scattered back to their owners
    (`reduce_scatter_rows`). The loss equals the reference loss at B = B_g; gradients
    are the full-loss gradients, summed (not averaged) across ranks.

The helpers take any process group; on `gloo` (CPU tests) the tensor collectives that
gloo lacks are composed from all_reduce / all_gather.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world_rank(group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _is_nccl(group):
    return dist.get_backend(group) == "nccl"


def gather_keys(local: torch.Tensor, out_rows: int, group=None) -> torch.Tensor:
    """All-gather equal row blocks [rows_l][...] -> [out_rows][...] (rank-major), zero tail."""
    W, _ = world_rank(group)
    rows_l = local.shape[0]
    out = torch.empty((out_rows,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    body = out[:W * rows_l]
    if _is_nccl(group):
        dist.all_gather_into_tensor(body, local.contiguous(), group=group)
    else:
        dist.all_gather(list(body.chunk(W)), local.contiguous(), group=group)
    if out_rows > W * rows_l:
        out[W * rows_l:].zero_()
    return out


def gather_rows(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather row blocks of a matrix: (rows_l, n) per rank -> (W*rows_l, n)."""
    return gather_keys(local, world_rank(group)[0] * local.shape[0], group)


def allreduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def reduce_scatter_rows(full: torch.Tensor, rows_l: int, group=None) -> torch.Tensor:
    """Sum row-blocked contributions over ranks and keep this rank's block:
    full [>= W*rows_l][...] (rank-major blocks) -> [rows_l][...]."""
    W, r = world_rank(group)
    body = full[:W * rows_l].contiguous()
    out = torch.empty((rows_l,) + tuple(full.shape[1:]), dtype=full.dtype, device=full.device)
    if _is_nccl(group):
        dist.reduce_scatter_tensor(out, body, op=dist.ReduceOp.SUM, group=group)
    else:
        dist.all_reduce(body, op=dist.ReduceOp.SUM, group=group)
        out.copy_(body[r * rows_l:(r + 1) * rows_l])
    return out


def agree_touched(space, group=None):
    """After a data-parallel reduction: a parameter has a gradient iff SOME rank's backward
    produced one (OR of the ranks' touched sets, every rank ends with the same set).

    The reduced buffer then holds the same value for every parameter on every rank -- the
    average (or sum) with zeros for ranks that did not produce it (HuBERT's LayerDrop draws
    differ per rank) -- so those parameters are stepped, counted and clipped identically
    everywhere, as DDP's reduced buckets are. A parameter no rank produced a gradient for (the
    idle modality of an av_focus / tv_warmup step, or a layer every rank dropped) stays
    untouched, so AdamW skips it exactly as torch skips a parameter whose .grad is None
    (SajayR/TRIAD train.py:1010-1040) -- no weight decay, no momentum step, no step count.

    The touched set is host state that the gradient hooks fill as backward runs on the host, so
    the OR needs no device work: on a `gloo` group it is a host collective that does not wait for
    the GPU (TriadTrainer passes a gloo group for an RCCL job); on an `nccl` group it goes through
    the device and synchronises once."""
    W, _ = world_rank(group)
    if W <= 1:
        return
    import numpy as np
    trainable = np.array([bool(p.requires_grad) for p in space.params], dtype=bool)
    local = torch.from_numpy((space.touched & trainable).astype(np.uint8))
    if _is_nccl(group):
        t = local.to(space.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        local = t.cpu()
    else:
        dist.all_reduce(local, op=dist.ReduceOp.MAX, group=group)
    space.touched[:] = local.numpy().astype(bool)


def allreduce_grads(flat: torch.Tensor, bucket_elems: int, average: bool, group=None):
    """Bucketed all-reduce of a flat gradient buffer (Mode R: average, Mode G: sum)."""
    W, _ = world_rank(group)
    if W <= 1:
        return
    # SUM then scale: ReduceOp.AVG needs the collective library's avg op, not guaranteed on
    # every RCCL build; the scale is one streaming pass per bucket
    for s in range(0, flat.numel(), bucket_elems):
        b = flat[s:s + bucket_elems]
        dist.all_reduce(b, op=dist.ReduceOp.SUM, group=group)
        if average:
            b.mul_(1.0 / W)


class GradBucketReducer:
    """Mode R / Mode G gradient reduction overlapped with backward.

    The flat fp32 gradient buffer of a FlatParamSpace is cut into contiguous buckets of about
    `bucket_mb` (parameter-aligned ranges of the buffer). A post-accumulate-grad hook on every
    parameter counts arrivals; when a bucket's last expected gradient has been accumulated, the
    bucket is handed to a dedicated communication stream (which first waits on every stream its
    gradients were produced on) and all-reduced asynchronously while autograd continues with the
    earlier layers. `finish()` flushes buckets whose gradients never came (unused in this phase),
    makes the caller's stream wait on every reduction, and scatters bf16 wire buffers back.

    Launch order is a property of the job, not of one rank's timing: a bucket is launched only
    after every bucket before it in `order` -- collectives must be issued in the same sequence on
    every rank. The first reducing step reduces after backward in buffer order while recording
    when each parameter's gradient arrived; `order` is then rank 0's arrival order of the buckets,
    broadcast to all ranks, and from the next step on the reductions overlap backward.

    Wire format: "fp32" all-reduces the buffer in place (prescaled by 1/W when averaging);
    "bf16" prescales, casts each bucket to bf16 and all-reduces that (half the xGMI bytes; the
    sum of W bf16 terms carries bf16 rounding, ~2^-9 relative per element). Bucket size: ring
    all-reduce over point-to-point xGMI is per-link bound, so buckets are sized for a few
    ms of link time each (64 MB default) rather than for latency.

    Gathered parameters (FlatParamSpace.gathered: the bf16 model weights and, on a GPU, the fp32
    ones): their autograd gradient is folded into the flat fp32 buffer inside the hook (so it can
    join a bucket) instead of by the single after-backward `gather_shadow_grads` launch.
    """

    def __init__(self, space, bucket_mb: float = 64.0, wire: str = "fp32", average: bool = True, group=None,
                 mask_group=None):
        if wire not in ("fp32", "bf16"):
            raise ValueError(f"wire must be 'fp32' or 'bf16', not {wire!r}")
        self.space, self.wire, self.average, self.group = space, wire, average, group
        self.mask_group = mask_group   # host (gloo) group for the touched-set OR; None: `group`
        self.world, _ = world_rank(group)
        self.cuda = space.device.type == "cuda"
        n = len(space.params)
        bounds, acc, start = [], 0, 0
        limit = max(1, int(bucket_mb * (1 << 20) / 4))
        for i in range(n):
            acc += space.params[i].numel()
            if acc >= limit or i == n - 1:
                bounds.append((start, i + 1))
                start, acc = i + 1, 0
        self.buckets = bounds                                   # parameter-index ranges
        self.bucket_of = [0] * n
        for b, (s, e) in enumerate(bounds):
            for i in range(s, e):
                self.bucket_of[i] = b
        self.order = None                                       # launch order (bucket ids)
        self._trainable = None                                  # requires_grad pattern `order` was fixed for
        self.active = False
        self.comm = torch.cuda.Stream(space.device) if self.cuda else None
        self.launched_in_backward = 0                           # overlap evidence (tests, logs)
        self._hooks = {}   # registered lazily: a frozen parameter (requires_grad False) takes no hook
        # correctness gate (bench.py --gpus N > 1): with `check` set for a step, each
        # bucket's local gradient is snapshotted right before its overlapped all-reduce, and after the
        # step the same buckets are all-reduced again from the snapshots in the same order with the
        # device otherwise idle; `check_result` compares the two bit for bit (max over ranks)
        self.check = False
        self.check_result = None
        self._snap = None

    def _arm_hooks(self):
        for i, p in enumerate(self.space.params):
            if p.requires_grad and i not in self._hooks:
                self._hooks[i] = p.register_post_accumulate_grad_hook(self._hook(i))

    # -- per step ------------------------------------------------------------------------
    def begin(self, accumulate: bool):
        """Arm the hooks for the backward that completes an accumulation window."""
        sp = self.space
        self._arm_hooks()
        trainable = tuple(bool(p.requires_grad) for p in sp.params)
        if trainable != self._trainable:
            # a staged unfreeze (train.py:527-548) changed which buckets take part: re-derive the
            # launch order at this step (reduce after backward, record, broadcast) -- every rank
            # flips at the same global step, so every rank resets here
            self.order = None
            self._trainable = trainable
        self.accumulate = accumulate
        self.expected = [0] * len(self.buckets)
        for i, p in enumerate(sp.params):
            if p.requires_grad:
                self.expected[self.bucket_of[i]] += 1
        self.arrived = [0] * len(self.buckets)
        self.streams = [set() for _ in self.buckets]
        self.ready = [False] * len(self.buckets)
        self.works = {}
        self.next = 0                                           # position in self.order
        self.arrival = [] if self.order is None else None
        self.launched_in_backward = 0
        self.active = True

    def _hook(self, i):
        def hook(p):
            if not self.active:
                return
            sp = self.space
            cur = torch.cuda.current_stream(sp.device) if self.cuda else None
            if sp.gathered[i] and p.grad is not None:
                view = sp.flat_g[sp.offsets[i]:sp.offsets[i] + p.numel()].view(p.shape)
                if cur is not None:
                    # a bf16 weight gradient may still be in flight on the side stream
                    # (linear.on_side_stream: autograd stored it without a main-stream wait), so
                    # fold it on that stream, after the work this stream has queued so far
                    from .linear import _side_stream
                    side = _side_stream(sp.device)
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        view.add_(p.grad) if self.accumulate else view.copy_(p.grad)
                    p.grad.record_stream(side)
                    cur = side
                elif self.accumulate:
                    view.add_(p.grad)
                else:
                    view.copy_(p.grad)
                p.grad = None
                sp.touched[i] = True
            b = self.bucket_of[i]
            self.arrived[b] += 1
            if cur is not None:
                self.streams[b].add(cur)
            if self.arrival is not None:
                self.arrival.append(b)
            if self.arrived[b] == self.expected[b]:
                self.ready[b] = True
                if self.order is not None:
                    self._drain(in_backward=True)
        return hook

    def _drain(self, in_backward=False, flush=False):
        while self.next < len(self.order):
            b = self.order[self.next]
            if not (self.ready[b] or flush):
                return
            self._launch(b)
            self.next += 1
            if in_backward:
                self.launched_in_backward += 1

    def _range(self, b):
        s, e = self.buckets[b]
        sp = self.space
        hi = sp.offsets[e] if e < len(sp.params) else sp.numel
        return sp.flat_g[sp.offsets[s]:hi]

    def _launch(self, b):
        if self.expected[b] == 0:       # every parameter frozen (identically on all ranks): nothing to reduce
            self.works[b] = None
            return
        g = self._range(b)
        scale = 1.0 / self.world if self.average else 1.0
        if not self.cuda:
            if self.check:
                self._snap_range(b).copy_(g)
            if scale != 1.0:
                g.mul_(scale)
            buf = g.to(torch.bfloat16) if self.wire == "bf16" else g
            self.works[b] = (dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True), buf)
            return
        for s in self.streams[b] or {torch.cuda.current_stream(self.space.device)}:
            self.comm.wait_stream(s)
        with torch.cuda.stream(self.comm):
            if self.check:
                self._snap_range(b).copy_(g)
            if scale != 1.0:
                g.mul_(scale)
            buf = g.to(torch.bfloat16) if self.wire == "bf16" else g
            work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.works[b] = (work, buf)

    def _snap_range(self, b):
        if self._snap is None or self._snap.numel() != self.space.flat_g.numel():
            self._snap = torch.empty_like(self.space.flat_g)
        s, e = self.buckets[b]
        sp = self.space
        hi = sp.offsets[e] if e < len(sp.params) else sp.numel
        return self._snap[sp.offsets[s]:hi]

    def _check_reference(self):
        """The same buckets all-reduced again from their pre-reduction snapshots, in the same order,
        one at a time with the device otherwise idle (no backward kernel co-resident with the
        collective); compared bit for bit with what the overlapped reductions produced."""
        dev = self.space.device
        if self.cuda:
            torch.cuda.synchronize(dev)
        scale = 1.0 / self.world if self.average else 1.0
        launched = [b for b in self.order if self.expected[b] > 0]
        max_abs, differ = 0.0, 0
        for b in launched:
            ref = self._snap_range(b)
            if scale != 1.0:
                ref.mul_(scale)
            buf = ref.to(torch.bfloat16) if self.wire == "bf16" else ref
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            if self.wire == "bf16":
                ref.copy_(buf)
            got = self._range(b)
            d = (got - ref).abs()
            max_abs = max(max_abs, float(d.max())) if d.numel() else max_abs
            differ += int((got != ref).sum())
        if self.cuda:
            torch.cuda.synchronize(dev)
        t = torch.tensor([max_abs, float(differ)], dtype=torch.float64,
                         device=dev if _is_nccl(self.group) else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        self.check_result = {"equal": bool(t[1] == 0), "max_abs": float(t[0]), "differing_elements_max_rank": int(t[1]),
                             "world_size": self.world, "backend": dist.get_backend(self.group),
                             "buckets": len(launched), "launched_in_backward": self.launched_in_backward,
                             "wire": self.wire}

    def finish(self):
        """After backward: flush, then order the caller's stream after every reduction."""
        if not self.active:
            return
        self.active = False
        if self.order is None:
            # first reducing step: fix the launch order from rank 0's arrival order
            first = {}
            for k, b in enumerate(self.arrival):
                first[b] = k                                    # last arrival = bucket ready time
            rank_order = sorted(range(len(self.buckets)), key=lambda b: (first.get(b, 1 << 60), b))
            t = torch.tensor(rank_order, dtype=torch.int64,
                             device=self.space.device if _is_nccl(self.group) else "cpu")
            dist.broadcast(t, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0,
                           group=self.group)
            self.order = [int(x) for x in t.cpu()]
            self.arrival = None
        self._drain(flush=True)
        agree_touched(self.space, self.mask_group if self.mask_group is not None else self.group)
        cur = torch.cuda.current_stream(self.space.device) if self.cuda else None
        for b in self.order:
            item = self.works.pop(b)
            if item is None:
                continue
            work, buf = item
            work.wait()                                         # cur stream (GPU) / host (gloo) waits
            if self.wire == "bf16":
                if cur is not None:
                    buf.record_stream(cur)
                self._range(b).copy_(buf)
        if self.check:
            self._check_reference()
            self.check = False
