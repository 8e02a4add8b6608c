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
