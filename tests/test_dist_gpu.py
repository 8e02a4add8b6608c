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
        dt += gt
    assert abs(dt - float(t.grad)) <= 1e-3 * abs(float(t.grad)) + 1e-6
