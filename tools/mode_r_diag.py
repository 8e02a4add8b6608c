"""Diagnose Mode R parity: per parameter group, relative difference of the two-step update of
(a) a second single-process run, (b) 2 ranks with the serial all-reduce, (c) 2 ranks with the
overlapped bucket reducer -- each against the single-process accumulated run. (Found: two
single-process runs already differ by 0.2-0.6 in the update -- AdamW's first steps are
~lr*sign(g), which turns noise in near-zero gradients into full-size differences -- so
tests/test_dist_gpu.py compares reduced gradients instead.)"""
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_dist_gpu as T  # noqa: E402


def groups(tr):
    sp = tr.space
    out = {}
    for name, ps in tr.groups.items():
        ids = sp.param_ids(ps)
        out[name] = [(sp.offsets[i], sp.params[i].numel()) for i in ids]
    return out


def worker(rank, world, port, overlap, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from triad_amd.train import TriadTrainer
    m = T._mode_r_model()
    tr = TriadTrainer(m, learning_rate=1e-4, total_updates=50, gradient_accumulation_steps=1, unfreeze_audio_step=0,
                      unfreeze_text_step=0, process_group=dist.group.WORLD, bucket_mb=16.0,
                      overlap_grad_reduce=overlap)
    p0 = tr.space.flat_p.clone()
    for step in range(2):
        f, a, t, ak, tk = T._mode_r_batch(step, rank)
        tr.step(f, a, t, phase="full_joint", av_keep=ak, tv_keep=tk)
    torch.cuda.synchronize()
    q.put((rank, (tr.space.flat_p - p0).cpu().numpy()))
    dist.destroy_process_group()


def dist_run(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = T._port()
    ps = [ctx.Process(target=worker, args=(r, 2, port, overlap, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(2)], key=lambda r: r[0])
    for p in ps:
        p.join()
    return res[0][1], res[1][1]


def single():
    m = T._mode_r_model()
    tr = T._trainer(m, 2)
    p0 = tr.space.flat_p.clone()
    for step in range(2):
        for rank in range(2):
            f, a, t, ak, tk = T._mode_r_batch(step, rank)
            tr.step(f, a, t, phase="full_joint", av_keep=ak, tv_keep=tk)
    return (tr.space.flat_p - p0).cpu().numpy(), groups(tr)


def report(tag, d, ref, gr):
    parts = []
    for name, spans in gr.items():
        if not spans:
            continue
        a = np.concatenate([d[o:o + n] for o, n in spans])
        b = np.concatenate([ref[o:o + n] for o, n in spans])
        parts.append(f"{name} {np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30):.2e}")
    print(tag, " | ".join(parts), flush=True)


if __name__ == "__main__":
    ref, gr = single()
    ref2, _ = single()
    report("single vs single", ref2, ref, gr)
    for ov in (False, True):
        d0, d1 = dist_run(ov)
        report(f"dist overlap={ov} rank0", d0, ref, gr)
        report(f"dist overlap={ov} rank1", d1, ref, gr)
