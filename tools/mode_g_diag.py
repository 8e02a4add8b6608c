"""Diagnostic for the Mode G TriadTrainer comparison (tests/test_dist_gpu.py): two gloo ranks on
the box's one GPU against one process at B_g = 4, per parameter group and the worst parameters of
each group, for a chosen unfreeze step.

    python tools/mode_g_diag.py [unfreeze_audio_step]   [nostreams]
"""
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_dist_gpu as T  # noqa: E402


def main():
    unf = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    if "nostreams" in sys.argv[2:]:
        os.environ["TRIAD_MODALITY_STREAMS"] = "0"
    world = 2
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = T._port()
    procs = [ctx.Process(target=T._mode_g_trainer_worker, args=(r, world, port, qo, unf)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([qo.get(timeout=600) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        if isinstance(r[1], str):
            print(r[2])
            return 1
    (_, g0, p0, l0, t0), (_, g1, p1, l1, t1) = res
    print(f"unfreeze_audio_step={unf} streams={os.environ.get('TRIAD_MODALITY_STREAMS', '1')}: losses {l0} / {l1}; "
          f"ranks' reduced gradients equal: {[bool(np.array_equal(a, b)) for a, b in zip(g0, g1)]}")
    m = T._mode_r_model()
    m.audio_embedder.normalize = T._no_znorm
    m.visual_embedder.set_global_mask(1, 0)
    T._embed_in_chunks(m, 2)
    tr = T._mode_g_trainer(m, None, unf)
    for step in range(2):
        b0, b1 = T._mode_r_batch(step, 0), T._mode_r_batch(step, 1)
        out = tr.step(torch.cat([b0[0], b1[0]]), torch.cat([b0[1], b1[1]]), list(b0[2]) + list(b1[2]),
                      phase="full_joint")
        ref = tr.reduced[step].cpu().numpy()
        print(f"step {step}: loss {float(out['loss'])} vs {l0[step]}; group rel {T._group_rel(tr, g0[step], ref)}")
        for name, ps in tr.groups.items():
            print(f"  worst {name}: {T._worst_params(m, tr, g0[step], ref, ps, k=5)}")
        sp = tr.space
        zero_rank = [i for i, p in enumerate(sp.params) if p.requires_grad
                     and not np.any(g0[step][sp.offsets[i]:sp.offsets[i] + p.numel()])
                     and np.any(ref[sp.offsets[i]:sp.offsets[i] + p.numel()])]
        print(f"  params zero on the ranks but not in the single process: {len(zero_rank)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
