"""Which side of the Mode G TriadTrainer comparison (tests/test_dist_gpu.py::
test_mode_g_trainer_two_ranks_with_unfreeze_flip) moves when HuBERT is trainable: the two gloo
ranks and the single process at B_g = 4, each with the modality streams + side-stream weight
gradients on ("on") and fully serialised ("off"), the single process twice per mode. Prints the
step-1 audio / others group errors of every pair of runs (the single processes start step 1 from
rank 0's parameters after step 0, as the test does).

    python tools/mode_g_diag2.py
"""
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_dist_gpu as T  # noqa: E402
from triad_amd import linear as L  # noqa: E402


def _set_mode(on):
    os.environ["TRIAD_MODALITY_STREAMS"] = "1" if on else "0"
    os.environ["TRIAD_SIDE_STREAM_DW"] = "1" if on else "0"
    L.SIDE_STREAM_DW = on


def ranks(on):
    _set_mode(on)
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = T._port()
    procs = [ctx.Process(target=T._mode_g_trainer_worker, args=(r, 2, port, qo, 1)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([qo.get(timeout=600) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        if isinstance(r[1], str):
            raise RuntimeError(r[2])
    (_, g0, p0, l0, _), (_, g1, _, l1, _) = res
    assert all(np.array_equal(a, b) for a, b in zip(g0, g1)), "ranks' reduced gradients differ"
    return g0, p0, l0


def single(on, p0):
    _set_mode(on)
    m = T._mode_r_model()
    m.audio_embedder.normalize = T._no_znorm
    m.visual_embedder.set_global_mask(1, 0)
    T._embed_in_chunks(m, 2)
    tr = T._mode_g_trainer(m, None)
    losses = []
    for step in range(2):
        if step:
            T._load_flat_params(tr, p0[step - 1])
        b0, b1 = T._mode_r_batch(step, 0), T._mode_r_batch(step, 1)
        out = tr.step(torch.cat([b0[0], b1[0]]), torch.cat([b0[1], b1[1]]), list(b0[2]) + list(b1[2]),
                      phase="full_joint")
        losses.append(float(out["loss"]))
    torch.cuda.synchronize()
    return [g.cpu().numpy() for g in tr.reduced], losses, (m, tr)


def main():
    runs = {}
    g, p0, l = ranks(True)
    runs["ranks_on"] = (g, l)
    print("ranks_on losses", l, flush=True)
    g, _, l = ranks(False)
    runs["ranks_off"] = (g, l)
    print("ranks_off losses", l, flush=True)
    mt = None
    for tag, on in (("single_on_a", True), ("single_on_b", True), ("single_off", False)):
        g, l, mt = single(on, p0)
        runs[tag] = (g, l)
        print(tag, "losses", l, flush=True)
    m, tr = mt
    names = list(runs)
    for i, a in enumerate(names):
        for b in names[i + 1:]:
            ga, gb = runs[a][0][1], runs[b][0][1]
            rel = T._group_rel(tr, ga, gb)
            worst = T._worst_params(m, tr, ga, gb, tr.groups["audio"], k=4)
            print(f"step 1 {a} vs {b}: equal {bool(np.array_equal(ga, gb))} rel {rel}\n   worst audio {worst}",
                  flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
