"""Which backward nodes make a modality / main stream wait for the weight-gradient side stream?

Builds the bench model and trainer, runs warm-up steps, then one step with linear.side_stream_ok
wrapped: every call that returns False because the weight was already claimed in this backward
pass (its second use, linear.py) -- the path that makes the calling stream wait for the side
stream -- is logged with the weight's shape and the calling stream. Experiments only.

usage: python tools/side_waits.py
"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from triad_amd import _lib, blas
    blas.configure()
    import bench
    from triad_amd import linear
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer
    dev = torch.device("cuda", 0)
    _lib.load()
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(1234)
    model = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.80, patch_sparsity_weight=0.01,
                            visual_dropout_prob=0.25, use_amp=True).to(dev)
    model.train()
    tr = TriadTrainer(model, learning_rate=1e-4, total_updates=100000, unfreeze_audio_step=0,
                      unfreeze_text_step=0, unfreeze_vit_step=0, device=dev)
    frames, audio, text = bench.synthetic(256, 0, dev)
    names = {id(p): n for n, p in model.named_parameters()}
    names.update({id(p): "shadow:" + n for n, p in getattr(tr, "named_shadows", lambda: [])()})
    log = collections.Counter()
    calls = collections.Counter()
    orig = linear.side_stream_ok

    def wrapped(*ws):
        dev_ = ws[0].device
        di = linear._dev_index(dev_)
        task = torch._C._current_graph_task_id()
        t, seen = linear._CLAIMED.get(di, (None, None))
        second = t == task and seen is not None and any(id(w) in seen for w in ws)
        r = orig(*ws)
        key = (tuple(tuple(w.shape) for w in ws), torch.cuda.current_stream(dev_).stream_id)
        calls[(r, second)] += 1
        if second:
            log[key + (",".join(names.get(id(w), "?") for w in ws),)] += 1
        return r

    linear.side_stream_ok = wrapped
    for _ in range(2):
        tr.step(frames, audio, text, phase="full_joint")
    torch.cuda.synchronize()
    log.clear()
    calls.clear()
    tr.step(frames, audio, text, phase="full_joint")
    torch.cuda.synchronize()
    print("side_stream_ok calls (returned, second use):", dict(calls))
    for k, v in log.most_common():
        print("second use:", v, "x", k)


if __name__ == "__main__":
    main()
