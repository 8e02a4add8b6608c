"""Host lead over the GPU inside the bench step: is the device ever waiting for the host?

Builds the bench model / trainer (bench.py's configuration), runs warm-up steps, then times steps
with a host timestamp AND an event on the main stream at each phase boundary of the step (step
begin, forward enqueued, backward enqueued, optimizer enqueued). Aligned at a synchronised start,
the host timestamp says when the host had enqueued the phase, the event when the GPU reached it;
lead = GPU time - host time. A lead near zero means the GPU waited for the host there.
Prints one JSON line per timed step. Experiments only.

usage: python tools/host_lead.py [--steps 4] [--warmup 2]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    from triad_amd import _lib, blas
    blas.configure()
    import bench
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
    marks = []

    def mark(tag):
        e = torch.cuda.Event(enable_timing=True)
        e.record()   # on the current stream (inside a gradient hook: the producing node's stream)
        marks.append((tag + "@s%d" % torch.cuda.current_stream().stream_id, time.perf_counter(), e))

    # phase boundaries: wrap backward and the optimizer step
    orig_backward = torch.Tensor.backward
    orig_opt = tr._optimizer_step

    def backward(self, *args, **kw):
        mark("fwd_enqueued")
        r = orig_backward(self, *args, **kw)
        mark("bwd_enqueued")
        return r

    def opt():
        r = orig_opt()
        mark("opt_enqueued")
        return r

    torch.Tensor.backward = backward
    tr._optimizer_step = opt
    # per-modality markers inside the backward: the gradient of each backbone output (the
    # projection head's input) is ready -> an event on the stream that produced it (the head's
    # backward stream), i.e. where that backbone's own backward begins
    from triad_amd import model as tmodel
    orig_project = tmodel._project
    kinds = {}

    def project(emb, h):
        kind = kinds.setdefault(type(emb).__name__, type(emb).__name__)
        if h.requires_grad:
            h.register_hook(lambda g, k=kind: (mark("bwd_backbone_start:" + k), g)[1])
        return orig_project(emb, h)

    tmodel._project = project
    for _ in range(a.warmup):
        tr.step(frames, audio, text, phase="full_joint")
    torch.cuda.synchronize()
    marks.clear()
    mark("start")
    for i in range(a.steps):
        mark(f"step{i}")
        tr.step(frames, audio, text, phase="full_joint")
    mark("end")
    for st in (tmodel._STREAMS.get(0) or ()):   # each modality stream's own end of the last step
        with torch.cuda.stream(st):
            mark("end")
    torch.cuda.synchronize()
    h0, e0 = marks[0][1], marks[0][2]
    rows = [(tag, (h - h0) * 1e3, e0.elapsed_time(e)) for tag, h, e in marks]
    for tag, hms, gms in rows:
        print(json.dumps({"mark": tag, "host_ms": round(hms, 2), "gpu_ms": round(gms, 2),
                          "lead_ms": round(gms - hms, 2)}), flush=True)


if __name__ == "__main__":
    main()
