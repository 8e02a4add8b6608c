"""Where does the multi-stream text-bias residual come from: the bias reduction, or its input?

One TriadTrainer step as in tools/stream_repeat.py (single-stream reference, then N multi-stream
reps, fresh model each). Every DistilBERT Linear output gets a gradient hook that keeps a copy
of dy (the bias reduction's input); the text biases' .grad is copied just before the gather.
After the step (device idle) each bias gradient is recomputed from its captured dy by the same
reduction run alone, and compared bit for bit with the in-step result:
  * in-step != alone-recompute  -> the reduction itself returned a wrong result (victim);
  * dy(multi) != dy(single)      -> the input already differed (upstream).
--tokens 6: the stream test's captions (768 rows: stock nn.Linear, PyTorch's sum_to reduction);
--tokens 32: the bench's captions (TriadLinear: triad_colsum)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

dev = "cuda"


def run(streams, frames, audio, text):
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer
    from triad_amd import ops
    os.environ["TRIAD_MODALITY_STREAMS"] = "1" if streams else "0"
    torch.manual_seed(0)
    m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.8, patch_sparsity_weight=0.01,
                        visual_dropout_prob=0.25, use_amp=True).to(dev)
    m.train()
    tr = TriadTrainer(m, total_updates=100, unfreeze_audio_step=0, unfreeze_text_step=0, unfreeze_vit_step=0,
                      device=dev)
    enc = m.text_embedder.encoder
    dys, hooks = {}, []
    lin = {n: mod for n, mod in enc.named_modules() if isinstance(mod, torch.nn.Linear)}

    def cap(name):
        def h(g):
            dys[name] = g.detach().clone()
        return h

    def fwd_hook(n):
        def h(mod, inp, out):   # must return None (a returned value replaces the output)
            if out.requires_grad:
                out.register_hook(cap(n))
        return h

    for n, mod in lin.items():
        hooks.append(mod.register_forward_hook(fwd_hook(n)))
    grads = {}
    inner = tr.space.gather_shadow_grads

    def gather(accumulate):
        for n, mod in lin.items():
            if mod.bias is not None and mod.bias.grad is not None:
                grads[n] = mod.bias.grad.detach().clone()
        return inner(accumulate)
    tr.space.gather_shadow_grads = gather
    torch.manual_seed(1)
    np.random.seed(1)
    out = tr.step(frames, audio, text)
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    # recompute every bias gradient alone from its captured input, with the op the step used
    alone = {}
    for n, dy in dys.items():
        O = dy.shape[-1]
        d2 = dy.reshape(-1, O).to(torch.bfloat16).contiguous()
        M = d2.shape[0]
        if M >= 4096 and M % 64 == 0:   # TriadLinear path (linear._eligible): triad_colsum
            alone[n] = ops.colsum(d2, torch.bfloat16, backbone=True)
        else:                           # stock F.linear: autograd's sum_to of the bias
            alone[n] = dy.reshape(-1, O).sum(0)
        torch.cuda.synchronize()
    loss = [float(out[k]) for k in ("loss", "loss_av", "loss_tv")]
    return loss, {k: v.cpu() for k, v in dys.items()}, {k: v.cpu() for k, v in grads.items()}, \
        {k: v.cpu() for k, v in alone.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=6)
    ap.add_argument("--B", type=int, default=128)
    a = ap.parse_args()
    B = a.B
    g = torch.Generator().manual_seed(5)
    frames = torch.randn(B, 3, 224, 224, generator=g).to(dev)
    audio = (torch.randn(B, 16000, generator=g) * 0.1).to(dev)
    words = ["caption", "number", "of", "a", "scene", "with", "red", "blue", "dog", "cat", "tree", "sky"]
    text = [" ".join(["caption", "number", str(i)] + [words[(i + j) % len(words)] for j in range(a.tokens - 3)])
            for i in range(B)]
    l_ref, dy_ref, g_ref, al_ref = run(False, frames, audio, text)
    self_bad = [n for n in g_ref if n in al_ref and not torch.equal(g_ref[n], al_ref[n])]
    print(f"single-stream: {len(g_ref)} text biases, in-step != alone: {self_bad}", flush=True)
    summary = dict(reps=a.reps, tokens=a.tokens, B=B, differs=0, reduction_victim=0, input_differs=0)
    for r in range(a.reps):
        l, dy, gr, al = run(True, frames, audio, text)
        diff = [n for n in g_ref if not torch.equal(gr[n], g_ref[n])]
        victim = [(n, int((gr[n] != al[n]).sum())) for n in gr if n in al and not torch.equal(gr[n], al[n])]
        upstream = [n for n in dy_ref if not torch.equal(dy[n], dy_ref[n])]
        summary["differs"] += bool(diff) or l != l_ref
        summary["reduction_victim"] += bool(victim)
        summary["input_differs"] += bool(upstream)
        print(f"rep {r}: losses_equal={l == l_ref} bias_grads_differ={diff[:6]} "
              f"in-step!=alone={victim[:6]} dy_differs={upstream[:6]}", flush=True)
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
