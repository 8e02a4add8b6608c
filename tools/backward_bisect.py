"""Which backward launch of the text backbone first returns different values when the backbones
run on concurrent streams?

Every backward of the library's autograd Functions on TEXT-sized tensors (numel <= --max-numel:
the 6-token captions of tools/stream_repeat.py; the ViT / HuBERT tensors are far larger) is
wrapped: clones of its incoming gradients and of its outputs are kept, in call order. One
single-stream step is the reference; concurrent steps repeat until one differs anywhere in the
recorded text chain (up to --reps); then the first recorded backward whose INPUTS are
bit-identical to the reference's but whose OUTPUTS are not is named -- that launch computed
differently, not its producer. One JSON line per differing step.

  python tools/backward_bisect.py [--reps 20]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

dev = "cuda"
REC = None
MAXN = 4 << 20


def _wrap(cls):
    orig = cls.backward

    def backward(ctx, *grads):
        out = orig(ctx, *grads)
        big = max((g.numel() for g in grads if isinstance(g, torch.Tensor)), default=0)
        if REC is not None and 0 < big <= MAXN:
            outs = out if isinstance(out, tuple) else (out,)
            REC.append((cls.__name__, [g.detach().clone() if isinstance(g, torch.Tensor) else None for g in grads],
                        [o.detach().clone() if isinstance(o, torch.Tensor) else None for o in outs]))
        return out
    cls.backward = staticmethod(backward)


def install():
    from triad_amd import attention, linear, postln
    for cls in (linear._LinearFn, linear._QKVFn, postln._DropAddLN, postln._GeluDrop, attention._Attention,
                attention._AttentionQKV):
        _wrap(cls)


def step(streams, frames, audio, text):
    global REC
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer
    os.environ["TRIAD_MODALITY_STREAMS"] = "1" if streams else "0"
    torch.manual_seed(0)
    m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.8, patch_sparsity_weight=0.01,
                        visual_dropout_prob=0.25, use_amp=True).to(dev)
    m.train()
    tr = TriadTrainer(m, total_updates=100, unfreeze_audio_step=0, unfreeze_text_step=0, unfreeze_vit_step=0,
                      device=dev)
    REC = []
    torch.manual_seed(1)
    np.random.seed(1)
    tr.step(frames, audio, text)
    torch.cuda.synchronize()
    rec, REC = REC, None
    return rec


def same(a, b):
    return all((x is None and y is None) or (x is not None and y is not None and torch.equal(x, y))
               for x, y in zip(a, b))


def main():
    global MAXN
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--max-numel", type=int, default=MAXN)
    a = ap.parse_args()
    MAXN = a.max_numel
    install()
    B = 128
    g = torch.Generator().manual_seed(5)
    frames = torch.randn(B, 3, 224, 224, generator=g).to(dev)
    audio = (torch.randn(B, 16000, generator=g) * 0.1).to(dev)
    words = ["of", "a", "scene", "with", "red", "blue", "dog", "cat", "tree", "sky", "sea", "car"]
    text = [" ".join(["caption", "number", str(i)] + [words[(i + j) % len(words)] for j in range(3)]) for i in range(B)]
    ref = step(False, frames, audio, text)
    print(json.dumps({"reference_backwards": len(ref), "kinds": sorted({n for n, _, _ in ref})}), flush=True)
    found = 0
    for r in range(a.reps):
        rec = step(True, frames, audio, text)
        if len(rec) != len(ref) or any(x[0] != y[0] for x, y in zip(rec, ref)):
            print(json.dumps({"rep": r, "note": "different backward sequence", "n": len(rec)}), flush=True)
            continue
        first_out = None
        first_in = None
        for i, ((n, gi, go), (_, ri, ro)) in enumerate(zip(rec, ref)):
            if first_in is None and not same(gi, ri):
                first_in = (i, n)
            if not same(go, ro) and same(gi, ri):
                first_out = (i, n)
                bad = [j for j, (x, y) in enumerate(zip(go, ro)) if x is not None and not torch.equal(x, y)]
                detail = []
                for j in bad:
                    d = (go[j].float() != ro[j].float())
                    detail.append({"output": j, "shape": list(go[j].shape), "differing": int(d.sum()),
                                   "dtype": str(go[j].dtype)})
                break
        if first_out is None and first_in is None:
            print(json.dumps({"rep": r, "text_chain": "identical"}), flush=True)
            continue
        found += 1
        print(json.dumps({"rep": r, "first_differing_input_at": first_in,
                          "first_launch_with_equal_inputs_and_different_outputs": first_out,
                          "outputs": detail if first_out else None}), flush=True)
    print(json.dumps({"reps": a.reps, "differing_text_chains": found}), flush=True)


if __name__ == "__main__":
    main()
