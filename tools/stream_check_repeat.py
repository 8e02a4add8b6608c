"""bench.py's serial-vs-concurrent product-shape check (stream_bit_identity), repeated in one
process, naming the parameters whose reduced gradients differ. Experiments only.

usage: python tools/stream_check_repeat.py [--reps 3] [--B 256]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--second", default="concurrent", choices=["concurrent", "serial"])
    a = ap.parse_args()
    from triad_amd import _lib, blas
    blas.configure()
    import bench
    from triad_amd.model import MultiModalModel, set_concurrent_streams
    from triad_amd.train import TriadTrainer
    dev = torch.device("cuda", 0)
    _lib.load()
    torch.backends.cudnn.benchmark = False
    frames, audio, text = bench.synthetic(a.B, 0, dev)

    from triad_amd import ops
    orig_pd = ops.patch_dropout
    grads = []

    def pd(x, keep_mask, n_out=None):   # capture the gradient reaching each dropout output
        out = orig_pd(x, keep_mask, n_out)
        if out.requires_grad:
            out.register_hook(lambda g: grads.append(g.detach().clone()))
        return out
    ops.patch_dropout = pd

    def run(concurrent):
        grads.clear()
        set_concurrent_streams(concurrent)
        torch.manual_seed(4321)
        m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.80, patch_sparsity_weight=0.01,
                            visual_dropout_prob=0.25, use_amp=True).to(dev)
        m.train()
        tr = TriadTrainer(m, learning_rate=1e-4, total_updates=100000, unfreeze_audio_step=0,
                          unfreeze_text_step=0, unfreeze_vit_step=0, device=dev)
        snap = []

        def grab():
            tr._allreduce_grads()
            snap.append(tr.space.flat_g.clone())
            return {}
        tr._optimizer_step = grab
        torch.manual_seed(1)
        np.random.seed(1)
        out = tr.step(frames, audio, text, phase="full_joint")
        torch.cuda.synchronize()
        loss = torch.stack([out["loss"], out["loss_av"], out["loss_tv"]]).clone()
        names = {id(p): n for n, p in m.named_parameters()}
        layout = [(names.get(id(p), "?"), int(o), p.numel()) for p, o in zip(tr.space.params, tr.space.offsets)]
        del tr, m
        return loss, snap[0], layout, list(grads)

    for r in range(a.reps):
        l_s, g_s, layout, d_s = run(False)
        l_c, g_c, _, d_c = run(a.second == "concurrent")
        dropout_grads_equal = [bool(torch.equal(x, y)) for x, y in zip(d_s, d_c)]
        set_concurrent_streams(True)
        diff = (g_s != g_c)
        bad = []
        for n, o, k in layout:
            d = int(diff[o:o + k].sum())
            if d:
                bad.append((n, d, k, float((g_s[o:o + k] - g_c[o:o + k]).abs().max())))
        print(json.dumps({"rep": r, "losses_equal": bool(torch.equal(l_s, l_c)), "dropout_out_grads_equal":
                          dropout_grads_equal, "differing": int(diff.sum()),
                          "params": bad[:20], "n_params": len(bad)}), flush=True)


if __name__ == "__main__":
    main()
