"""How often does the multi-stream tri-modal step differ from the single-stream one?

One TriadTrainer step (c3 model, B=128, dropout / LayerDrop / SpecAugment on -- the setting of
tests/test_ops_gpu.py::test_modality_streams_match_single_stream) from identical models and seeds:
once single-stream as the reference, then `--reps` times with the modality streams, each compared
bit for bit (losses and the reduced fp32 gradient buffer). Prints one line per rep (the differing
parameters, if any) and a JSON summary. TRIAD_GATHER_FP32_GRADS=0 selects the old route of the
fp32 gradients (autograd's add into views of the flat buffer) for an A/B.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

dev = "cuda"


SIDE = False


def run(streams, frames, audio, text):
    from triad_amd import linear
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer
    os.environ["TRIAD_MODALITY_STREAMS"] = "1" if streams else "0"
    linear.SIDE_STREAM_DW = bool(streams and SIDE)   # the dW side stream with the concurrent runs (--side)
    torch.manual_seed(0)
    m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.8, patch_sparsity_weight=0.01,
                        visual_dropout_prob=0.25, use_amp=True).to(dev)
    m.train()
    tr = TriadTrainer(m, total_updates=100, unfreeze_audio_step=0, unfreeze_text_step=0, unfreeze_vit_step=0,
                      device=dev)
    snap = []
    inner = tr._allreduce_grads

    def grab():
        inner()
        snap.append(tr.space.flat_g.clone())
    tr._allreduce_grads = grab
    torch.manual_seed(1)
    np.random.seed(1)
    out = tr.step(frames, audio, text)
    torch.cuda.synchronize()
    names = {id(p): n for n, p in m.named_parameters()}
    layout = [(names[id(p)], tr.space.offsets[i], p.numel()) for i, p in enumerate(tr.space.params)]
    return [float(out[k]) for k in ("loss", "loss_av", "loss_tv")], snap[0].cpu(), layout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--math-sdpa", action="store_true", help="PyTorch's masked SDPA (the DistilBERT attention) "
                    "on its math backend only")
    ap.add_argument("--det", action="store_true", help="torch.use_deterministic_algorithms(True, warn_only=True)")
    ap.add_argument("--configs", default="", help="A/B within one process: 'name:VAR=val,VAR2=val;name2:...' -- "
                    "the multi-stream reps alternate over these environments (each counted on its own)")
    ap.add_argument("--tokens", type=int, default=6, help="caption words (6: the stream test; 32: the bench)")
    ap.add_argument("--ref-per-config", action="store_true", help="each config against its own single-stream "
                    "reference (for configs that change the arithmetic)")
    ap.add_argument("--side", action="store_true", help="concurrent runs also put the backbone weight gradients "
                    "on the side stream (set_concurrent_streams(True) as a whole)")
    a = ap.parse_args()
    global SIDE
    SIDE = a.side
    if a.math_sdpa:
        torch.backends.cuda.enable_flash_sdp(False)
        torch.backends.cuda.enable_mem_efficient_sdp(False)
        torch.backends.cuda.enable_math_sdp(True)
    if a.det:
        torch.use_deterministic_algorithms(True, warn_only=True)
    B = 128
    g = torch.Generator().manual_seed(5)
    frames = torch.randn(B, 3, 224, 224, generator=g).to(dev)
    audio = (torch.randn(B, 16000, generator=g) * 0.1).to(dev)
    words = ["of", "a", "scene", "with", "red", "blue", "dog", "cat", "tree", "sky", "sea", "car"]
    text = [" ".join(["caption", "number", str(i)] + [words[(i + j) % len(words)] for j in range(a.tokens - 3)])
            for i in range(B)]
    l_ref, g_ref, layout = run(False, frames, audio, text)
    configs = [("default", {})]
    if a.configs:
        configs = []
        for item in a.configs.split(";"):
            name, _, kv = item.partition(":")
            configs.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    per = {n: [0, 0] for n, _ in configs}
    refs = {}

    def under(env, streams):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            return run(streams, frames, audio, text)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    bad = 0
    for r in range(a.reps):
        cname, env = configs[r % len(configs)]
        if a.ref_per_config:
            if cname not in refs:   # this config's own single-stream reference (its arithmetic may differ)
                refs[cname] = under(env, False)[:2]
            l_ref, g_ref = refs[cname]
        l, gm, _ = under(env, True)
        diff = []
        for name, off, n in layout:
            x, y = gm[off:off + n], g_ref[off:off + n]
            if not torch.equal(x, y):
                rel = float((x.double() - y.double()).norm() / y.double().norm().clamp(min=1e-300))
                diff.append((name, int((x != y).sum()), n, f"{rel:.2g}"))
        ok = l == l_ref and not diff
        bad += not ok
        per[cname][0] += 1
        per[cname][1] += not ok
        print(f"rep {r} [{cname}]: {'equal' if ok else 'DIFFERS'} losses_equal={l == l_ref} params={diff[:6]}",
              flush=True)
    print(json.dumps({"per_config": {n: {"reps": v[0], "differing": v[1]} for n, v in per.items()},
                      "tokens": a.tokens}), flush=True)
    print(json.dumps({"reps": a.reps, "differing": bad, "math_sdpa": a.math_sdpa, "det": a.det,
                      "gather_fp32": os.environ.get("TRIAD_GATHER_FP32_GRADS", "1")}), flush=True)


if __name__ == "__main__":
    main()
