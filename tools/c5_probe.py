"""Debug probe for the c5 configuration (DINOv2-L + HuBERT-large, 518 px, 10 s): runs a
base-model step first (as the config tests do), then the c5 step with a backward hook on every
backbone submodule that prints (flushed) when its backward starts, so a hang names its op."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def log(m):
    print(f"[c5 {time.strftime('%H:%M:%S')}] {m}", file=sys.stderr, flush=True)


def run(kw, B, px, secs, hooks):
    from triad_amd.model import MultiModalModel
    torch.manual_seed(1234)
    m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.8, patch_sparsity_weight=0.01,
                        visual_dropout_prob=0.25, **kw).cuda().train()
    if hooks:
        for name, mod in m.named_modules():
            if name.count(".") <= 4 and name:
                mod.register_full_backward_pre_hook(lambda mm, g, n=name: log(f"bwd start {n}"))
    g = torch.Generator(device="cuda").manual_seed(1)
    frames = torch.randn(B, 3, px, px, generator=g, device="cuda")
    audio = torch.randn(B, 16000 * secs, generator=g, device="cuda") * 0.1
    text = {"input_ids": torch.randint(1000, 30522, (B, 32)), "attention_mask": torch.ones(B, 32, dtype=torch.long)}
    (av, tv) = m.forward_triad(frames, audio, text)
    torch.cuda.synchronize()
    log(f"forward {kw} ok loss {float(av[0]):.4f} {float(tv[0]):.4f}")
    (av[0] + tv[0]).backward()
    torch.cuda.synchronize()
    log(f"backward {kw} ok")


if __name__ == "__main__":
    os.environ.setdefault("TRIAD_MODALITY_STREAMS", "0")
    run({}, 64, 224, 4, False)
    run({"audio_model_name": "facebook/hubert-large-ls960-ft", "vit_arch": "dinov2_vitl14_reg"}, 32, 518, 10, True)
