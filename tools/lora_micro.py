"""Microbench of one ViT-B LoRA Linear (qkv: 66,816 x 768 -> 2304, proj: -> 768) forward+backward
on the HIP LoRA kernels vs the plain autocast chain base(x) + B(A(x)) * s. One JSON line each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd.vit import LoRALinear  # noqa: E402


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for O in (2304, 768):
    M, K = 256 * 261, 768
    base = torch.nn.Linear(K, O).cuda().to(torch.bfloat16)
    for p in base.parameters():
        p.requires_grad = False
    m = LoRALinear(base, 8, 16).cuda()
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    gy = torch.randn(M, O, device="cuda", dtype=torch.bfloat16)

    def fast():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.backward(gy)

    def ref():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = base(x) + torch.nn.functional.linear(torch.nn.functional.linear(x, m.lora_A), m.lora_B) * m.scaling
        y.backward(gy)
    print(json.dumps({"O": O, "hip_ms": round(bench(fast), 4), "torch_chain_ms": round(bench(ref), 4)}), flush=True)
