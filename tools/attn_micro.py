"""Backbone attention shapes: HIP kernels (triad_amd.attention) vs torch SDPA, fwd and fwd+bwd."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import attention  # noqa: E402


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for name, B, N, H in (("vit", 256, 261, 12), ("hubert", 256, 199, 12), ("distilbert", 256, 32, 12)):
    qkv = torch.randn(B, N, 3 * H * 64, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    go = torch.randn(B, N, H * 64, device="cuda", dtype=torch.bfloat16)

    def ours_f():
        with torch.no_grad():
            attention.attention_qkv(qkv, H)

    def ours_fb():
        attention.attention_qkv(qkv, H).backward(go)

    def torch_o():
        x = qkv.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
        return F.scaled_dot_product_attention(x[0], x[1], x[2]).transpose(1, 2).reshape(B, N, H * 64)

    def torch_f():
        with torch.no_grad():
            torch_o()

    def torch_fb():
        torch_o().backward(go)
    fl = 4.0 * B * H * N * N * 64
    r = {"shape": name, "B": B, "N": N, "H": H}
    for k, f in (("ours_fwd", ours_f), ("ours_fwdbwd", ours_fb), ("torch_fwd", torch_f), ("torch_fwdbwd", torch_fb)):
        ms = bench(f)
        r[k + "_ms"] = round(ms, 4)
        r[k + "_TFLOPs"] = round(fl * (3.5 if "bwd" in k else 1.0) / ms / 1e9, 1)
    print(json.dumps(r), flush=True)
