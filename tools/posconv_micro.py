"""HuBERT positional conv kernels at the c3 shape (B=256, T=199, C=768, 16 groups, 128 taps):
forward (= input-gradient form) and weight gradient, ms and TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def bench(fn, iters=20):
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


def main():
    B, T, C, G, K, pad = 256, 199, 768, 16, 128, 64
    st = stream_ptr(torch.device("cuda"))
    x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
    dy = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
    wt = (torch.randn(G, 48, K * 48, device="cuda") * 0.02).to(torch.bfloat16)
    y = torch.empty_like(x)
    flops = 2.0 * B * T * C * 48 * K
    fwd = bench(lambda: call("triad_posconv", ptr(x), ptr(wt), None, ptr(y), B, T, C, G, pad, st))
    part = torch.empty(int(call("triad_posconv_dw_part_bytes", C, G, 16)) // 4, device="cuda")
    dw = bench(lambda: call("triad_posconv_dw", ptr(x), ptr(dy), B, T, C, G, pad, 16, ptr(part), st))
    print(json.dumps({"fwd_ms": round(fwd, 4), "fwd_TFLOPs": round(flops / fwd / 1e9, 1), "dw_ms": round(dw, 4),
                      "dw_TFLOPs": round(flops / dw / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
