"""Microbench of the backbone linear-layer GEMM shapes of the c3 step (bf16, torch.mm on
hipBLASLt): forward y = x W^T, dX = dy W, dW = dy^T x for the ViT-B (66,816 tokens), HuBERT-base
(50,944) and DistilBERT (8,192) layers. Prints one JSON line per shape with ms and TFLOP/s, so
the step profile's GEMM time can be read against what the library reaches on each shape."""
import json

import torch


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
    dt = torch.bfloat16
    for name, M in (("vit", 66816), ("hubert", 50944), ("distilbert", 8192)):
        for K, N in ((768, 2304), (768, 768), (768, 3072), (3072, 768)):
            x = torch.randn(M, K, device="cuda", dtype=dt)
            w = torch.randn(N, K, device="cuda", dtype=dt)
            dy = torch.randn(M, N, device="cuda", dtype=dt)
            flops = 2.0 * M * K * N
            for kind, fn in (("fwd", lambda: torch.mm(x, w.t())), ("dX", lambda: torch.mm(dy, w)),
                             ("dW", lambda: torch.mm(dy.t(), x))):
                ms = bench(fn)
                print(json.dumps({"model": name, "M": M, "K": K, "N": N, "gemm": kind, "ms": round(ms, 4),
                                  "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
