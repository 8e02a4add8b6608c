"""The projection head's GEMMs on the library (torch.matmul -> hipBLASLt, bf16 in / bf16 out) at
the c3 row counts, for comparison with the fused row-panel kernels (tools/projhead_micro.py):
fwd y1 = x W1^T (K = H), y = ln W2^T (K = 512); bwd dX GEMMs dy W2, dy1 W1; dW GEMMs dy^T ln,
dy1^T x. Prints one JSON line per (rows, GEMM): ms and TFLOP/s."""
import json

import torch


def timed(fn, iters=30):
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
    dev = "cuda"
    bf = torch.bfloat16
    for M in (65536, 50944, 8192):
        H = 768
        x = torch.randn(M, H, device=dev, dtype=bf)
        ln = torch.randn(M, 512, device=dev, dtype=bf)
        dy = torch.randn(M, 512, device=dev, dtype=bf)
        W1 = torch.randn(512, H, device=dev, dtype=bf)
        W2 = torch.randn(512, 512, device=dev, dtype=bf)
        cases = {"fwd1 x W1^T": (lambda: x @ W1.t(), M * H * 512),
                 "fwd2 ln W2^T": (lambda: ln @ W2.t(), M * 512 * 512),
                 "dX2 dy W2": (lambda: dy @ W2, M * 512 * 512),
                 "dX1 dy1 W1": (lambda: dy @ W1, M * 512 * H),
                 "dW2 dy^T ln": (lambda: dy.t() @ ln, M * 512 * 512),
                 "dW1 dy1^T x": (lambda: dy.t() @ x, M * 512 * H)}
        tot = 0.0
        for name, (fn, mac) in cases.items():
            ms = timed(fn)
            tot += ms
            print(json.dumps({"rows": M, "gemm": name, "ms": round(ms, 4), "TFLOPs": round(2 * mac / ms / 1e9, 1)}),
                  flush=True)
        print(json.dumps({"rows": M, "gemm": "all six", "ms": round(tot, 4)}), flush=True)


if __name__ == "__main__":
    main()
