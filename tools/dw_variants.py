"""Weight-gradient GEMM (dW = dy^T x, contraction over the 50-67 K token rows) variants on the
HuBERT / ViT shapes: operand order, an explicit transpose copy, and rocBLAS vs hipBLASLt.
One JSON line per (shape, variant): ms and TFLOP/s."""
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
    for M, K, N in ((50944, 768, 2304), (50944, 768, 768), (50944, 768, 3072), (50944, 3072, 768)):
        x = torch.randn(M, K, device="cuda", dtype=dt)
        dy = torch.randn(M, N, device="cuda", dtype=dt)
        out32 = torch.empty(N, K, device="cuda", dtype=torch.float32)
        flops = 2.0 * M * K * N
        variants = {
            "dyT_x": lambda: torch.mm(dy.t(), x),
            "xT_dy_T": lambda: torch.mm(x.t(), dy).t(),
            "dyTc_x": lambda: torch.mm(dy.t().contiguous(), x),
            "dyT_x_f32out": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32) if hasattr(torch.mm, "__call__") else None,
        }
        for lib in ("cublaslt", "cublas"):
            torch.backends.cuda.preferred_blas_library(lib)
            for name, fn in variants.items():
                try:
                    ms = bench(fn)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"M": M, "K": K, "N": N, "lib": lib, "variant": name, "error": str(e)[:80]}))
                    continue
                print(json.dumps({"M": M, "K": K, "N": N, "lib": lib, "variant": name, "ms": round(ms, 4),
                                  "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)
        torch.backends.cuda.preferred_blas_library("cublaslt")


def triad_splitk(M=50944):
    """triad_gemm_bf16_splitk (csrc/gemm.hip, 128x128x64 tiles, fp32 slabs) on the same shapes,
    next to torch.mm(dy^T, x)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from triad_amd._lib import call, ptr, stream_ptr
    dt = torch.bfloat16
    for K, N in ((768, 2304), (768, 768), (768, 3072), (3072, 768)):
        x = torch.randn(M, K, device="cuda", dtype=dt)
        dy = torch.randn(M, N, device="cuda", dtype=dt)
        ref = torch.mm(dy.t().float(), x.float())
        ms = bench(lambda: torch.mm(dy.t(), x))
        print(json.dumps({"M": M, "K": K, "N": N, "lib": "torch", "ms": round(ms, 4),
                          "TFLOPs": round(2.0 * M * K * N / ms / 1e9, 1)}), flush=True)
        one = torch.ones(1, device="cuda")
        flops = 2.0 * M * K * N
        for sp in [int(v) for v in os.environ.get("TRIAD_DW_SPLITS", "2,4,8,16").split(",")]:
            slabs = torch.empty(sp * N * K, device="cuda")
            out = torch.empty(N, K, device="cuda")
            fn = lambda: call("triad_gemm_bf16_splitk", ptr(dy), N, 0, ptr(x), K, 0, N, K, M, sp, ptr(one),  # noqa: E731
                              ptr(slabs), ptr(out), 0, stream_ptr())
            ms = bench(fn)
            err = float((out - ref).norm() / ref.norm())
            print(json.dumps({"M": M, "K": K, "N": N, "lib": "triad_splitk", "splits": sp, "ms": round(ms, 4),
                              "TFLOPs": round(flops / ms / 1e9, 1), "rel_err": err}), flush=True)


if __name__ == "__main__":
    import sys
    triad_splitk(int(sys.argv[1]) if len(sys.argv) > 1 else 50944)
