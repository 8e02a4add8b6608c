"""GEMM form comparison (triad_gemm_set_form): 128 x 128, 256 x 128 ring and 256 x 256 four-wave
tiles on the step's shapes -- HuBERT conv layer GEMMs (overlapping A rows), split-K weight
gradients (both operands transposed), and the backbone linear forward against torch.mm
(hipBLASLt). Prints one JSON line per shape with ms per form and the max error vs torch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


def main():
    st = stream_ptr(torch.device("cuda"))
    dev = "cuda"
    forms = (1, 2, 3)
    # conv: A rows overlap (lda = 2C = 1024 < K = 1536), B [512][K]
    for M in (256 * 6400, 256 * 1600):
        K, N, lda = 1536, 512, 1024
        buf = torch.randn((M + 2) * lda, device=dev).to(torch.bfloat16)
        b = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ref = torch.mm(buf.as_strided((M, K), (lda, 1)), b.t())
        r = {"shape": "conv", "M": M, "N": N, "K": K, "torch": bench(lambda: torch.mm(buf.as_strided((M, K), (lda, 1)),
                                                                                       b.t()))}
        for f in forms:
            call("triad_gemm_set_form", f)
            r[f"form{f}"] = bench(lambda: call("triad_gemm_bf16", ptr(buf), lda, 1, ptr(b), K, 1, M, N, K, None,
                                               ptr(c), N, 1, st))
            r[f"err{f}"] = rel(c, ref)
        print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del buf, b, c, ref
    # weight gradients: dW[O][I] = dy^T x over T tokens (A = dy [T][O], B = x [T][I], both k-major)
    for T, O, I in ((50944, 768, 2304), (50944, 768, 768), (50944, 3072, 768), (50944, 768, 3072), (66816, 768, 768)):
        dy = torch.randn(T, O, device=dev).to(torch.bfloat16)
        x = torch.randn(T, I, device=dev).to(torch.bfloat16)
        ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
        r = {"shape": "dW", "M": O, "N": I, "K": T, "torch": bench(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))}
        out = torch.empty(O, I, device=dev)
        for f in forms:
            call("triad_gemm_set_form", f)
            for sp in ((8,) if f != 3 else (8, 16, 32)):
                slabs = torch.empty(sp * O * I, device=dev)
                r[f"form{f}_s{sp}"] = bench(lambda: call("triad_gemm_bf16_splitk", ptr(dy), O, 0, ptr(x), I, 0, O, I,
                                                          T, sp, None, ptr(slabs), ptr(out), 0, st))
                r[f"err{f}_s{sp}"] = rel(out, ref)
        print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del dy, x, ref, slabs
    # linear forward y = x W^T
    for M, K, N in ((66816, 768, 2304), (66816, 768, 3072), (66816, 3072, 768), (50944, 768, 768)):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ref = torch.mm(x, w.t())
        r = {"shape": "linear", "M": M, "N": N, "K": K, "torch": bench(lambda: torch.mm(x, w.t()))}
        for f in forms:
            call("triad_gemm_set_form", f)
            r[f"form{f}"] = bench(lambda: call("triad_gemm_bf16", ptr(x), K, 1, ptr(w), K, 1, M, N, K, None, ptr(y), N,
                                               1, st))
            r[f"err{f}"] = rel(y, ref)
        print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    call("triad_gemm_set_form", 0)


if __name__ == "__main__":
    main()
