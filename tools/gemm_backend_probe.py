"""Backbone forward / input-gradient GEMM shapes of the c3 step on (a) torch -> the BLAS library
triad_amd.blas selects (rocBLAS without its hipBLASLt forwarding, by default) and (b) the HIP
GEMM of gemm.hip in each tile form (1: 128 x 128, 2: 256 x 128 ring, 3: 256 x 256 four-wave, 4: eight-wave),
bf16 out. Prints one JSON line per (shape, path): microseconds and TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import triad_amd  # noqa: E402,F401  (BLAS selection happens at import)
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def timed(fn, iters=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = "cuda"
    bf = torch.bfloat16
    shapes = []
    for M in (66816, 50944, 8192):
        for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
            shapes.append(("fwd", M, N, K))     # y = x W^T
            shapes.append(("dX", M, K, N))      # dx = dy W   (dy [M][N], W [N][K])
    one = torch.ones(1, device=dev)
    forms = tuple(int(f) for f in os.environ.get("PROBE_FORMS", "1,2,3,4").split(","))
    min_m = int(os.environ.get("PROBE_MIN_M", "0"))
    shapes = [sh for sh in shapes if sh[1] >= min_m]
    for kind, M, N, K in shapes:
        fl = 2.0 * M * N * K
        if kind == "fwd":
            A = torch.randn(M, K, device=dev, dtype=bf)
            W = torch.randn(N, K, device=dev, dtype=bf)
            lib = lambda: A @ W.t()   # noqa: E731
            args = (A, K, 1, W, K, 1)
        else:
            A = torch.randn(M, K, device=dev, dtype=bf)   # dy, contraction K (= out features)
            W = torch.randn(K, N, device=dev, dtype=bf)   # W [out][in]: B is [Kd][N]
            lib = lambda: A @ W       # noqa: E731
            args = (A, K, 1, W, N, 0)
        C = torch.empty(M, N, device=dev, dtype=bf)
        ref = lib().float()
        res = {"kind": kind, "M": M, "N": N, "K": K, "lib_us": round(timed(lib), 1) if not min_m else None,
               "variant": os.environ.get("TRIAD_LIB_VARIANT", "default")}
        for form in forms:
            call("triad_gemm_set_form", form)
            a, lda, ak, b, ldb, bk = args

            def ours():
                call("triad_gemm_bf16", ptr(a), lda, ak, ptr(b), ldb, bk, M, N, K, ptr(one), ptr(C), N, 1,
                     stream_ptr())
            try:
                us = timed(ours)
                err = float((C.float() - ref).norm() / ref.norm())
                res[f"form{form}_us"] = round(us, 1)
                res[f"form{form}_err"] = round(err, 5)
            except Exception as e:   # shape outside the form
                res[f"form{form}_us"] = None
        call("triad_gemm_set_form", 0)
        best = min(v for k, v in res.items() if k.endswith("_us") and v)
        res["best_TFLOPs"] = round(fl / best / 1e6, 1)
        res["lib_TFLOPs"] = round(fl / res["lib_us"] / 1e6, 1) if res["lib_us"] else None
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
