"""HuBERT conv-stack forward / input-gradient GEMMs (frontend._gemm_rows) at the c3 sizes, every
tile form of triad_gemm_bf16_form: the size policy (form 0) sends K < 1024 to the 256 x 128 ring
(gemm_big), which ran the odd-frame input gradients (M = 1.6 M, N = K = 512, output rows strided
2C) at ~340 TFLOP/s in the step profile (profiles/r04_bench_kernel_stats_final2.csv).

  python tools/conv_gemm_ab.py [--iters 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import _lib  # noqa: E402
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def bench(fn, iters):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    _lib.load()
    # (label, M, N, K, lda, ldc)
    shapes = [("odd dX k3", 1638400, 512, 512, 512, 1024), ("odd dX k3", 819200, 512, 512, 512, 1024),
              ("odd dX k3", 409600, 512, 512, 512, 1024), ("odd dX k3", 204800, 512, 512, 512, 1024),
              ("dX k2", 102400, 1024, 512, 512, 1024), ("dX k2", 51200, 1024, 512, 512, 1024),
              ("even dX k3", 819200, 512, 1024, 512, 1024), ("fwd k3", 819200, 512, 1536, 1024, 512)]
    for label, M, N, K, lda, ldc in shapes:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        a = torch.randn(M + 4, lda, device="cuda", generator=g).to(torch.bfloat16)
        b = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
        c = torch.empty(M + 1, ldc, device="cuda", dtype=torch.bfloat16)
        outs = {}
        for rnd in range(2):
            res = {}
            for form in (0, 2, 3, 4):
                def run():
                    call("triad_gemm_bf16_form", ptr(a), lda, 1, ptr(b), K, 1, M, N, K, None, ptr(c), ldc, 1, form,
                         stream_ptr())
                res[form] = round(bench(run, args.iters), 4)
                if rnd == 0:
                    outs[form] = c[:M, :N].clone()
            same = {f: bool(torch.equal(outs[f], outs[0])) for f in outs} if rnd == 0 else None
            best = min(res, key=res.get)
            print(json.dumps(dict(label=label, M=M, N=N, K=K, round=rnd, ms=res, best_form=best,
                                  TFLOPs={f: round(2.0 * M * N * K / v / 1e9, 1) for f, v in res.items()},
                                  bit_identical_to_form0=same)), flush=True)
            del same


if __name__ == "__main__":
    main()
