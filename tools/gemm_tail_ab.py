"""Last-round tile occupancy of the backbone GEMMs: at 50,944 rows (the c3 audio backbone) the
eight-wave 256 x 256 form has 199 x 3 = 597 tiles at N = 768, 2.33 rounds of 256 CUs -- the third
round runs a third full. Times every tile form of triad_gemm_bf16_form at the c3 backbone /
head shapes, forward (B [N][K]) and input-gradient (B [K][N]) operand layouts, alternated rounds.

  python tools/gemm_tail_ab.py [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import _lib  # noqa: E402
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def bench(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    _lib.load()
    shapes = [(50944, 768, 768), (50944, 768, 3072), (50944, 2304, 768), (50944, 3072, 768),
              (65536, 768, 768), (65536, 768, 3072), (50944, 512, 768), (50944, 512, 512)]
    for M, N, K in shapes:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
        wt = w.t().contiguous()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for rnd in range(2):
            for layout, bk, B, ldb in (("fwd", 1, w, K), ("dX", 0, wt, N)):
                res = {}
                for form in (1, 2, 3, 4):
                    def run():
                        call("triad_gemm_bf16_form", ptr(a), K, 1, ptr(B), ldb, bk, M, N, K, None, ptr(c), N, 1,
                             form, stream_ptr())
                    ms = bench(run, args.iters)
                    res[form] = round(ms, 4)
                best = min(res, key=res.get)
                print(json.dumps(dict(M=M, N=N, K=K, layout=layout, round=rnd, ms=res, best_form=best,
                                      TFLOPs_best=round(2.0 * M * N * K / res[best] / 1e9, 1),
                                      tiles_w8=(M // 256) * (N // 256), tiles_256x128=(M // 256) * (N // 128))),
                      flush=True)


if __name__ == "__main__":
    main()
