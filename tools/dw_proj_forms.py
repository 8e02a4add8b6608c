"""Projection-head weight-gradient GEMMs (dW2 = dy^T ln [512 x 512], dW1 = dy1^T h [512 x 768],
contraction over the token rows) on the split-K GEMM in its 128 x 128 form (1) and its 256 x 256
four-wave (3) and eight-wave (4) forms at several split counts, slab reduction included (HIP
events, c3 row counts; triad_gemm_bf16_splitk_form)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def timed(fn, iters=20):
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
    for K in (65536, 50944, 8192):
        for N in (512, 768):
            dy = torch.randn(K, 512, device=dev).to(torch.bfloat16)
            x = torch.randn(K, N, device=dev).to(torch.bfloat16)
            ref = dy.float().t() @ x.float()
            out = torch.empty(512, N, device=dev)
            for form, tiles in ((1, (512 // 128) * (N // 128)), (3, (512 // 256) * (N // 256)),
                                (4, (512 // 256) * (N // 256))):
                for sp in sorted({max(1, w // tiles) for w in (64, 128, 192, 256, 384)}):
                    if K // sp < 256 or K % 64:
                        continue
                    slabs = torch.empty(sp * 512 * N, device=dev)

                    def run():
                        call("triad_gemm_bf16_splitk_form", ptr(dy), 512, 0, ptr(x), N, 0, 512, N, K, sp, None,
                             ptr(slabs), ptr(out), 0, form, stream_ptr())
                    ms = timed(run)
                    err = float((out - ref).norm() / ref.norm())
                    print(json.dumps({"K": K, "N": N, "form": form, "splits": sp, "us": round(ms * 1e3, 1),
                                      "TFLOPs": round(2 * 512 * N * K / ms / 1e9, 1), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
