"""Split-K weight-gradient GEMM (triad_amd.linear.weight_grad) at the c3 dW shapes: ms per call.
Run against a variant build with TRIAD_LIB_VARIANT to compare staging forms."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    from triad_amd import _lib
    from triad_amd.linear import weight_grad
    _lib.load()
    for M, O, K in ((50944, 768, 768), (50944, 3072, 768), (50944, 768, 3072), (50944, 2304, 768),
                    (8192, 768, 768), (8192, 3072, 768)):
        dy = torch.randn(M, O, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        ref = torch.mm(dy.t().float(), x.float())
        got = weight_grad(dy, x).float()
        err = float((got - ref).norm() / ref.norm())
        print(json.dumps({"M": M, "O": O, "K": K, "ms": round(bench(lambda: weight_grad(dy, x)), 4),
                          "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
