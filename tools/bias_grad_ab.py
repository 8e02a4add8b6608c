"""Column sums of the step's bias gradients: ops.bias_grad (split-K MFMA GEMM, x^T . ones) vs
triad_colsum, ms per call at the c3 backbone / head shapes (alternated, HIP events)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402


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


for rows, cols in ((50944, 768), (50944, 2304), (50944, 3072), (65536, 768), (65536, 3072), (8192, 768),
                   (8192, 3072), (65536, 512)):
    x = (torch.randn(rows, cols, device="cuda") * 0.05).to(torch.bfloat16)
    for r in range(2):
        os.environ["TRIAD_DB_FORM"] = "gemm"
        a = bench(lambda: ops.bias_grad(x))
        os.environ["TRIAD_DB_FORM"] = "dma"
        d = bench(lambda: ops.bias_grad(x))
        ref = x.float().sum(0)
        err = float((ops.bias_grad(x).float() - ref).norm() / ref.norm())
        os.environ["TRIAD_DB_FORM"] = "gemm"
        b = bench(lambda: ops.colsum(x, backbone=True))
        print(json.dumps(dict(rows=rows, cols=cols, round=r, gemm_ms=round(a, 4), dma_ms=round(d, 4),
                              colsum_ms=round(b, 4), dma_rel_err=err)), flush=True)
