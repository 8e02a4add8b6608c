"""Backbone weight-gradient GEMMs (dW = dY^T X, both operands token-major: a_kcontig = b_kcontig = 0)
of the c3 step on the split-K HIP GEMM: the current policy (linear._splits, size-policy form) against
the eight-wave 256 x 256 form (triad_gemm_set_form(4)) at several split counts. One JSON line per
shape: microseconds per call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import linear  # noqa: E402
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
    bf = torch.bfloat16
    spec = os.environ.get("PROBE_SHAPES")  # "M:O:K,..." (default: the HuBERT / DistilBERT shapes)
    if spec:
        shapes = [tuple(int(v) for v in t.split(":")) for t in spec.split(",")]
    else:
        shapes = [(M, O, K) for M in (50944, 8192) for O, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072))]
    splits = tuple(int(v) for v in os.environ.get("PROBE_SPLITS", "2,4,8,12,16,24,32").split(","))
    for M, O, K in shapes:
        if True:
            dy = torch.randn(M, O, device="cuda", dtype=bf)
            x = torch.randn(M, K, device="cuda", dtype=bf)
            ref = (dy.float().t() @ x.float())
            res = {"M": M, "O": O, "K": K}

            def run(sp, form):
                slabs = torch.empty(sp * O * K, dtype=torch.float32, device="cuda")
                dw = torch.empty(O, K, dtype=bf, device="cuda")
                call("triad_gemm_set_form", form)

                def f():
                    call("triad_gemm_bf16_splitk", ptr(dy), O, 0, ptr(x), K, 0, O, K, M, sp, None, ptr(slabs),
                         ptr(dw), 1, stream_ptr())
                us = timed(f)
                err = float((dw.float() - ref).norm() / ref.norm())
                call("triad_gemm_set_form", 0)
                return round(us, 1), round(err, 5)
            sp0 = linear._splits(M, O, K)
            res["policy"] = (sp0,) + run(sp0, 0)
            for sp in splits:
                res[f"w8_s{sp}"] = run(sp, 4)
                res[f"f1_s{sp}"] = run(sp, 1)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
