"""GELU passes (postln.gelu: geludrop kernels at p = 0, table-driven) at the step's largest
shapes: fwd / bwd ms and effective HBM rate."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


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
    from triad_amd.postln import gelu_table
    st = stream_ptr(torch.device("cuda"))
    tab = gelu_table(torch.device("cuda"))
    for name, n in (("vit_mlp", 66816 * 3072), ("conv1", 1638400 * 512), ("hubert_ffn", 50944 * 3072)):
        u = torch.randn(n, device="cuda").to(torch.bfloat16)
        dv = torch.randn(n, device="cuda").to(torch.bfloat16)
        v = torch.empty_like(u)
        f = bench(lambda: call("triad_geludrop_fwd", ptr(u), n, 0.0, 0, ptr(tab), ptr(v), st))
        b = bench(lambda: call("triad_geludrop_bwd", ptr(u), ptr(dv), n, 0.0, 0, ptr(tab), ptr(v), st))
        fd = bench(lambda: call("triad_geludrop_fwd", ptr(u), n, 0.1, 7, ptr(tab), ptr(v), st))
        print(json.dumps({"shape": name, "n": n, "fwd_ms": round(f, 4), "fwd_TBps": round(4 * n / f / 1e9, 2),
                          "bwd_ms": round(b, 4), "bwd_TBps": round(6 * n / b / 1e9, 2), "fwd_drop_ms": round(fd, 4)}),
              flush=True)
        del u, dv, v


if __name__ == "__main__":
    main()
