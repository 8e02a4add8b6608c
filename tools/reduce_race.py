"""Do column reductions return different values when another stream's kernels share the GPU?

The multi-stream residual only ever hit column sums: bias gradients of the text
layers (PyTorch's sum_to reduction at the stream test's 768-row shape) and HuBERT's
masked_spec_embed (a reduction over the masked rows). Here each victim runs (a) alone ->
reference, then (b) `iters` times while a noise stream keeps the CUs busy with GEMMs, each result
compared bit for bit. Victims: torch .sum(0) of bf16 / fp32 matrices at the bias-gradient
shapes, triad_colsum (two launches), a masked-row sum. One JSON line per (victim, noise)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
ITERS = int(os.environ.get("ITERS", "200"))


def noise_gemm(form):
    a = torch.randn(33280, 768, device=dev).to(torch.bfloat16)
    w = torch.randn(3072, 768, device=dev).to(torch.bfloat16)
    out = torch.empty(33280, 3072, device=dev, dtype=torch.bfloat16)

    def run(n=3):
        for _ in range(n):
            call("triad_gemm_bf16_form", ptr(a), 768, 1, ptr(w), 768, 1, 33280, 3072, 768, None, ptr(out), 3072, 1,
                 form, stream_ptr(dev))
    return run


def noise_torch():
    a = torch.randn(16384, 1024, device=dev).to(torch.bfloat16)
    b = torch.randn(1024, 4096, device=dev).to(torch.bfloat16)

    def run(n=3):
        for _ in range(n):
            torch.mm(a, b)
    return run


def victims():
    g = torch.Generator(device=dev).manual_seed(3)
    out = {}
    for rows, cols in ((768, 768), (768, 2304), (768, 3072), (6272, 768), (8192, 768)):
        xb = (torch.randn(rows, cols, device=dev, generator=g) * 0.01).to(torch.bfloat16)
        xf = torch.randn(rows, cols, device=dev, generator=g)
        out[f"torch sum0 bf16 {rows}x{cols}"] = (lambda x=xb: x.sum(0))
        out[f"torch sum0 fp32 {rows}x{cols}"] = (lambda x=xf: x.sum(0))
        if rows % 16 == 0:
            out[f"triad_colsum bf16 {rows}x{cols}"] = (lambda x=xb: ops.colsum(x, torch.bfloat16))
    h = (torch.randn(128, 49, 768, device=dev, generator=g) * 0.01).to(torch.bfloat16)
    m = torch.rand(128, 49, device=dev, generator=g) < 0.3
    out["torch masked-row sum bf16 (128x49x768, 30 %)"] = lambda: h[m].sum(0)
    return out


def check(name, fn, noise, noise_name):
    side = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    ref = fn().clone()
    torch.cuda.synchronize()
    bad, worst, nel = 0, 0.0, 0
    for _ in range(ITERS):
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        noise()
        with torch.cuda.stream(side):
            got = fn().clone()
        noise()
        torch.cuda.synchronize()
        if not torch.equal(got, ref):
            bad += 1
            d = (got.float() - ref.float()).abs()
            worst = max(worst, float(d.max()))
            nel = max(nel, int((d > 0).sum()))
    print(json.dumps(dict(victim=name, noise=noise_name, iters=ITERS, mismatching=bad, max_abs=worst,
                          max_elems=nel)), flush=True)
    return bad


def kernels_of(fn):
    """Device kernels (and memsets) one call launches: a global (cross-workgroup) reduction shows
    as a semaphore memset + the reduce kernel."""
    from torch.profiler import ProfilerActivity, profile
    fn()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return [e.name[:90] for e in prof.events() if e.device_type.name == "CUDA"]


def main():
    tot = 0
    vs = victims()
    for name, fn in vs.items():
        print(json.dumps(dict(victim=name, kernels=kernels_of(fn))), flush=True)
    noises = {"none": lambda: None, "gemm form 1 (128x128)": noise_gemm(1), "gemm form 4 (8-wave)": noise_gemm(4),
              "torch.mm (rocBLAS)": noise_torch()}
    for nn, noise in noises.items():
        for name, fn in vs.items():
            tot += check(name, fn, noise, nn)
    print(json.dumps(dict(total_mismatching=tot)), flush=True)


if __name__ == "__main__":
    main()
