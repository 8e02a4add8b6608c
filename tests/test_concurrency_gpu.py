"""Our kernels' results must not depend on what else shares the CUs (the default concurrent step
runs three backbone streams). Regression test of the round-2 nondeterminism: the HuBERT conv-0 +
GroupNorm + GELU kernel (triad_c0gn_fwd) returned wrong values in lanes 48-63 whenever a 128 x 128
MFMA GEMM workgroup (triad_gemm_bf16 form 1) shared its CU, until round 3 changed its weight loads
and dropped packed-FP32 ops library-wide (which of the two mattered is not established, DESIGN.md
§2b; plain-load bf16 column-sum reductions were victims, so every column sum of the step now reads
its rows by LDS-DMA). Every output buffer
of c0gn, computed on a side stream while the GEMM runs on the main stream, must equal the quiet
run bit for bit (tools/concurrency_repro.py has the wider matrix of kernel pairs)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def test_c0gn_bit_identical_beside_128x128_gemm():
    from triad_amd._lib import call, ptr, stream_ptr
    B, T, C = 64, 3199, 512
    Tp = T + 1
    Lp = 5 * (Tp - 1) + 10
    g = torch.Generator(device=dev).manual_seed(3)
    xw = torch.randn(B, Lp, device=dev, generator=g).to(torch.bfloat16)
    w0 = (torch.randn(C, 10, device=dev, generator=g) * 0.3).to(torch.bfloat16)
    gam = torch.rand(C, device=dev, generator=g) + 0.5
    bet = torch.randn(C, device=dev, generator=g) * 0.1
    nb = int(call("triad_chgn_workspace_bytes", B, T, C))

    def bufs():
        return [torch.zeros(nb, dtype=torch.uint8, device=dev), torch.zeros(B, C, device=dev),
                torch.zeros(B, C, device=dev), torch.zeros(B * Tp + 2, C, device=dev, dtype=torch.bfloat16),
                torch.zeros(B * Tp, C, device=dev, dtype=torch.bfloat16)]

    def c0gn(b):
        ws, mean, rstd, out, y0 = b
        call("triad_c0gn_fwd", ptr(xw), Lp, ptr(w0), B, T, Tp, C, ptr(gam), ptr(bet), 1e-5, ptr(mean), ptr(rstd),
             ptr(ws), ptr(out), ptr(y0), stream_ptr(dev))

    M, N, K = 33280, 3072, 768
    a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

    def gemm():
        for _ in range(4):
            call("triad_gemm_bf16_form", ptr(a), K, 1, ptr(w), K, 1, M, N, K, None, ptr(c), N, 1, 1, stream_ptr(dev))

    ref = bufs()
    c0gn(ref)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    for it in range(3):
        got = bufs()
        side.wait_stream(torch.cuda.current_stream(dev))
        gemm()
        with torch.cuda.stream(side):
            c0gn(got)
        gemm()
        torch.cuda.synchronize()
        for name, x, y in zip(("ws", "mean", "rstd", "out", "y0"), got, ref):
            assert torch.equal(x, y), (it, name)
