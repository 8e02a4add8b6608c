"""HuBERT conv layer 1 (C=512, k=3, stride 2, 12 800 padded frames x 256) as GEMMs: the current
im2col + hipBLASLt form vs overlapping-row operands (lda = 2C < K = 3C) on triad_gemm_bf16,
forward, dX (K = 2O over consecutive dY rows) and dW (split-K). JSON lines: ms, TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def bench(fn, iters=10):
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


B, Tp, C, O = 256, 12800, 512, 512
M = B * Tp // 2
dt = torch.bfloat16
x = torch.randn(B * Tp + 2, C, device="cuda", dtype=dt)
w = torch.randn(O, 3 * C, device="cuda", dtype=dt) * 0.02
dy = torch.randn(M + 2, O, device="cuda", dtype=dt)
fl = 2.0 * M * 3 * C * O


def im2col_fwd():
    xv = x[:B * Tp].view(B, Tp, C)
    To = Tp // 2
    cols = torch.empty(B, To, 3, C, dtype=dt, device="cuda")
    for j in range(3):
        cols[:, :To - 1, j].copy_(xv[:, j:j + 2 * (To - 1):2])
    return torch.mm(cols.view(-1, 3 * C), w.t())


y = torch.empty(M, O, device="cuda", dtype=dt)
one = torch.ones(1, device="cuda")


def ov_fwd():
    call("triad_gemm_bf16", ptr(x), 2 * C, 1, ptr(w), 3 * C, 1, M, O, 3 * C, ptr(one), ptr(y), O, 1, stream_ptr())


wd = torch.randn(2 * C, 2 * O, device="cuda", dtype=dt) * 0.02
dx2 = torch.empty(M + 1, 2 * C, device="cuda", dtype=dt)


def ov_dx():
    call("triad_gemm_bf16", ptr(dy), O, 1, ptr(wd), 2 * O, 1, M, 2 * C, 2 * O, ptr(one), ptr(dx2[1:]), 2 * C, 1,
         stream_ptr())


dw = torch.empty(O, 3 * C, device="cuda")


def ov_dw(sp):
    slabs = torch.empty(sp * O * 3 * C, device="cuda")

    def f():
        call("triad_gemm_bf16_splitk", ptr(dy), O, 0, ptr(x), 2 * C, 0, O, 3 * C, M, sp, ptr(one), ptr(slabs),
             ptr(dw), 0, stream_ptr())
    return f


def torch_dw():
    xv = x[:B * Tp].view(B, Tp, C)
    To = Tp // 2
    cols = torch.empty(B, To, 3, C, dtype=dt, device="cuda")
    for j in range(3):
        cols[:, :To - 1, j].copy_(xv[:, j:j + 2 * (To - 1):2])
    return torch.mm(dy[:M].t(), cols.view(-1, 3 * C))


# correctness of the overlapping-row forward against im2col (rows that do not cross a sample)
ov_fwd()
ref = im2col_fwd()
torch.cuda.synchronize()
yv = y.view(B, Tp // 2, O)[:, :-1].float()
rv = ref.view(B, Tp // 2, O)[:, :-1].float()
print(json.dumps({"check_fwd_rel": float((yv - rv).norm() / rv.norm())}))
for name, fn in (("im2col+hipblaslt fwd", im2col_fwd), ("overlap triad fwd", ov_fwd), ("overlap triad dX", ov_dx),
                 ("im2col+hipblaslt dW", torch_dw), ("overlap triad dW sp4", ov_dw(4)),
                 ("overlap triad dW sp8", ov_dw(8)), ("overlap triad dW sp16", ov_dw(16))):
    ms = bench(fn)
    f = fl * (2.0 / 3.0 if "dX" in name else 1.0)
    print(json.dumps({"case": name, "ms": round(ms, 3), "TFLOPs": round(f / ms / 1e9, 1)}), flush=True)
