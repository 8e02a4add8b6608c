"""HuBERT conv-stack weight gradients (frontend._weight_grad_rows: dW [512][3C or 2C] = dY^T X over
the layer's B*Tp/2 frame-pair rows, X rows overlapping) at the c3 sizes: the policy's 8 splits of
256 x 128 tiles put 24 x 8 = 192 workgroups on 256 CUs. Times tile form x split count, GEMM + slab
sum per call, with the relative error against an fp32 torch product.

  python tools/conv_dw_ab.py [--iters 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import _lib  # noqa: E402
from triad_amd._lib import TriadError, call, ptr, stream_ptr  # noqa: E402


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
    O, C = 512, 512
    # (rows, N): kernel-3 layers (N = 3C over pair rows of stride 2C) and kernel-2 layers (N = 2C)
    shapes = [(1638400, 3 * C), (819200, 3 * C), (409600, 3 * C), (204800, 3 * C), (102400, 2 * C)]
    variants = [("policy f0 s8", 0, 8), ("f2 s10", 2, 10), ("f2 s16+xcd", 2 | 8, 16), ("f4 s21", 4, 21),
                ("f4 s16+xcd", 4 | 8, 16), ("f4 s24+xcd", 4 | 8, 24), ("f1 s5", 1, 5), ("f2 s8", 2, 8)]
    for rows, N in shapes:
        g = torch.Generator(device="cuda").manual_seed(rows + N)
        dy = (torch.randn(rows, O, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        ldx = 2 * C
        xbuf = torch.randn(rows + 2, ldx, device="cuda", generator=g).to(torch.bfloat16)
        X = xbuf.view(-1).as_strided((rows, N), (ldx, 1))
        ref = torch.mm(dy.t().float(), X.float()) if rows <= 409600 else None
        for rnd in range(2):
            for name, form, sp in variants:
                slabs = torch.empty(sp * O * N, dtype=torch.float32, device="cuda")
                out = torch.empty(O, N, dtype=torch.float32, device="cuda")

                def run():
                    call("triad_gemm_bf16_splitk_form", ptr(dy), O, 0, ptr(xbuf), ldx, 0, O, N, rows, sp, None,
                         ptr(slabs), ptr(out), 0, form, stream_ptr())
                try:
                    ms = bench(run, args.iters)
                except TriadError as e:
                    print(json.dumps(dict(rows=rows, N=N, variant=name, error=str(e))), flush=True)
                    continue
                rec = dict(rows=rows, N=N, round=rnd, variant=name, ms=round(ms, 4),
                           TFLOPs=round(2.0 * O * N * rows / ms / 1e9, 1))
                if ref is not None and rnd == 0:
                    rec["rel_err"] = float((out - ref).norm() / ref.norm())
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
