"""Projection head (ops.projection_head) forward / backward at the c3 row counts: ms per call and
algorithmic TFLOP/s (fwd 2 rows (H 512 + 512 512), bwd twice that), HIP-event timed, plus the
parity of one call against the bf16-autocast emulation (oracle/ref_cpu.projection_head on the
device, fp32, autograd).

usage: python tools/projhead_micro.py [--iters N]"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
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
    ap.add_argument("--forms", default="fused,passes")
    a = ap.parse_args()
    from oracle import ref_cpu
    from triad_amd import _lib, ops
    _lib.load()
    dev = "cuda"
    cases = [(f, n, M, H) for n, M, H in (("visual", 65536, 768), ("audio", 50944, 768), ("text", 8192, 768),
                                         ("c5-visual", 43808, 1024)) for f in a.forms.split(",")]
    for form, name, M, H in cases:
        torch.manual_seed(0)
        p1, ln, p2 = nn.Linear(H, 512).to(dev), nn.LayerNorm(512).to(dev), nn.Linear(512, 512).to(dev)
        with torch.no_grad():
            ln.weight.uniform_(0.5, 1.5)
            ln.bias.uniform_(-0.2, 0.2)
        h = torch.randn(M, H, device=dev).to(torch.bfloat16).requires_grad_(True)
        gy = (torch.randn(M, 512, device=dev) * 0.01).to(torch.bfloat16)
        y = ops.projection_head(h, p1, ln, p2, form=form)
        fwd_ms = timed(lambda: ops.projection_head(h, p1, ln, p2, form=form), a.iters)

        def fb():
            out = ops.projection_head(h, p1, ln, p2, form=form)
            out.backward(gy)
        fb_ms = timed(fb, a.iters)
        fl = 2.0 * M * (H * 512 + 512 * 512)
        # parity vs the autocast emulation (fp32 autograd through bf16 roundings)
        hr = h.detach().float().requires_grad_(True)
        ws = [t.detach().float().requires_grad_(True) for t in (p1.weight, p1.bias, ln.weight, ln.bias, p2.weight, p2.bias)]
        yr = ref_cpu.projection_head(hr, *ws, amp=True)
        yr.backward(gy.float())
        for m in (p1, ln, p2):
            for t in m.parameters():
                t.grad = None
        h.grad = None
        y = ops.projection_head(h, p1, ln, p2, form=form)
        y.float().backward(gy.float())
        rel = lambda g, r: float((g.float() - r).norm() / r.norm())
        errs = {"y": rel(y.detach(), yr.detach()), "dh": rel(h.grad, hr.grad),
                "dW1": rel(p1.weight.grad, ws[0].grad), "db1": rel(p1.bias.grad, ws[1].grad),
                "dgamma": rel(ln.weight.grad, ws[2].grad), "dbeta": rel(ln.bias.grad, ws[3].grad),
                "dW2": rel(p2.weight.grad, ws[4].grad), "db2": rel(p2.bias.grad, ws[5].grad)}
        print(json.dumps({"form": form, "head": name, "M": M, "H": H, "fwd_ms": round(fwd_ms, 4), "fwd_TFLOPs": fl / fwd_ms / 1e9,
                          "fwd_bwd_ms": round(fb_ms, 4), "bwd_ms": round(fb_ms - fwd_ms, 4),
                          "bwd_TFLOPs": 2 * fl / (fb_ms - fwd_ms) / 1e9,
                          "rel_err": {k: round(v, 5) for k, v in errs.items()}}), flush=True)


if __name__ == "__main__":
    main()
