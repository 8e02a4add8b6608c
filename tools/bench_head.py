"""Micro-benchmark of the fused contrastive head (fwd+bwd) at config-3 shapes."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402


def run(kind, B, Nq, Nk, iters, warm):
    g = torch.Generator(device="cuda").manual_seed(0)
    q = (torch.randn(B, Nq, 512, device="cuda", generator=g) * 0.58).to(torch.bfloat16).requires_grad_(True)
    k = (torch.randn(B, Nk, 512, device="cuda", generator=g) * 0.58).to(torch.bfloat16).requires_grad_(True)
    t = torch.tensor(1.5, device="cuda", requires_grad=True)
    mask = torch.ones(B, Nq, device="cuda") if kind == ops.TV else None

    def step():
        losses, _, _ = ops.contrastive_head(kind, q, k, t, q_mask=mask, threshold=0.8, sparsity_weight=0.01)
        losses[0].backward()
        return losses
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    flops = 6.0 * B * B * Nq * Nk * 512
    return dt, flops


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--B", type=int, default=256)
    a = ap.parse_args()
    for name, kind, Nq, Nk in (("AV", ops.AV, 199, 205), ("TV", ops.TV, 32, 205)):
        dt, fl = run(kind, a.B, Nq, Nk, a.iters, a.warm)
        print(json.dumps({"head": name, "B": a.B, "Nq": Nq, "Nk": Nk, "ms": dt * 1e3,
                          "algo_TFLOPs": fl / dt / 1e12}), flush=True)
