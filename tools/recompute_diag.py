"""Gradient error of the AV head against the fp64 oracle by backward form (fast materialised dS,
recompute in one chunk, recompute in 4-sample chunks) at a given shape: prints one JSON line per
form with the relative L2 errors of dQ / dK and d/dtemp."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_cpu  # noqa: E402
from triad_amd import ops  # noqa: E402


def rel(a, b):
    return float((a.double().cpu() - b.double()).norm() / b.double().norm())


def main(B, Na, Nv, seed):
    g = torch.Generator().manual_seed(seed)
    A = (torch.randn(B, Na, 512, generator=g) * 0.58).to(torch.bfloat16).float()
    V = (torch.randn(B, Nv, 512, generator=g) * 0.58).to(torch.bfloat16).float()
    Ar, Vr = A.double().requires_grad_(True), V.double().requires_grad_(True)
    tr = torch.tensor(1.4, dtype=torch.float64, requires_grad=True)
    ref_cpu.av_loss(Ar, Vr, tr)[0].backward()
    geo = ops.Geometry(B, Na, B, ((Nv + 31) // 32) * 32)
    per = (geo.R_pad // 32) * (geo.Nk_pad // 32) * 2048
    for name, budget, mix in (("fast", None, False), ("recompute1", None, True), ("chunk4", 4 * per, False)):
        Ag = A.to("cuda", torch.bfloat16).requires_grad_(True)
        Vg = V.to("cuda", torch.bfloat16).requires_grad_(True)
        tg = torch.tensor(1.4, device="cuda", requires_grad=True)
        losses, st, clip = ops.contrastive_head(ops.AV, Ag, Vg, tg, ds_budget=budget)
        # mix: route the same total through its components (forces the recompute backward)
        (losses[1] + losses[2] if mix else losses[0]).backward()
        print(json.dumps({"form": name, "B": B, "Na": Na, "Nv": Nv, "dA": rel(Ag.grad, Ar.grad),
                          "dV": rel(Vg.grad, Vr.grad), "dtemp": float(tg.grad), "dtemp_ref": float(tr.grad)}),
              flush=True)


if __name__ == "__main__":
    for B, Na, Nv in ((5, 300, 40), (5, 61, 40), (10, 61, 90), (5, 300, 96), (4, 300, 40)):
        main(B, Na, Nv, 500 + B)
