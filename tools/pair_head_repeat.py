"""The training pair head (ops.contrastive_heads_av_tv) on fixed c3-shaped inputs whose keys come
from ops.patch_dropout (compact key tiles), repeated in one process: every repeat's key / query
gradients compared bit for bit with the first; for a differing one, which key rows differ (sample,
key, tile). Experiments only.

usage: python tools/pair_head_repeat.py [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402

dev = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(7)
    B, N, Na, Nt = 256, 256, 199, 32
    A = (torch.randn(B, Na, 512, generator=g) * 0.58).to(torch.bfloat16)
    T = (torch.randn(B, Nt, 512, generator=g) * 0.58).to(torch.bfloat16)
    X = (torch.randn(B, N, 512, generator=g) * 0.58).to(torch.bfloat16)
    keep_av = torch.rand(B, N, generator=g) < 0.75
    keep_tv = torch.rand(B, N, generator=g) < 0.75
    mask = torch.ones(B, Nt, dtype=torch.long, device=dev)
    first = None
    heads = []
    orig_compact = ops._compact

    def spy(h):   # keep each head's compact dS to compare it across repeats
        orig_compact(h)
        heads.append(h)
    ops._compact = spy

    def valid_ds(h):   # the stored tiles' part of the tiled dS: [R_pad/32][nct] tiles of 1024
        return h.dS.view(h.g.R_pad // 32, h.CT, 1024)[:, :h.nct].clone()
    for r in range(a.reps):
        heads.clear()
        a_ = A.to(dev).requires_grad_(True)
        t_ = T.to(dev).requires_grad_(True)
        x = X.to(dev)
        va0, vt0 = ops.patch_dropout(x, keep_av), ops.patch_dropout(x, keep_tv)
        va, vt = va0.detach().requires_grad_(True), vt0.detach().requires_grad_(True)
        for v, v0 in ((va, va0), (vt, vt0)):   # detach() drops the attribute: carry it over
            setattr(v, ops.KEPT_ROWS_ATTR, getattr(v0, ops.KEPT_ROWS_ATTR))
        tg = torch.tensor(1.5, device=dev, requires_grad=True)
        (la, _, _), (lt, _, _) = ops.contrastive_heads_av_tv(a_, va, t_, vt, tg, mask, threshold=0.8,
                                                             sparsity_weight=0.01)
        torch.cuda.synchronize()
        fwd_ds = [valid_ds(h) for h in heads]
        (la[0] + lt[0]).backward()
        torch.cuda.synchronize()
        cur = {"gA": a_.grad, "gT": t_.grad, "gVa": va.grad, "gVt": vt.grad}
        if len(heads) == 2:
            cur.update(dS_fwd_av=fwd_ds[0], dS_fwd_tv=fwd_ds[1], dS_bwd_av=valid_ds(heads[0]),
                       dS_bwd_tv=valid_ds(heads[1]))
        if first is None:
            first = cur
            continue
        rep = {"rep": r}
        for k in cur:
            d = cur[k] != first[k]
            n = int(d.sum())
            rep[k] = n
            if n and k.startswith("dS"):
                rows = torch.nonzero((cur[k] != first[k]).any(-1))
                rep[k + "_tiles(rt,ct)"] = rows[:8].tolist()
            if n and k.startswith("gV"):
                rows = torch.nonzero(d.any(-1))
                keys = rows[:, 1]
                rep[k + "_samples"] = sorted(set(rows[:, 0].tolist()))[:12]
                rep[k + "_tiles"] = sorted(set((keys // 32).tolist()))
                rep[k + "_nrows"] = int(rows.shape[0])
        print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
