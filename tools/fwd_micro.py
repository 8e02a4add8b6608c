"""Microbench of the fused forward alone (triad_pairsim_fwd) at the c3 AV / TV shapes, with and
without the training dS output. Loads TRIAD_LIB_VARIANT if set (tools/build_variants.py).
Prints one JSON line per case: average ms over `iters` launches (HIP events)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def run(kind, B, Nq, Nk, train, iters, patch=False):
    g = ops.Geometry(B, Nq, B, Nk)
    gen = torch.Generator(device="cuda").manual_seed(0)
    q = (torch.randn(B, Nq, 512, device="cuda", generator=gen) * 0.58).to(torch.bfloat16)
    k = (torch.randn(B, Nk, 512, device="cuda", generator=gen) * 0.58).to(torch.bfloat16)
    Qb, Kb = ops.pack_queries(q, g), ops.pack_keys(k, g)
    temp = torch.tensor([1.5], device="cuda")
    nparts = 2 * call("triad_pairsim_nparts", g.R_pad, g.Bk)  # room for 128-row workgroup variants
    rowmax = torch.empty(g.Bk, g.R_pad, device="cuda")
    argmax = torch.empty(g.Bk, g.R_pad, dtype=torch.int32, device="cuda")
    nn = torch.empty(nparts, dtype=torch.float64, device="cuda")
    diagS = torch.empty(B, Nq, g.Nk_pad, device="cuda")
    CT = ops._rup(g.C_pad // 32, 4)
    dS = torch.empty((g.R_pad // 32) * CT * 1024, dtype=torch.bfloat16, device="cuda") if train else None
    stp = torch.empty(nparts, dtype=torch.float64, device="cuda") if train else None

    def launch():
        call("triad_pairsim_fwd", ptr(Qb), ptr(Kb), g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, 512,
             ptr(temp), ops.CLAMP_LO[kind], 0, 0, ptr(rowmax), ptr(argmax), ptr(nn), None, ptr(dS), CT, ptr(stp),
             None, stream_ptr())
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2.0 * g.R * g.Bk * g.Nk_eff * 512
    if not patch:
        return ms, flops / ms / 1e9
    # the max-term patch over this forward's dS and argmax (full key tiles, no diagonal term)
    dclip = torch.randn(g.Bq, g.Bk, device="cuda", generator=gen) * 1e-3
    qw = torch.rand(g.R_pad, device="cuda", generator=gen)
    nmp = int(os.environ.get("TRIAD_PATCH_NMP", "1024"))
    mp = torch.empty(nmp, dtype=torch.float64, device="cuda")

    def patch_launch():
        call("triad_dS_patch_tiles", ptr(dS), CT, g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, 0, ptr(argmax),
             ptr(rowmax), ptr(dclip), ptr(qw), 1.0, None, 0.0, ptr(mp), nmp, ptr(temp), None, stream_ptr())
    for _ in range(3):
        patch_launch()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        patch_launch()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters, 0.0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default=os.environ.get("TRIAD_LIB_VARIANT", "default"))
    ap.add_argument("--patch", action="store_true", help="time triad_dS_patch_tiles (max term) instead")
    a = ap.parse_args()
    if a.patch:
        for name, kind, Nq, Nk in (("AV", ops.AV, 199, 205), ("TV", ops.TV, 32, 205)):
            ms, _ = run(kind, 256, Nq, Nk, True, a.iters, patch=True)
            print(json.dumps({"tag": os.path.basename(a.tag), "head": name, "patch_ms": round(ms, 4),
                              "nmp": int(os.environ.get("TRIAD_PATCH_NMP", "1024"))}), flush=True)
        sys.exit(0)
    for name, kind, Nq, Nk in (("AV", ops.AV, 199, 205), ("TV", ops.TV, 32, 205)):
        for train in (True, False):
            ms, tf = run(kind, 256, Nq, Nk, train, a.iters)
            print(json.dumps({"tag": os.path.basename(a.tag), "head": name, "train": train, "ms": round(ms, 4),
                              "algo_TFLOPs": round(tf, 1)}), flush=True)
