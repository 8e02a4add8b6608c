"""A/B of the head backward forms: the materialised tiled dS (forward writes
the unit l_nonneg gradient, dS_patch, two tile GEMMs) against the memory-bounded recompute form
(eval forward, then ops.recompute_backward: S recomputed per key-sample chunk, dS written one
chunk at a time, dQ partials summed). At the c3 AV / TV head shapes (256 x 256 samples) and at
the c4 per-rank Mode G shape (256 query samples x 2048 key samples, materialised dS 47 GB).
Prints one JSON line per (shape, form): ms of forward + backward, peak dS bytes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402

D = 512


def setup(kind, Bq, Nq, Bk, Nk):
    g = ops.Geometry(Bq, Nq, Bk, Nk)
    gen = torch.Generator(device="cuda").manual_seed(0)
    q = (torch.randn(Bq, Nq, D, device="cuda", generator=gen) * 0.58).to(torch.bfloat16)
    k = (torch.randn(Bk, Nk, D, device="cuda", generator=gen) * 0.58).to(torch.bfloat16)
    t = dict(g=g, Qb=ops.pack_queries(q, g), Kb=ops.pack_keys(k, g),
             temp=torch.tensor([1.5], device="cuda"),
             rowmax=torch.empty(g.Bk, g.R_pad, device="cuda"),
             argmax=torch.empty(g.Bk, g.R_pad, dtype=torch.int32, device="cuda"),
             diagS=torch.empty(Bq, Nq, g.Nk_pad, device="cuda"),
             qw=torch.full((g.R,), 1.0 / Nq, device="cuda"),
             dclip=torch.randn(Bq, Bk, device="cuda", generator=gen) * 1e-3,
             gdiag=torch.zeros(Bq, Nq, g.Nk_pad, device="cuda"),
             coef=torch.tensor([1.0, 0.15 * 2 / (Bq * Bk * Nq * Nk), 0.01, 20.0], device="cuda"))
    t["nparts"] = call("triad_pairsim_nparts", g.R_pad, g.Bk)
    return t


def forward(kind, t, dS, CT):
    g = t["g"]
    nn = torch.empty(t["nparts"], dtype=torch.float64, device="cuda")
    stp = torch.empty(t["nparts"], dtype=torch.float64, device="cuda") if dS is not None else None
    call("triad_pairsim_fwd", ptr(t["Qb"]), ptr(t["Kb"]), g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, D,
         ptr(t["temp"]), ops.CLAMP_LO[kind], 1, 0, ptr(t["rowmax"]), ptr(t["argmax"]), ptr(nn), ptr(t["diagS"]),
         ptr(dS), CT, ptr(stp), None, stream_ptr())


def materialised(kind, t, dS, CT):
    g = t["g"]
    st = stream_ptr()
    forward(kind, t, dS, CT)
    mp = torch.empty(1024, dtype=torch.float64, device="cuda")
    call("triad_dS_patch", ptr(dS), CT, g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, 0, ptr(t["argmax"]),
         ptr(t["rowmax"]), ptr(t["dclip"]), ptr(t["qw"]), 1.0, ptr(t["gdiag"]), 1.0, ptr(mp), 1024, ptr(t["temp"]), st)
    dQ = torch.empty(g.R_pad, D, dtype=torch.bfloat16, device="cuda")
    dK = torch.empty(CT * 32, D, dtype=torch.bfloat16, device="cuda")
    ops.tile_gemm(dS, CT, 0, t["Kb"], g.R_pad, g.C_pad // 32, t["temp"], dQ, st)
    ops.tile_gemm(dS, CT, 1, t["Qb"], CT * 32, g.R_pad // 32, t["temp"], dK, st)


def recompute(kind, t, chunk):
    g = t["g"]
    forward(kind, t, None, 0)
    ops.recompute_backward(g, t["Qb"], t["Kb"], t["temp"], kind, 0, t["argmax"], t["dclip"], t["qw"], t["gdiag"],
                           t["coef"], True, True, chunk, stream_ptr())


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    cases = [("c3 AV", ops.AV, 256, 199, 256, 205, 5), ("c3 TV", ops.TV, 256, 32, 256, 205, 5),
             ("c4 AV per rank", ops.AV, 256, 199, 2048, 205, 2)]
    for name, kind, Bq, Nq, Bk, Nk, iters in cases:
        t = setup(kind, Bq, Nq, Bk, Nk)
        g = t["g"]
        CT = ops._rup(g.C_pad // 32, 4)
        full = ops.ds_bytes(g)
        dS = torch.empty(full // 2, dtype=torch.bfloat16, device="cuda")
        ms = timeit(lambda: materialised(kind, t, dS, CT), iters)
        print(json.dumps({"shape": name, "form": "materialised", "ms": round(ms, 3), "dS_bytes": full}), flush=True)
        del dS
        torch.cuda.empty_cache()
        for budget in (16 << 30, 4 << 30, 1 << 30):
            chunk = ops.ds_chunk_samples(g, budget)
            if chunk == g.Bk:   # fits: the product would materialise; time the one-chunk recompute form
                chunk = g.Bk
            per = (g.R_pad // 32) * (g.Nk_pad // 32) * 2048
            ms = timeit(lambda: recompute(kind, t, chunk), iters)
            print(json.dumps({"shape": name, "form": f"recompute chunk={chunk}", "ms": round(ms, 3),
                              "dS_bytes": per * chunk}), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
