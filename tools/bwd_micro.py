"""Microbench of the backward tile GEMMs alone (triad_tile_gemm dQ = dS K and dK = dS^T Q) at
the c3 AV / TV shapes over a random tiled dS. Loads TRIAD_LIB_VARIANT if set
(tools/build_variants.py). Prints one JSON line per case: average ms over `iters` launches
(HIP events) and algorithmic TFLOP/s (2 R Bk Nk_eff 512 per GEMM)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402


def run(B, Nq, Nk, dk, iters, force_sp=None, form=0, ct=0):
    g = ops.Geometry(B, Nq, B, Nk)
    gen = torch.Generator(device="cuda").manual_seed(0)
    q = (torch.randn(B, Nq, 512, device="cuda", generator=gen) * 0.58).to(torch.bfloat16)
    k = (torch.randn(B, Nk, 512, device="cuda", generator=gen) * 0.58).to(torch.bfloat16)
    Qb, Kb = ops.pack_queries(q, g), ops.pack_keys(k, g)
    CT = ops._rup(g.C_pad // 32, 4) if not ct else ct   # ct: compact key tiles (ops._compact's CT)
    dS = (torch.randn((g.R_pad // 32) * CT * 1024, device="cuda", generator=gen) * 1e-3).to(torch.bfloat16)
    alpha = torch.tensor([1.5], device="cuda")
    if dk:
        M, nkt, Bm = CT * 32, g.R_pad // 32, Qb
    else:
        M, nkt, Bm = g.R_pad, (ct or g.C_pad // 32), Kb
    sp = ops._gemm_splits(M // 128, nkt, M) if force_sp is None else force_sp
    out = torch.empty(M, 512, dtype=torch.bfloat16, device="cuda")
    slabs = torch.empty(sp * M * 512, dtype=torch.float32, device="cuda") if sp > 1 else None

    Bp = None
    if form == 16:   # on v_mfma_f32_16x16x32_bf16 (triad_tile_gemm_packed16), vs the 32x32x16 ring form
        Bp = torch.empty(nkt * 32 * 512, dtype=torch.bfloat16, device="cuda")
        call("triad_bfrag_pack16", ptr(Bm), nkt, dk, ptr(Bp), stream_ptr())
        ref = torch.empty_like(out)
        call("triad_tile_gemm", ptr(dS), CT, dk, ptr(Bm), M, nkt, ptr(alpha), sp, ptr(slabs), ptr(ref), stream_ptr())
        call("triad_tile_gemm_packed16", ptr(dS), CT, dk, ptr(Bp), M, nkt, ptr(alpha), sp, ptr(slabs), ptr(out),
             stream_ptr())
        torch.cuda.synchronize()
        d = (out.float() - ref.float()).abs()
        rel = float(d.max() / ref.float().abs().max())
        print(json.dumps({"check": "packed16 vs ring", "dk": dk, "M": M, "max_rel": rel,
                          "frac_differing": float((d > 0).float().mean())}), flush=True)
        assert rel < 1e-2
    def launch():
        if form == 16:
            call("triad_tile_gemm_packed16", ptr(dS), CT, dk, ptr(Bp), M, nkt, ptr(alpha), sp, ptr(slabs), ptr(out),
                 stream_ptr())
        elif form:   # a variant entry point (tools/build_variants.py builds): triad_tile_gemm_form
            call("triad_tile_gemm_form", ptr(dS), CT, dk, ptr(Bm), M, nkt, ptr(alpha), sp, ptr(slabs), ptr(out), form,
                 stream_ptr())
        else:
            call("triad_tile_gemm", ptr(dS), CT, dk, ptr(Bm), M, nkt, ptr(alpha), sp, ptr(slabs), ptr(out),
                 stream_ptr())
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
    return ms, flops / ms / 1e9, sp


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default=os.environ.get("TRIAD_LIB_VARIANT", "default"))
    ap.add_argument("--sweep", action="store_true", help="every split count 1..8 (else the product rule)")
    ap.add_argument("--forms", default="0", help="comma-separated triad_tile_gemm_form forms, alternated")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--ct", default="0", help="AV,TV key-tile counts (compact layout; 0 = padded)")
    ap.add_argument("--heads", default="AV,TV")
    a = ap.parse_args()
    cts = dict(zip(("AV", "TV"), (int(v) for v in a.ct.split(","))))
    for r in range(a.rounds):
        for name, Nq, Nk in (("AV", 199, 212), ("TV", 32, 212)):
            if name not in a.heads.split(","):
                continue
            for dk in (0, 1):
                for fsp in (range(1, 9) if a.sweep else (None,)):
                    for form in (int(f) for f in a.forms.split(",")):
                        res = run(256, Nq, Nk, dk, a.iters, fsp, form, cts.get(name, 0))
                        if res is None:
                            continue
                        ms, tf, sp = res
                        print(json.dumps({"tag": os.path.basename(a.tag), "form": form, "round": r, "head": name,
                                          "gemm": "dK" if dk else "dQ", "ct": cts.get(name, 0), "splits": sp, "ms": round(ms, 4),
                                          "algo_TFLOPs": round(tf, 1)}), flush=True)
