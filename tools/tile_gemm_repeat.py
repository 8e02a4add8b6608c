"""Repeat one tile-GEMM case many times in one process and compare every result bit for bit with
the first (and the first with an fp32 torch product): a determinism check for an intermittent
mismatch (tests/test_head_gpu.py::test_tile_gemm_vs_torch). Prints one JSON line per case: the
number of differing repeats and, for the first differing one, the differing rows / columns.
Experiments only.

usage: python tools/tile_gemm_repeat.py [--reps 200]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402
from triad_amd._lib import stream_ptr  # noqa: E402

dev = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--cases", default="7x36,16x64,400x24,3x4", help="panels x key tiles (x dk-only)")
    a = ap.parse_args()
    for case in a.cases.split(","):
        panels, ct = (int(v) for v in case.split("x"))
        g = torch.Generator(device=dev).manual_seed(panels * 100 + ct)
        R_pad, CT = panels * 128, ct
        dS = (torch.randn(R_pad // 32 * CT * 1024, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        K = torch.randn(CT * 32, 512, device=dev, generator=g).to(torch.bfloat16)
        Q = torch.randn(R_pad, 512, device=dev, generator=g).to(torch.bfloat16)
        alpha = torch.tensor([0.75], device=dev)
        for dk in (0, 1):
            if dk and CT % 4:
                continue
            M, nkt, B = (CT * 32, R_pad // 32, Q) if dk else (R_pad, CT, K)
            first = None
            bad = 0
            info = None
            for r in range(a.reps):
                out = torch.empty(M, 512, dtype=torch.bfloat16, device=dev)
                ops.tile_gemm(dS, CT, dk, B, M, nkt, alpha, out, stream_ptr())
                if first is None:
                    torch.cuda.synchronize()
                    first = out
                    continue
                if not torch.equal(out, first):
                    bad += 1
                    if info is None:
                        d = (out != first)
                        rows = torch.nonzero(d.any(1)).flatten().tolist()
                        cols = torch.nonzero(d.any(0)).flatten().tolist()
                        info = {"rep": r, "rows": rows[:40], "n_rows": len(rows), "cols": cols[:16],
                                "n_cols": len(cols)}
            torch.cuda.synchronize()
            print(json.dumps({"panels": panels, "ct": ct, "dk": dk, "reps": a.reps, "differing_repeats": bad,
                              "first_diff": info}), flush=True)


if __name__ == "__main__":
    main()
