"""Split-K weight gradients with each split's workgroups on ONE XCD (form flag 8, gemm.hip
tile_split) against the default tile remap, at the projection-head and backbone dW shapes of the
c3 step: ms per call (GEMM + slab reduction), and a bit-identity check of the flag at equal
form / splits (placement must not change a result).

  python tools/dw_xcd_ab.py [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import _lib  # noqa: E402
from triad_amd._lib import TriadError, call, ptr, stream_ptr  # noqa: E402
from triad_amd.linear import _form_splits  # noqa: E402
from triad_amd.ops import _splitk  # noqa: E402


def bench(fn, iters):
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
    args = ap.parse_args()
    _lib.load()
    shapes = [("proj", 65536, 512, 512), ("proj", 65536, 512, 768), ("proj", 50944, 512, 512),
              ("proj", 50944, 512, 768), ("proj", 8192, 512, 512), ("proj", 8192, 512, 768),
              ("backbone", 50944, 768, 768), ("backbone", 50944, 2304, 768), ("backbone", 50944, 3072, 768),
              ("backbone", 50944, 768, 3072), ("backbone", 8192, 768, 768), ("backbone", 8192, 3072, 768)]
    for kind, M, O, K in shapes:
        g = torch.Generator(device="cuda").manual_seed(M + O + K)
        dy = (torch.randn(M, O, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        ref = torch.mm(dy.t().float(), x.float())
        if kind == "proj":
            base = (0, _splitk(M, (O // 128) * (K // 128)))
        else:
            base = _form_splits(M, O, K)
        variants = [("policy", base[0], base[1])]
        for form in (1, 4):
            for sp in (8, 16, 24, 32):
                if M // sp < 512:
                    continue
                variants.append((f"f{form}s{sp}", form, sp))
                variants.append((f"f{form}s{sp}+xcd", form | 8, sp))
        outs = {}
        for name, form, sp in variants:
            slabs = torch.empty(sp * O * K, device="cuda")
            dw = torch.empty(O, K, dtype=torch.bfloat16, device="cuda")

            def run():
                call("triad_gemm_bf16_splitk_form", ptr(dy), O, 0, ptr(x), K, 0, O, K, M, sp, None, ptr(slabs),
                     ptr(dw), 1, form, stream_ptr())
            try:
                ms = bench(run, args.iters)
            except TriadError as e:
                print(json.dumps(dict(kind=kind, M=M, O=O, K=K, variant=name, error=str(e))), flush=True)
                continue
            outs[name] = dw.clone()
            err = float((dw.float() - ref).norm() / ref.norm())
            rec = dict(kind=kind, M=M, O=O, K=K, variant=name, splits=sp, ms=round(ms, 4),
                       TFLOPs=round(2.0 * M * O * K / ms / 1e9, 1), rel_err=round(err, 6))
            if name.endswith("+xcd"):
                rec["bit_identical_to_default_map"] = bool(torch.equal(dw, outs[name[:-4]]))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
