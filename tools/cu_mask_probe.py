"""Do CU-masked streams keep the round-4 co-residency hazard away?

1. Placement: for single-bit CU masks, where do a masked stream's workgroups run (XCC id and
   the HW_ID register's CU / SH / SE fields, read in tools/hazard/hazard.hip where_kernel)?
2. Hazard: PyTorch's bf16 column sum (the measured victim) on one stream beside the MFMA +
   LDS-DMA aggressor (mix_loop) and the library's eight-wave GEMM on another, with the two
   streams (a) unmasked, (b) on disjoint XCDs, (c) on disjoint CU halves of every XCD.
One JSON line per result.  python tools/cu_mask_probe.py [--reps 100]"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from triad_amd._lib import call, ptr  # noqa: E402

dev = torch.device("cuda")


def hip():
    h = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    h.hipExtStreamCreateWithCUMask.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]
    h.hipStreamDestroy.argtypes = [C.c_void_p]
    return h


def masked_stream(h, bits, ncu):
    words = (C.c_uint32 * ((ncu + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = C.c_void_p()
    rc = h.hipExtStreamCreateWithCUMask(C.byref(s), len(words), words)
    assert rc == 0, rc
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    args = ap.parse_args()
    torch.zeros(1, device=dev)
    h = hip()
    import hazard_probe
    hz = hazard_probe.lib()
    hz.hz_where.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(2 * 64, dtype=torch.int32, device=dev)
    bit_xcc, bit_cu = {}, {}
    for b in range(ncu):
        s = masked_stream(h, [b], ncu)
        assert hz.hz_where(C.c_void_p(out.data_ptr()), 64, s) == 0
        torch.cuda.synchronize()
        v = out.view(64, 2).cpu()
        places = sorted({(int(x), (int(w) >> 8) & 0xff) for x, w in v.tolist()})
        h.hipStreamDestroy(s)
        bit_xcc[b] = places[0][0] if len(places) == 1 else None
        bit_cu[b] = places
        if b < 40 or len(places) != 1:
            print(json.dumps(dict(bit=b, places=places)), flush=True)
    by_xcc = {}
    for b, x in bit_xcc.items():
        by_xcc.setdefault(x, []).append(b)
    print(json.dumps(dict(bits_per_xcc={str(k): v for k, v in sorted(by_xcc.items(), key=lambda kv: str(kv[0]))})),
          flush=True)
    if None in by_xcc or len(by_xcc) != 8:
        print(json.dumps(dict(note="placement not one XCC per bit; hazard part skipped")))
        return

    # hazard: aggressors / victim on two streams, masked three ways
    g = torch.Generator(device=dev).manual_seed(1)
    src = torch.randn(1 << 22, device=dev, generator=g)
    scratch = torch.empty(1 << 20, device=dev)
    a = torch.randn(33280, 768, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(3072, 768, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    gout = torch.empty(33280, 3072, device=dev, dtype=torch.bfloat16)
    sb = (torch.randn(768, 2304, device=dev, generator=g) * 0.01).to(torch.bfloat16)

    def mix(stream):
        rc = hz.hz_aggressor(2, C.c_void_p(src.data_ptr()), src.numel() // 4, C.c_void_p(scratch.data_ptr()), 256,
                             1000, C.c_void_p(stream.cuda_stream))
        assert rc == 0, rc

    def gemm(stream):
        call("triad_gemm_bf16_form", ptr(a), 768, 1, ptr(w), 768, 1, 33280, 3072, 768, None, ptr(gout), 3072, 1, 4,
             C.c_void_p(stream.cuda_stream))

    xccs = sorted(by_xcc)
    half_a = [b for x in xccs[:4] for b in by_xcc[x]]
    half_b = [b for x in xccs[4:] for b in by_xcc[x]]
    cu_a = [b for x in xccs for b in sorted(by_xcc[x])[:len(by_xcc[x]) // 2]]
    cu_b = [b for x in xccs for b in sorted(by_xcc[x])[len(by_xcc[x]) // 2:]]
    layouts = {"unmasked": None, "disjoint XCDs (4 + 4)": (half_a, half_b),
               "same XCDs, disjoint CU halves": (cu_a, cu_b)}
    for lname, masks in layouts.items():
        if masks is None:
            sa, sv = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
            raw = []
        else:
            ra, rv = masked_stream(h, masks[0], ncu), masked_stream(h, masks[1], ncu)
            raw = [ra, rv]
            sa, sv = torch.cuda.ExternalStream(ra.value, device=dev), torch.cuda.ExternalStream(rv.value, device=dev)
        for aname, agg in (("mix_loop", mix), ("triad_gemm eight-wave", gemm)):
            with torch.cuda.stream(sv):
                ref = sb.sum(0).clone()
            torch.cuda.synchronize()
            bad = 0
            for _ in range(args.reps):
                sa.wait_stream(torch.cuda.current_stream())
                sv.wait_stream(torch.cuda.current_stream())
                agg(sa)
                with torch.cuda.stream(sv):
                    got = sb.sum(0).clone()
                agg(sa)
                torch.cuda.synchronize()
                bad += int(not torch.equal(got, ref))
            print(json.dumps(dict(layout=lname, aggressor=aname, victim="torch bf16 sum(0) 768x2304",
                                  reps=args.reps, mismatching=bad)), flush=True)
        torch.cuda.synchronize()
        for r in raw:
            h.hipStreamDestroy(r)


if __name__ == "__main__":
    main()
