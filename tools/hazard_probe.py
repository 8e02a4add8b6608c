"""Which ingredient of the library's GEMMs disturbs co-resident packed-FP32 arithmetic?
(kernels: tools/hazard/hazard.hip -> tools/hazard/libhazard.so, built by this script if absent)

tools/reduce_race.py showed PyTorch's bf16 column sums returning different values in 40-95 % of
launches while triad_gemm_bf16 (128 x 128 or eight-wave form) ran on another stream -- and never
beside rocBLAS GEMMs, alone, or for fp32 sums (whose inner loop is scalar). Each victim runs
alone (reference), then `reps` times beside each aggressor (queued first on the main stream,
the victim on a second stream so its workgroups share the CUs), compared bit for bit.
One JSON line per (aggressor, victim): mismatching launches, worst elements. Third probe
(lds_colsum / xblk_colsum*): is it the LDS hand-off inside a workgroup or the cross-workgroup
hand-off of one launch that goes wrong (every disturbed victim has the latter)?"""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402

HZ = os.path.join(ROOT, "tools", "hazard", "libhazard.so")
dev = torch.device("cuda")
REPS = int(os.environ.get("REPS", "100"))


def lib():
    if not os.path.exists(HZ):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-shared", "-fPIC",
                        os.path.join(ROOT, "tools", "hazard", "hazard.hip"), "-o", HZ], check=True)
    h = C.CDLL(HZ)
    h.hz_aggressor.argtypes = [C.c_int, C.c_void_p, C.c_longlong, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    h.hz_victim.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    h.hz_victim2.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                             C.c_void_p]
    h.hz_copy.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_longlong, C.c_int, C.c_void_p]
    return h


def main():
    h = lib()
    g = torch.Generator(device=dev).manual_seed(1)
    src = torch.randn(1 << 22, device=dev, generator=g)
    scratch = torch.empty(1 << 20, device=dev)
    a = torch.randn(33280, 768, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(3072, 768, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    gout = torch.empty(33280, 3072, device=dev, dtype=torch.bfloat16)
    ma = torch.randn(16384, 1024, device=dev, generator=g).to(torch.bfloat16)
    mb = torch.randn(1024, 4096, device=dev, generator=g).to(torch.bfloat16)

    def agg(kind, blocks, iters):
        def run():
            rc = h.hz_aggressor(kind, C.c_void_p(src.data_ptr()), src.numel() // 4, C.c_void_p(scratch.data_ptr()),
                                blocks, iters, C.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
        return run

    def gemm(form):
        def run():
            call("triad_gemm_bf16_form", ptr(a), 768, 1, ptr(w), 768, 1, 33280, 3072, 768, None, ptr(gout), 3072, 1,
                 form, stream_ptr(dev))
        return run

    aggressors = {
        "none": lambda: None,
        "mfma_loop (32x32x16 chains, registers only)": agg(0, 256, 20000),
        "dma_loop (global_load_lds + vmcnt + barrier, no MFMA)": agg(1, 256, 1000),
        "mix_loop (both)": agg(2, 256, 1000),
        "valu_loop (scalar fp32 FMAs)": agg(3, 256, 200000),
        "triad_gemm form 1 (128x128)": gemm(1),
        "triad_gemm form 4 (eight-wave)": gemm(4),
        "torch.mm (rocBLAS)": lambda: torch.mm(ma, mb),
        "dma_valu_loop (global_load_lds beside scalar VALU, no MFMA)": agg(4, 256, 1000),
    }
    if os.environ.get("AGGRESSORS"):
        keep = os.environ["AGGRESSORS"].split("|")
        aggressors = {k: v for k, v in aggressors.items() if any(k.startswith(x) for x in keep)}
    n = 65536
    x = torch.randn(n, 2, device=dev, generator=g)
    rows = 768
    m = torch.randn(rows, 2304 // 2, 2, device=dev, generator=g)
    sb = (torch.randn(768, 2304, device=dev, generator=g) * 0.01).to(torch.bfloat16)

    def vic(kind, inp, cnt, r=0):
        def run():
            out = torch.empty_like(inp if kind != 2 else inp[0])
            rc = h.hz_victim(kind, C.c_void_p(inp.data_ptr()), C.c_void_p(out.data_ptr()), cnt, r,
                             C.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
            return out
        return run

    u16 = (torch.randn(rows, 2304, device=dev, generator=g) * 0.01).to(torch.bfloat16).view(torch.int16)

    def vic16(kind):
        def run():
            out = torch.empty(2304, device=dev)
            rc = h.hz_victim(kind, C.c_void_p(u16.data_ptr()), C.c_void_p(out.data_ptr()), 2304 // 2, rows,
                             C.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
            return out
        return run

    def vic2(kind, nsplit=8):
        def run():   # staging / semaphores allocated per launch on the launching stream, as PyTorch does
            out = torch.empty(2304, device=dev)
            staging = torch.empty(nsplit * 2304, device=dev)
            sem = torch.zeros(16, dtype=torch.int32, device=dev)
            rc = h.hz_victim2(kind, C.c_void_p(u16.data_ptr()), C.c_void_p(staging.data_ptr()),
                              C.c_void_p(sem.data_ptr()), C.c_void_p(out.data_ptr()), 2304, rows, nsplit,
                              C.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
            return out
        return run

    cp_in = torch.randint(-2**31, 2**31 - 1, (768 * 2304 // 2,), dtype=torch.int32, device=dev, generator=g)

    def vcopy(kind):
        def run():   # out = in, 16-byte loads (1 or 4 in flight per thread, or sc1): any differing word is a bad load
            out = torch.empty_like(cp_in)
            rc = h.hz_copy(kind, C.c_void_p(cp_in.data_ptr()), C.c_void_p(out.data_ptr()), cp_in.numel() // 4, 256,
                           C.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
            return out
        return run

    victims = {
        "copy16 depth1 (one 16-byte load per thread in flight)": vcopy(13),
        "copy16 depth4 (four 16-byte loads in flight, as colsum8)": vcopy(14),
        "copy16 depth4 sc1 (the same, loads bypass L1)": vcopy(15),
        "lds_colsum (8 row-threads per column combined through LDS, one launch, no cross-WG hand-off)": vic2(6),
        "xblk_colsum plain (cross-WG hand-off: threadfence + atomic semaphore, last WG plain loads)": vic2(7),
        "xblk_colsum acquire (the same + agent-scope acquire fence after the semaphore)": vic2(8),
        "xblk_colsum atomic-load (the same, partials read by agent-scope atomic loads)": vic2(9),
        "torchform_colsum plain (PyTorch's form: sc1 partial stores, vmcnt(0), barrier, atomic, PLAIN loads)": vic2(10),
        "torchform_colsum acquire (the same + agent-scope acquire after the semaphore)": vic2(11),
        "torchform_colsum sc1-load (the same, partials read by sc1 loads)": vic2(12),
        "ld16_victim d16 (global_load_short_d16 / _d16_hi into one VGPR)": vic16(3),
        "ld16_victim ushort (two zero-extending 16-bit loads)": vic16(4),
        "ld16_victim dword (one 32-bit load)": vic16(5),
        "pk_victim (v_pk_fma_f32 chain)": vic(0, x, n),
        "fma_victim (v_fma_f32 chain)": vic(1, x, n),
        "pk_add_victim (v_pk_add_f32 column sums)": vic(2, m, 2304 // 2, rows),
        "torch bf16 sum(0) 768x2304": lambda: sb.sum(0),
        "torch fp32 sum(0) 768x2304": lambda: sb.float().sum(0),
    }
    if os.environ.get("VICTIMS"):
        keep = os.environ["VICTIMS"].split("|")
        victims = {k: v for k, v in victims.items() if any(k.startswith(x) for x in keep)}
    side = torch.cuda.Stream(device=dev)
    total = 0
    for an, af in aggressors.items():
        for vn, vf in victims.items():
            torch.cuda.synchronize()
            ref = vf().clone()
            torch.cuda.synchronize()
            bad, nel = 0, 0
            for _ in range(REPS):
                main = torch.cuda.current_stream()
                side.wait_stream(main)
                af()
                with torch.cuda.stream(side):
                    got = vf().clone()
                af()
                torch.cuda.synchronize()
                if not torch.equal(got, ref):
                    bad += 1
                    nel = max(nel, int((got != ref).sum()))
            total += bad
            print(json.dumps(dict(aggressor=an, victim=vn, reps=REPS, mismatching=bad, max_elems=nel)), flush=True)
    print(json.dumps(dict(total_mismatching=total)), flush=True)


if __name__ == "__main__":
    main()
