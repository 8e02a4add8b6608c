"""DESIGN.md §2b, VERDICT r5 #5: is the co-residency disturbance of PyTorch's bf16 column sum a
stale-cache-line effect in its cross-workgroup hand-off? (diagnostic, not product code)

Round 4 (profiles/r04_hazard_probe_torchform.log, tools/hazard/hazard.hip): beside `mix_loop` (a
20-line MFMA + LDS-DMA loop whose DMA destinations stay in its own 16 KB ring) PyTorch's bf16
sum(0) of a 768 x 2304 matrix returned different values in 93 of 100 launches, while a replica of
its hand-off (partials stored sc1, vmcnt(0), barrier, returning atomic, the last workgroup reading
the partials with PLAIN loads) was 0 of 100 -- with and without an agent-scope acquire, and with sc1
loads. Variant (iii) of the verdict (an acquire in the victim) is therefore that round's result.
This probe runs the verdict's other two variants ONCE each, with PyTorch's own kernel as the victim:

  base      as round 4 (every allocation from the caching allocator; the victim on a side stream)
  fresh     (i)  the victim's input, output, staging and semaphore buffers from a private memory
                 pool created for it: memory no aggressor launch has ever touched
  confined  (ii) the aggressor's source / scratch buffers in their own pool, between 256 MB guard
                 allocations, so none of its loads or stores can reach the victim's memory
  both      (i) + (ii)

One JSON line per (variant, victim); `mismatching` counts launches whose result differs from the
victim's solo result bit for bit.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HZ = os.path.join(ROOT, "tools", "hazard", "libhazard.so")
REPS = int(os.environ.get("REPS", "100"))
dev = torch.device("cuda")


def lib():
    if not os.path.exists(HZ):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-shared", "-fPIC",
                        os.path.join(ROOT, "tools", "hazard", "hazard.hip"), "-o", HZ], check=True)
    h = C.CDLL(HZ)
    h.hz_aggressor.argtypes = [C.c_int, C.c_void_p, C.c_longlong, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    return h


def aggressor(h, confined):
    """mix_loop (kind 2) over a 16 MB source; with `confined` its buffers sit in a pool of their own
    between guard allocations."""
    def alloc():
        g = torch.Generator(device=dev).manual_seed(1)
        return torch.randn(1 << 22, device=dev, generator=g), torch.empty(1 << 20, device=dev)
    if confined:
        pool = torch.cuda.MemPool()
        with torch.cuda.use_mem_pool(pool):
            guard0 = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
            src, scratch = alloc()
            guard1 = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
        keep = (pool, guard0, guard1)
    else:
        src, scratch = alloc()
        keep = ()

    def run():
        rc = h.hz_aggressor(2, C.c_void_p(src.data_ptr()), src.numel() // 4, C.c_void_p(scratch.data_ptr()), 256,
                            1000, C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
    run.keep = (src, scratch) + keep
    return run


def victim(rows, cols, fresh):
    """PyTorch's bf16 sum(0); with `fresh` its input and every allocation of its launches (output,
    the reduction's staging buffer and semaphores) come from a private pool."""
    g = torch.Generator(device=dev).manual_seed(3)
    pool = torch.cuda.MemPool() if fresh else None
    if fresh:
        with torch.cuda.use_mem_pool(pool):
            x = (torch.randn(rows, cols, device=dev, generator=g) * 0.01).to(torch.bfloat16)
    else:
        x = (torch.randn(rows, cols, device=dev, generator=g) * 0.01).to(torch.bfloat16)

    def run():
        if fresh:
            with torch.cuda.use_mem_pool(pool):
                return x.sum(0).clone()
        return x.sum(0).clone()
    run.keep = (pool, x)
    return run


def main():
    h = lib()
    side = torch.cuda.Stream(device=dev)
    total = 0
    for variant, fresh, confined in (("base", False, False), ("fresh", True, False), ("confined", False, True),
                                     ("both", True, True)):
        agg = aggressor(h, confined)
        for rows, cols in ((768, 2304), (8192, 768)):
            vf = victim(rows, cols, fresh)
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                ref = vf()
            torch.cuda.synchronize()
            bad, nel = 0, 0
            for _ in range(REPS):
                main_s = torch.cuda.current_stream()
                side.wait_stream(main_s)
                agg()
                with torch.cuda.stream(side):
                    got = vf()
                agg()
                torch.cuda.synchronize()
                if not torch.equal(got, ref):
                    bad += 1
                    nel = max(nel, int((got != ref).sum()))
            total += bad
            print(json.dumps(dict(variant=variant, victim=f"torch bf16 sum(0) {rows}x{cols}", aggressor="mix_loop",
                                  reps=REPS, mismatching=bad, max_elems=nel)), flush=True)
    print(json.dumps(dict(total_mismatching=total)), flush=True)


if __name__ == "__main__":
    main()
