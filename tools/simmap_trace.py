"""rocprofv3 evidence for the one-launch similarity maps: run under
`rocprofv3 --kernel-trace`, calls ops.similarity_maps `--calls` times on a (B, N1, N2, 512) problem
between marker launches (triad_l2norm_rows on a tiny tensor); `--parse <kernel_trace.csv>` then
prints the kernels between consecutive markers, i.e. per call."""
import argparse
import csv
import os
import sys


def run(calls, B, N1, N2):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from triad_amd import ops
    g = torch.Generator(device="cuda").manual_seed(0)
    f1 = torch.randn(B, N1, 512, device="cuda", generator=g).to(torch.bfloat16)
    f2 = torch.randn(B, N2, 512, device="cuda", generator=g).to(torch.bfloat16)
    temp = torch.tensor(1.5, device="cuda")
    mark = torch.ones(4, 512, device="cuda", dtype=torch.bfloat16)
    ops.similarity_maps(f1, f2, temp)   # warm-up (allocator)
    torch.cuda.synchronize()
    for _ in range(calls):
        ops.l2_normalize(mark)
        ops.similarity_maps(f1, f2, temp)
    ops.l2_normalize(mark)
    torch.cuda.synchronize()


def parse(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "l2norm_rows_kernel" in r["Kernel_Name"]]
    for n, (a, b) in enumerate(zip(marks, marks[1:])):
        ks = [r for r in rows[a + 1:b]]
        names = [r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0] for r in ks]
        us = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks) / 1e3
        print(f"call {n}: {len(ks)} launch(es), {us:.1f} us: {names}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--shape", default="256,199,256", help="B,N1,N2")
    ap.add_argument("--parse")
    a = ap.parse_args()
    if a.parse:
        parse(a.parse)
    else:
        run(a.calls, *map(int, a.shape.split(",")))
