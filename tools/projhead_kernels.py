"""Device time of the projection head per call, kernel durations only (host overhead excluded):
run under rocprofv3 --kernel-trace, each (form, rows) case does `iters` forward calls and `iters`
backward calls, each segment fenced by a marker launch (triad_l2norm_rows on a tiny tensor,
rows = a segment id). Then `python tools/projhead_kernels.py --parse <kernel_trace.csv>` sums the
kernel durations between markers (one stream, so kernels do not overlap) and prints per call
fwd / bwd microseconds and algorithmic TFLOP/s (fwd 2 M (H 512 + 512 512), bwd twice that).
Gradients are released after each backward, so no accumulation kernels are counted (round 3;
the round-2 figures included ~45-75 us of them at 65,536 rows). --detail: per-kernel times."""
import argparse
import csv
import json
import os
import sys

CASES = (("visual", 65536, 768), ("audio", 50944, 768), ("text", 8192, 768), ("c5-visual", 43808, 1024),
         ("visual-view", 65536, 768))   # the ViT's patch tokens as a strided view of (256, 261, 768)
FORMS = tuple(os.environ.get("TRIAD_PROJHEAD_FORMS", "rows,passes").split(","))
# the trainer keeps bf16 shadows of projection1 / projection2 (round 4, train.py bf16_weight_params):
# bf16 weights are the product configuration; fp32 = the round-2 / round-3 figures
WDTYPE = os.environ.get("TRIAD_PROJHEAD_WDTYPE", "bf16")


def run(iters):
    import torch
    import torch.nn as nn
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from triad_amd import ops
    dev = "cuda"
    seg = 1

    def mark(i):
        ops.l2_normalize(torch.ones(i, 512, device=dev, dtype=torch.bfloat16))

    for form in FORMS:
        for name, M, H in CASES:
            torch.manual_seed(0)
            p1, ln, p2 = nn.Linear(H, 512).to(dev), nn.LayerNorm(512).to(dev), nn.Linear(512, 512).to(dev)
            if WDTYPE == "bf16":
                p1, p2 = p1.to(torch.bfloat16), p2.to(torch.bfloat16)
            if name.endswith("-view"):
                full = torch.randn(M // 256, 261, H, device=dev).to(torch.bfloat16).requires_grad_(True)
                h = full[:, 5:]
            else:
                h = torch.randn(M, H, device=dev).to(torch.bfloat16).requires_grad_(True)
            gy = (torch.randn(*h.shape[:-1], 512, device=dev) * 0.01).to(torch.bfloat16)
            for _ in range(2):   # warm-up (library heuristics, allocator)
                ops.projection_head(h, p1, ln, p2, form=form).backward(gy)
            outs = []
            torch.cuda.synchronize()
            mark(seg)
            for _ in range(iters):
                outs.append(ops.projection_head(h, p1, ln, p2, form=form))
            mark(seg + 1)
            for y in outs:
                y.backward(gy)
                (full if name.endswith("-view") else h).grad = None   # stored, not added (no add kernels)
                for mod in (p1, ln, p2):
                    for prm in mod.parameters():
                        prm.grad = None
            mark(seg + 2)
            torch.cuda.synchronize()
            seg += 3


def parse(path, iters, detail=False):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [(i, r) for i, r in enumerate(rows) if "l2norm_rows_kernel" in r["Kernel_Name"]]
    seg_of = {}
    for (i, r), (j, _) in zip(marks, marks[1:]):
        seg_of[int(r["Grid_Size_X"])] = (i, j)
    # marker grid = ceil(rows / 4) workgroups x 256 threads; recover the segment order instead
    order = [i for i, _ in marks]
    k = 0
    for form in FORMS:
        for name, M, H in CASES:
            a, b, c = order[k], order[k + 1], order[k + 2]
            k += 3
            fw = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a + 1:b]) / iters / 1e3
            bw = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[b + 1:c]) / iters / 1e3
            fl = 2.0 * M * (H * 512 + 512 * 512)
            if detail:
                for tag, lo, hi in (("fwd", a, b), ("bwd", b, c)):
                    per = {}
                    for r in rows[lo + 1:hi]:
                        kn = r["Kernel_Name"].replace("void ", "")
                        kn = kn[:kn.find("(")] if kn.find("(") > 0 else kn
                        kn = kn[:110]
                        per[kn] = per.get(kn, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / iters / 1e3
                    for kn, us in sorted(per.items(), key=lambda kv: -kv[1]):
                        print(f"   {form} {name} {tag} {us:8.1f} us  {kn}")
            print(json.dumps({"form": form, "head": name, "M": M, "H": H, "fwd_us": round(fw, 1),
                              "fwd_TFLOPs": round(fl / fw / 1e6, 1), "bwd_us": round(bw, 1),
                              "bwd_TFLOPs": round(2 * fl / bw / 1e6, 1),
                              "fwd_frac": round(fl / fw / 1e6 / 2500, 3), "bwd_frac": round(2 * fl / bw / 1e6 / 2500, 3)}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--parse")
    ap.add_argument("--detail", action="store_true", help="per-kernel-name microseconds per call")
    a = ap.parse_args()
    if a.parse:
        parse(a.parse, a.iters, a.detail)
    else:
        run(a.iters)
