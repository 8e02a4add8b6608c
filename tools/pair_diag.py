"""The inputs of tests/test_head_gpu.py::test_pair_launch_matches_two_heads[5-300-8-40-mixed]
(same generator draws): AV head gradient error against the fp64 oracle by ds_budget (None: fast
path; the TV dS size: chunked recompute) and by padding (as drawn / none)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_cpu  # noqa: E402
from triad_amd import ops  # noqa: E402


def feats(g, shape):
    return (torch.randn(*shape, generator=g) * 0.58).to(torch.bfloat16).float()


def rel(a, b):
    return float((a.double().cpu() - b.double()).norm() / b.double().norm())


B, Na, Nt, Nv = 5, 300, 8, 40
g = torch.Generator().manual_seed(500 + B)
A = feats(g, (B, Na, 512))
T = feats(g, (B, Nt, 512))
Va = feats(g, (B, Nv, 512))
Vt = feats(g, (B, Nv - 3, 512))
Va_nopad = Va.clone()
for V in (Va, Vt):
    lens = torch.randint(V.shape[1] // 2, V.shape[1] + 1, (B,), generator=g)
    lens[0] = V.shape[1]
    print("lens", lens.tolist())
    for j in range(B):
        V[j, lens[j]:] = 0
gt = ops.Geometry(B, Nt, B, Vt.shape[1])
for pad_name, V in (("padded", Va), ("nopad", Va_nopad)):
    Ar, Vr = A.double().requires_grad_(True), V.double().requires_grad_(True)
    tr = torch.tensor(1.4, dtype=torch.float64, requires_grad=True)
    ref_cpu.av_loss(Ar, Vr, tr)[0].backward()
    for name, budget in (("fast", None), ("chunked", ops.ds_bytes(gt))):
        Ag = A.to("cuda", torch.bfloat16).requires_grad_(True)
        Vg = V.to("cuda", torch.bfloat16).requires_grad_(True)
        tg = torch.tensor(1.4, device="cuda", requires_grad=True)
        losses, st, clip = ops.contrastive_head(ops.AV, Ag, Vg, tg, ds_budget=budget)
        losses[0].backward()
        err = (Ag.grad.double().cpu() - Ar.grad).norm(dim=-1) / Ar.grad.norm(dim=-1).clamp(min=1e-30)
        worst = torch.topk(err.flatten(), 5)
        print(json.dumps({"pad": pad_name, "form": name, "dA": rel(Ag.grad, Ar.grad), "dV": rel(Vg.grad, Vr.grad),
                          "worst_rows": [(int(i) // Na, int(i) % Na, round(float(v), 4)) for v, i in
                                         zip(worst.values, worst.indices)],
                          "dA_norm_ref": float(Ar.grad.norm()), "loss": float(losses[0]),
                          "loss_ref": float(ref_cpu.av_loss(A.double(), V.double(), torch.tensor(1.4,
                                                            dtype=torch.float64))[0])}), flush=True)
