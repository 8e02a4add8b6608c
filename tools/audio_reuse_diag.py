"""Diagnostic: does the audio backbone give the same parameter gradients when it runs twice inside
one autograd graph (two B=2 chunks, features concatenated) as when each chunk runs in a graph of
its own (gradients accumulated)? And at B=4 in one call? Prints per-parameter relative L2.

    python tools/audio_reuse_diag.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_dist_gpu import _mode_r_model  # noqa: E402


def grads(ae):
    return {n: p.grad.detach().clone() for n, p in ae.named_parameters() if p.grad is not None}


def main():
    m = _mode_r_model()
    ae = m.audio_embedder
    ae.normalize = lambda a: a.float()
    for p in ae.parameters():
        p.requires_grad_(True)
    g = torch.Generator().manual_seed(7)
    audio = (torch.randn(4, 32000, generator=g) * 0.1).cuda()
    runs = {}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        probe = ae(audio[:2])
    gy = torch.randn(4, *probe.shape[1:], generator=g).cuda() * 0.01

    def run(kind):
        ae.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if kind == "full":
                y = ae(audio)
                (y.float() * gy).sum().backward()
            elif kind == "chunked":
                y = torch.cat([ae(audio[:2]), ae(audio[2:])])
                (y.float() * gy).sum().backward()
            else:
                for i in (0, 2):
                    y = ae(audio[i:i + 2])
                    (y.float() * gy[i:i + 2]).sum().backward()
        torch.cuda.synchronize()
        return grads(ae)

    for kind in ("separate", "chunked", "full", "separate"):
        runs.setdefault(kind, []).append(run(kind))
    ref = runs["separate"][0]

    def cmp(name, other):
        rows = []
        for n, r in ref.items():
            o = other.get(n)
            if o is None:
                rows.append((float("inf"), n))
                continue
            rows.append((float((o.double() - r.double()).norm() / r.double().norm().clamp(min=1e-30)), n))
        rows.sort(reverse=True)
        tot_n = sum(float((other[n].double() - ref[n].double()).norm() ** 2) for n in ref if n in other)
        tot_d = sum(float(ref[n].double().norm() ** 2) for n in ref)
        print(f"{name}: total rel {tot_n ** 0.5 / tot_d ** 0.5:.3e}; worst {[(f'{r:.2e}', n) for r, n in rows[:6]]}",
              flush=True)

    cmp("separate (repeat)", runs["separate"][1])
    cmp("chunked one graph", runs["chunked"][0])
    cmp("full B=4", runs["full"][0])


if __name__ == "__main__":
    main()
