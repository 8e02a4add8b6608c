"""Run-to-run determinism of one training step's gradients (c1-sized model, dropout off): two
fresh models from the same seed take the same micro-batch; print the parameters whose reduced
fp32 gradients differ most (relative L2)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_dist_gpu as T  # noqa: E402


def grads(shared=True):
    m = T._mode_r_model()
    tr = T._trainer(m, 1)
    f, a, t, ak, tk = T._mode_r_batch(0, 0)
    tr.step(f, a, t, phase="full_joint", av_keep=ak, tv_keep=tk)
    torch.cuda.synchronize()
    names = {id(p): n for n, p in m.named_parameters()}
    sp = tr.space
    g = tr.reduced[0].cpu().numpy()
    return {names[id(p)]: g[sp.offsets[i]:sp.offsets[i] + p.numel()] for i, p in enumerate(sp.params)}


if __name__ == "__main__":
    a = grads()
    b = grads()
    rows = []
    for k in a:
        na = np.linalg.norm(a[k])
        rows.append((float(np.linalg.norm(a[k] - b[k]) / max(na, 1e-30)), float(na), k))
    rows.sort(reverse=True)
    for r in rows[:40]:
        print(f"{r[0]:.3e}  |g| {r[1]:.3e}  {r[2]}")
    print("identical params:", sum(1 for r in rows if r[0] == 0.0), "of", len(rows))
