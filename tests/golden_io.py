"""Helpers to read the committed golden fixtures (tests/golden/*.npz)."""
import glob
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names(kind=None):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        if kind is None or str(np.load(p)["kind"]) == kind:
            out.append(os.path.splitext(os.path.basename(p))[0])
    return out


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def bf16(u16):
    """uint16 bf16 bit patterns -> fp32 torch tensor (exact)."""
    a = np.asarray(u16).astype(np.uint32) << 16
    return torch.from_numpy(a.view(np.float32).copy())
