"""Repeat the two-rank Mode G trainer run of tests/test_dist_gpu.py (two processes on the box's one
GPU, gloo, audio unfrozen at step 1) and compare the ranks' reduced gradients across repetitions:
NaN count per step and whether each repetition is bit-identical to the first. One JSON line per
repetition, then a summary. Diagnosis of a one-off NaN in that test.

  python tools/mode_g_repeat.py [--reps 4]        (environment passes to the rank processes)"""
import argparse
import json
import os
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    from triad_amd import blas
    blas.configure()                     # as tests/conftest.py does (inherited by the rank processes)
    import test_dist_gpu as T
    ctx = mp.get_context("spawn")
    first = None
    bad = 0
    env = {k: os.environ.get(k) for k in ("TRIAD_MODALITY_STREAMS", "TRIAD_SIDE_STREAM_DW")}
    for r in range(args.reps):
        qo = ctx.Queue()
        port = T._port()
        procs = [ctx.Process(target=T._mode_g_trainer_worker, args=(k, 2, port, qo)) for k in range(2)]
        for p in procs:
            p.start()
        res = sorted([qo.get(timeout=600) for _ in range(2)], key=lambda x: x[0])
        for p in procs:
            p.join(timeout=60)
        if any(isinstance(x[1], str) for x in res):
            print(json.dumps({"rep": r, "error": [x[2] for x in res if isinstance(x[1], str)][0][-2000:]}), flush=True)
            return 1
        g = res[0][1]
        nans = [int(np.isnan(s).sum()) for s in g]
        same = None if first is None else [bool(np.array_equal(a, b)) for a, b in zip(g, first)]
        if first is None:
            first = g
        ranks_equal = all(np.array_equal(a, b, equal_nan=True) for a, b in zip(res[0][1], res[1][1]))
        bad += int(any(nans) or (same is not None and not all(same)))
        print(json.dumps({"rep": r, "nan_per_step": nans, "bit_identical_to_rep0": same,
                          "ranks_equal": ranks_equal, "losses": res[0][3]}), flush=True)
    print(json.dumps({"reps": args.reps, "differing_or_nan": bad, "env": env}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
