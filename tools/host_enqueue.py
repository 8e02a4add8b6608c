"""Host enqueue time per c3 step vs GPU time per step (is the step launch-bound anywhere?).

Runs bench.py's model / trainer setup, then times each step() call on the host (no sync inside)
and the whole run with a final sync. Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from triad_amd import _lib
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer
    _lib.load()
    torch.manual_seed(1234)
    model = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.80, patch_sparsity_weight=0.01,
                            visual_dropout_prob=0.25, use_amp=True).to(dev)
    model.train()
    tr = TriadTrainer(model, learning_rate=1e-4, total_updates=100000, unfreeze_audio_step=0,
                      unfreeze_text_step=0, unfreeze_vit_step=0, device=dev)
    frames, audio, text = bench.synthetic(256, 0, dev)
    for _ in range(2):
        tr.step(frames, audio, text, phase="full_joint")
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(6):
        h0 = time.perf_counter()
        tr.step(frames, audio, text, phase="full_joint")
        host.append((time.perf_counter() - h0) * 1e3)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / 6
    print(json.dumps({"host_enqueue_ms": [round(x, 2) for x in host], "wall_ms_per_step": round(wall, 2)}), flush=True)


if __name__ == "__main__":
    main()
