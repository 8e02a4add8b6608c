"""Does PyTorch's TunableOp (per-shape hipBLASLt / rocBLAS solution search) speed up the c3 step's
library GEMMs? Times K steps with TunableOp off, tunes during W steps, then times K steps with
the tuned solutions; torch writes the results to gpurun_out/tunableop_results.csv (the source of
triad_amd/tuning/tunableop_gfx950_c3.csv). usage: python tools/tunable_probe.py [K] [max_tuning_ms]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(K=5, max_ms=30):
    import bench
    from triad_amd import _lib
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer
    K, max_ms = int(K), int(max_ms)
    _lib.load()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(1234)
    model = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.80, patch_sparsity_weight=0.01,
                            visual_dropout_prob=0.25, use_amp=True).to(dev)
    model.train()
    trainer = TriadTrainer(model, learning_rate=1e-4, total_updates=100000, unfreeze_audio_step=0,
                           unfreeze_text_step=0, unfreeze_vit_step=0, device=dev)
    frames, audio, text = bench.synthetic(256, 0, dev)

    def step():
        return trainer.step(frames, audio, text, phase="full_joint", shared_frames=True, frames_tv=None)

    def timed(n):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    for _ in range(2):
        step()
    base = timed(K)
    print(f"baseline {base:.2f} ms/step", flush=True)
    tun = torch.cuda.tunable
    os.makedirs("gpurun_out", exist_ok=True)
    tun.set_filename("gpurun_out/tunableop_results.csv")
    tun.set_max_tuning_duration(max_ms)
    tun.set_max_tuning_iterations(100)
    tun.enable(True)
    tun.tuning_enable(True)
    t0 = time.perf_counter()
    for i in range(2):
        step()
        torch.cuda.synchronize()
        print(f"tuning step {i}: {time.perf_counter() - t0:.1f} s", flush=True)
    tun.tuning_enable(False)
    tuned = timed(K)
    print(f"tuned {tuned:.2f} ms/step ({base / tuned:.3f}x)", flush=True)
    tun.enable(False)
    again = timed(K)
    print(f"tunable off again {again:.2f} ms/step", flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:3])
