"""aten ops of one c3 training step (bench.py's model and trainer, B=256) by input shape and
device time (torch.profiler, CPU + CUDA activities), to attribute the step's elementwise kernels
(copies, casts, adds) to the ops that launch them. usage: python tools/step_ops.py [rows]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rows=60):
    import bench
    from torch.profiler import ProfilerActivity, profile
    from triad_amd import _lib
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer
    _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.80, patch_sparsity_weight=0.01,
                            visual_dropout_prob=0.25, use_amp=True).to(dev)
    model.train()
    trainer = TriadTrainer(model, learning_rate=1e-4, total_updates=100000, unfreeze_audio_step=0,
                           unfreeze_text_step=0, unfreeze_vit_step=0, device=dev)
    frames, audio, text = bench.synthetic(256, 0, dev)

    def step():
        return trainer.step(frames, audio, text, phase="full_joint", shared_frames=True, frames_tv=None)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total", row_limit=int(rows),
                                                             max_name_column_width=36, max_shapes_column_width=100))
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40, max_name_column_width=50))
    # where the copy / cast kernels come from: copy_ by input shape, with the python stack
    copies = [e for e in prof.key_averages(group_by_input_shape=True) if e.key in ("aten::copy_", "aten::add_")]
    for e in sorted(copies, key=lambda e: -e.self_device_time_total)[:30]:
        print(f"{e.key:12s} {e.count:5d} {e.self_device_time_total / 1e3:8.3f} ms  {str(e.input_shapes)[:150]}")


if __name__ == "__main__":
    main(*sys.argv[1:2])
