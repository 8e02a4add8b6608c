"""Per-kernel time of one backbone's forward+backward alone (torch.profiler over 3 iterations
after 2 warmups, B=256, bf16 autocast, training mode, synthetic inputs), to attribute the step
profile's elementwise time to modules. usage: python tools/backbone_profile.py vit|hubert|distilbert"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(which, B):
    from triad_amd import model as M
    if which == "vit":
        m = M.ViTLoRAEmbedder(arch="dinov2_vitb14_reg").cuda()
        from triad_amd.vit import store_frozen_base_bf16
        store_frozen_base_bf16(m.model)
        x = torch.randn(B, 3, 224, 224, device="cuda")
        return m.model, lambda: m.model.get_intermediate_layers(x, n=1)[0]
    if which == "hubert":
        m = M.AudioEmbedder().cuda()
        h = m.hubert
        x = torch.randn(B, 64000, device="cuda") * 0.1
        return h, lambda: h(x).last_hidden_state
    m = M.TextEmbedder().cuda()
    enc = m.encoder
    ids = torch.randint(1000, 30000, (B, 32), device="cuda")
    return enc, lambda: enc(input_ids=ids).last_hidden_state


def main(which, B=256):
    mod, fwd = build(which, B)
    mod.train()
    for p in mod.parameters():
        if p.dtype == torch.float32 and p.requires_grad and p.dim() >= 2 and which != "vit":
            p.data = p.data.to(torch.bfloat16)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = fwd()
        y.float().square().mean().backward()
        for p in mod.parameters():
            p.grad = None
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    shapes = "--shapes" in sys.argv
    acts = [ProfilerActivity.CUDA] + ([ProfilerActivity.CPU] if shapes else [])
    with profile(activities=acts, record_shapes=shapes) as prof:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
    if shapes:  # aten ops by input shape, by device time (attribute copies / adds to their callers)
        print(prof.key_averages(group_by_input_shape=True).table(sort_by="device_time_total", row_limit=45,
                                                                 max_name_column_width=40,
                                                                 max_shapes_column_width=90))
        return
    rows = []
    for e in prof.key_averages():
        t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
        if t > 0:
            rows.append((t / 3 / 1e3, e.count / 3, e.key[:110]))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"== {which}: {tot:.2f} ms/iter device time")
    for ms, n, k in rows[:40]:
        print(f"{ms:8.3f} ms {n:6.1f}x  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
