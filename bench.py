"""Throughput benchmark: tri-modal triples/sec of the TRIAD full_joint training step.

Workload (BASELINE.json configs[2], "c3"): full tri-modal V+A+T training step,
B=256 triples per GPU -- DINOv2-B/14-reg (+LoRA r8) on 224x224 frames, HuBERT-base
on 4 s @ 16 kHz audio, DistilBERT on 32-token captions, projection heads, patch
dropout 0.25, fused AV + TV similarity / InfoNCE heads, backward, grad norms +
clip, four AdamW + OneCycleLR steps; every module trainable (the post-unfreeze
worst case), grad-accum 1. Random-init weights, synthetic data
resident in HBM before the timed region.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5] [--global-negatives]
       (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
Prints ONE JSON line on rank 0. The default (c3, Mode R) is the headline line; --config c2 / c5 time
BASELINE.json's other single-GPU-sized configurations with their own per-kernel fractions, and
--global-negatives times Mode G (BASELINE c4: every rank contrasts its queries against the keys of
all ranks, RCCL all-gather / reduce-scatter inside the head).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "tri-modal triples/sec (whole node) + loss parity, B=256 at 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
# every hot-path entry point of the library's C ABI (triad_amd/_lib.py: all launching entry points
# but the backbone-only ones), so a kernel added or renamed on the path cannot drop out of the
# per-kernel timing; backbone launches of the shared GEMM / column-sum entry points are tagged
# and reported apart (kernel_report)
from triad_amd._lib import hot_path_entry_points  # noqa: E402
TRACKED = hot_path_entry_points()


# BASELINE.json configurations a single GPU runs (configs[1], [2], [4] per rank; c1 is the CPU plumbing
# case, c4 is c3 x 8 ranks with --global-negatives). phase: the trainer's loss mix (train.py:972-984)
CONFIGS = {
    "c3": dict(batch=256, px=224, audio_s=4, n_text=32, phase="full_joint", unit="triples/s",
               audio_model="facebook/hubert-base-ls960", vit_arch="dinov2_vitb14_reg",
               workload="c3: full tri-modal V+A+T train step, DINOv2-B/14-reg+LoRA / HuBERT-base / DistilBERT, "
                        "full_joint, all modules trainable, patch dropout 0.25"),
    "c2": dict(batch=128, px=224, audio_s=4, n_text=32, phase="av_focus", unit="pairs/s",
               audio_model="facebook/hubert-base-ls960", vit_arch="dinov2_vitb14_reg",
               workload="c2: image-audio train step (forward_audio_visual, train.py:954), DINOv2-B/14-reg+LoRA / "
                        "HuBERT-base, B=128, 4 s audio, av_focus, all modules trainable, patch dropout 0.25"),
    "c5": dict(batch=32, px=518, audio_s=10, n_text=32, phase="full_joint", unit="triples/s",
               audio_model="facebook/hubert-large-ls960-ft", vit_arch="dinov2_vitl14_reg",
               workload="c5 per rank: full tri-modal train step, DINOv2-L/14-reg+LoRA on 518 px frames (1369 "
                        "patches) / HuBERT-large on 10 s audio (Na=499) / DistilBERT, full_joint, all modules "
                        "trainable, patch dropout 0.25"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3",
                    help="BASELINE configuration (c3 = the headline; c2 / c5 = their own lines)")
    ap.add_argument("--global-negatives", action="store_true",
                    help="Mode G: contrast against the keys of every rank (BASELINE c4 at N > 1)")
    ap.add_argument("--batch", type=int, default=None, help="samples per GPU (default: the config's)")
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--cpu-head-batch", type=int, default=48, help="batch of the CPU hot-path timing (extrapolated)")
    ap.add_argument("--separate-steps", type=int, default=3,
                    help="timed steps of the --separate-frames variant reported beside the headline (0 = skip)")
    ap.add_argument("--single-stream-steps", type=int, default=3,
                    help="timed steps in the OTHER execution mode (serial <-> concurrent streams), reported "
                         "beside the headline (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stream-check", dest="stream_check", action="store_false",
                    help="skip the serial-vs-concurrent bit-identity check at the product shape (N = 1)")
    ap.add_argument("--separate-frames", action="store_true",
                    help="encode the AV and TV frame batches separately (2x ViT work)")
    return ap.parse_args()


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knob for the N>1 code path on a one-GPU box (never the measured configuration):
    # TRIAD_BENCH_BACKEND=gloo puts every rank on device LOCAL_RANK % device_count over gloo.
    backend = os.environ.get("TRIAD_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def synthetic(B, rank, device, px=224, audio_s=4, n_text=32):
    """SURVEY §8d inputs: frames N(0,1) (px x px), audio N(0,0.1) audio_s s @ 16 kHz, n_text random
    token ids."""
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    frames = torch.randn(B, 3, px, px, generator=g, device=device)
    audio = torch.randn(B, 16000 * audio_s, generator=g, device=device) * 0.1
    # token ids / mask stay on the host like the reference tokenizer's output (model.py:102-112);
    # the text embedder moves them with a pinned async copy each step
    ids = torch.randint(1000, 30522, (B, n_text), generator=torch.Generator().manual_seed(1234 + rank))
    mask = torch.ones(B, n_text, dtype=torch.long)
    return frames, audio, {"input_ids": ids.pin_memory(), "attention_mask": mask.pin_memory()}


def pmc_traffic(kernel_prefix, grid):
    """HBM bytes per launch of this kernel/grid from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py: FETCH_SIZE x2 x1024 + WRITE_SIZE x1024, separate passes), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if grid is None or not os.path.exists(path):
        return None
    for k, v in json.load(open(path)).items():
        if k.startswith(kernel_prefix) and k.endswith(f"@grid{grid}"):
            return v["hbm_bytes_per_launch"]
    return None


def kernel_report(timers):
    rep = {}
    for name, evs in timers.items():
        for e0, e1, meta in evs:
            key = name
            if meta is not None and meta.get("backbone"):
                key += "[backbone]"  # the same entry points serve backbone layers (linear.py, frontend.py, postln.py)
            elif meta is not None and "tag" in meta:
                key += "[" + meta["tag"] + "]"   # projection heads: per (width x rows)
            elif meta is not None:
                kind = meta.get("kind")
                if kind in (0, 1):
                    key += "[" + ("AV" if kind == 0 else "TV") + ("/" + meta["what"] if "what" in meta else "") + "]"
                else:  # one launch over several heads (triad_pairsim_fwd_multi): "AV+TV"
                    key += "[" + meta.get("what", "?") + "]"
            ms = e0.elapsed_time(e1)
            r = rep.setdefault(key, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "grid": None})
            r["launches"] += 1
            r["ms"] += ms
            r["flops"] += (meta or {}).get("flops", 0.0)
            r["bytes"] += (meta or {}).get("bytes", 0.0)
            r["ds_bytes"] = r.get("ds_bytes", 0.0) + (meta or {}).get("ds_bytes", 0.0)
            r["grid"] = (meta or {}).get("grid")
    return rep


def model_streams():
    """Does forward_triad run the audio / text backbones on their own streams (the headline mode)?"""
    from triad_amd.model import modality_streams_enabled
    return modality_streams_enabled()


def stream_bit_identity(dev, frames, audio, text):
    """the concurrent default must give the serial step's results bit for bit at the
    PRODUCT shape (c3, B = 256), not only at the tests' B = 128. Two fresh models / trainers from
    the same seed, one step each (dropout, LayerDrop, SpecAugment and patch dropout drawn from the
    same seeds), serial then concurrent; the losses and the reduced flat gradient (taken before
    clipping / AdamW) are compared bit for bit."""
    import numpy as np
    from triad_amd.model import MultiModalModel, modality_streams_enabled, set_concurrent_streams
    from triad_amd.train import TriadTrainer

    def run(concurrent):
        set_concurrent_streams(concurrent)
        torch.manual_seed(4321)
        m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.80, patch_sparsity_weight=0.01,
                            visual_dropout_prob=0.25, use_amp=True).to(dev)
        m.train()
        tr = TriadTrainer(m, learning_rate=1e-4, total_updates=100000, unfreeze_audio_step=0,
                          unfreeze_text_step=0, unfreeze_vit_step=0, device=dev)
        snap = []

        def grab():   # the reduced gradient, then no optimizer step (the models are discarded)
            tr._allreduce_grads()
            snap.append(tr.space.flat_g.clone())
            return {}
        tr._optimizer_step = grab
        torch.manual_seed(1)
        np.random.seed(1)   # SpecAugment masks (transformers draws them from numpy)
        out = tr.step(frames, audio, text, phase="full_joint")
        torch.cuda.synchronize()
        loss = torch.stack([out["loss"], out["loss_av"], out["loss_tv"]]).clone()
        del tr, m
        return loss, snap[0]

    prev = modality_streams_enabled()
    try:
        l_s, g_s = run(False)
        l_c, g_c = run(True)
    finally:
        set_concurrent_streams(prev)
    diff = int((g_s != g_c).sum())
    return {"equal": bool(torch.equal(l_s, l_c) and diff == 0), "B": int(frames.shape[0]),
            "losses_serial": [float(x) for x in l_s], "losses_concurrent": [float(x) for x in l_c],
            "gradient_elements": int(g_s.numel()), "differing_elements": diff,
            "max_abs": float((g_s - g_c).abs().max())}


def main():
    a = parse()
    cfg = CONFIGS[a.config]
    if a.batch is None:
        a.batch = cfg["batch"]
    headline = a.config == "c3"
    shared = cfg["phase"] == "full_joint"   # one frame batch for both heads (forward_triad)
    from triad_amd import _lib, blas
    blas.configure()   # torch's own GEMMs on rocBLAS, before the HIP runtime starts (triad_amd/blas.py)
    world, rank, local = setup_dist()
    dev = torch.device("cuda", local)
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer

    _lib.load()
    # The only MIOpen convolution left is HuBERT's positional conv (the feature encoder and the
    # patch embedding run as GEMMs, triad_amd.frontend): immediate mode, no per-shape search /
    # runtime kernel compilation on a fresh box.
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(1234)
    model = MultiModalModel(audio_model_name=cfg["audio_model"], temperature=1.5, patch_sparsity_threshold=0.80,
                            patch_sparsity_weight=0.01, visual_dropout_prob=0.25, use_amp=True,
                            vit_arch=cfg["vit_arch"]).to(dev)
    model.train()
    trainer = TriadTrainer(model, learning_rate=1e-4, total_updates=100000, unfreeze_audio_step=0,
                           unfreeze_text_step=0, unfreeze_vit_step=0, device=dev,
                           global_negatives=a.global_negatives)
    frames, audio, text = synthetic(a.batch, rank, dev, cfg["px"], cfg["audio_s"], cfg["n_text"])
    frames_tv = frames.roll(1, 0).contiguous() if (a.separate_frames and shared) else None

    # step watchdog (hang forensics): per-stream markers after every HIP entry point,
    # a monitor thread that writes which launch is in flight and exits non-zero when a step stalls
    wd = None
    if os.environ.get("TRIAD_WATCHDOG", "1") != "0":
        from triad_amd import watchdog
        out_dir = "gpurun_out" if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else "."
        wd = watchdog.arm(dev, os.path.join(ROOT, out_dir, f"bench_watchdog_rank{rank}.json"),
                          ops=os.environ.get("TRIAD_WATCHDOG_OPS", "0") == "1").__enter__()

    def step():
        if wd is not None:
            wd.step_begin()
        out = trainer.step(frames, audio, text, phase=cfg["phase"], shared_frames=not a.separate_frames,
                           frames_tv=frames_tv)
        if wd is not None:
            wd.step_end()
        return out

    for i in range(a.warmup):
        t_w = time.perf_counter()
        out = step()
        torch.cuda.synchronize()
        if rank == 0:  # progress (the first step includes MIOpen's conv-algorithm search)
            print(f"[bench] warmup step {i + 1}/{a.warmup}: {time.perf_counter() - t_w:.1f} s", file=sys.stderr,
                  flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if os.environ.get("TRIAD_PROFILE_MARK"):  # marker launch for tools/trace_summary.py (never in a step)
        from triad_amd import ops
        ops.l2_normalize(torch.ones(64, 512, device=dev, dtype=torch.bfloat16))
        torch.cuda.synchronize()
    _lib.TIMERS = {k: [] for k in TRACKED}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    timers, _lib.TIMERS = _lib.TIMERS, None
    if wd is not None:
        wd.__exit__(None, None, None)
        wd = None
    if rank == 0:
        print(f"[bench] {a.steps} timed steps: {dt:.2f} s", file=sys.stderr, flush=True)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    loss = float(out["loss"])
    rep = kernel_report(timers)
    sep = None
    if a.separate_steps > 0 and not a.separate_frames and shared:
        # the --separate-frames figure beside the headline: AV and TV frames encoded separately
        frames_sep = frames.roll(1, 0).contiguous()

        def step_sep():
            return trainer.step(frames, audio, text, phase="full_joint", shared_frames=False, frames_tv=frames_sep)
        step_sep()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(a.separate_steps):
            step_sep()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dts = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([dts], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dts = float(t)
        sep = world * a.batch * a.separate_steps / dts
        if rank == 0:
            print(f"[bench] {a.separate_steps} separate-frames steps: {dts:.2f} s", file=sys.stderr, flush=True)

    rcheck = None
    if world > 1 and trainer.reducer is not None:
        # correctness gate of the overlapped gradient reduction: one more step with
        # every bucket's pre-reduction gradient snapshotted; after it the same buckets are
        # all-reduced again from the snapshots, one at a time with the device otherwise idle, and
        # compared bit for bit with what the all-reduces overlapped with backward produced
        trainer.reducer.check = True
        step()
        torch.cuda.synchronize()
        rcheck = trainer.reducer.check_result
        if rank == 0:
            print(f"[bench] reducer check: {rcheck}", file=sys.stderr, flush=True)

    single = None
    if a.single_stream_steps > 0:
        # the same step in the other execution mode, reported beside the headline: the serial step
        # (one stream) beside the concurrent default (backbones on three streams + the dW side stream)
        from triad_amd import linear as _lin
        from triad_amd.model import set_concurrent_streams
        prev = (os.environ.get("TRIAD_MODALITY_STREAMS"), _lin.SIDE_STREAM_DW)
        headline_concurrent = model_streams()
        set_concurrent_streams(not headline_concurrent)
        try:
            step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            _lib.TIMERS = {k: [] for k in TRACKED}
            t1 = time.perf_counter()
            for _ in range(a.single_stream_steps):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            dtss = time.perf_counter() - t1
            timers_other, _lib.TIMERS = _lib.TIMERS, None
        finally:
            if prev[0] is None:
                os.environ.pop("TRIAD_MODALITY_STREAMS", None)
            else:
                os.environ["TRIAD_MODALITY_STREAMS"] = prev[0]
            _lin.SIDE_STREAM_DW = prev[1]
        if world > 1:
            t = torch.tensor([dtss], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dtss = float(t)
        single = {"value": world * a.batch * a.single_stream_steps / dtss, "unit": "triples/s",
                  "steps": a.single_stream_steps, "ms_per_step": dtss / a.single_stream_steps * 1e3,
                  "concurrent_streams": not headline_concurrent,
                  "note": ("concurrent streams (backbones on three streams + dW side stream)" if not headline_concurrent
                           else "serial step (one stream), bit-identical results")}
        # per-kernel figures of this mode too: on concurrent streams a launch shares the CUs with the
        # other streams' kernels, so its duration (and fraction of peak) reads lower than alone
        rep_o = kernel_report(timers_other)
        single["kernels_frac"] = {k: v["flops"] / max(1, v["launches"]) / (v["ms"] / max(1, v["launches"]) * 1e-3)
                                  / 1e12 / PEAK_BF16_TFLOPS
                                  for k, v in sorted(rep_o.items()) if v["flops"] and not k.endswith("[backbone]")
                                  and ("pairsim" in k or "tile_gemm" in k)}
        # every hot-path launch of this mode too (the projection heads' GEMMs / passes included), so
        # a launch's time alone on the CUs can be read beside its time on concurrent streams
        single["kernels_ms"] = {k: {"avg_ms": v["ms"] / max(1, v["launches"]),
                                    "launches_per_step": v["launches"] / a.single_stream_steps}
                                for k, v in sorted(rep_o.items()) if not k.endswith("[backbone]")}
        pko = [k for k in rep_o if "[proj" in k]
        po_ms = sum(rep_o[k]["ms"] for k in pko) / a.single_stream_steps
        po_fl = sum(rep_o[k]["flops"] for k in pko) / a.single_stream_steps
        if po_ms > 0:
            single["projection_heads"] = {"ms_per_step": po_ms, "achieved_TFLOPs": po_fl / po_ms / 1e9,
                                          "frac": po_fl / po_ms / 1e9 / PEAK_BF16_TFLOPS}
        if rank == 0:
            print(f"[bench] {a.single_stream_steps} steps with concurrent streams "
                  f"{'on' if single['concurrent_streams'] else 'off'}: {dtss:.2f} s", file=sys.stderr, flush=True)

    if rank == 0:
        value = world * a.batch * a.steps / dt
        mode_g = bool(trainer.global_negatives)
        # dominant hot-path kernel: the similarity forward of both heads in one launch (S = temp*Q K^T,
        # max/argmax, l_nonneg; S never leaves registers). Algorithmic FLOPs = 2*B^2*Nq*Nk_eff*512 per
        # head (AV: Nq = Na, TV: Nq = Nt). With TRIAD_PAIR_FWD=0 (two launches): the AV launch.
        roof_key, roof_sym = "triad_pairsim_fwd_multi[AV+TV]", "pairsim_fwd_multi_kernel<true>"
        if roof_key not in rep:
            roof_key, roof_sym = "triad_pairsim_fwd[AV]", "pairsim_fwd2_kernel<true, false>"
        fwd = rep.get(roof_key, {"launches": 0, "ms": 1.0, "flops": 0.0, "bytes": 0.0, "grid": None})
        avg_ms = fwd["ms"] / max(1, fwd["launches"])
        achieved = (fwd["flops"] / max(1, fwd["launches"])) / (avg_ms * 1e-3) / 1e12
        # every hand-written kernel of the hot path (heads fwd+bwd, projection heads, trainer
        # optimizer); launches tagged as backbone work (the same GEMM / column-sum entry points serve the
        # backbones) are kept apart
        head_keys = [k for k in rep if not k.endswith("[backbone]")]
        head_ms = sum(rep[k]["ms"] for k in head_keys) / a.steps
        head_flops = sum(rep[k]["flops"] for k in head_keys) / a.steps

        def kstats(k):
            v = rep[k]
            avg = v["ms"] / max(1, v["launches"])
            out = {"avg_ms": avg, "launches": v["launches"]}
            if v["flops"]:
                tf = v["flops"] / max(1, v["launches"]) / (avg * 1e-3) / 1e12
                out.update(achieved_TFLOPs=tf, frac=tf / PEAK_BF16_TFLOPS)
            return out
        res = {
            "metric": METRIC if headline else f"{a.config} {cfg['unit'].replace('/s', '')}/sec (whole node)",
            "value": value, "unit": cfg["unit"], "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": f"synthetic (frames N(0,1) {cfg['px']}px, audio N(0,0.1) {cfg['audio_s']}s@16kHz, "
                    f"{cfg['n_text']} random token ids); random-init weights",
            "config": {"workload": cfg["workload"]
                                   + ("" if not shared else ", AV/TV frames encoded separately" if a.separate_frames
                                      else ", one frame batch per triple (dropout masks drawn per head)"),
                       "name": a.config, "phase": cfg["phase"],
                       "global_batch": a.batch * world, "per_gpu_batch": a.batch, "parallelism": f"dp{world}",
                       "negatives": (f"global (Mode G): each rank's queries against all {a.batch * world} key "
                                     f"samples (key all-gather, clip-row gather and key-gradient reduce-scatter inside the head, "
                                     f"on the {dist.get_backend() if world > 1 else 'nccl'} backend)" if mode_g else
                                     "local (Mode R): each rank's reference loss over its own batch"),
                       "gradient_accumulation_steps": 1,
                       "gradient_accumulation_note": "one triple = one sample through one optimizer step at "
                                                     "grad-accum 1 (SURVEY 8d); the reference's __main__ "
                                                     "accumulates 4 micro-batches (train.py:1167), which changes only "
                                                     "how often the optimizer runs"},
            "loss": loss,
            "roofline": {"kernel": roof_key, "symbol": roof_sym, "bound": "mfma", "achieved": achieved,
                         "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": achieved / PEAK_BF16_TFLOPS,
                         "traffic": pmc_traffic(roof_sym, fwd["grid"]), "avg_ms": avg_ms,
                         "algorithmic_bytes": fwd["bytes"] / max(1, fwd["launches"]),
                         "ds_stream_bytes": fwd.get("ds_bytes", 0.0) / max(1, fwd["launches"]),
                         "traffic_source": "profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                                           "same kernel and grid; FETCH x2 gfx950 correction); algorithmic bytes = "
                                           "Q + K features + rowmax/argmax (SURVEY 8d); the training forward also "
                                           "streams the tiled unit-dS gradient (ds_stream_bytes), which is traffic"},
            "head": {"ms_per_step": head_ms, "algo_TFLOPs_per_step": head_flops / 1e12,
                     "achieved_TFLOPs": head_flops / max(head_ms, 1e-9) / 1e9,
                     "kernels": {k: kstats(k) for k in sorted(rep) if k in head_keys}},
            "backbone_hip_gemm_ms_per_step": sum(v["ms"] for k, v in rep.items() if k not in head_keys) / a.steps,
        }
        # the three projection heads as one figure: every launch tagged proj-* /
        # proj{H}x{M} (GEMMs, LayerNorm passes, bias column sums, slab sums) against their algorithmic
        # flops, 6 x rows x (H x 512 + 512 x 512) per step (forward 2, backward 4)
        pk = [k for k in head_keys if "[proj" in k]
        p_ms = sum(rep[k]["ms"] for k in pk) / a.steps
        p_fl = sum(rep[k]["flops"] for k in pk) / a.steps
        if p_ms > 0:
            res["projection_heads"] = {"ms_per_step": p_ms, "algo_TFLOP_per_step": p_fl / 1e12,
                                       "achieved_TFLOPs": p_fl / p_ms / 1e9,
                                       "frac": p_fl / p_ms / 1e9 / PEAK_BF16_TFLOPS, "launches": len(pk)}
        res["config"]["execution"] = ("concurrent streams: audio / text backbones and the backbone dW on their own "
                                      "streams (the default; bit-identical to the serial step, DESIGN.md 2b)"
                                      if model_streams() else "serial: one stream")
        if rcheck is not None:
            res["reducer_check"] = rcheck
        if single is not None:
            res["other_stream_mode"] = single
        if sep is not None:
            res["separate_frames"] = {"value": sep, "unit": "triples/s", "steps": a.separate_steps,
                                      "note": "AV and TV frame batches encoded separately, as the reference's "
                                              "two data loaders do (2x ViT work)"}
        if world == 1 and a.stream_check and headline:
            del trainer, model
            torch.cuda.empty_cache()
            bit = stream_bit_identity(dev, frames, audio, text)
            res["stream_bit_identity"] = bit
            print(f"[bench] serial vs concurrent step at B={a.batch}: {bit}", file=sys.stderr, flush=True)
        if world == 1 and not a.no_cpu_baseline and headline:
            from oracle import cpu_step
            # the threads this process may use: torch's intra-op pool honours OMP_NUM_THREADS (the GPU box
            # sets it to the job's CPU share; its affinity mask shows the whole machine, and oversubscribing
            # that stalls the run)
            threads = torch.get_num_threads()
            if hasattr(os, "sched_getaffinity"):
                threads = min(threads, len(os.sched_getaffinity(0)))
            print(f"[bench] cpu baseline on {threads} threads", file=sys.stderr, flush=True)
            model = "unknown"
            try:
                for line in open("/proc/cpuinfo"):
                    if line.startswith("model name"):
                        model = line.split(":", 1)[1].strip()
                        break
            except OSError:
                pass
            sec = cpu_step.time_steps(B=a.cpu_batch, steps=a.cpu_steps, warmup=1, threads=threads)
            print(f"[bench] cpu full step: {sec:.2f} s", file=sys.stderr, flush=True)
            hb = a.cpu_head_batch
            hsec = cpu_step.time_head(B=hb, steps=a.cpu_steps, warmup=1, threads=threads)
            print(f"[bench] cpu hot path B={hb}: {hsec:.2f} s", file=sys.stderr, flush=True)
            res["cpu_baseline"] = {"value": a.cpu_batch / sec, "unit": "triples/s", "cores": threads, "kind": "port",
                                   "cpu_model": model,
                                   "sample": f"oracle/cpu_step.py full_joint step (fp32 CPU backbones + materialising "
                                             f"reference loss), B={a.cpu_batch}, {a.cpu_steps} timed steps after 1 "
                                             f"warmup: {sec:.2f} s/step on {threads} threads",
                                   "hot_path": {"measured_B": hb, "s_per_step": hsec,
                                                "extrapolated_B": a.batch,
                                                "extrapolated_s_per_step": hsec * (a.batch / hb) ** 2,
                                                "note": "AV+TV losses fwd+bwd of the reference on random features "
                                                        "(Na=199, Nv=205, Nt=32); B^2-extrapolated to the bench batch "
                                                        "(EXTRAPOLATED, not measured at that size)"}}
        print(json.dumps(res), flush=True)
        if not res.get("stream_bit_identity", {"equal": True})["equal"]:
            print("[bench] ERROR: the concurrent step's results differ from the serial step's at the product "
                  "shape (stream_bit_identity); the default execution mode is not trustworthy", file=sys.stderr,
                  flush=True)
            sys.exit(1)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
