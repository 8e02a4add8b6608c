"""Why does the three-stream tri-modal step differ from the single-stream one?

Runs one TriadTrainer step (c3 model, B=128 as tests/test_ops_gpu.py::
test_modality_streams_match_single_stream) from identical models / seeds in several execution
modes, twice each, and prints for every pair: the loss deltas (total, AV, TV), the relative L2
delta of the reduced fp32 gradient per parameter group, and the parameters that differ most.
Modes: single / multi stream (TRIAD_MODALITY_STREAMS) x side-stream weight gradients on / off.
`--nodrop` turns every dropout / LayerDrop / SpecAugment off (isolates RNG-order effects).
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

dev = "cuda"


def _nodrop(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    for cfg_owner in (m.audio_embedder.hubert, m.text_embedder.encoder):
        cfg = cfg_owner.config
        for k in ("hidden_dropout", "attention_dropout", "activation_dropout", "feat_proj_dropout",
                  "layerdrop", "mask_time_prob", "mask_feature_prob", "dropout", "attention_dropout",
                  "final_dropout"):
            if hasattr(cfg, k):
                setattr(cfg, k, 0.0)
    m.audio_embedder.hubert.config.apply_spec_augment = False


def run(streams, side, nodrop, B, frames, audio, text):
    from triad_amd import linear as L
    from triad_amd.model import MultiModalModel
    from triad_amd.train import TriadTrainer, split_param_groups
    os.environ["TRIAD_MODALITY_STREAMS"] = "1" if streams else "0"
    L.SIDE_STREAM_DW = side
    torch.manual_seed(0)
    m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.8, patch_sparsity_weight=0.01,
                        visual_dropout_prob=0.25, use_amp=True).to(dev)
    m.train()
    if nodrop:
        _nodrop(m)
    tr = TriadTrainer(m, total_updates=100, unfreeze_audio_step=0, unfreeze_text_step=0, unfreeze_vit_step=0,
                      device=dev)
    snap = []
    inner = tr._allreduce_grads

    def grab():   # the reduced gradient buffer before clipping / AdamW / zero_grad
        inner()
        snap.append(tr.space.flat_g.detach().cpu().numpy().copy())
    tr._allreduce_grads = grab
    torch.manual_seed(1)
    np.random.seed(1)
    out = tr.step(frames, audio, text)
    torch.cuda.synchronize()
    names = {id(p): n for n, p in m.named_parameters()}
    groups = split_param_groups(m)
    gid = {id(p): k for k, ps in groups.items() for p in ps}
    sp = tr.space
    g = snap[0]
    per = {}
    for i, p in enumerate(sp.params):
        per[names[id(p)]] = (gid[id(p)], g[sp.offsets[i]:sp.offsets[i] + p.numel()].astype(np.float64))
    res = dict(loss=float(out["loss"]), av=float(out["loss_av"]), tv=float(out["loss_tv"]), per=per)
    del tr, m
    torch.cuda.empty_cache()
    return res


def compare(tag, a, b, top=8):
    print(f"== {tag}")
    for k in ("loss", "av", "tv"):
        print(f"   {k:5s} {a[k]:.8f} vs {b[k]:.8f}  rel {abs(a[k] - b[k]) / max(abs(a[k]), 1e-30):.3e}")
    num, den = {}, {}
    rows = []
    for n, (grp, ga) in a["per"].items():
        gb = b["per"][n][1]
        d2, n2 = float(((ga - gb) ** 2).sum()), float((ga ** 2).sum())
        num[grp] = num.get(grp, 0.0) + d2
        den[grp] = den.get(grp, 0.0) + n2
        rows.append((np.sqrt(d2 / max(n2, 1e-300)), np.sqrt(n2), n))
    tot = np.sqrt(sum(num.values()) / max(sum(den.values()), 1e-300))
    print(f"   flat grad rel {tot:.3e}; per group: " +
          ", ".join(f"{k} {np.sqrt(num[k] / max(den[k], 1e-300)):.2e}" for k in sorted(num)))
    rows.sort(reverse=True)
    nz = sum(1 for r in rows if r[0] > 0)
    print(f"   params differing: {nz} of {len(rows)}")
    for r in rows[:top]:
        print(f"     {r[0]:.3e}  |g| {r[1]:.3e}  {r[2]}")
    sys.stdout.flush()


def poison(B, frames, audio, text, streams):
    """Every torch.empty / empty_like filled with NaN (torch's deterministic-mode memory fill):
    run the tri-modal forward and name the first module of each embedder whose output holds a
    NaN / Inf -- a kernel that reads memory nobody wrote (an uninitialised-read is deterministic
    on one stream, where the allocator hands out the same blocks every run, and not with three)."""
    from triad_amd.model import MultiModalModel
    os.environ["TRIAD_MODALITY_STREAMS"] = "1" if streams else "0"
    torch.manual_seed(0)
    m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.8, patch_sparsity_weight=0.01,
                        visual_dropout_prob=0.25, use_amp=True).to(dev)
    m.train()
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = True
    bad = []

    def hook(name):
        def h(mod, inp, out):
            outs = out if isinstance(out, (tuple, list)) else (out,)
            for o in outs:
                if hasattr(o, "last_hidden_state"):
                    o = o.last_hidden_state
                if isinstance(o, torch.Tensor) and o.is_floating_point() and not bool(torch.isfinite(o).all()):
                    bad.append((name, type(mod).__name__, tuple(o.shape)))
        return h
    for root in ("audio_embedder", "text_embedder", "visual_embedder"):
        for n, mod in getattr(m, root).named_modules():
            mod.register_forward_hook(hook(root + "." + n))
    torch.manual_seed(1)
    np.random.seed(1)
    av, tv = m.forward_triad(frames, audio, text)
    torch.cuda.synchronize()
    print(f"poison streams={streams}: av {float(av[0]):.6f} tv {float(tv[0]):.6f}")
    seen = set()
    for b in bad:   # forward hooks fire innermost first: the first entries are the sources
        if b[0] not in seen:
            seen.add(b[0])
            print("   non-finite output:", b)
        if len(seen) >= 25:
            break
    torch.use_deterministic_algorithms(False)
    torch.utils.deterministic.fill_uninitialized_memory = False


def bisect(B, frames, audio, text, modes, nodrop, trainer=False, hooks=True):
    """Per-module output checksums (fp64 sum and sum of squares, taken on the module's own stream)
    of the tri-modal forward in each mode; prints, per embedder, the first module (execution order)
    whose output differs from the first run's."""
    from triad_amd.model import MultiModalModel
    runs = []
    for md in modes:
        os.environ["TRIAD_MODALITY_STREAMS"] = "1" if md == "M" else "0"
        torch.manual_seed(0)
        m = MultiModalModel(temperature=1.5, patch_sparsity_threshold=0.8, patch_sparsity_weight=0.01,
                            visual_dropout_prob=0.25, use_amp=True).to(dev)
        m.train()
        if nodrop:
            _nodrop(m)
        if trainer:   # bf16 shadow weights over fp32 masters, flat parameter / gradient buffers
            from triad_amd.train import TriadTrainer
            TriadTrainer(m, total_updates=100, unfreeze_audio_step=0, unfreeze_text_step=0, unfreeze_vit_step=0,
                         device=dev)
        rec = []

        def hook(name):
            def h(mod, inp, out):
                o = out[0] if isinstance(out, (tuple, list)) else out
                if hasattr(o, "last_hidden_state"):
                    o = o.last_hidden_state
                if isinstance(o, torch.Tensor) and o.is_floating_point():
                    od = o.detach().double()
                    rec.append((name, torch.stack([od.sum(), (od * od).sum()])))
            return h
        def prehook(name):
            def h(mod, args):
                for i, a in enumerate(args):
                    if isinstance(a, torch.Tensor) and a.is_floating_point():
                        ad = a.detach().double()
                        rec.append((f"{name}:in{i}", torch.stack([ad.sum(), (ad * ad).sum()])))
            return h
        hs = []
        for root in ("audio_embedder", "text_embedder", "visual_embedder") if hooks else ():
            for n, mod in getattr(m, root).named_modules():
                hs.append(mod.register_forward_pre_hook(prehook(root + "." + n)))
                hs.append(mod.register_forward_hook(hook(root + "." + n)))
        torch.manual_seed(1)
        np.random.seed(1)
        av, tv = m.forward_triad(frames, audio, text)
        torch.cuda.synchronize()
        runs.append((md, float(av[0]), [(n, v.cpu().tolist()) for n, v in rec]))
        del m
        torch.cuda.empty_cache()
    base = runs[0]
    for md, av, rec in runs[1:]:
        print(f"mode {md}: av {av:.8f} vs {base[1]:.8f}")
        first = {}
        bmap = {}
        for n, v in base[2]:
            bmap.setdefault(n, []).append(v)
        seen = {}
        for n, v in rec:
            k = seen.get(n, 0)
            seen[n] = k + 1
            ref = bmap.get(n, [None] * (k + 1))[k] if k < len(bmap.get(n, [])) else None
            root = n.split(".")[0]
            if ref is not None and ref != v and root not in first:
                first[root] = (n, k, v, ref)
        for root, (n, k, v, ref) in first.items():
            print(f"   first differing module in {root}: {n} (call {k}) {v} vs {ref}")
        if not first:
            print("   every module output identical")
        sys.stdout.flush()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--poison", action="store_true")
    ap.add_argument("--bisect", default="")
    ap.add_argument("--trainer", action="store_true")
    ap.add_argument("--nohooks", action="store_true")
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--nodrop", action="store_true")
    ap.add_argument("--modes", default="S1,S1,M1,M1,M0,S0")
    args = ap.parse_args()
    B = args.B
    g = torch.Generator().manual_seed(5)
    frames = torch.randn(B, 3, 224, 224, generator=g).to(dev)
    audio = (torch.randn(B, 16000, generator=g) * 0.1).to(dev)
    text = [f"caption number {i} of a scene" for i in range(B)]
    if args.bisect:
        bisect(B, frames, audio, text, args.bisect.split(","), args.nodrop, args.trainer, not args.nohooks)
        sys.exit(0)
    if args.poison:
        poison(B, frames, audio, text, False)
        poison(B, frames, audio, text, True)
        sys.exit(0)
    res = []
    for md in args.modes.split(","):
        r = run(md[0] == "M", md[1] == "1", args.nodrop, B, frames, audio, text)
        print(f"run {md}: loss {r['loss']:.8f} av {r['av']:.8f} tv {r['tv']:.8f}")
        sys.stdout.flush()
        res.append((md, r))
    base = res[0]
    for i, (md, r) in enumerate(res[1:], 1):
        compare(f"{base[0]}#0 vs {md}#{i}", base[1], r)
    # multi vs multi (run to run) when present
    ms = [(i, r) for i, (md, r) in enumerate(res) if md.startswith("M")]
    if len(ms) >= 2:
        compare(f"multi #{ms[0][0]} vs multi #{ms[1][0]}", ms[0][1], ms[1][1])
