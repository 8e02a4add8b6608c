"""Does a HIP kernel give different results when another stream's kernels share the CUs?

The tri-modal step runs HuBERT on its own stream beside the ViT (model.forward_triad);
tools/stream_diag.py localised run-to-run differences of that mode to HuBERT's conv feature
encoder. Here each candidate launch runs (a) alone -> reference, then (b) N times while a noise
stream keeps the CUs busy with other kernels, and every result is compared bit for bit.

Candidates: triad_gemm_bf16_form in each tile form on the feature encoder's layer-1 shape
(overlapping A rows, lda = 2C < K = 3C) and on a plain shape; the fused conv0 + GroupNorm + GELU;
the whole feature encoder module.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd._lib import call, ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
ITERS = int(os.environ.get("ITERS", "12"))


def noise_fn():
    """A stream's worth of other GEMM work (ViT-like shapes, eight-wave form) + elementwise."""
    a = torch.randn(66816, 768, device=dev).to(torch.bfloat16)
    w = torch.randn(2304, 768, device=dev).to(torch.bfloat16)
    out = torch.empty(66816, 2304, device=dev, dtype=torch.bfloat16)

    def run(n=6):
        for _ in range(n):
            call("triad_gemm_bf16_form", ptr(a), 768, 1, ptr(w), 768, 1, 66816, 2304, 768, None, ptr(out), 2304, 1, 0,
                 stream_ptr(dev))
            out.mul_(0.5)
    return run


def check(name, fn, noise):
    side = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    ref = fn().clone()
    torch.cuda.synchronize()
    bad = 0
    worst = 0.0
    for _ in range(ITERS):
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        noise()                      # queued on main first ...
        with torch.cuda.stream(side):
            got = fn()               # ... then the candidate beside it
            got = got.clone()
        noise()
        torch.cuda.synchronize()
        if not torch.equal(got, ref):
            bad += 1
            d = (got.float() - ref.float()).abs().max().item()
            worst = max(worst, d)
    print(f"{name:48s} mismatching runs {bad}/{ITERS}  max|diff| {worst:.3e}", flush=True)
    return bad


def gemm_case(M, N, K, lda, form, rows_total):
    g = torch.Generator(device=dev).manual_seed(M + N + K + form)
    a = torch.randn(rows_total, lda, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)

    def fn():
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        call("triad_gemm_bf16_form", ptr(a), lda, 1, ptr(b), K, 1, M, N, K, None, ptr(out), N, 1, form,
             stream_ptr(dev))
        return out
    return fn


def feature_encoder_case(B):
    import transformers
    from triad_amd import frontend
    hub = frontend.install_hubert_frontend(transformers.HubertModel(transformers.HubertConfig())).to(dev)
    fe = hub.feature_extractor
    x = torch.randn(B, 16000, device=dev) * 0.1

    def fn():
        with torch.autocast("cuda", dtype=torch.bfloat16), torch.no_grad():
            return fe(x).contiguous()
    return fn


def model_noise(which):
    """The tri-modal step's other streams as the noise: the DINOv2-B (+LoRA) patch encoder on the
    current stream and / or DistilBERT on a third stream (forward under autocast, train mode)."""
    from triad_amd.model import MultiModalModel
    torch.manual_seed(0)
    m = MultiModalModel(temperature=1.5, visual_dropout_prob=0.25).to(dev).train()
    frames = torch.randn(128, 3, 224, 224, device=dev)
    ids = torch.randint(1000, 30522, (128, 32))
    text = {"input_ids": ids, "attention_mask": torch.ones(128, 32, dtype=torch.long)}
    s_text = torch.cuda.Stream(device=dev)

    def run():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if "text" in which:
                s_text.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(s_text):
                    m.text_embedder(text)
            if "vit" in which:
                m.visual_embedder.encode_patches(frames)
            if "text" in which:
                torch.cuda.current_stream(dev).wait_stream(s_text)
    return m, run


def audio_case(m, B):
    """The whole audio embedder in eval mode (dropout / LayerDrop / SpecAugment draw per call)."""
    x = torch.randn(B, 16000, device=dev) * 0.1
    m.audio_embedder.eval()

    def fn():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return m.audio_embedder(x).detach().contiguous()
    return fn


def feature_case(m, B):
    x = torch.randn(B, 16000, device=dev) * 0.1
    fe = m.audio_embedder.hubert.feature_extractor

    def fn():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return fe(m.audio_embedder.normalize(x)).detach().contiguous()
    return fn


def vit_part_noises(m):
    """The ViT forward cut into parts (each run under autocast as encode_patches runs it)."""
    from triad_amd import attention, vit as V
    vit = m.visual_embedder.model
    frames = torch.randn(128, 3, 224, 224, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        t = vit.prepare_tokens(frames).float()
        ln = torch.nn.functional.layer_norm(t, (768,), vit.blocks[0].norm1.weight, vit.blocks[0].norm1.bias, 1e-6)
        ln = ln.to(torch.bfloat16)
    blk = vit.blocks[0]

    def ac(fn):
        def run():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                for _ in range(4):
                    fn()
        return run
    return {
        "prepare_tokens (patch GEMM, pos-embed)": ac(lambda: vit.prepare_tokens(frames)),
        "qkv LoRA linear": ac(lambda: blk.attn.qkv(ln)),
        "attention kernel": ac(lambda: attention.attention_qkv(blk.attn.qkv(ln), blk.attn.heads)),
        "proj LoRA linear": ac(lambda: blk.attn.proj(ln)),
        "mlp (fc1, gelu, fc2)": ac(lambda: blk.mlp(ln)),
        "add_scale_ln": ac(lambda: V.add_scale_ln(t, ln, blk.ls1, blk.norm2)),
        "torch layer_norm": ac(lambda: torch.nn.functional.layer_norm(t, (768,), blk.norm1.weight, blk.norm1.bias)),
    }


def encoder_part_victims(m, B=128):
    """The HuBERT feature encoder cut into its launches (layer-0 conv+GroupNorm+GELU, each frame
    conv GEMM, the GELU pass), each on its real input."""
    from triad_amd import frontend
    from triad_amd.postln import gelu
    fe = m.audio_embedder.hubert.feature_extractor
    x = m.audio_embedder.normalize(torch.randn(B, 16000, device=dev) * 0.1)
    l0 = fe.conv_layers[0]
    plan = frontend._frame_stack_plan(fe, x.to(torch.bfloat16)) if False else None
    T = (16000 - 10) // 5 + 1
    Tp = T + (T & 1)
    out = {}
    with torch.no_grad():
        h = frontend._Conv0GNGelu.apply(x, l0.conv.weight, l0.layer_norm.weight, l0.layer_norm.bias,
                                         float(l0.layer_norm.eps), Tp)
        out["c0gn (conv0+GN+GELU)"] = lambda: frontend._Conv0GNGelu.apply(
            x, l0.conv.weight, l0.layer_norm.weight, l0.layer_norm.bias, float(l0.layer_norm.eps), Tp).clone()
        Tc = Tp
        for i, layer in enumerate(fe.conv_layers[1:], 1):
            hin, Tin = h, Tc

            def conv(hin=hin, Tin=Tin, w=layer.conv.weight):
                return frontend._FrameConvS2.apply(hin, w.to(torch.bfloat16), B, Tin).clone()
            out[f"frame conv {i} (M={B * Tin // 2})"] = conv
            y = frontend._FrameConvS2.apply(hin, layer.conv.weight.to(torch.bfloat16), B, Tin)
            if i == 1:
                out["gelu pass"] = lambda y=y: gelu(y).clone()
            h = gelu(y)
            Tc = Tin // 2
    return out


def kernel_noises():
    """Single launches of the ViT MLP's pieces at its c3 shapes (M = 128 x 261 tokens)."""
    from triad_amd import gemm as G
    from triad_amd.postln import gelu
    M = 128 * 261
    x = torch.randn(M, 768, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(3072, 768, device=dev) * 0.02).to(torch.bfloat16)
    b1 = torch.zeros(3072, device=dev, dtype=torch.bfloat16)
    h = torch.randn(M, 3072, device=dev).to(torch.bfloat16)
    w2 = (torch.randn(768, 3072, device=dev) * 0.02).to(torch.bfloat16)

    def rep(fn):
        def run():
            for _ in range(6):
                fn()
        return run
    return {
        "fc1 GEMM 33408x3072x768 (bias)": rep(lambda: G.linear(x, w1, b1)),
        "fc2 GEMM 33408x768x3072": rep(lambda: G.linear(h, w2, None)),
        "gelu pass (table) 33408x3072": rep(lambda: gelu(h)),
        "torch copy 33408x3072": rep(lambda: h.clone()),
    }


def gemm_form_fn(M, N, K, form):
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)

    def fn():
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        call("triad_gemm_bf16_form", ptr(a), K, 1, ptr(w), K, 1, M, N, K, None, ptr(out), N, 1, form, stream_ptr(dev))
        return out
    return fn


def c0gn_direct(noise, iters=ITERS, B=128):
    """triad_c0gn_fwd on PRE-ALLOCATED buffers (no allocator traffic in the loop) on a side stream
    beside `noise`; per output buffer (chunk partials, mean, rstd, out, y0): mismatching runs and
    where the differing elements sit."""
    T, C = 3199, 512
    Tp = T + 1
    Lp = 5 * (Tp - 1) + 10
    g = torch.Generator(device=dev).manual_seed(3)
    xw = (torch.randn(B, Lp, device=dev, generator=g)).to(torch.bfloat16)
    w0 = (torch.randn(C, 10, device=dev, generator=g) * 0.3).to(torch.bfloat16)
    gam = torch.rand(C, device=dev, generator=g) + 0.5
    bet = torch.randn(C, device=dev, generator=g) * 0.1
    nb = int(call("triad_chgn_workspace_bytes", B, T, C))
    bufs = lambda: dict(ws=torch.zeros(nb, dtype=torch.uint8, device=dev),  # noqa: E731
                        mean=torch.zeros(B, C, device=dev), rstd=torch.zeros(B, C, device=dev),
                        out=torch.zeros(B * Tp + 2, C, device=dev, dtype=torch.bfloat16),
                        y0=torch.zeros(B * Tp, C, device=dev, dtype=torch.bfloat16))

    def launch(bb):
        call("triad_c0gn_fwd", ptr(xw), Lp, ptr(w0), B, T, Tp, C, ptr(gam), ptr(bet), 1e-5, ptr(bb["mean"]),
             ptr(bb["rstd"]), ptr(bb["ws"]), ptr(bb["out"]), ptr(bb["y0"]), stream_ptr(dev))
    ref = bufs()
    launch(ref)
    torch.cuda.synchronize()
    inputs = dict(xw=xw, w0=w0, gam=gam, bet=bet)
    saved = {k: v.clone() for k, v in inputs.items()}
    got = bufs()
    side = torch.cuda.Stream(device=dev)
    bad = {k: 0 for k in ref}
    for _ in range(iters):
        for v in got.values():
            v.zero_()
        side.wait_stream(torch.cuda.current_stream(dev))
        noise()
        with torch.cuda.stream(side):
            launch(got)
        noise()
        torch.cuda.synchronize()
        for k in ref:
            if not torch.equal(got[k], ref[k]):
                bad[k] += 1
                if k == "out":
                    d = (got[k][:B * Tp].float() - ref[k][:B * Tp].float()).abs().view(B, Tp, C) > 0
                    bs = d.any(2).any(1).nonzero().flatten().tolist()
                    ts = d.any(2).any(0).nonzero().flatten()
                    print(f"   out differs: {int(d.sum())} elements, samples {bs[:8]}.., frames "
                          f"{ts[:6].tolist()}.. chunks {sorted(set((ts // 128).tolist()))[:10]}, "
                          f"channels {d.any(1).any(0).nonzero().flatten()[:8].tolist()}..", flush=True)
                if k == "mean":
                    d = (got[k] - ref[k]).abs() > 0
                    print(f"   mean differs at {int(d.sum())} (b, c): samples {d.any(1).nonzero().flatten()[:8].tolist()}",
                          flush=True)
    print("c0gn direct, pre-allocated buffers: mismatching runs per buffer", bad, flush=True)
    for k, v in inputs.items():   # were the launch's INPUTS overwritten (by someone else's writes)?
        if not torch.equal(v, saved[k]):
            d = (v.float() - saved[k].float()).abs() > 0
            idx = d.reshape(-1).nonzero().flatten()
            print(f"   INPUT {k} changed: {int(d.sum())} elements, flat index {idx[:4].tolist()} .. "
                  f"{idx[-4:].tolist()} of {v.numel()} ({v.dtype}, ptr {v.data_ptr():#x})", flush=True)
        else:
            print(f"   input {k} unchanged", flush=True)
    again = bufs()
    launch(again)
    torch.cuda.synchronize()
    print("   quiet re-run equal to the reference:", {k: bool(torch.equal(again[k], ref[k])) for k in ref}, flush=True)


def vit_train_noise(m, B=128):
    """The ViT (+LoRA) patch encoder forward AND backward (LoRA / head gradients), train mode."""
    frames = torch.randn(B, 3, 224, 224, device=dev)
    ve = m.visual_embedder

    def run():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ve.encode_patches(frames)
        y.float().square().mean().backward()
    return run


def audio_train_noise(m, B=128):
    x = torch.randn(B, 16000, device=dev) * 0.1
    ae = m.audio_embedder

    def run():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ae(x)
        y.float().square().mean().backward()
    return run


def text_grad_case(m, B=128):
    """DistilBERT + projection head forward AND backward (eval mode: no dropout draws), the
    flattened gradients of every text parameter as the result."""
    te = m.text_embedder
    te.eval()
    ids = torch.randint(1000, 30522, (B, 32), generator=torch.Generator().manual_seed(11))
    text = {"input_ids": ids, "attention_mask": torch.ones(B, 32, dtype=torch.long)}
    ps = [p for p in te.parameters() if p.requires_grad]
    gy = None

    def fn():
        nonlocal gy
        for p in ps:
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = te(text)
            y = y[0] if isinstance(y, tuple) else y
        if gy is None:
            gy = torch.randn(y.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(12))
        (y.float() * gy).sum().backward()
        return torch.cat([p.grad.float().reshape(-1) for p in ps if p.grad is not None])
    return fn


def torch_victims():
    """PyTorch's own fp32 kernels (built with the compiler's defaults, packed-FP32 VALU ops
    included): elementwise FMA chain, add, LayerNorm, softmax, reductions."""
    g = torch.Generator(device=dev).manual_seed(21)
    x = torch.randn(8192, 768, device=dev, generator=g)
    y = torch.randn(8192, 768, device=dev, generator=g)
    w = torch.randn(768, device=dev, generator=g)
    b = torch.randn(768, device=dev, generator=g)
    return {
        "torch x*y+x (fp32)": lambda: torch.addcmul(x, x, y),
        "torch add (fp32)": lambda: x + y,
        "torch layer_norm (fp32)": lambda: torch.nn.functional.layer_norm(x, (768,), w, b),
        "torch softmax (fp32)": lambda: torch.softmax(x, -1),
        "torch sum(0) (fp32)": lambda: x.sum(0),
        "torch gelu (fp32)": lambda: torch.nn.functional.gelu(x),
    }


if __name__ == "__main__":
    torch.manual_seed(0)
    if len(sys.argv) > 1 and sys.argv[1] == "torchops":
        def rep(fn, n=6):
            def run():
                for _ in range(n):
                    fn()
            return run
        tot = 0
        for form in (1, 2, 4):
            noise = rep(gemm_form_fn(33280, 3072, 768, form))
            for name, victim in torch_victims().items():
                tot += check(f"{name} beside gemm form {form}", victim, noise)
        print("total mismatching runs", tot)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "text":
        from triad_amd.model import MultiModalModel
        m = MultiModalModel(temperature=1.5, visual_dropout_prob=0.25).to(dev).train()
        victim = text_grad_case(m)

        def rep(fn, n=6):
            def run():
                for _ in range(n):
                    fn()
            return run
        tot = check("text fwd+bwd beside nothing", victim, lambda: None)
        for form in (1, 2, 4):
            tot += check(f"text fwd+bwd beside gemm form {form}", victim, rep(gemm_form_fn(33280, 3072, 768, form)))
        for name, noise in vit_part_noises(m).items():
            tot += check(f"text fwd+bwd beside {name}", victim, noise)
        _, vit_fwd = model_noise("vit")
        tot += check("text fwd+bwd beside the ViT forward", victim, vit_fwd)
        tot += check("text fwd+bwd beside the ViT fwd+bwd", victim, vit_train_noise(m))
        tot += check("text fwd+bwd beside HuBERT fwd+bwd", victim, audio_train_noise(m))
        tot += check("text fwd+bwd beside HuBERT forward", victim, rep(audio_case(m, 128), 1))
        print("total mismatching runs", tot)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "direct":
        def rep(fn, n=6):
            def run():
                for _ in range(n):
                    fn()
            return run
        c0gn_direct(rep(gemm_form_fn(33280, 3072, 768, 1)), iters=3)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "pair":
        from triad_amd.model import MultiModalModel
        m = MultiModalModel(temperature=1.5, visual_dropout_prob=0.25).to(dev).train()
        c0 = encoder_part_victims(m)["c0gn (conv0+GN+GELU)"]

        def rep(fn, n=6):
            def run():
                for _ in range(n):
                    fn()
            return run
        tot = 0
        # the GEMM as the victim, c0gn as the noise: is the GEMM's own result disturbed too?
        tot += check("gemm form 1 33408x3072x768 beside c0gn", gemm_form_fn(33408, 3072, 768, 1), rep(c0, 3))
        for form in (1, 2, 3, 4):
            tot += check(f"c0gn beside gemm form {form} 33280x3072x768", c0, rep(gemm_form_fn(33280, 3072, 768, form)))
        print("total mismatching runs", tot)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "c0gn":
        from triad_amd.model import MultiModalModel
        m = MultiModalModel(temperature=1.5, visual_dropout_prob=0.25).to(dev).train()
        victim = encoder_part_victims(m)["c0gn (conv0+GN+GELU)"]
        tot = 0
        for name, noise in kernel_noises().items():
            tot += check(f"c0gn beside {name}", victim, noise)
        print("total mismatching runs", tot)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "encparts":
        from triad_amd.model import MultiModalModel
        m = MultiModalModel(temperature=1.5, visual_dropout_prob=0.25).to(dev).train()
        noise = vit_part_noises(m)["mlp (fc1, gelu, fc2)"]
        tot = 0
        for name, victim in encoder_part_victims(m).items():
            tot += check(f"{name} beside the ViT MLP", victim, noise)
        print("total mismatching runs", tot)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "vitparts":
        from triad_amd.model import MultiModalModel
        m = MultiModalModel(temperature=1.5, visual_dropout_prob=0.25).to(dev).train()
        victim = feature_case(m, 128)
        tot = 0
        for name, noise in vit_part_noises(m).items():
            tot += check(f"feature encoder beside {name}", victim, noise)
        print("total mismatching runs", tot)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "model":
        # victim: HuBERT (feature encoder / whole audio embedder, autograd recording as in training)
        # beside the real ViT / DistilBERT forwards
        tot = 0
        for which in ("vit+text", "vit", "text"):
            m, noise = model_noise(which)
            tot += check(f"feature encoder beside {which}", feature_case(m, 128), noise)
            tot += check(f"audio embedder beside {which}", audio_case(m, 128), noise)
            del m
            torch.cuda.empty_cache()
        print("total mismatching runs", tot)
        sys.exit(0)
    noise = noise_fn()
    # feature encoder layer 1 at B = 128 x 1 s: frames Tp = 3200 -> M = 204,800 pair rows, K = 3 x 512
    M, C = 204800, 512
    tot = 0
    for form in (0, 1, 2, 3, 4):
        tot += check(f"gemm overlap rows M={M} N=512 K=1536 lda=1024 form {form}",
                     gemm_case(M, 512, 3 * C, 2 * C, form, M + 2), noise)
    for form in (0, 4):
        tot += check(f"gemm plain M={M} N=512 K=1024 form {form}", gemm_case(M, 512, 2 * C, 2 * C, form, M), noise)
    tot += check("hubert feature encoder B=128 (1 s)", feature_encoder_case(128), noise)
    print("total mismatching runs", tot)
