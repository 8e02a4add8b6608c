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
    x = torch.randn(B, 16000, device=dev) * 0.1

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


if __name__ == "__main__":
    torch.manual_seed(0)
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
