"""Every LDS-DMA kernel of the library on fixed inputs, with a digest of each output: run it once
per library build and compare the digests (do the counted `s_waitcnt vmcnt(N)`
waits retire everything read, and do LDS-DMA destinations stay inside each kernel's LDS?).

  python tools/kernel_tour.py out.json                         # product library
  TRIAD_LIB_VARIANT=tools/variants/lib_vmcnt0.so  python ...   # counted waits -> vmcnt(0)
  TRIAD_LIB_VARIANT=tools/variants/lib_ldscheck.so python ...  # bounds check on every LDS-DMA

Identical digests across the three = the counted waits read nothing early (a premature read
of a ring slot would see another stage's data in some launch), and the check build's stdout
carries no "TRIAD_LDS_CHECK OOB" line. Launches: both heads' fused forward (training and eval
forms) and backward at c3-like shapes, the recompute backward, the ring / direct-B / 16x16x32
tile GEMMs, the tiled bf16 GEMM in its five forms (+ split-K, bias), both projection-head
forms, HuBERT's positional convolution and conv feature encoder."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import ops  # noqa: E402
from triad_amd._lib import TriadError, call, ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")


def digest(*ts):
    h = hashlib.sha256()
    for t in ts:
        if t is None:
            continue
        h.update(t.detach().reshape(-1).contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def gen(seed):
    return torch.Generator(device=dev).manual_seed(seed)


def feats(shape, seed, scale=0.58):
    return (torch.randn(*shape, device=dev, generator=gen(seed)) * scale).to(torch.bfloat16)


def heads(out):
    B = 48
    qa, ka = feats((B, 199, 512), 1), feats((B, 212, 512), 2)
    qt, kt = feats((B, 32, 512), 3), feats((B, 212, 512), 4)
    ka[5, 180:] = 0
    mask = (torch.arange(32, device=dev)[None] < torch.randint(4, 33, (B, 1), device=dev, generator=gen(5))).long()
    for label, budget in (("pair", None), ("pair-recompute", 1 << 26)):
        xs = [x.clone().requires_grad_(True) for x in (qa, ka, qt, kt)]
        t = torch.tensor(1.5, device=dev, requires_grad=True)
        (la, sa, ca), (lt, st, ct) = ops.contrastive_heads_av_tv(*xs, t, mask, threshold=0.8, sparsity_weight=0.01,
                                                                 ds_budget=budget)
        (la[0] + lt[0]).backward()
        out[label] = digest(*[x.grad for x in xs], t.grad, ca, ct, sa, st)
    with torch.no_grad():
        (la, sa, ca), _ = ops.contrastive_heads_av_tv(qa, ka, qt, kt, torch.tensor(1.5, device=dev), mask)
    out["pair-eval"] = digest(ca, sa)


def tile_gemms(out):
    R_pad, CT = 7 * 128, 36
    dS = feats((R_pad // 32 * CT * 1024,), 11, 0.1)
    K, Q = feats((CT * 32, 512), 12, 1.0), feats((R_pad, 512), 13, 1.0)
    alpha = torch.tensor([0.75], device=dev)
    st = stream_ptr()
    for dk, Bm, M, nkt in ((0, K, R_pad, CT), (1, Q, CT * 32, R_pad // 32)):
        for splits in (1, 3):
            slabs = torch.empty(splits * M * 512, device=dev) if splits > 1 else None
            c = torch.empty(M, 512, dtype=torch.bfloat16, device=dev)
            call("triad_tile_gemm", ptr(dS), CT, dk, ptr(Bm), M, nkt, ptr(alpha), splits, ptr(slabs), ptr(c), st)
            out[f"tile-ring-dk{dk}-sp{splits}"] = digest(c)
            Bp = torch.empty(nkt * 32 * 512, dtype=torch.bfloat16, device=dev)
            call("triad_bfrag_pack16", ptr(Bm), nkt, dk, ptr(Bp), st)
            call("triad_tile_gemm_packed16", ptr(dS), CT, dk, ptr(Bp), M, nkt, ptr(alpha), splits, ptr(slabs),
                 ptr(c), st)
            out[f"tile-packed16-dk{dk}-sp{splits}"] = digest(c, Bp)


def gemms(out):
    st = stream_ptr()
    for (M, N, K) in ((33280, 768, 768), (4096, 2304, 768), (8192, 512, 512)):
        a, w = feats((M, K), 21), feats((N, K), 22, 0.05)
        for form in range(5):
            c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            try:
                call("triad_gemm_bf16_form", ptr(a), K, 1, ptr(w), K, 1, M, N, K, None, ptr(c), N, 1, form, st)
            except TriadError:   # a form that does not tile this shape
                continue
            out[f"gemm-{M}x{N}x{K}-form{form}"] = digest(c)
        b = torch.randn(N, device=dev, generator=gen(23)).to(torch.bfloat16).float()
        c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        call("triad_gemm_bf16_bias", ptr(a), K, 1, ptr(w), K, 1, M, N, K, ptr(b), ptr(c), N, st)
        out[f"gemm-bias-{M}x{N}x{K}"] = digest(c)
        # weight gradient shape: dW [N][K] = dy^T x over M rows, split-K
        dy = feats((M, N), 24, 0.1)
        for form in (0, 4):
            sp = 8
            slabs = torch.empty(sp * N * K, device=dev)
            dw = torch.empty(N, K, dtype=torch.bfloat16, device=dev)
            call("triad_gemm_bf16_splitk_form", ptr(dy), N, 0, ptr(a), K, 0, N, K, M, sp, None, ptr(slabs), ptr(dw), 1,
                 form, st)
            out[f"gemm-splitk-{N}x{K}x{M}-form{form}"] = digest(dw)


def projheads(out):
    torch.manual_seed(31)
    for H, M in ((768, 8192), (1024, 4096)):
        p1, ln, p2 = torch.nn.Linear(H, 512).to(dev), torch.nn.LayerNorm(512).to(dev), torch.nn.Linear(512, 512).to(dev)
        h = feats((M // 64, 64, H), 32, 1.0).requires_grad_(True)
        for form in ("passes", "rows"):
            for p in (*p1.parameters(), *ln.parameters(), *p2.parameters()):
                p.grad = None
            h.grad = None
            y = ops.projection_head(h, p1, ln, p2, form=form)
            (y.float() * torch.linspace(-1, 1, 512, device=dev)).sum().backward()
            out[f"projhead-{form}-{M}x{H}"] = digest(y, h.grad, p1.weight.grad, p2.weight.grad, ln.weight.grad)


def hubert_front(out):
    """HuBERT-base with the channels-last conv feature encoder and the positional-conv kernels
    (triad_amd.frontend), eval mode (no random draws), forward + backward under bf16 autocast."""
    import transformers
    from triad_amd import frontend
    torch.manual_seed(41)
    hub = frontend.install_hubert_frontend(transformers.HubertModel(transformers.HubertConfig())).to(dev).eval()
    x = torch.randn(8, 16000, device=dev, generator=gen(42)) * 0.1
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = hub(x).last_hidden_state
    y.float().square().mean().backward()
    grads = [p.grad for p in hub.parameters() if p.grad is not None]
    out["hubert"] = digest(y, *grads)


def main(path):
    out = {"lib": os.environ.get("TRIAD_LIB_VARIANT", "product")}
    for fn in (heads, tile_gemms, gemms, projheads, hubert_front):
        fn(out)
        torch.cuda.synchronize()
        print(f"[tour] {fn.__name__} done", flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
