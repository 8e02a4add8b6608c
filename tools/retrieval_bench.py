"""1000-way retrieval timed on the device: av_retrieval_metrics and
tv_retrieval_metrics (both directions, N x N aggregated similarities in one pairsim launch each,
ranks and R@1/5/10/20) at N = 1000 items with the c3 token counts (199 audio tokens, 256 visual
tokens, ragged 8-32 caption tokens), features L2-normalised bf16; then the fp32 mode on the same
values (one timed run per direction pair). Beside it the CPU restatement
of retrieval.py's per-pair aggregation (its double loop over pairs, fp32 torch on the host's
threads; written out here, not imported) timed on a small N and scaled by N^2 (labelled
EXTRAPOLATED).
Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triad_amd import retrieval  # noqa: E402


def feats(n, lens, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.functional.normalize(torch.randn(int(l), 512, generator=g), dim=-1).to(torch.bfloat16)
            for l in lens[:n]]


def main():
    N = int(os.environ.get("TRIAD_RETRIEVAL_N", "1000"))
    g = torch.Generator().manual_seed(7)
    t_lens = torch.randint(8, 33, (N,), generator=g).tolist()
    audio = feats(N, [199] * N, 1)
    video = feats(N, [256] * N, 2)
    text = feats(N, t_lens, 3)
    out = {"N": N}
    for name, fn, q, k in (("av", retrieval.av_retrieval_metrics, audio, video),
                           ("tv", retrieval.tv_retrieval_metrics, text, video)):
        fn(q[:8], k[:8], 0.07)   # warm-up
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            m = fn(q, k, 0.07)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[f"{name}_s"] = round(min(ts), 4)
        out[f"{name}_r1"] = round(list(m.values())[0], 4)
        # the reference-precision mode (model.use_amp=False): the same lists in fp32, fp32 scorer
        q32, k32 = [x.float() for x in q], [x.float() for x in k]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m32 = fn(q32, k32, 0.07, precision="fp32")
        torch.cuda.synchronize()
        out[f"{name}_fp32_s"] = round(time.perf_counter() - t0, 4)
        out[f"{name}_fp32_r1"] = round(list(m32.values())[0], 4)
    # the reference's per-pair loops on the host (both directions), small N, scaled by N^2
    n_cpu = int(os.environ.get("TRIAD_RETRIEVAL_CPU_N", "24"))
    qa, kv = [a.float() for a in audio[:n_cpu]], [v.float() for v in video[:n_cpu]]
    t0 = time.perf_counter()
    for i in range(n_cpu):
        for j in range(n_cpu):
            float((qa[i] @ kv[j].t() / 0.07).max(dim=1).values.mean())
            float((qa[j] @ kv[i].t() / 0.07).max(dim=0).values.mean())
    dt = time.perf_counter() - t0
    out["cpu_av_sample"] = f"N={n_cpu}: {dt:.2f} s on {torch.get_num_threads()} threads"
    out["cpu_av_s_EXTRAPOLATED"] = round(dt * (N / n_cpu) ** 2, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
