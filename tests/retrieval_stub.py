"""Deterministic stand-ins for the retrieval drop-in's end-to-end fixture (tests/golden/
gen_retrieval_e2e.py freezes the reference's compute_{av,tv}_retrieval_metrics on them;
tests/test_retrieval_gpu.py runs triad_amd.retrieval's on the same ones).

The embedders are elementwise-only maps (unfold / reshape / sin / cos / tanh / cat): autocast
leaves them in fp32, so the reference (no autocast, CPU) and the drop-in (bf16 autocast, GPU)
embed the same items to the same features up to fp32 evaluation order. Datasets follow the
reference's item formats: AV `__getitem__(idx, apply_augmentation=...)` -> {video_frames, audio,
video_path} with variable-length waveforms (the collate pads them, retrieval.py:46-64); TV
`__getitem__(idx)` -> (image, caption) with captions of different lengths (the embed trims
to the attention mask, retrieval.py:243-244)."""
import zlib

import torch
import torch.nn as nn

D = 512


def _expand(x):
    """(..., n) -> (..., 512): [x, sin 3x, cos 2x, tanh x] truncated (n >= 128)."""
    y = torch.cat([x, torch.sin(3.0 * x), torch.cos(2.0 * x), torch.tanh(x)], -1)
    return y[..., :D].contiguous()


class StubVisual(nn.Module):
    def forward(self, frames):            # (B, 3, 32, 32) -> (B, 24, 512): 128-value tokens
        return _expand(frames.reshape(frames.shape[0], 24, 128))


class StubAudio(nn.Module):
    def forward(self, audio):             # (B, T) -> (B, T // 128, 512)
        B, T = audio.shape
        return _expand(audio[:, :(T // 128) * 128].reshape(B, -1, 128))


def word_vector(w):
    """The 128 raw values a caption word stands for (its hash)."""
    i = zlib.crc32(w.encode()) % 99991 + 1
    return torch.sin(i * 0.00731 * torch.arange(1, 129, dtype=torch.float32))


class StubText(nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("dev", torch.zeros(1))

    def forward(self, captions):          # list[str] -> ((B, Nt, 512), mask (B, Nt)), zero-padded
        rows = [[word_vector(w) for w in c.split()] for c in captions]
        n = max(len(r) for r in rows)
        raw = torch.zeros(len(rows), n, 128)
        mask = torch.zeros(len(rows), n, dtype=torch.long)
        for i, r in enumerate(rows):
            raw[i, :len(r)] = torch.stack(r)
            mask[i, :len(r)] = 1
        raw, mask = raw.to(self.dev.device), mask.to(self.dev.device)
        return _expand(raw) * mask[..., None], mask


class StubModel(nn.Module):
    def __init__(self, temperature=1.3):
        super().__init__()
        self.visual_embedder = StubVisual()
        self.audio_embedder = StubAudio()
        self.text_embedder = StubText()
        self.temperature = nn.Parameter(torch.tensor(float(temperature)))
        self.use_amp = True
        self.amp_dtype = torch.bfloat16


class AVStubDataset(torch.utils.data.Dataset):
    """Item i: random frames; its waveform is 0.9 x the first T samples of the flattened frames +
    noise, so its 128-sample windows resemble the frames' first visual tokens."""

    def __init__(self, n=40):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, idx, apply_augmentation=True):
        g = torch.Generator().manual_seed(1000 + idx)
        frames = torch.randn(3, 32, 32, generator=g)
        T = 128 * (6 + idx % 5)           # 768 .. 1280 samples: padded per batch
        audio = 0.9 * frames.flatten()[:T] + 6.0 * torch.randn(T, generator=g)
        return {"video_frames": frames, "audio": audio, "video_path": f"clip_{idx:03d}.mp4"}


class TVStubDataset(torch.utils.data.Dataset):
    """Item i: a caption of 3-8 words unique to it; the image's 24 tokens are its words' vectors
    (cycled) + noise, so each word finds its own token in the matching image."""

    def __init__(self, n=40):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(2000 + idx)
        words = [f"w{idx}x{j}" for j in range(3 + idx % 6)]
        toks = torch.stack([word_vector(words[j % len(words)]) for j in range(24)])
        image = (toks + 12.0 * torch.randn(24, 128, generator=g)).reshape(3, 32, 32)
        return image, " ".join(words)
