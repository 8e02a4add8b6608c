"""Drop-in mirror of SajayR/TRIAD src/model.py on MI355X.

Same class names, constructor arguments, attribute names (for parameter grouping
by name in the trainer, train.py:251-261) and method return tuples as the
reference. The backbones run on PyTorch-ROCm; the hot path -- projection heads,
patch-dropout compaction, the B x B x Nq x Nk token-similarity contraction,
max/mean aggregation, InfoNCE, regularisers and their backward -- runs in the
HIP kernels of libtriad_hip.so (triad_amd.ops).

Offline differences (documented in DESIGN.md):
  * pretrained weights / tokenizers cannot be downloaded: backbones are random-
    init `transformers` HuBERT / DistilBERT and the local DINOv2 restatement
    (triad_amd.vit); if a local HF cache holds the named checkpoint it is used;
  * the text tokenizer falls back to a deterministic hashing word tokenizer when
    the DistilBERT vocabulary is unavailable; pre-tokenised input is accepted;
  * the patch-dropout Bernoulli mask is drawn on the host (one B x N draw) so the
    compacted length is known without a device sync.
"""
from __future__ import annotations

import math
import os
import re
import types
import warnings
import zlib
from collections.abc import Mapping
from typing import Dict, List, Optional, Sequence, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, attention, dense, frontend, ops
from .linear import install_fast_linear
from .postln import install_fused_distilbert, install_fused_encoder
from .vit import DinoVisionTransformer, apply_lora, store_frozen_base_bf16

warnings.filterwarnings("ignore", message=".*torch.cuda.amp.*")

_AV_KEYS = ("av_pos_sim_mean", "av_pos_sim_std", "av_neg_sim_mean", "av_neg_sim_std", "av_separation",
            "av_hardest_negative")
_TV_KEYS = tuple("tv_" + k[3:] for k in _AV_KEYS)


class LazyStats(Mapping):
    """The reference's stats dict of Python floats (model.py:463-470, 584-591).

    Values stay on the device until first read, so a training step that never
    logs them has no host synchronisation (the reference does 5 `.item()` syncs
    per head, model.py:443-447 / 561-565).
    """

    def __init__(self, keys, values: torch.Tensor):
        self._keys = tuple(keys)
        self._dev = values.detach()
        self._host = None

    def _materialise(self):
        if self._host is None:
            v = self._dev[:6].double().cpu().tolist()
            self._host = dict(zip(self._keys, v))
        return self._host

    def __getitem__(self, k):
        return self._materialise()[k]

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)

    def __repr__(self):
        return repr(dict(self._materialise()))


RANDOM_INIT = {}  # backbone / tokenizer name -> reason it is NOT the pretrained one (reported by bench)


def _hub_online():
    """from_pretrained may reach the network only when asked to (TRIAD_HF_ONLINE=1): this build
    runs on machines without egress, where a download attempt would stall, not fail."""
    import os
    return os.environ.get("TRIAD_HF_ONLINE", "0") == "1"


def _fallback(name, what, err):
    """Record and announce LOUDLY that `name` runs without its pretrained weights / vocabulary."""
    RANDOM_INIT[name] = f"{what}: {type(err).__name__}: {str(err).splitlines()[0][:160] if str(err) else ''}"
    warnings.warn(f"triad_amd: '{name}' is not available locally ({type(err).__name__}); using {what}. "
                  "Results are NOT those of the pretrained model (set TRIAD_HF_ONLINE=1 to allow a "
                  "download, or populate the HF cache).", RuntimeWarning, stacklevel=3)


# architecture of a checkpoint NAME when only its name is known offline (AutoModel resolves it from
# the checkpoint's config.json, which is not there): (name substring, model class, config class,
# whether the HIP attention kernels serve it)
_ARCH_BY_NAME = (("modernbert", "ModernBertModel", "ModernBertConfig", False),
                 ("distilbert", "DistilBertModel", "DistilBertConfig", True),
                 ("hubert", "HubertModel", "HubertConfig", True))


def _hf_model(kind, name, config_overrides=None):
    """Load `name` from the HF cache (or the hub with TRIAD_HF_ONLINE=1) with `kind`
    ("AutoModel" as model.py:80, or a concrete class as model.py:30); when it is not there
    (OSError -- the only failure that means "no such local checkpoint"), random-init the
    architecture its name denotes, warn and record it in RANDOM_INIT. Any other error propagates."""
    import transformers
    try:
        return install_fast_linear(getattr(transformers, kind).from_pretrained(
            name, local_files_only=not _hub_online()))
    except OSError as e:
        err = e
    low = name.lower()
    arch = next((a for a in _ARCH_BY_NAME if (a[1] == kind if kind != "AutoModel" else a[0] in low)), None)
    if arch is None:
        raise OSError(f"triad_amd: '{name}' is not available locally and its architecture is not one this "
                      f"offline build can random-init ({', '.join(a[0] for a in _ARCH_BY_NAME)})") from err
    _, model_cls, cfg_cls, triad_attn = arch
    _fallback(name, "random-init " + model_cls, err)
    cfg = getattr(transformers, cfg_cls)(**(config_overrides or {}))
    if triad_attn:
        try:
            cfg._attn_implementation = _register_attention()
        except Exception:
            pass
    return install_fast_linear(getattr(transformers, model_cls)(cfg))


def _register_attention():
    """transformers attention-interface entry "triad": the HIP attention kernels (attention dropout
    included) for unmasked short sequences, the stock sdpa function otherwise (triad_amd.attention)."""
    from transformers import AttentionInterface
    from transformers.masking_utils import ALL_MASK_ATTENTION_FUNCTIONS, AttentionMaskInterface
    AttentionInterface.register("triad", attention.hf_attention_forward)
    AttentionMaskInterface.register("triad", ALL_MASK_ATTENTION_FUNCTIONS["sdpa"])  # same masks as sdpa
    return "triad"


_HUBERT_LARGE = dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096,
                     feat_extract_norm="layer", do_stable_layer_norm=True)


class ProjectionHead(nn.Module):
    """Holder so `projection1`, `layer_norm`, `projection2` keep the reference names."""


def _project(emb, h):
    """proj2(LN(proj1(h))) (model.py:68,116,201,326) via the fused HIP projection head."""
    return ops.projection_head(h, emb.projection1, emb.layer_norm, emb.projection2)


def hubert_execution_tweaks(hubert):
    """Execution-only changes to the HF HuBERT model (results unchanged up to summation order):
    the conv feature encoder runs as channels-last im2col + GEMM with a fused HIP GroupNorm +
    GELU for layer 0, and the positional convolution as an implicit-GEMM HIP kernel
    (triad_amd.frontend) -- no MIOpen; the raw waveform gets no gradient (HF marks it
    requires_grad only as a gradient-checkpointing workaround); the post-LN encoder layers run
    their residual / dropout / LayerNorm / GELU passes fused (triad_amd.postln)."""
    return install_fused_encoder(frontend.install_hubert_frontend(hubert))


class AudioEmbedder(nn.Module):
    """HuBERT + projection head (model.py:22-70)."""

    def __init__(self, embedding_dim=512, hubert_name="facebook/hubert-base-ls960"):
        super().__init__()
        over = _HUBERT_LARGE if "large" in hubert_name else None
        self.hubert = hubert_execution_tweaks(_hf_model("HubertModel", hubert_name, over))
        self.projection1 = nn.Linear(self.hubert.config.hidden_size, 512)
        self.layer_norm = nn.LayerNorm(512)
        self.projection2 = nn.Linear(512, embedding_dim)
        for p in self.parameters():
            p.requires_grad = True

    def normalize(self, audio: torch.Tensor) -> torch.Tensor:
        """The reference's processor call (model.py:56-62): Wav2Vec2FeatureExtractor with
        do_normalize=True treats the (B,T) batch as ONE utterance: (x - mean) / sqrt(var + 1e-7)
        over all B*T samples (measured). Done on the device: no host round trip."""
        return ops.global_znorm(audio, 1e-7)

    def forward(self, audio_input: torch.Tensor) -> torch.Tensor:
        if audio_input.dim() == 3:
            audio_input = audio_input.squeeze(0)
        x = self.normalize(audio_input.to(next(self.parameters()).device))
        h = self.hubert(x).last_hidden_state
        return _project(self, h)


class HashTokenizer:
    """Deterministic offline stand-in for the DistilBERT word-piece tokenizer.

    Lower-cased words/punctuation hashed into [1000, vocab); padding=True,
    truncation to max_length, no special tokens (model.py:102-109). Token ids
    differ from the real vocabulary (parity unpinned), shapes and masks do not.
    """

    def __init__(self, vocab_size=30522):
        self.vocab_size = vocab_size

    def __call__(self, texts, padding=True, truncation=True, add_special_tokens=False, max_length=128,
                 return_tensors="pt"):
        rows = []
        for t in texts:
            toks = re.findall(r"\w+|[^\w\s]", t.lower())
            ids = [1000 + zlib.crc32(w.encode()) % (self.vocab_size - 1000) for w in toks]
            rows.append(ids[:max_length] if truncation else ids)
        n = max(1, max(len(r) for r in rows))
        ids = torch.zeros(len(rows), n, dtype=torch.long)
        mask = torch.zeros(len(rows), n, dtype=torch.long)
        for i, r in enumerate(rows):
            ids[i, :len(r)] = torch.tensor(r, dtype=torch.long)
            mask[i, :len(r)] = 1
        return {"input_ids": ids, "attention_mask": mask}


class TextEmbedder(nn.Module):
    """BERT-like encoder + projection head (model.py:72-118). Like the reference, the default
    encoder is ModernBERT-base (model.py:77) and MultiModalModel passes DistilBERT (model.py:335);
    the encoder is whatever AutoModel resolves `model_name` to (model.py:80)."""

    def __init__(self, embedding_dim=512, model_name="answerdotai/ModernBERT-base"):
        super().__init__()
        try:
            from transformers import AutoTokenizer
            self.tokenizer = AutoTokenizer.from_pretrained(model_name, local_files_only=not _hub_online())
        except OSError as e:
            _fallback(model_name + " (tokenizer)", "HashTokenizer (hashed word ids)", e)
            self.tokenizer = HashTokenizer()
        self.encoder = install_fused_distilbert(_hf_model("AutoModel", model_name))  # no-op unless DistilBERT
        self.projection1 = nn.Linear(self.encoder.config.hidden_size, 512)
        self.layer_norm = nn.LayerNorm(512)
        self.projection2 = nn.Linear(512, embedding_dim)
        for p in self.parameters():
            p.requires_grad = True

    def tokenize(self, text_list):
        return self.tokenizer(text_list, padding=True, truncation=True, add_special_tokens=False,
                              max_length=128, return_tensors="pt")

    def forward(self, text_list):
        """text_list: list[str], or a pre-tokenised dict {input_ids, attention_mask}.
        Returns (text_feats (B,Nt,512), attention_mask (B,Nt))."""
        inputs = dict(text_list) if isinstance(text_list, Mapping) else self.tokenize(text_list)
        device = next(self.parameters()).device
        mask = inputs["attention_mask"]
        # A host-side mask with no padding is dropped before the encoder (identical math): HF
        # would otherwise test it on the device (`mask.all()`, a host sync) every step.
        no_pad = not mask.is_cuda and bool(mask.all())
        inputs = {k: (_lib.h2d(v, device) if not v.is_cuda and device.type == "cuda" else v.to(device))
                  for k, v in inputs.items()}
        h = self.encoder(input_ids=inputs["input_ids"],
                         attention_mask=None if no_pad else inputs["attention_mask"]).last_hidden_state
        return _project(self, h), inputs["attention_mask"]


def _dist_rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _load_dinov2_base(vit, arch):
    """The reference fetches pretrained DINOv2 through torch.hub (model.py:218). Offline, a hub
    state dict saved to a file can be named by TRIAD_DINOV2_WEIGHTS (loaded weights_only); the
    hub parameter names match this restatement. Without it the base is random-init (warned,
    recorded in RANDOM_INIT)."""
    import os
    path = os.environ.get("TRIAD_DINOV2_WEIGHTS")
    if path:
        sd = torch.load(path, map_location="cpu", weights_only=True)
        vit.load_state_dict(sd, strict=True)
        return
    _fallback(f"facebookresearch/dinov2:{arch}", "random-init DINOv2 restatement (triad_amd.vit)",
              OSError("torch.hub is not reachable offline and TRIAD_DINOV2_WEIGHTS is not set"))


class _PatchTokenEmbedder(nn.Module):
    """What ViTEmbedder (model.py:120-205) and ViTLoRAEmbedder (model.py:207-329) share: the DINOv2
    patch tokens (get_intermediate_layers(x, n=1)[0]), the projection head and the patch dropout
    (model.py:143-183 == 268-308: per-sample Bernoulli keep mask, kept tokens in order, zero-padded
    to the longest), on the HIP head and gather kernels."""

    def _init_head(self, embedding_dim, dropout_prob):
        self.projection1 = nn.Linear(self.model.embed_dim, 512)
        self.layer_norm = nn.LayerNorm(512)
        self.projection2 = nn.Linear(512, embedding_dim)
        self.patch_dropout_rate = dropout_prob
        # host generator of the patch-dropout masks; its state is saved in trainer checkpoints (one
        # per rank, checkpoint.trainer_checkpoint). It is seeded at the FIRST draw, not here, with
        # the data-parallel rank mixed in, so replicas seeded alike still draw different masks even
        # when the model is built before init_process_group
        self._mask_gen = torch.Generator()
        self._mask_seed_base = torch.initial_seed()
        self._mask_seeded = False
        self.mask_world = (1, 0)  # (W, rank): draw the global (W*B, N) mask, keep this rank's rows

    def mask_generator(self) -> torch.Generator:
        """The patch-mask generator, seeded on first use (initial seed + rank mix, or the shared
        seed of set_global_mask)."""
        if not self._mask_seeded:
            self._mask_gen.manual_seed((self._mask_seed_base + 0x9E3779B1 * _dist_rank()) % (2 ** 63))
            self._mask_seeded = True
        return self._mask_gen

    def set_global_mask(self, world, rank, seed=1234):
        """Global negatives: every rank draws the same global mask from a shared seed, so the
        padded key length (the global max kept count) agrees without any communication."""
        self.mask_world = (world, rank)
        self._mask_gen.manual_seed(seed)
        self._mask_seeded = True

    def draw_keep_mask(self, B, N):
        """Bernoulli(1 - drop) keep mask (model.py:157-159 / 282-284), drawn on the host.
        Returns (this rank's (B, N) mask, padded output length)."""
        W, r = self.mask_world
        full = torch.bernoulli(torch.full((W * B, N), 1.0 - self.patch_dropout_rate),
                               generator=self.mask_generator()).bool()
        return full[r * B:(r + 1) * B], int(full.sum(1).max())

    def patch_dropout(self, x, drop_rate, keep_mask=None):
        """model.py:143-183 / 268-308: keep tokens of each sample in order, zero-pad to the longest."""
        if not self.training or drop_rate == 0:
            return x
        B, N = x.shape[0], x.shape[1]
        n_out = None
        if keep_mask is None:
            keep_mask, n_out = self.draw_keep_mask(B, N)
        return ops.patch_dropout(x, keep_mask, n_out)

    def encode_patches(self, x):
        if x.dim() == 5:
            x = x.squeeze(0)
        if x.dim() == 3:
            x = x.unsqueeze(0)
        patches = self.model.get_intermediate_layers(x, n=1)[0]
        return _project(self, patches)

    def forward(self, x, keep_mask=None):
        feats = self.encode_patches(x)
        return self.patch_dropout(feats, self.patch_dropout_rate, keep_mask)


class ViTEmbedder(_PatchTokenEmbedder):
    """DINOv2 (no LoRA, every parameter trainable) + projection head + patch dropout
    (model.py:120-205). The reference's default arch has no register tokens ('dinov2_vitb14');
    MultiModalModel uses ViTLoRAEmbedder, this class completes the import surface."""

    def __init__(self, model_name="facebookresearch/dinov2", arch="dinov2_vitb14", embedding_dim=512,
                 dropout_prob=0.1):
        super().__init__()
        self.model = DinoVisionTransformer(arch)
        _load_dinov2_base(self.model, arch)
        self.model = install_fast_linear(self.model)
        self._init_head(embedding_dim, dropout_prob)
        for p in self.parameters():   # model.py:136-141
            p.requires_grad = True


class ViTLoRAEmbedder(_PatchTokenEmbedder):
    """DINOv2(-reg) + LoRA + projection head + patch dropout (model.py:207-329)."""

    def __init__(self, model_name="facebookresearch/dinov2", arch="dinov2_vitb14", embedding_dim=512,
                 dropout_prob=0.1, lora_rank=8, lora_alpha=16):
        super().__init__()
        self.model = DinoVisionTransformer(arch)
        _load_dinov2_base(self.model, arch)
        self.model = install_fast_linear(apply_lora(self.model, lora_rank, lora_alpha))  # MLP fc1 / fc2
        self._init_head(embedding_dim, dropout_prob)


class MultiModalModel(nn.Module):
    """model.py:331-637 with the fused HIP loss head."""

    def __init__(self, audio_model_name="facebook/hubert-base-ls960",
                 text_model_name="distilbert/distilbert-base-uncased", temperature=1.2,
                 patch_sparsity_threshold=0.3, patch_sparsity_weight=0.1, visual_dropout_prob=0.1, use_amp=True,
                 vit_arch="dinov2_vitb14_reg"):
        super().__init__()
        self.audio_embedder = AudioEmbedder(embedding_dim=512, hubert_name=audio_model_name)
        self.text_embedder = TextEmbedder(embedding_dim=512, model_name=text_model_name)
        self.visual_embedder = ViTLoRAEmbedder(arch=vit_arch, embedding_dim=512, dropout_prob=visual_dropout_prob)
        if use_amp:
            store_frozen_base_bf16(self.visual_embedder.model)
        self.temperature = nn.Parameter(torch.tensor(temperature))
        self.patch_sparsity_threshold = patch_sparsity_threshold
        self.patch_sparsity_weight = patch_sparsity_weight
        self.use_amp = use_amp
        self.amp_dtype = torch.bfloat16
        self.negatives_group = None  # process group for global negatives (SURVEY §8e Mode G)
        self.ds_budget = None        # bytes of tiled dS a head may materialise (None: ops.DS_BUDGET_BYTES)

    def enable_global_negatives(self, group=None):
        """Contrast every local query against the keys of all data-parallel ranks."""
        import torch.distributed as dist
        self.negatives_group = group if group is not None else dist.group.WORLD
        self.visual_embedder.set_global_mask(dist.get_world_size(group), dist.get_rank(group))

    # ---- inference similarity maps (model.py:355-368) -------------------------------
    def compute_similarity_matrix(self, feats1, feats2):
        """(B,N1,D) x (B,N2,D) -> (B,N1,N2) = normalize(f1) . normalize(f2)^T * temperature."""
        return ops.similarity_maps(feats1, feats2, self.temperature)

    # ---- fused training heads -------------------------------------------------------
    def _av_head(self, audio_feats, visual_feats):
        losses, stats, clip = ops.contrastive_head(ops.AV, audio_feats, visual_feats, self.temperature,
                                                   group=self.negatives_group,
                                                   ds_budget=getattr(self, "ds_budget", None))
        return (losses[0], losses[1], losses[2], losses[3], LazyStats(_AV_KEYS, stats)), clip

    def _tv_head(self, text_feats, visual_feats, attention_mask):
        losses, stats, clip = ops.contrastive_head(ops.TV, text_feats, visual_feats, self.temperature,
                                                   q_mask=attention_mask, threshold=self.patch_sparsity_threshold,
                                                   sparsity_weight=self.patch_sparsity_weight,
                                                   group=self.negatives_group,
                                                   ds_budget=getattr(self, "ds_budget", None))
        return (losses[0], LazyStats(_TV_KEYS, stats)), clip

    # ---- materialising debug path (small B), reference model.py:370-593 -------
    # Same names, arguments, composition and return tuples as the reference; every piece is a
    # differentiable HIP op of triad_amd.dense, so autograd through these matches the reference's.
    def compute_all_similarities_av(self, audio_feats, visual_feats):
        """-> (clip_sims (B,B), token_sims (B,B,Na,Nv) fp32) (model.py:370-392)."""
        return dense.all_similarities(audio_feats, visual_feats, self.temperature)

    def compute_temporal_smoothness_loss(self, token_sims):
        """mean of squared steps along Na over the diagonal pairs (model.py:394-408)."""
        return dense.diag_smoothness(token_sims)

    def compute_regularization_losses_av(self, token_sims):
        """-> (20 l_cal + 0.15 l_nonneg + 0.01 l_smooth, 0.01 l_smooth) (model.py:410-428)."""
        l_nonneg = dense.nonneg(token_sims, ops.CLAMP_LO[ops.AV])
        l_cal = torch.clamp(-torch.log(self.temperature), min=0) ** 2   # log(1) - log(temp); temp_high unused
        l_smooth = self.compute_temporal_smoothness_loss(token_sims)
        reg_loss = 20 * l_cal + 0.15 * l_nonneg + 0.01 * l_smooth
        return reg_loss, 0.01 * l_smooth

    def compute_contrastive_loss_av(self, clip_sims, token_sims):
        """-> (contrastive + reg, contrastive, reg, 0.01 l_smooth, stats) (model.py:430-472)."""
        contrastive_loss, st = dense.clip_ce(clip_sims)
        reg_loss, l_smooth = self.compute_regularization_losses_av(token_sims)
        return contrastive_loss + reg_loss, contrastive_loss, reg_loss, l_smooth, LazyStats(_AV_KEYS, st)

    def compute_all_similarities_tv(self, text_feats, visual_feats, attention_mask):
        """-> (clip_sims (B,B) masked mean over Nt, token_sims (B,B,Nt,Nv) fp32) (model.py:490-514)."""
        return dense.all_similarities(text_feats, visual_feats, self.temperature, q_mask=attention_mask)

    def compute_regularization_losses_tv(self, token_sims):
        """-> 0.15 l_nonneg + w * sparsity (model.py:516-542)."""
        l_nonneg = dense.nonneg(token_sims, ops.CLAMP_LO[ops.TV])
        loss_sparsity = dense.diag_sparsity(token_sims, self.patch_sparsity_threshold)
        return 0.15 * l_nonneg + self.patch_sparsity_weight * loss_sparsity

    def compute_contrastive_loss_tv(self, clip_sims, token_sims):
        """-> (contrastive + reg, stats) (model.py:544-593)."""
        contrastive_loss, st = dense.clip_ce(clip_sims)
        reg_loss = self.compute_regularization_losses_tv(token_sims)
        return contrastive_loss + reg_loss, LazyStats(_TV_KEYS, st)

    def forward_audio_visual(self, frames, audio):
        """-> (total, contrastive, reg, 0.01*l_smooth, stats) (model.py:474-488)."""
        with torch.autocast("cuda", enabled=self.use_amp, dtype=self.amp_dtype):
            visual_feats = self.visual_embedder(frames)
            audio_feats = self.audio_embedder(audio)
        return self._av_head(audio_feats, visual_feats)[0]

    def forward_text_visual(self, frames, text_list):
        """-> (total, stats) (model.py:595-608)."""
        with torch.autocast("cuda", enabled=self.use_amp, dtype=self.amp_dtype):
            visual_feats = self.visual_embedder(frames)
            text_feats, attention_mask = self.text_embedder(text_list)
        return self._tv_head(text_feats, visual_feats, attention_mask)[0]

    def forward_triad(self, frames, audio, text_list, av_keep=None, tv_keep=None):
        """One tri-modal triple batch: the frames are encoded once; AV and TV draw
        independent patch-dropout masks after the head (dropout follows the head,
        model.py:326-327, so this equals two separate encodes given the masks).
        Returns (av_tuple, tv_tuple) as forward_audio_visual / forward_text_visual."""
        ve = self.visual_embedder
        streams = _modality_streams(frames)
        with torch.autocast("cuda", enabled=self.use_amp, dtype=self.amp_dtype):
            if streams is None:
                patches = ve.encode_patches(frames)
                v_av = ve.patch_dropout(patches, ve.patch_dropout_rate, av_keep)
                v_tv = ve.patch_dropout(patches, ve.patch_dropout_rate, tv_keep)
                audio_feats = self.audio_embedder(audio)
                text_feats, attention_mask = self.text_embedder(text_list)
            else:
                # the three backbones are independent until the heads: audio and text run on
                # their own streams beside the ViT (and, since autograd runs each backward op on
                # its forward op's stream, so do their backward chains)
                # (the same host-side call order as above, so every RNG draw is unchanged)
                main, s_audio, s_text = streams
                s_audio.wait_stream(main)
                s_text.wait_stream(main)
                patches = ve.encode_patches(frames)
                v_av = ve.patch_dropout(patches, ve.patch_dropout_rate, av_keep)
                v_tv = ve.patch_dropout(patches, ve.patch_dropout_rate, tv_keep)
                with torch.cuda.stream(s_audio):
                    audio_feats = self.audio_embedder(audio)
                with torch.cuda.stream(s_text):
                    text_feats, attention_mask = self.text_embedder(text_list)
                main.wait_stream(s_audio)
                main.wait_stream(s_text)
                for t in (audio_feats, text_feats, attention_mask):
                    if isinstance(t, torch.Tensor) and t.is_cuda:
                        t.record_stream(main)
                if os.environ.get("TRIAD_STREAM_HANDOFF", "1") != "0":
                    audio_feats = _Handoff.apply(audio_feats, s_audio)
                    text_feats = _Handoff.apply(text_feats, s_text)
        return self._triad_heads(audio_feats, v_av, text_feats, v_tv, attention_mask)

    def _triad_heads(self, audio_feats, v_av, text_feats, v_tv, attention_mask):
        """Both heads with ONE similarity-forward launch (ops.contrastive_heads_av_tv); the same
        tuples as forward_audio_visual / forward_text_visual. TRIAD_PAIR_FWD=0: two launches."""
        import os
        if os.environ.get("TRIAD_PAIR_FWD", "1") == "0":
            return self._av_head(audio_feats, v_av)[0], self._tv_head(text_feats, v_tv, attention_mask)[0]
        (la, sa, _), (lt, st, _) = ops.contrastive_heads_av_tv(
            audio_feats, v_av, text_feats, v_tv, self.temperature, attention_mask,
            threshold=self.patch_sparsity_threshold, sparsity_weight=self.patch_sparsity_weight,
            group=self.negatives_group, ds_budget=getattr(self, "ds_budget", None))
        return (la[0], la[1], la[2], la[3], LazyStats(_AV_KEYS, sa)), (lt[0], LazyStats(_TV_KEYS, st))

    def forward(self, frames=None, audio=None, text_list=None):
        """Embeddings + L2-normalised similarity maps (model.py:610-637). `frames` is an
        image path (as in the reference) or a (3,H,W)/(B,3,H,W) tensor."""
        assert frames is not None or audio is not None or text_list is not None, \
            "At least one modality must be provided"
        if isinstance(frames, str):
            frames = _load_image(frames, next(self.parameters()).device)
        emb = {}
        if frames is not None:
            emb["visual_feats"] = self.visual_embedder(frames)
        if audio is not None:
            emb["audio_feats"] = self.audio_embedder(audio)
        if text_list is not None:
            emb["text_feats"], _ = self.text_embedder(text_list)
        if frames is not None and text_list is not None:
            emb["vis_text_sim_matrix"] = self.compute_similarity_matrix(emb["text_feats"], emb["visual_feats"])
        if audio is not None and frames is not None:
            emb["vis_audio_sim_matrix"] = self.compute_similarity_matrix(emb["audio_feats"], emb["visual_feats"])
        if audio is not None and text_list is not None:
            emb["text_audio_sim_matrix"] = self.compute_similarity_matrix(emb["text_feats"], emb["audio_feats"])
        return emb


_STREAMS = {}


class _Handoff(torch.autograd.Function):
    """Identity on the caller's (main) stream at a modality stream's output. Its backward runs on
    main, where the heads produce the feature gradient; the modality's backward then consumes
    that tensor on its own stream. The gradient is recorded for that stream (and the stream made
    to wait), so the caching allocator cannot hand its block to another main-stream tensor while
    the modality stream's kernels still read it -- whatever the autograd engine itself does at
    the stream boundary."""

    @staticmethod
    def forward(ctx, x, stream):
        ctx.stream = stream
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if g is not None and g.is_cuda:
            ctx.stream.wait_stream(torch.cuda.current_stream(g.device))
            g.record_stream(ctx.stream)
        return g, None


def modality_streams_enabled() -> bool:
    """forward_triad's execution mode: audio / text on their own HIP streams beside the ViT
    (default, TRIAD_MODALITY_STREAMS unset or 1) or all three backbones on the caller's stream
    (TRIAD_MODALITY_STREAMS=0). Both modes give bit-identical results
    (test_ops_gpu.py::test_step_bit_identical_serial_and_concurrent): every column-sum reduction of
    the step reads its rows by LDS-DMA (ops.bias_grad) -- plain-load reductions were what
    co-running streams disturbed."""
    return os.environ.get("TRIAD_MODALITY_STREAMS", "1") != "0"


def set_concurrent_streams(on: bool):
    """Switch the step between the concurrent default and the serial mode: the modality streams
    of forward_triad AND the weight-gradient side stream (triad_amd.linear)."""
    from . import linear
    os.environ["TRIAD_MODALITY_STREAMS"] = "1" if on else "0"
    linear.SIDE_STREAM_DW = bool(on)


def _modality_streams(frames):
    """(current, audio, text) streams for forward_triad's concurrent backbones, or None (CPU
    tensors, or the single-stream mode)."""
    if not (isinstance(frames, torch.Tensor) and frames.is_cuda) or not modality_streams_enabled():
        return None
    dev = frames.device
    pair = _STREAMS.get(dev.index)
    if pair is None:
        pair = _STREAMS[dev.index] = (torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev))
    return (torch.cuda.current_stream(dev),) + pair


def _load_image(path, device):
    """Resize 224, ToTensor, ImageNet normalise (model.py:615-622) without torchvision."""
    from PIL import Image
    import numpy as np
    img = Image.open(path).convert("RGB").resize((224, 224), Image.BILINEAR)
    x = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
    mean = torch.tensor([0.485, 0.456, 0.406])[:, None, None]
    std = torch.tensor([0.229, 0.224, 0.225])[:, None, None]
    return ((x - mean) / std).to(device)
