"""DINOv2 ViT with register tokens + LoRA adapters (PyTorch-ROCm backbone).

The reference loads `torch.hub.load('facebookresearch/dinov2', 'dinov2_vitb14_reg')`
(src/model.py:218,346) and wraps it with peft LoRA (r=8, alpha=16, dropout 0) on
`attn.qkv` and `attn.proj` (model.py:227-248). Neither the hub code nor peft is
available offline, so this module restates that architecture with the hub's
parameter names (patch_embed.proj, cls_token, register_tokens, pos_embed,
blocks.N.{norm1,attn.qkv,attn.proj,ls1,norm2,mlp.fc1,mlp.fc2,ls2}, norm), so a hub
state_dict loads into it, and implements LoRA directly (`lora_A` / `lora_B`
parameters, names containing "lora" as train.py:256-258 expects).
Backbone numerics are "parity unpinned": no pretrained weights exist offline.
Attention uses torch's fused scaled_dot_product_attention (ROCm flash kernels).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import attention
from . import gemm as hipgemm
from ._lib import call, ptr, stream_ptr
from .frontend import patch_embed
from .postln import gelu

ARCHS = {
    # name: (embed_dim, depth, heads)
    "dinov2_vits14_reg": (384, 12, 6),
    "dinov2_vitb14_reg": (768, 12, 12),
    "dinov2_vitl14_reg": (1024, 24, 16),
    "dinov2_vits14": (384, 12, 6),
    "dinov2_vitb14": (768, 12, 12),
    "dinov2_vitl14": (1024, 24, 16),
}


class _LoRALinear(torch.autograd.Function):
    """y = x W^T + b + (s B)(A x) for a frozen base under bf16 autocast, as ONE base GEMM plus an
    in-place rank-8 update, with the skinny products on the HIP kernels of csrc/lora.hip:
    forward t = x A^T (triad_rows_nt) and y += t (sB)^T (triad_lora_update); backward ONE pass
    over dy for both dt = dy (sB) and dB = s dy^T t (triad_lora_tn), dX = dy W on the library
    GEMM plus dx += dt A (triad_lora_update), and one pass over x for dA = dt^T x. Same
    operands and rounding class as autocast's F.linear chain; LoRA gradients accumulate in fp32."""

    @staticmethod
    def forward(ctx, x, w, b, A, B, scaling):
        lead, K = x.shape[:-1], x.shape[-1]
        O, r = B.shape
        xb = x.reshape(-1, K).to(torch.bfloat16).contiguous()
        M = xb.shape[0]
        dev = x.device
        st = stream_ptr(dev)
        Ab = A.detach().to(torch.bfloat16).contiguous()
        sB = (B.detach() * scaling).to(torch.bfloat16).contiguous()
        y = hipgemm.linear(xb, w.to(torch.bfloat16), None if b is None else b.to(torch.bfloat16)).contiguous()
        t = torch.empty(M, r, dtype=torch.bfloat16, device=dev)
        call("triad_rows_nt", ptr(xb), K, M, K, ptr(Ab), r, ptr(t), st)
        call("triad_lora_update", ptr(y), O, M, O, ptr(t), ptr(sB), st)
        ctx.save_for_backward(xb, w, Ab, sB, t)
        ctx.meta = (lead, x.dtype, float(scaling), A.dtype, B.dtype)
        return y.view(*lead, O)

    @staticmethod
    def backward(ctx, dy):
        xb, w, Ab, sB, t = ctx.saved_tensors
        lead, x_dtype, scaling, a_dtype, b_dtype = ctx.meta
        M, K = xb.shape
        O, r = sB.shape
        dev = xb.device
        dy2 = dy.reshape(M, O).to(torch.bfloat16).contiguous()
        st = stream_ptr(dev)
        dt = torch.empty(M, r, dtype=torch.bfloat16, device=dev)
        G = call("triad_lora_tn_blocks", M)
        slabs = torch.empty(G * max(O, K) * r, dtype=torch.float32, device=dev)
        # dt = dy (sB) and dB = s dy^T t in one pass over dy
        wt = torch.zeros(16, O, dtype=torch.bfloat16, device=dev)
        wt[:r].copy_(sB.t())
        dB = torch.empty(O, r, dtype=torch.float32, device=dev)
        call("triad_lora_tn", ptr(dy2), O, M, O, ptr(t), ptr(wt), ptr(dt), scaling, ptr(slabs), ptr(dB), st)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = hipgemm.mm(dy2, w.to(torch.bfloat16))
            At = Ab.t().contiguous()   # referenced across the launch
            call("triad_lora_update", ptr(dx), K, M, K, ptr(dt), ptr(At), st)
            dx = dx.view(*lead, K).to(x_dtype)
        dAt = torch.empty(K, r, dtype=torch.float32, device=dev)
        call("triad_lora_tn", ptr(xb), K, M, K, ptr(dt), None, None, 1.0, ptr(slabs), ptr(dAt), st)
        return dx, None, None, dAt.t().to(a_dtype), dB.to(b_dtype), None


def lora_linear(x, w, b, A, B, scaling):
    return _LoRALinear.apply(x, w, b, A, B, scaling)


class LoRALinear(nn.Module):
    """y = base(x) + (alpha/r) * B(A(x)); base frozen by the caller, B zero-initialised."""

    def __init__(self, base: nn.Linear, r: int = 8, alpha: int = 16):
        super().__init__()
        self.base = base
        self.lora_A = nn.Parameter(torch.empty(r, base.in_features))
        self.lora_B = nn.Parameter(torch.zeros(base.out_features, r))
        nn.init.kaiming_uniform_(self.lora_A, a=math.sqrt(5))
        self.scaling = alpha / r

    @property
    def weight(self):
        return self.base.weight

    def forward(self, x):
        if x.is_cuda and torch.is_autocast_enabled("cuda") and not self.base.weight.requires_grad \
                and (self.base.bias is None or not self.base.bias.requires_grad) and self.lora_A.shape[0] == 8 \
                and self.lora_A.shape[1] % 256 == 0 and self.lora_B.shape[0] % 256 == 0:
            return lora_linear(x, self.base.weight, self.base.bias, self.lora_A, self.lora_B, self.scaling)
        return self.base(x) + F.linear(F.linear(x, self.lora_A), self.lora_B) * self.scaling


class Attention(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim, bias=True)

    def forward(self, x):
        B, N, C = x.shape
        qkv = self.qkv(x)
        if attention.supported(qkv, N, C // self.heads):  # HIP kernels (triad_amd.attention)
            return self.proj(attention.attention_qkv(qkv, self.heads))
        qkv = qkv.reshape(B, N, 3, self.heads, C // self.heads).permute(2, 0, 3, 1, 4)
        o = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2])
        return self.proj(o.transpose(1, 2).reshape(B, N, C))


class LayerScale(nn.Module):
    def __init__(self, dim, init=1e-5):
        super().__init__()
        self.gamma = nn.Parameter(torch.full((dim,), init))

    def forward(self, x):
        return x * self.gamma


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(gelu(self.fc1(x)))


class _AddScaleLN(torch.autograd.Function):
    """(xn, ln) = (x + g * y, LayerNorm(x + g * y)) for the frozen DINOv2 blocks under bf16
    autocast, as one HIP row pass each way (csrc/resid_ln.hip): y is the bf16 branch output
    (attention proj / fc2), g the LayerScale gamma, ln bf16 (the next GEMM's operand) or fp32
    (the final norm). Backward: dx = dxn + LN'(dln), dy = bf16(g dx); LayerNorm / LayerScale
    parameters are frozen (model.py:223-224) and get no gradient."""

    @staticmethod
    def forward(ctx, x, y, g, w, b, eps, out_f32):
        M, D = x.numel() // x.shape[-1], x.shape[-1]
        dev = x.device
        # the kernels index x / xn as fp32 and y as bf16 rows of D: check before launching
        if not (x.dtype == torch.float32 and y.dtype == torch.bfloat16 and y.shape == x.shape
                and all(p.dtype == torch.float32 and p.numel() == D for p in (g, w, b))):
            raise TypeError(f"add_scale_ln: x {x.dtype} {tuple(x.shape)}, y {y.dtype} {tuple(y.shape)}")
        x = x.contiguous()
        y = y.contiguous()
        xn = torch.empty_like(x)
        ln = torch.empty(x.shape, dtype=torch.float32 if out_f32 else torch.bfloat16, device=dev)
        mean = torch.empty(M, dtype=torch.float32, device=dev)
        rstd = torch.empty(M, dtype=torch.float32, device=dev)
        call("triad_addln_fwd", ptr(x), ptr(y), ptr(g), ptr(w), ptr(b), eps, M, D, ptr(xn), ptr(ln), int(out_f32),
             ptr(mean), ptr(rstd), stream_ptr(dev))
        ctx.save_for_backward(xn, mean, rstd, w, g)
        return xn, ln

    @staticmethod
    def backward(ctx, dxn, dln):
        xn, mean, rstd, w, g = ctx.saved_tensors
        M, D = xn.numel() // xn.shape[-1], xn.shape[-1]
        dev = xn.device
        if dln is None:
            dln = torch.zeros_like(xn)
        dln = dln.contiguous()
        if dln.shape != xn.shape or dln.dtype not in (torch.float32, torch.bfloat16) or \
                (dxn is not None and (dxn.shape != xn.shape or dxn.dtype != torch.float32)):
            raise TypeError("add_scale_ln backward: unexpected gradient layout")
        dxn = None if dxn is None else dxn.contiguous()
        dx = torch.empty_like(xn)
        dy = torch.empty(xn.shape, dtype=torch.bfloat16, device=dev)
        call("triad_addln_bwd", ptr(dln), int(dln.dtype == torch.float32), ptr(dxn), ptr(xn), ptr(mean), ptr(rstd),
             ptr(w), ptr(g), M, D, ptr(dx), ptr(dy), stream_ptr(dev))
        return dx, dy, None, None, None, None, None


def add_scale_ln(x, y, ls, norm, out_f32=False):
    return _AddScaleLN.apply(x, y, ls.gamma, norm.weight, norm.bias, norm.eps, out_f32)


class Block(nn.Module):
    def __init__(self, dim, heads, mlp_ratio=4.0, ls_init=1e-5):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, heads)
        self.ls1 = LayerScale(dim, ls_init)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))
        self.ls2 = LayerScale(dim, ls_init)

    def forward(self, x):
        x = x + self.ls1(self.attn(self.norm1(x)))
        return x + self.ls2(self.mlp(self.norm2(x)))


class PatchEmbed(nn.Module):
    def __init__(self, patch, dim):
        super().__init__()
        self.proj = nn.Conv2d(3, dim, kernel_size=patch, stride=patch)

    def forward(self, x):
        # = self.proj(x).flatten(2).transpose(1, 2), as one GEMM over the reshaped patches
        return patch_embed(x, self.proj.weight, self.proj.bias, self.proj.stride[0])


class DinoVisionTransformer(nn.Module):
    """dinov2_vit*14(_reg): 518 px pretraining grid (37x37), bicubic pos-embed interpolation."""

    def __init__(self, arch="dinov2_vitb14_reg", img_size=518, patch=14):
        super().__init__()
        dim, depth, heads = ARCHS[arch]
        self.embed_dim = dim
        self.patch_size = patch
        self.num_register_tokens = 4 if arch.endswith("_reg") else 0
        self.interpolate_antialias = self.num_register_tokens > 0
        self.interpolate_offset = 0.0 if self.num_register_tokens > 0 else 0.1
        grid = img_size // patch
        self.patch_embed = PatchEmbed(patch, dim)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, 1 + grid * grid, dim))
        self.register_tokens = (nn.Parameter(torch.zeros(1, self.num_register_tokens, dim))
                                if self.num_register_tokens else None)
        self.mask_token = nn.Parameter(torch.zeros(1, dim))
        self.blocks = nn.ModuleList([Block(dim, heads) for _ in range(depth)])
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=1e-6)
        if self.register_tokens is not None:
            nn.init.normal_(self.register_tokens, std=1e-6)
        self.apply(self._init)
        self._pos_cache = {}

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)

    def refresh_frozen_copies(self):
        """Called after a state_dict load: drop the cached interpolated positional embedding."""
        self._pos_cache = {}

    def interpolate_pos_encoding(self, n_patches_h, n_patches_w, dtype):
        key = (n_patches_h, n_patches_w, dtype, self.pos_embed._version)
        if not self.pos_embed.requires_grad and key in self._pos_cache:
            return self._pos_cache[key]
        pos = self.pos_embed.float()
        cls_pos, patch_pos = pos[:, :1], pos[:, 1:]
        M = int(math.sqrt(patch_pos.shape[1]))
        if (n_patches_h, n_patches_w) != (M, M):
            patch_pos = F.interpolate(patch_pos.reshape(1, M, M, -1).permute(0, 3, 1, 2),
                                      size=(n_patches_h, n_patches_w), mode="bicubic",
                                      antialias=self.interpolate_antialias)
            patch_pos = patch_pos.permute(0, 2, 3, 1).reshape(1, -1, pos.shape[-1])
        out = torch.cat([cls_pos, patch_pos], dim=1).to(dtype)
        if not self.pos_embed.requires_grad:
            self._pos_cache = {key: out.detach()}
        return out

    def prepare_tokens(self, x):
        B, _, H, W = x.shape
        t = self.patch_embed(x)
        t = torch.cat([self.cls_token.expand(B, -1, -1).to(t.dtype), t], dim=1)
        t = t + self.interpolate_pos_encoding(H // self.patch_size, W // self.patch_size, t.dtype)
        if self.register_tokens is not None:
            t = torch.cat([t[:, :1], self.register_tokens.expand(B, -1, -1).to(t.dtype), t[:, 1:]], dim=1)
        return t

    def _fused_ok(self, t, n, norm):
        return (t.is_cuda and n == 1 and norm and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16 and self.embed_dim % 256 == 0
                and self.embed_dim <= 1536
                and not any(p.requires_grad for blk in self.blocks
                            for m in (blk.norm1, blk.norm2, blk.ls1, blk.ls2) for p in m.parameters())
                and not any(p.requires_grad for p in self.norm.parameters()))

    def _blocks_fused(self, t):
        """The blocks with every residual + LayerScale + LayerNorm step as one HIP row pass
        (_AddScaleLN); attention and MLP branches unchanged. Returns the final norm (fp32).
        The token embedding comes out of the patch GEMM in bf16; autocast's first residual add
        promotes it to fp32 exactly, as t.float() does here."""
        t = t.float()
        ln = F.layer_norm(t, (self.embed_dim,), self.blocks[0].norm1.weight, self.blocks[0].norm1.bias,
                          self.blocks[0].norm1.eps)
        last = len(self.blocks) - 1
        for i, blk in enumerate(self.blocks):
            t, ln = add_scale_ln(t, blk.attn(ln), blk.ls1, blk.norm2)
            nxt = self.norm if i == last else self.blocks[i + 1].norm1
            t, ln = add_scale_ln(t, blk.mlp(ln), blk.ls2, nxt, out_f32=i == last)
        return ln

    def get_intermediate_layers(self, x, n=1, norm=True):
        """Hub semantics for an int n: outputs of the last n blocks, normed, patch tokens only."""
        t = self.prepare_tokens(x)
        if self._fused_ok(t, n, norm):
            return (self._blocks_fused(t)[:, 1 + self.num_register_tokens:],)
        outs = []
        start = len(self.blocks) - n
        for i, blk in enumerate(self.blocks):
            t = blk(t)
            if i >= start:
                outs.append(t)
        if norm:
            outs = [self.norm(o) for o in outs]
        skip = 1 + self.num_register_tokens
        return tuple(o[:, skip:] for o in outs)

    def forward(self, x):
        t = self.prepare_tokens(x)
        for blk in self.blocks:
            t = blk(t)
        return self.norm(t)[:, 0]


def apply_lora(vit: DinoVisionTransformer, r=8, alpha=16, targets=("attn.qkv", "attn.proj")):
    """Freeze the ViT and wrap the target Linears with LoRA (model.py:223-266)."""
    for p in vit.parameters():
        p.requires_grad = False
    for blk in vit.blocks:
        if "attn.qkv" in targets:
            blk.attn.qkv = LoRALinear(blk.attn.qkv, r, alpha)
        if "attn.proj" in targets:
            blk.attn.proj = LoRALinear(blk.attn.proj, r, alpha)
    for n, p in vit.named_parameters():
        p.requires_grad = "lora_" in n
    return vit


def store_frozen_base_bf16(vit: nn.Module):
    """Keep the frozen (non-LoRA) Linear / Conv weights of the ViT in bf16.

    Under bf16 autocast (model.py:483,603) every forward casts these fp32 weights to bf16;
    they never change (frozen, model.py:223-224,261-262), so storing the cast once gives
    bit-identical matmul operands and removes ~86 M x 6 B of cast traffic and ~170 cast
    launches per step. LayerNorm / LayerScale / token parameters stay fp32 (autocast keeps
    their ops in fp32).

    The fp32 values are kept (host memory, `vit.frozen_fp32`, keyed by parameter name): they
    are what a checkpoint saves (the reference keeps the frozen base in fp32, train.py:413), so
    a reference checkpoint loaded here and saved again comes back bit-exact."""
    masters = {}
    for mname, mod in vit.named_modules():
        if isinstance(mod, (nn.Linear, nn.Conv2d)):
            for pname, p in mod.named_parameters(recurse=False):
                if not p.requires_grad and p.dtype != torch.bfloat16:
                    masters[f"{mname}.{pname}" if mname else pname] = p.data.detach().to("cpu", torch.float32,
                                                                                            copy=True)
                    p.data = p.data.to(torch.bfloat16)
    vit.frozen_fp32 = {**getattr(vit, "frozen_fp32", {}), **masters}
    return vit
