"""HuBERT post-LN encoder layers with the residual / dropout / LayerNorm / GELU passes fused
(csrc/postln.hip).

The reference trains HubertModel end to end under bf16 autocast (SajayR/TRIAD model.py:29-30,
48-70, 483; train.py:527-548). transformers' HubertEncoderLayer runs, per layer,

    h1 = LN1(res + dropout(attn(res)));  h2 = LN2(h1 + dropout(fc2(dropout(gelu(fc1(h1))))))

as ~20 elementwise ATen launches forward and backward over the fp32 residual stream (dropout
masks stored, every LayerNorm output cast to bf16 again by each of q/k/v/fc1). Here each
residual step is ONE row pass that also emits the bf16 GEMM operand, GELU + dropout is one pass,
and dropout keep bits are regenerated from a counter hash instead of stored. Module structure,
parameters and state-dict keys are unchanged (the encoder's forward is swapped per instance);
anything outside training-mode bf16 autocast on the GPU runs the stock transformers code.

Numerics: same operation order and roundings as the autocast chain; the dropout masks are drawn
from the hash instead of torch's Philox stream (same distribution, p to 1.5e-5), so parity
tests pin the kernels against torch on the SAME masks (triad_dropout_keep).
"""
from __future__ import annotations

import types

import torch

from ._lib import call, ptr, stream_ptr


class _Seeds:
    """Per-call 32-bit dropout seeds from a host generator (no device sync)."""

    def __init__(self):
        self.gen = torch.Generator()
        self.gen.manual_seed(torch.initial_seed() % (2 ** 63))

    def __call__(self):
        return int(torch.randint(0, 2 ** 32 - 1, (1,), generator=self.gen))


class _DropAddLN(torch.autograd.Function):
    """(h, hb) = (LN(res + dropout(y)), bf16 copy); res fp32 [..., D], y bf16 [..., D]."""

    @staticmethod
    def forward(ctx, res, y, w, b, eps, p, seed):
        D = res.shape[-1]
        M = res.numel() // D
        dev = res.device
        if not (res.dtype == torch.float32 and y.dtype == torch.bfloat16 and y.shape == res.shape
                and w.dtype == b.dtype == torch.float32 and w.numel() == b.numel() == D):
            raise TypeError(f"drop_add_ln: res {res.dtype} {tuple(res.shape)}, y {y.dtype} {tuple(y.shape)}")
        res = res.contiguous()
        y = y.contiguous()
        h = torch.empty_like(res)
        hb = torch.empty(res.shape, dtype=torch.bfloat16, device=dev)
        mean = torch.empty(M, dtype=torch.float32, device=dev)
        rstd = torch.empty(M, dtype=torch.float32, device=dev)
        call("triad_dropaddln_fwd", ptr(res), ptr(y), ptr(w), ptr(b), eps, M, D, p, seed, ptr(h), ptr(hb), ptr(mean),
             ptr(rstd), stream_ptr(dev))
        ctx.save_for_backward(res, y, w, mean, rstd)
        ctx.meta = (p, seed)
        return h, hb

    @staticmethod
    def backward(ctx, dh, dhb):
        res, y, w, mean, rstd = ctx.saved_tensors
        p, seed = ctx.meta
        D = res.shape[-1]
        M = res.numel() // D
        dev = res.device
        dh = None if dh is None else dh.contiguous()
        dhb = None if dhb is None else dhb.contiguous()
        if (dh is not None and (dh.dtype != torch.float32 or dh.shape != res.shape)) or \
                (dhb is not None and (dhb.dtype != torch.bfloat16 or dhb.shape != res.shape)):
            raise TypeError("drop_add_ln backward: unexpected gradient layout")
        dres = torch.empty_like(res)
        dy = torch.empty(res.shape, dtype=torch.bfloat16, device=dev)
        nb = call("triad_dropaddln_bwd_blocks", M)
        part = torch.empty(nb * 2 * D, dtype=torch.float32, device=dev)
        st = stream_ptr(dev)
        call("triad_dropaddln_bwd", ptr(dh), ptr(dhb), ptr(res), ptr(y), ptr(mean), ptr(rstd), ptr(w), M, D, p, seed,
             ptr(dres), ptr(dy), ptr(part), st)
        gwb = torch.empty(2 * D, dtype=torch.float32, device=dev)
        call("triad_sum_slabs", ptr(part), nb, 2 * D, None, 0, ptr(gwb), st, meta=dict(backbone=True))
        return dres, dy, gwb[:D], gwb[D:], None, None, None


_GELU_TABLES = {}


def gelu_table(device):
    """Per-device GELU value / slope table (triad_gelu_table), built once."""
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    t = _GELU_TABLES.get(key)
    if t is None:
        t = torch.empty(int(call("triad_gelu_table_bytes")), dtype=torch.uint8, device=device)
        call("triad_gelu_table", ptr(t), stream_ptr(device))
        torch.cuda.current_stream(device).synchronize()  # once: other streams read it without a wait
        _GELU_TABLES[key] = t
    return t


class _GeluDrop(torch.autograd.Function):
    """v = dropout(gelu(u)) on bf16 u (exact erf GELU, as ACT2FN['gelu'])."""

    @staticmethod
    def forward(ctx, u, p, seed):
        if u.dtype != torch.bfloat16 or u.numel() % 8:
            raise TypeError(f"gelu_drop: u {u.dtype} {tuple(u.shape)}")
        u = u.contiguous()
        v = torch.empty_like(u)
        call("triad_geludrop_fwd", ptr(u), u.numel(), p, seed, ptr(gelu_table(u.device)), ptr(v),
             stream_ptr(u.device))
        ctx.save_for_backward(u)
        ctx.meta = (p, seed)
        return v

    @staticmethod
    def backward(ctx, dv):
        (u,) = ctx.saved_tensors
        p, seed = ctx.meta
        dv = dv.to(torch.bfloat16).contiguous()
        du = torch.empty_like(u)
        call("triad_geludrop_bwd", ptr(u), ptr(dv), u.numel(), p, seed, ptr(gelu_table(u.device)), ptr(du),
             stream_ptr(u.device))
        return du, None, None


def drop_add_ln(res, y, norm, p, seed):
    return _DropAddLN.apply(res, y, norm.weight, norm.bias, norm.eps, p, seed)


def gelu_drop(u, p, seed):
    return _GeluDrop.apply(u, p, seed)


def gelu(u):
    """Exact-erf GELU of a bf16 CUDA tensor on the geludrop kernels with p = 0 (same value and
    gradient roundings as aten gelu / gelu_backward, one pass each way at HBM rate); anything
    else through F.gelu."""
    if u.is_cuda and u.dtype == torch.bfloat16 and u.numel() % 8 == 0 and u.numel() > 0:
        return _GeluDrop.apply(u, 0.0, 0)
    return torch.nn.functional.gelu(u)


def dropout_keep(n, p, seed, device):
    """The keep bits (u8) the kernels use for `n` elements at (p, seed): test view."""
    out = torch.empty(n, dtype=torch.uint8, device=device)
    call("triad_dropout_keep", n, p, seed, ptr(out), stream_ptr(out.device))
    return out


def _attn_parts(attn):
    """(q, k, v, out, heads, head_dim, scaling, dropout p) of a transformers HubertAttention or
    DistilBertSelfAttention."""
    if hasattr(attn, "q_proj"):
        return (attn.q_proj, attn.k_proj, attn.v_proj, attn.out_proj, attn.num_heads, attn.head_dim, attn.scaling,
                float(attn.dropout))
    return (attn.q_lin, attn.k_lin, attn.v_lin, attn.out_lin, attn.n_heads, attn.attention_head_size, attn.scaling,
            float(attn.dropout.p))


def self_attention(attn, x):
    """transformers HubertAttention / DistilBertSelfAttention forward (self-attention, no mask)
    with q / k / v as ONE projection GEMM (linear.qkv_projection) and the fused-qkv HIP
    attention kernels on its output; anything the fused form does not cover runs the module."""
    from . import attention as A
    from .linear import qkv_eligible, qkv_projection
    B, N, E = x.shape
    q, k, v, o, H, d, scaling, p = _attn_parts(attn)
    if not (qkv_eligible(q, k, v, x) and q.out_features == k.out_features == v.out_features == E == H * d
            and A.supported(x, N, d) and not getattr(attn, "is_causal", False)):
        return attn(x)[0]
    p = p if attn.training else 0.0
    return o(A.attention_qkv(qkv_projection(q, k, v, x), H, scaling, dropout=p))


def fused_layer(layer, res, res_b, seeds):
    """One HubertEncoderLayer (post-LN) on (fp32 residual, its bf16 copy) -> the same pair."""
    p_h = layer.dropout.p if layer.training else 0.0
    ff = layer.feed_forward
    p_a = ff.intermediate_dropout.p if layer.training else 0.0
    a = self_attention(layer.attention, res_b)
    h1, h1b = drop_add_ln(res, a, layer.layer_norm, p_h, seeds())
    v = gelu_drop(ff.intermediate_dense(h1b), p_a, seeds())
    f = ff.output_dense(v)
    p_o = ff.output_dropout.p if layer.training else 0.0
    return drop_add_ln(h1, f, layer.final_layer_norm, p_o, seeds())


def _fused_ok(enc, hidden_states, attention_mask, output_attentions, output_hidden_states):
    cfg = enc.config
    return (hidden_states.is_cuda and attention_mask is None and not output_attentions and not output_hidden_states
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and cfg.hidden_size % 256 == 0 and cfg.hidden_size <= 1024 and cfg.hidden_act == "gelu"
            and (hidden_states.shape[0] * hidden_states.shape[1] * cfg.intermediate_size) % 8 == 0)


def _encoder_forward(self, hidden_states, attention_mask=None, output_attentions=False, output_hidden_states=False,
                     return_dict=True):
    """HubertEncoder.forward (post-LN) with the fused layers; same pre-layer steps and LayerDrop."""
    if not _fused_ok(self, hidden_states, attention_mask, output_attentions, output_hidden_states):
        return self._triad_stock_forward(hidden_states, attention_mask=attention_mask,
                                         output_attentions=output_attentions,
                                         output_hidden_states=output_hidden_states, return_dict=return_dict)
    from transformers.modeling_outputs import BaseModelOutput
    position_embeddings = self.pos_conv_embed(hidden_states)
    hidden_states = hidden_states + position_embeddings.to(hidden_states.device)
    hidden_states = self.layer_norm(hidden_states)
    hidden_states = self.dropout(hidden_states)
    res = hidden_states.float()
    res_b = res.to(torch.bfloat16)
    for layer in self.layers:
        dropout_probability = torch.rand([])  # LayerDrop, as the stock loop draws it
        if self.training and dropout_probability < self.config.layerdrop:
            continue
        res, res_b = fused_layer(layer, res, res_b, self._triad_seeds)
    if not return_dict:
        return (res,)
    return BaseModelOutput(last_hidden_state=res)


def install_fused_encoder(hubert):
    """Swap the post-LN HubertEncoder's forward for the fused one (stable-LN encoders, e.g.
    HuBERT-large, keep the stock code)."""
    from transformers.models.hubert.modeling_hubert import HubertEncoder
    enc = hubert.encoder
    if type(enc) is HubertEncoder and not hasattr(enc, "_triad_stock_forward"):
        enc._triad_stock_forward = enc.forward
        enc._triad_seeds = _Seeds()
        enc.forward = types.MethodType(_encoder_forward, enc)
    return hubert


# ---- DistilBERT (model.py:79-80, 102-116: DistilBertModel trained after unfreeze_text_step) ----
# TransformerBlock: h1 = sa_LN(attn(h) + h); h2 = out_LN(dropout(lin2(gelu(lin1(h1)))) + h1),
# the same passes with p = 0 where DistilBERT has no dropout.

def fused_distilbert_block(block, res, res_b, seeds):
    ffn = block.ffn
    p = ffn.dropout.p if block.training else 0.0
    a = self_attention(block.attention, res_b)
    h1, h1b = drop_add_ln(res, a, block.sa_layer_norm, 0.0, 0)
    v = gelu_drop(ffn.lin1(h1b), 0.0, 0)
    return drop_add_ln(h1, ffn.lin2(v), block.output_layer_norm, p, seeds())


def _distilbert_transformer_forward(self, hidden_states, attention_mask=None, **kwargs):
    """transformers DistilBERT Transformer.forward with the fused residual / LayerNorm passes."""
    cfg = self.config
    if not (hidden_states.is_cuda and attention_mask is None and not kwargs.get("output_attentions")
            and not kwargs.get("output_hidden_states") and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16 and cfg.dim % 256 == 0 and cfg.dim <= 1024
            and cfg.activation == "gelu" and getattr(cfg, "chunk_size_feed_forward", 0) == 0
            and (hidden_states.shape[0] * hidden_states.shape[1] * cfg.hidden_dim) % 8 == 0):
        return self._triad_stock_forward(hidden_states, attention_mask, **kwargs)
    from transformers.modeling_outputs import BaseModelOutput
    res = hidden_states.float()
    res_b = res.to(torch.bfloat16)
    for block in self.layer:
        res, res_b = fused_distilbert_block(block, res, res_b, self._triad_seeds)
    return BaseModelOutput(last_hidden_state=res)


def install_fused_distilbert(encoder):
    """Swap a DistilBertModel's Transformer.forward for the fused one (per instance)."""
    tr = getattr(encoder, "transformer", None)
    if tr is not None and hasattr(tr, "layer") and not hasattr(tr, "_triad_stock_forward"):
        tr._triad_stock_forward = tr.forward
        tr._triad_seeds = _Seeds()
        tr.config = encoder.config
        tr.forward = types.MethodType(_distilbert_transformer_forward, tr)
    return encoder
