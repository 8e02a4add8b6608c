"""Convolutional front-ends of the backbones, executed as GEMMs (no MIOpen).

The reference's audio path (SajayR/TRIAD model.py:29-30,64-66) runs HuBERT's conv
feature encoder -- 7 strided conv1d layers over the 64 000-sample waveform, layer 0
followed by GroupNorm(512 groups) and GELU, the others by GELU -- and its visual path
(model.py:218-227) a 14x14 / stride-14 patch-embedding conv. On MI355X these are
re-expressed without changing their parameters or math:

  * every conv layer is im2col + ONE hipBLASLt GEMM over channels-last (B, T, C) tensors
    (`conv1d_gemm`; M = B*T_out rows, K = kernel*C_in): MIOpen, its NCHW<->NHWC transposes
    and its per-shape kernel search / runtime compilation on a fresh box are gone;
  * layer 0's GroupNorm + GELU is one fused HIP kernel pair over the channels-last conv
    output (`triad_chgn_gelu_fwd/bwd`, csrc/frontend.hip), writing the bf16 value the next
    conv reads instead of fp32 GroupNorm and GELU tensors;
  * the patch embedding is a reshape (non-overlapping patches) + one GEMM.

The GEMMs run in the autocast dtype (bf16) with fp32 accumulation, as autocast would run
the convolutions. On a CPU tensor the original transformers modules run unchanged.
"""
from __future__ import annotations

import types
from ctypes import c_void_p as C_void_p

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import call, ptr, stream_ptr


def _compute_dtype(x):
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return x.dtype


class _Conv1dGemm(torch.autograd.Function):
    """y[b, t, o] = sum_{j, c} x[b, s*t + j, c] * w[o, c, j] (+ bias[o]): a 'valid' strided
    conv1d over channels-last x (B, T, C), as im2col (cols[b, t, j, c]) + one GEMM with the
    weight viewed as wr[o, j*C + c]."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, need_dx, cd):
        B, T, C = x.shape
        O, Cw, k = w.shape
        if Cw != C:
            raise ValueError(f"conv1d_gemm: weight expects {Cw} input channels, got {C}")
        To = (T - k) // stride + 1
        if To <= 0:
            raise ValueError("conv1d_gemm: input shorter than the kernel")
        xc = x.to(cd)
        if C == 1:
            cols = xc.reshape(B, T).unfold(1, k, stride).reshape(B * To, k)
        else:
            cols4 = torch.empty(B, To, k, C, dtype=cd, device=x.device)
            span = stride * (To - 1) + 1
            for j in range(k):
                cols4[:, :, j].copy_(xc[:, j:j + span:stride])
            cols = cols4.view(B * To, k * C)
        wr = w.to(cd).permute(0, 2, 1).reshape(O, k * C)
        if bias is None:
            y = torch.mm(cols, wr.t())
        else:
            y = torch.addmm(bias.to(cd), cols, wr.t())
        ctx.save_for_backward(cols, wr)
        ctx.shape = (B, T, C, O, k, To, stride)
        ctx.need_dx, ctx.has_bias, ctx.w_dtype, ctx.x_dtype = need_dx, bias is not None, w.dtype, x.dtype
        ctx.b_dtype = bias.dtype if bias is not None else None
        return y.view(B, To, O)

    @staticmethod
    def backward(ctx, dy):
        cols, wr = ctx.saved_tensors
        B, T, C, O, k, To, stride = ctx.shape
        dy2 = dy.reshape(B * To, O).to(cols.dtype)
        dw = torch.mm(dy2.t(), cols).view(O, k, C).permute(0, 2, 1).to(ctx.w_dtype)
        acc = torch.float32 if dy2.dtype in (torch.bfloat16, torch.float16) else dy2.dtype
        db = torch.sum(dy2, 0, dtype=acc).to(ctx.b_dtype) if ctx.has_bias else None
        dx = None
        if ctx.need_dx:
            dcols = torch.mm(dy2, wr).view(B, To, k, C)
            dx = torch.zeros(B, T, C, dtype=cols.dtype, device=cols.device)
            span = stride * (To - 1) + 1
            for j in range(k):
                dx[:, j:j + span:stride] += dcols[:, :, j]
            dx = dx.to(ctx.x_dtype)
        return dx, dw, db, None, None, None


def conv1d_gemm(x, weight, bias, stride, need_dx=True):
    """Channels-last strided conv1d (no padding, dilation 1, groups 1) as im2col + GEMM."""
    return _Conv1dGemm.apply(x, weight, bias, int(stride), bool(need_dx), _compute_dtype(x))


class _ChannelGroupNormGelu(torch.autograd.Function):
    """gelu(GroupNorm(num_groups=C)(x)) over channels-last x (B, T, C) bf16 -> bf16 (HIP). With
    `frames` = (B, T, Tp), x is a flat padded frame buffer (sample b's valid frames at rows
    b*Tp .. b*Tp+T-1; padding frames come out 0 and get no gradient)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, frames=None):
        if frames is None:
            B, T, C = x.shape
            Tp = T
        else:
            (B, T, Tp), C = frames, x.shape[-1]
            if x.dim() != 2 or x.shape[0] < B * Tp:
                raise _lib.TriadError("channel_group_norm_gelu: frame buffer smaller than B * Tp rows")
        xc = x.contiguous()
        dev = x.device
        g = gamma.detach().float().contiguous()
        b = beta.detach().float().contiguous()
        mean = torch.empty(B, C, dtype=torch.float32, device=dev)
        rstd = torch.empty(B, C, dtype=torch.float32, device=dev)
        ws = torch.empty(int(call("triad_chgn_workspace_bytes", B, T, C)), dtype=torch.uint8, device=dev)
        y = torch.empty_like(xc)
        if y.shape[0] > B * Tp and frames is not None:
            y[B * Tp:].zero_()
        call("triad_chgn_gelu_fwd", ptr(xc), B, T, Tp, C, ptr(g), ptr(b), float(eps), ptr(mean), ptr(rstd), ptr(ws),
             ptr(y), stream_ptr(dev))
        ctx.save_for_backward(xc, g, b, mean, rstd)
        ctx.dtypes = (gamma.dtype, beta.dtype)
        ctx.frames = (B, T, Tp, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, g, b, mean, rstd = ctx.saved_tensors
        B, T, Tp, C = ctx.frames
        dev = xc.device
        dyc = dy.to(xc.dtype).contiguous()
        dx = torch.empty_like(xc)
        if dx.dim() == 2 and dx.shape[0] > B * Tp:
            dx[B * Tp:].zero_()
        dg = torch.empty(C, dtype=torch.float32, device=dev)
        db = torch.empty(C, dtype=torch.float32, device=dev)
        ws = torch.empty(int(call("triad_chgn_workspace_bytes", B, T, C)), dtype=torch.uint8, device=dev)
        call("triad_chgn_gelu_bwd", ptr(xc), ptr(dyc), B, T, Tp, C, ptr(g), ptr(b), ptr(mean), ptr(rstd), ptr(ws),
             ptr(dx), ptr(dg), ptr(db), stream_ptr(dev))
        return dx, dg.to(ctx.dtypes[0]), db.to(ctx.dtypes[1]), None, None


# ---- HuBERT conv stack over padded frame buffers ---------------------------------------------
# Activations of the feature encoder live in flat channels-last frame buffers [B*Tp + 2, C]
# (bf16): sample b's frames at rows b*Tp .. b*Tp+Tp-1 with Tp EVEN (the valid T frames, then one
# padding frame when T is odd), plus two spare zero frames at the end. Pairs of frames are then
# rows of a [B*Tp/2 + 1, 2C] matrix with a uniform stride, so a kernel-3 / stride-2 conv is ONE
# GEMM whose A operand has OVERLAPPING rows (row r = frames 2r .. 2r+2: lda = 2C < K = 3C) and a
# kernel-2 / stride-2 conv a plain GEMM over the pair rows -- no im2col copy; and the input
# gradient of the kernel-3 conv is one GEMM over overlapping rows of dY (row q = dY[q-1], dY[q]).
# Each layer produces B*Tp/2 rows of which the last per sample straddles the next sample: it is
# the padding frame of the next layer (finite, never read by a valid output, zero gradient).

def _addr(t, row, ld):
    return C_void_p(t.data_ptr() + 2 * row * ld)


def _gemm_rows(a, a_row, lda, M, K, b, out, out_row, ldc):
    """out[out_row + m][:N] = sum_k A[m][k] b[n][k] (bf16, fp32 accumulate) with A[m][k] =
    a.flat[(a_row + m) * lda + k] (rows may overlap), b [N][K] contiguous bf16."""
    N = b.shape[0]
    if M % 128 == 0 and N % 128 == 0 and K % 64 == 0 and lda % 8 == 0 and ldc % 8 == 0:
        # the eight-wave 256 x 256 tile for every tall product, K = 512 included (the size policy's
        # 256 x 128 ring ran the 512-deep input gradients at 605-690 TFLOP/s, this form 745-815;
        # bit-identical, profiles/r04_conv_gemm_ab.log; A/B tool in git history)
        form = 4 if M >= 32768 and M % 256 == 0 and N % 256 == 0 else 0
        call("triad_gemm_bf16_form", _addr(a, a_row, lda), lda, 1, ptr(b), K, 1, M, N, K, None,
             _addr(out, out_row, ldc), ldc, 1, form, stream_ptr(a.device), meta=dict(backbone=True))
    else:  # same product through torch (it copies the overlapping operand)
        A = a.as_strided((M, K), (lda, 1), a.storage_offset() + a_row * lda)
        out.as_strided((M, N), (ldc, 1), out.storage_offset() + out_row * ldc).copy_(torch.mm(A, b.t()))


def _conv_dw_plan(M, O, N):
    """(form, splits) of a conv-stack weight gradient ([O][N] over M frame-pair rows): the
    eight-wave 256 x 256 tile with one round of <= 256 workgroups (21 splits at N = 1536, 32 with
    each split on one XCD at N = 1024), >= 2,048 rows per split. 965 against 720 TFLOP/s for the
    former 8 splits of 256 x 128 tiles (192 workgroups) at 1.6 M rows x 1,536 -- 3.6 -> 2.65 ms per
    call, ~1.9 ms per c3 step over the conv stack (profiles/r04_conv_dw_ab.log; A/B tool in git history)."""
    if O % 256 or N % 256:
        return 0, 8
    sp = max(1, min(256 // ((O // 256) * (N // 256)), M // 2048))
    return (4 | 8 if sp % 8 == 0 else 4), sp


def _weight_grad_rows(dy, M, x, ldx, N):
    """fp32 [O][N] = sum_r dy[r][o] X[r][n] over r < M, X[r][n] = x.flat[r * ldx + n] (overlapping)."""
    O = dy.shape[1]
    if M % 64 == 0 and O % 128 == 0 and N % 128 == 0 and ldx % 8 == 0:
        form, sp = _conv_dw_plan(M, O, N)
        slabs = torch.empty(sp * O * N, dtype=torch.float32, device=dy.device)
        out = torch.empty(O, N, dtype=torch.float32, device=dy.device)
        call("triad_gemm_bf16_splitk_form", ptr(dy), O, 0, ptr(x), ldx, 0, O, N, M, sp, None, ptr(slabs), ptr(out), 0,
             form, stream_ptr(dy.device), meta=dict(backbone=True))
        return out
    X = x.as_strided((M, N), (ldx, 1), x.storage_offset())
    return torch.mm(dy[:M].t(), X, out_dtype=torch.float32)


class _FrameConv0(torch.autograd.Function):
    """HuBERT conv layer 0 (1 -> O channels, kernel k, stride s, no bias) from the (B, L)
    waveform into a padded frame buffer; the padding frame is computed from zero-padded
    samples. The waveform gets no gradient."""

    @staticmethod
    def forward(ctx, wave, w, stride, Tp):
        B, L = wave.shape
        O, _, k = w.shape
        need = (Tp - 1) * stride + k
        xw = F.pad(wave.to(torch.bfloat16), (0, max(0, need - L)))
        cols = xw.unfold(1, k, stride)[:, :Tp].reshape(B * Tp, k)
        wr = w.to(torch.bfloat16).reshape(O, k)
        y = torch.empty(B * Tp + 2, O, dtype=torch.bfloat16, device=wave.device)
        torch.mm(cols, wr.t(), out=y[:B * Tp])
        y[B * Tp:].zero_()
        ctx.save_for_backward(cols)
        ctx.meta = (B, Tp, w.shape, w.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        (cols,) = ctx.saved_tensors
        B, Tp, wshape, wdt = ctx.meta
        dw = torch.mm(dy[:B * Tp].t().to(torch.bfloat16), cols, out_dtype=torch.float32)
        return None, dw.view(wshape).to(wdt), None, None


class _Conv0GNGelu(torch.autograd.Function):
    """HuBERT conv layer 0 (1 -> C, kernel 10, stride 5, no bias) + GroupNorm(C groups) + GELU into
    a padded frame buffer. Forward: conv0 recomputed from the waveform in the statistics and the
    output pass (csrc/frontend.hip c0gn; neither pass reads conv0's output), which is written
    once for the backward; backward: the fused GroupNorm+GELU backward over it and dW0 contracted
    with the waveform windows (triad_conv0_dw). The waveform gets no gradient."""

    @staticmethod
    def forward(ctx, wave, w, gamma, beta, eps, Tp):
        B, L = wave.shape
        O = w.shape[0]
        T = (L - 10) // 5 + 1
        need = (Tp - 1) * 5 + 10
        xw = F.pad(wave.to(torch.bfloat16), (0, max(0, need - L))).contiguous()
        w0 = w.to(torch.bfloat16).reshape(O, 10).contiguous()
        g = gamma.detach().float().contiguous()
        b = beta.detach().float().contiguous()
        dev = wave.device
        mean = torch.empty(B, O, dtype=torch.float32, device=dev)
        rstd = torch.empty(B, O, dtype=torch.float32, device=dev)
        ws = torch.empty(int(call("triad_chgn_workspace_bytes", B, T, O)), dtype=torch.uint8, device=dev)
        out = torch.empty(B * Tp + 2, O, dtype=torch.bfloat16, device=dev)
        y0 = torch.empty(B * Tp, O, dtype=torch.bfloat16, device=dev)
        out[B * Tp:].zero_()
        call("triad_c0gn_fwd", ptr(xw), xw.shape[1], ptr(w0), B, T, Tp, O, ptr(g), ptr(b), float(eps), ptr(mean),
             ptr(rstd), ptr(ws), ptr(out), ptr(y0), stream_ptr(dev))
        ctx.save_for_backward(xw, y0, g, b, mean, rstd)
        ctx.meta = (B, T, Tp, w.shape, w.dtype, gamma.dtype, beta.dtype)
        return out

    @staticmethod
    def backward(ctx, dout):
        xw, y0, g, b, mean, rstd = ctx.saved_tensors
        B, T, Tp, wshape, wdt, gdt, bdt = ctx.meta
        O = y0.shape[1]
        dev = xw.device
        dy = dout[:B * Tp].to(torch.bfloat16).contiguous()
        ws = torch.empty(int(call("triad_chgn_workspace_bytes", B, T, O)), dtype=torch.uint8, device=dev)
        dy0 = torch.empty_like(y0)
        dg = torch.empty(O, dtype=torch.float32, device=dev)
        db = torch.empty(O, dtype=torch.float32, device=dev)
        call("triad_chgn_gelu_bwd", ptr(y0), ptr(dy), B, T, Tp, O, ptr(g), ptr(b), ptr(mean), ptr(rstd), ptr(ws),
             ptr(dy0), ptr(dg), ptr(db), stream_ptr(dev))
        dw = torch.empty(O, 10, dtype=torch.float32, device=dev)
        ws2 = torch.empty(int(call("triad_conv0_dw_workspace_bytes", B, T, O)), dtype=torch.uint8, device=dev)
        call("triad_conv0_dw", ptr(xw), xw.shape[1], ptr(dy0), B, T, Tp, O, ptr(ws2), ptr(dw), stream_ptr(dev))
        return None, dw.view(wshape).to(wdt), dg.to(gdt), db.to(bdt), None, None


class _FrameConvS2(torch.autograd.Function):
    """Kernel-k (2 or 3), stride-2 conv (C -> O, no bias) between padded frame buffers:
    x [B*Tp + 2, C] -> y [B*Tp/2 + 2, O]."""

    @staticmethod
    def forward(ctx, x, w, B, Tp):
        Cin = x.shape[1]
        O, Cw, k = w.shape
        if Cw != Cin or k not in (2, 3) or Tp % 2 or x.shape[0] != B * Tp + 2:
            raise _lib.TriadError("frame conv: expects a [B*Tp + 2, C] buffer, even Tp, kernel 2 or 3")
        M = B * Tp // 2
        wr = w.to(torch.bfloat16).permute(0, 2, 1).reshape(O, k * Cin).contiguous()
        y = torch.empty(M + 2, O, dtype=torch.bfloat16, device=x.device)
        _gemm_rows(x, 0, 2 * Cin, M, k * Cin, wr, y, 0, O)
        y[M:].zero_()
        ctx.save_for_backward(x, w)
        ctx.meta = (B, Tp, w.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        B, Tp, wdt = ctx.meta
        Cin = x.shape[1]
        O, _, k = w.shape
        M = B * Tp // 2
        dy = dy.to(torch.bfloat16).contiguous()
        wb = w.to(torch.bfloat16)
        wj = [wb[:, :, j] for j in range(k)]  # [O][C] each

        def weight_grad():  # [O][k*C] (column j*C + c) -> contiguous [O][C][k]
            dwr = _weight_grad_rows(dy, M, x, 2 * Cin, k * Cin)
            return dwr.view(O, k, Cin).permute(0, 2, 1).to(wdt).contiguous()

        from .linear import on_side_stream, side_stream_ok
        # bf16 shadow weight: dW on the side stream, queued before (and running beside) the dX GEMMs
        dw = on_side_stream(weight_grad, (dy, x)) if wdt == torch.bfloat16 and side_stream_ok(w) else None
        dx = torch.empty(M + 1, 2 * Cin, dtype=torch.bfloat16, device=x.device)  # = B*Tp + 2 frames
        if k == 3:
            # even frames 2q: dY[q-1] W2 + dY[q] W0 -- rows q = 1..M over overlapping dY rows
            be = torch.cat([wj[2].t(), wj[0].t()], dim=1).contiguous()  # [C][2O]
            _gemm_rows(dy, 0, O, M, 2 * O, be, dx, 1, 2 * Cin)
            dx[0, :Cin] = (dy[0:1] @ wj[0])[0]
            # odd frames 2q+1: dY[q] W1
            _gemm_rows(dy, 0, O, M, O, wj[1].t().contiguous(), dx[:, Cin:], 0, 2 * Cin)
        else:
            bk = torch.cat([wj[0].t(), wj[1].t()], dim=0).contiguous()  # [2C][O]
            _gemm_rows(dy, 0, O, M, O, bk, dx, 0, 2 * Cin)
        dx[M].zero_()  # spare frames: constants
        if dw is None:
            dw = weight_grad()
        return dx.view(2 * M + 2, Cin), dw, None, None


def channel_group_norm_gelu(x, gamma, beta, eps):
    """GroupNorm(C groups, affine) + exact GELU, channels-last bf16 on the HIP device."""
    if not x.is_cuda or x.dtype != torch.bfloat16:
        raise _lib.TriadError("channel_group_norm_gelu runs on a HIP device over bf16 input")
    return _ChannelGroupNormGelu.apply(x, gamma, beta, float(eps))


def _hip_act(act):
    """transformers' exact-erf GELUActivation -> postln.gelu (the same function and roundings as
    one HIP pass each way); any other activation unchanged."""
    from transformers.activations import GELUActivation
    from .postln import gelu
    return gelu if isinstance(act, GELUActivation) and act.act is F.gelu else act


def _frame_stack_plan(self, input_values):
    """[(T, Tp)] of layer 0's output and every later layer's input when HuBERT's layout runs
    over padded frame buffers (every Tp even), else None."""
    layers = self.conv_layers
    if len(layers) < 2 or _compute_dtype(input_values) != torch.bfloat16 or input_values.dim() != 2:
        return None
    c0 = layers[0].conv
    if c0.in_channels != 1 or c0.bias is not None or not isinstance(getattr(layers[0], "layer_norm", None),
                                                                     nn.GroupNorm):
        return None
    T = (input_values.shape[1] - c0.kernel_size[0]) // c0.stride[0] + 1
    Tp = T + (T & 1)
    plan = [(T, Tp)]
    for layer in layers[1:]:
        c = layer.conv
        if c.bias is not None or c.stride[0] != 2 or c.kernel_size[0] not in (2, 3) \
                or getattr(layer, "layer_norm", None) is not None or Tp % 2:
            return None
        T = (T - c.kernel_size[0]) // 2 + 1
        Tp //= 2
        if T <= 0:
            return None
        plan.append((T, Tp))
    return plan


def _hubert_feature_encoder_forward(self, input_values):
    """transformers HubertFeatureEncoder.forward in channels-last GEMM form. Returns the
    (B, C, T) feature map as a transposed view of (B, T, C) storage (HubertModel transposes it
    straight back). The waveform gets no gradient (the reference only marks it for gradient
    checkpointing). HuBERT's own layout (conv0 + GroupNorm, then bias-free stride-2 convs)
    runs over padded frame buffers (_FrameConv0 / _FrameConvS2); any other layout through
    conv1d_gemm."""
    if not input_values.is_cuda:
        return self._triad_hf_forward(input_values)
    plan = _frame_stack_plan(self, input_values)
    if plan is not None:
        B = input_values.shape[0]
        l0 = self.conv_layers[0]
        T, Tp = plan[0]
        norm = l0.layer_norm
        if l0.conv.kernel_size[0] == 10 and l0.conv.stride[0] == 5 and l0.conv.out_channels % 8 == 0 \
                and 256 % (l0.conv.out_channels // 8) == 0:
            h = _Conv0GNGelu.apply(input_values, l0.conv.weight, norm.weight, norm.bias, float(norm.eps), Tp)
        else:
            y = _FrameConv0.apply(input_values, l0.conv.weight, l0.conv.stride[0], Tp)
            h = _ChannelGroupNormGelu.apply(y, norm.weight, norm.bias, float(norm.eps), (B, T, Tp))
        for layer, (T, Tp_out) in zip(self.conv_layers[1:], plan[1:]):
            h = _hip_act(layer.activation)(_FrameConvS2.apply(h, layer.conv.weight, B, Tp))
            Tp = Tp_out
        return h[:B * Tp].view(B, Tp, -1)[:, :T].transpose(1, 2)
    h = input_values.unsqueeze(-1)
    cd = _compute_dtype(h)
    for i, layer in enumerate(self.conv_layers):
        conv = layer.conv
        y = conv1d_gemm(h, conv.weight, conv.bias, conv.stride[0], need_dx=i > 0)
        norm = getattr(layer, "layer_norm", None)
        if isinstance(norm, nn.GroupNorm) and cd == torch.bfloat16:
            h = channel_group_norm_gelu(y, norm.weight, norm.bias, norm.eps)
        elif isinstance(norm, nn.GroupNorm):
            h = layer.activation(F.group_norm(y.transpose(1, 2), norm.num_groups, norm.weight, norm.bias,
                                              norm.eps).transpose(1, 2))
        elif isinstance(norm, nn.LayerNorm):
            h = layer.activation(F.layer_norm(y, norm.normalized_shape, norm.weight, norm.bias, norm.eps))
        else:
            h = layer.activation(y)
    return h.transpose(1, 2)


class _PosConv(torch.autograd.Function):
    """Grouped conv1d(C, C, K=128, padding=pad, groups) over channels-last x (B, T, C), first T
    outputs (HubertSamePadLayer drops the last): forward and input gradient by the implicit-GEMM
    HIP kernel (triad_posconv), weight gradient by triad_posconv_dw (48 channels per group) or the
    overlapping-row GEMM of _posconv_dw_gemm (channels per group dividing 128)."""

    @staticmethod
    def forward(ctx, x, w, bias, groups, pad):
        B, T, C = x.shape
        Co, Cg, K = w.shape
        if Co != C or Cg * groups != C or K != 128:
            raise _lib.TriadError("posconv: expects Conv1d(C, C, 128, groups) weights")
        xb = x.to(torch.bfloat16).contiguous()
        wb = w.to(torch.bfloat16)
        wt = wb.view(groups, Cg, Cg, K).permute(0, 1, 3, 2).reshape(groups, Cg, K * Cg).contiguous()
        bf = None if bias is None else bias.detach().float().contiguous()
        y = torch.empty_like(xb)
        call("triad_posconv", ptr(xb), ptr(wt), ptr(bf), ptr(y), B, T, C, groups, pad, stream_ptr(x.device))
        ctx.save_for_backward(xb, wb)
        ctx.groups, ctx.pad, ctx.has_bias = groups, pad, bias is not None
        ctx.dtypes = (x.dtype, w.dtype, None if bias is None else bias.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, wb = ctx.saved_tensors
        B, T, C = xb.shape
        G, pad = ctx.groups, ctx.pad
        Co, Cg, K = wb.shape
        dyb = dy.to(torch.bfloat16).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wtb = wb.view(G, Cg, Cg, K).flip(-1).permute(0, 2, 3, 1).reshape(G, Cg, K * Cg).contiguous()
            dx = torch.empty_like(dyb)
            call("triad_posconv", ptr(dyb), ptr(wtb), None, ptr(dx), B, T, C, G, K - 1 - pad, stream_ptr(xb.device))
            dx = dx.to(ctx.dtypes[0])
        if ctx.needs_input_grad[1] and C // G == 48:
            # HIP weight gradient: fp32 partials over sample ranges, summed, then [g][j][n][c] -> [g*48+n][c][j]
            splits = max(1, min(B, 16))
            part = torch.empty(int(call("triad_posconv_dw_part_bytes", C, G, splits)) // 4, dtype=torch.float32,
                               device=dyb.device)
            call("triad_posconv_dw", ptr(xb), ptr(dyb), B, T, C, G, pad, splits, ptr(part), stream_ptr(dyb.device))
            cg = C // G
            dsum = torch.empty(part.numel() // splits, dtype=torch.float32, device=dyb.device)
            call("triad_sum_slabs", ptr(part), splits, dsum.numel(), None, 0, ptr(dsum), stream_ptr(dyb.device),
                 meta=dict(backbone=True))
            dw = dsum.view(G, K, cg, cg).permute(0, 2, 3, 1).reshape(C, cg, K)
            dw = dw.to(ctx.dtypes[1])
        elif ctx.needs_input_grad[1] and 128 % (C // G) == 0:
            dw = _posconv_dw_gemm(xb, dyb, G, pad, K).to(ctx.dtypes[1])
        elif ctx.needs_input_grad[1]:
            # the conv's full output has T_full = T + 2*pad - K + 1 steps; the dropped tail gets 0
            t_full = T + 2 * pad - K + 1
            dy_full = torch.zeros(B, t_full, C, dtype=torch.bfloat16, device=dyb.device)
            dy_full[:, :T] = dyb
            x4 = xb.transpose(1, 2).unsqueeze(2)          # (B, C, 1, T), channels-last storage
            dy4 = dy_full.transpose(1, 2).unsqueeze(2)
            dw = torch.ops.aten.convolution_backward(dy4, x4, wb.unsqueeze(2), None, [1, 1], [0, pad], [1, 1],
                                                     False, [0, 0], G, [False, True, False])[1]
            dw = dw.squeeze(2).to(ctx.dtypes[1])
        if ctx.has_bias and ctx.needs_input_grad[2]:
            from .ops import bias_grad
            db = bias_grad(dyb.view(B * T, C), torch.float32).to(ctx.dtypes[2])
        return dx, dw, db, None, None


def _posconv_dw_gemm(xb, dyb, G, pad, K):
    """Weight gradient of the grouped positional conv for CG = C / G dividing 128 (HuBERT-large:
    CG = 64) on the HIP split-K GEMM, no im2col and no MIOpen (whose grouped backward-weight solver
    choice depends on the free device memory it sees -- a multi-minute naive fallback was observed).

    For a block of P = 128 / CG consecutive groups (128 channels), with the padded channels-last
    copies xp[b][tp][c] = x[b][tp - pad][c] (zero outside [0, T), Tp = T + K - 1 rows per sample)
    and dyp[b][t][n] = dy (zero for t >= T):
        dWblk[n][j * 128 + c] = sum_{r = b Tp + t} dyp[r][n] * xp_flat[r * 128 + j * 128 + c]
    i.e. ONE GEMM whose B operand rows OVERLAP (row r = xp_flat[128 r .. 128 r + 128 K), ldb = 128);
    rows t >= T carry dy = 0. dW of group p of the block = dWblk[p CG:(p+1) CG][j, p CG:(p+1) CG]
    (the cross-group blocks are computed and dropped: P-fold work, acceptable for this config)."""
    from ._lib import call, ptr, stream_ptr
    B, T, C = xb.shape
    CG = C // G
    P = 128 // CG
    Tp = T + K - 1
    rows = B * Tp
    Kd = (rows + 63) // 64 * 64
    dev = xb.device
    out = torch.empty(C, CG, K, dtype=torch.float32, device=dev)
    splits = 4
    slabs = torch.empty(splits * 128 * 128 * K, dtype=torch.float32, device=dev)
    blk = torch.empty(128, K * 128, dtype=torch.float32, device=dev)
    st = stream_ptr(dev)
    for c0 in range(0, C, 128):
        xp = torch.zeros(Kd + K, 128, dtype=torch.bfloat16, device=dev)   # + K rows: the last windows
        xp[:rows].view(B, Tp, 128)[:, pad:pad + T] = xb[:, :, c0:c0 + 128]
        dyp = torch.zeros(Kd, 128, dtype=torch.bfloat16, device=dev)
        dyp[:rows].view(B, Tp, 128)[:, :T] = dyb[:, :, c0:c0 + 128]
        call("triad_gemm_bf16_splitk", ptr(dyp), 128, 0, ptr(xp), 128, 0, 128, K * 128, Kd, splits, None,
             ptr(slabs), ptr(blk), 0, st, meta=dict(backbone=True))
        v = blk.view(128, K, 128)
        for q in range(P):
            g0 = c0 + q * CG
            # dW[g0 + n][c][j] = blk[q CG + n][j][q CG + c]
            out[g0:g0 + CG] = v[q * CG:(q + 1) * CG, :, q * CG:(q + 1) * CG].permute(0, 2, 1)
    return out


def _hubert_pos_conv_forward(self, hidden_states):
    """transformers HubertPositionalConvEmbedding.forward (conv -> SamePad -> GELU) on the
    channels-last (B, T, C) hidden state, without the two transposes."""
    conv = self.conv
    if not hidden_states.is_cuda or getattr(self, "batch_norm", None) is not None \
            or _compute_dtype(hidden_states) != torch.bfloat16 or conv.kernel_size[0] != 128 \
            or getattr(self.padding, "num_pad_remove", 1) != 1:
        return self._triad_hf_forward(hidden_states)
    y = _PosConv.apply(hidden_states, conv.weight, conv.bias, conv.groups, conv.padding[0])
    return _hip_act(self.activation)(y)


class _SpecMask(torch.autograd.Function):
    """torch.where(mask[..., None], emb, h) with emb's gradient (the sum of h's gradient over the
    masked frames) taken by ops.bias_grad instead of PyTorch's bf16 reduction, which returned
    disturbed sums beside the concurrent streams' GEMMs."""

    @staticmethod
    def forward(ctx, h, m, emb):
        ctx.save_for_backward(m)
        ctx.emb_dtype = emb.dtype
        return torch.where(m[..., None], emb.to(h.dtype), h)

    @staticmethod
    def backward(ctx, g):
        (m,) = ctx.saved_tensors
        from .ops import bias_grad
        mm = m[..., None]
        gm = torch.where(mm, g, torch.zeros((), dtype=g.dtype, device=g.device))
        demb = bias_grad(gm.reshape(-1, g.shape[-1]).to(torch.bfloat16).contiguous(), torch.float32)
        return torch.where(mm, torch.zeros((), dtype=g.dtype, device=g.device), g), None, demb.to(ctx.emb_dtype)


def _spec_where(m, emb, h):
    if h.dtype == torch.bfloat16 and emb.requires_grad:
        return _SpecMask.apply(h, m, emb)
    return torch.where(m[..., None], emb.to(h.dtype), h)


def _hubert_mask_hidden_states(self, hidden_states, mask_time_indices=None, attention_mask=None):
    """transformers HubertModel._mask_hidden_states (SpecAugment in training) without host syncs:
    the numpy-drawn masks go up through pinned memory and are applied with torch.where instead of
    boolean-mask assignment (which needs a device->host count). Same masks, same values."""
    if not hidden_states.is_cuda:
        return self._triad_hf_mask(hidden_states, mask_time_indices=mask_time_indices, attention_mask=attention_mask)
    from transformers.models.hubert.modeling_hubert import _compute_mask_indices
    cfg = self.config
    if not getattr(cfg, "apply_spec_augment", True):
        return hidden_states
    B, T, C = hidden_states.shape
    dev = hidden_states.device
    if mask_time_indices is not None:
        hidden_states = _spec_where(mask_time_indices.to(dev), self.masked_spec_embed, hidden_states)
    elif cfg.mask_time_prob > 0 and self.training:
        # masked_spec_embed exists only when masking is configured
        m = _compute_mask_indices((B, T), mask_prob=cfg.mask_time_prob, mask_length=cfg.mask_time_length,
                                  attention_mask=attention_mask, min_masks=cfg.mask_time_min_masks)
        m = _lib.h2d(torch.from_numpy(m).to(torch.bool), dev)
        hidden_states = _spec_where(m, self.masked_spec_embed, hidden_states)
    if cfg.mask_feature_prob > 0 and self.training:
        mf = _compute_mask_indices((B, C), mask_prob=cfg.mask_feature_prob, mask_length=cfg.mask_feature_length,
                                   min_masks=cfg.mask_feature_min_masks)
        mf = _lib.h2d(torch.from_numpy(mf).to(torch.bool), dev)
        hidden_states = hidden_states.masked_fill(mf[:, None, :], 0)
    return hidden_states


def install_hubert_frontend(hubert):
    """Route a transformers HubertModel's conv feature encoder through the GEMM form above
    (CUDA tensors only; parameters and state_dict unchanged)."""
    fe = getattr(hubert, "feature_extractor", None)
    if fe is None or not hasattr(fe, "conv_layers"):
        return hubert
    for layer in fe.conv_layers:
        c = layer.conv
        if c.padding[0] != 0 or c.dilation[0] != 1 or c.groups != 1:
            return hubert  # not the HuBERT layout: leave it alone
    if hasattr(hubert, "_mask_hidden_states"):
        hubert._triad_hf_mask = hubert._mask_hidden_states
        hubert._mask_hidden_states = types.MethodType(_hubert_mask_hidden_states, hubert)
    fe._requires_grad = False
    fe._triad_hf_forward = fe.forward
    fe.forward = types.MethodType(_hubert_feature_encoder_forward, fe)
    pce = getattr(getattr(hubert, "encoder", None), "pos_conv_embed", None)
    if pce is not None and isinstance(getattr(pce, "conv", None), nn.Conv1d):
        pce._triad_hf_forward = pce.forward
        pce.forward = types.MethodType(_hubert_pos_conv_forward, pce)
    return hubert


def patch_embed(x, weight, bias, patch):
    """Conv2d(C, dim, kernel=patch, stride=patch) over (B, C, H, W) -> (B, N, dim) tokens in
    row-major patch order (= conv(x).flatten(2).transpose(1, 2)): non-overlapping patches are a
    reshape, so the conv is one GEMM with the weight viewed as (dim, C*patch*patch)."""
    B, C, H, W = x.shape
    gh, gw = H // patch, W // patch
    cd = _compute_dtype(x)
    xc = x[:, :, :gh * patch, :gw * patch].to(cd)
    cols = xc.reshape(B, C, gh, patch, gw, patch).permute(0, 2, 4, 1, 3, 5).reshape(B, gh * gw, C * patch * patch)
    w = weight.reshape(weight.shape[0], -1).to(cd)
    return F.linear(cols, w, None if bias is None else bias.to(cd))
