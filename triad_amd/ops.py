"""Autograd ops over the HIP kernels of libtriad_hip.so.

`contrastive_head` is the fused replacement of the reference's
`compute_all_similarities_{av,tv}` + `compute_contrastive_loss_{av,tv}` pair
(SajayR/TRIAD src/model.py:370-472 and 490-593): it returns the same scalar
losses and statistics without ever materialising the (B, B, Nq, Nk) token
similarity tensor, and its backward produces d/dq, d/dk and d/dtemperature.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import functools
import os

import numpy as np
import torch

from . import _lib
from . import gemm as hipgemm
from ._lib import TriadError, call, ptr, stream_ptr

D = 512
ROWS_PER_WG = 256
AV, TV = 0, 1
CLAMP_LO = {AV: -60.0, TV: -20.0}  # model.py:417 / 524


def _rup(x, m):
    return (x + m - 1) // m * m


def _check_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise TriadError("triad_amd ops run only on a HIP device (MI355X); got a CPU tensor. "
                             "There is no CPU fallback in the product path.")


@dataclass(frozen=True)
class Geometry:
    Bq: int
    Nq: int
    Bk: int
    Nk_eff: int

    @property
    def R(self):
        return self.Bq * self.Nq

    @property
    def R_pad(self):
        return _rup(max(self.R, 1), ROWS_PER_WG)

    @property
    def Nk_pad(self):
        return _rup(self.Nk_eff, 32)

    @property
    def C_pad(self):
        return self.Bk * self.Nk_pad

    @property
    def C_alloc(self):
        return _rup(self.C_pad, 128)


def pack_queries(q: torch.Tensor, g: Geometry) -> torch.Tensor:
    """(Bq, Nq, 512) -> zero-padded [R_pad][512] bf16 (layout of include/triad_hip.h)."""
    out = torch.empty(g.R_pad, D, dtype=torch.bfloat16, device=q.device)
    out[:g.R].copy_(q.reshape(g.R, D))
    if g.R_pad > g.R:
        out[g.R:].zero_()
    return out


def pack_keys(k: torch.Tensor, g: Geometry) -> torch.Tensor:
    """(Bk, Nk_eff, 512) -> [C_alloc][512] bf16, each sample padded to Nk_pad rows."""
    out = torch.empty(g.C_alloc, D, dtype=torch.bfloat16, device=k.device)
    if g.Nk_pad == g.Nk_eff:
        out[:g.C_pad].copy_(k.reshape(g.C_pad, D))
    else:
        v = out[:g.C_pad].view(g.Bk, g.Nk_pad, D)
        v[:, :g.Nk_eff].copy_(k)
        v[:, g.Nk_eff:].zero_()
    if g.C_alloc > g.C_pad:
        out[g.C_pad:].zero_()
    return out


def bias_grad(x, out_dtype=torch.float32, meta=None):
    """Column sums of a bf16 [rows][cols] matrix -- EVERY column sum of the step: the backbone and
    head bias gradients and SpecAugment's masked_spec_embed -- fp32 accumulation, by
    triad_colsum_dma (rows staged into an LDS ring by 16-byte LDS-DMA, VALU sums, a second pass
    over the per-split partials; HBM-bound, 4.8 TB/s at 50,944 x 2,304,
    profiles/r04_colsum_dma_ring.log). Why not a plain-load reduction (triad_colsum, PyTorch's
    sum): with the backbones on concurrent streams, column-sum REDUCTIONS beside the library's MFMA
    + LDS-DMA GEMMs returned disturbed partial sums in some launches (21-38 of 80 concurrent steps
    differing from the serial one), while sums whose rows arrive by LDS-DMA stayed bit-identical
    in every concurrent step (profiles/r04_stream_repeat_*.log). There is no other
    form: a shape the kernel does not take directly (cols % 8, a misaligned or column-strided view)
    is first copied into an aligned buffer padded to 8 columns (zeros), never summed another way.
    meta: launch tag (default: backbone work)."""
    if x.dim() != 2 or x.dtype != torch.bfloat16:
        raise TriadError(f"bias_grad expects a 2-D bf16 matrix, got {tuple(x.shape)} {x.dtype}")
    rows, cols = x.shape
    if rows == 0:
        return torch.zeros(cols, dtype=out_dtype, device=x.device)
    if cols % 8 or x.stride(1) != 1 or x.stride(0) % 8 or x.data_ptr() % 16:
        xp = torch.zeros(rows, _rup(cols, 8), dtype=torch.bfloat16, device=x.device)
        xp[:, :cols].copy_(x)
        return bias_grad(xp, out_dtype, meta)[:cols]
    part = torch.empty(call("triad_colsum_dma_splits", rows, cols) * cols, dtype=torch.float32, device=x.device)
    out = torch.empty(cols, dtype=out_dtype, device=x.device)
    call("triad_colsum_dma", ptr(x), rows, cols, x.stride(0), ptr(part), 1.0, int(out_dtype == torch.bfloat16),
         ptr(out), stream_ptr(x.device), meta=meta if meta is not None else dict(backbone=True))
    return out


def pack_b(B, nkt, dk, stream):
    """B [nkt*32][512] bf16 -> its v_mfma_f32_16x16x32_bf16 fragments in the direct-B GEMM's order
    (triad_bfrag_pack16): one pass over B, after which each wave of the GEMM streams its own columns
    into registers."""
    Bp = torch.empty(nkt * 32 * D, dtype=torch.bfloat16, device=B.device)
    call("triad_bfrag_pack16", ptr(B), nkt, dk, ptr(Bp), stream,
         meta=dict(tag="bfrag-pack", flops=0.0))
    return Bp


def tile_gemm(dS, CT, dk, B, M, nkt, alpha, out, stream, meta=None, Bp=None):
    """dQ = alpha dS K (dk=0) / dK = alpha dS^T Q (dk=1) over the tiled dS, split-K over the CUs
    when the row panels alone leave them idle. (A stream-K form -- one run of (row panel, k tile)
    units per CU, no slab round trip -- measured slower: runs start at different k offsets, so CUs
    of one XCD no longer share the streamed B panel in L2.) The direct-B form over pack_b's
    fragments on 16x16x32 MFMAs (triad_tile_gemm_packed16; the LDS-ring triad_tile_gemm is its
    parity reference): 9-12 % faster for dQ and 3-5 % for dK than the 32x32x16 direct-B form it
    replaced (profiles/r04_bwd_micro_mfma16.log), which was 6-7 % faster than the ring
    (profiles/r03_tile_gemm_db_ab.log); Bp: B already packed by pack_b."""
    sp = _gemm_splits(M // 128, nkt, M)
    slabs = torch.empty(sp * M * D, dtype=torch.float32, device=out.device) if sp > 1 else None
    if Bp is None:
        Bp = pack_b(B, nkt, dk, stream)
    call("triad_tile_gemm_packed16", ptr(dS), CT, dk, ptr(Bp), M, nkt,
         ptr(alpha), sp, ptr(slabs), ptr(out), stream, meta=meta)


def tile_gemm_slabs(dS, CT, dk, Bp, M, nkt, splits, slabs, stream, meta=None):
    """Unscaled fp32 split-K partial sums only (the recompute backward's per-chunk dQ), over pack_b's
    fragments."""
    call("triad_tile_gemm_packed16_slabs", ptr(dS), CT, dk,
         ptr(Bp), M, nkt, splits, ptr(slabs), stream, meta=meta)




def _gemm_splits(wgs, nkt, M, cus=256, max_splits=8, t_tile=1.0e-6, hbm=5.0e12):
    """Split-K factor of the tile GEMM minimising (dispatch rounds of one workgroup per CU) x
    (k tiles per workgroup) x t_tile + the fp32 slab round trip (write + reduce read of
    splits x M x 512 x 4 B). The slab term matters when the k loop is short: TV dK (448 row
    panels, 256 k tiles) ran 0.76 ms with 4 splits, of which ~0.38 ms was the 0.94 GB slab round
    trip (profiles/r02_bench.json); with the slab term it takes 1 split (0.48 ms), AV dQ 3 instead
    of 5 (2.98-3.01 vs 3.20 ms), AV dK stays at 4 (profiles/r02_tile_splits_ab.log)."""
    best, best_c = 1, None
    for sp in range(1, max_splits + 1):
        if sp > nkt:
            break
        rounds = -(-(wgs * sp) // cus)
        c = rounds * -(-nkt // sp) * t_tile + (sp * M * D * 8 / hbm if sp > 1 else 0.0)
        if best_c is None or c < best_c * 0.98:
            best, best_c = sp, c
    return best


DS_BUDGET_BYTES = None


def _default_budget(dev) -> int:
    if DS_BUDGET_BYTES is not None:
        return int(DS_BUDGET_BYTES)
    total = torch.cuda.get_device_properties(dev).total_memory
    return min(64 << 30, total // 4)


def ds_bytes(g: Geometry) -> int:
    """Bytes of the tiled bf16 dS of a head geometry ([R_pad/32][CT][1024])."""
    return (g.R_pad // 32) * _rup(g.C_pad // 32, 4) * 2048


def ds_chunk_samples(g: Geometry, budget: int) -> int:
    """Key samples per chunk of the memory-bounded backward: all of them when the whole dS fits
    the budget, else the largest multiple of 4 whose dS chunk PLUS the recompute path's fp32 dQ
    partial slabs (nchunks x splits x R_pad x 512 x 4 B) fit (at least 4)."""
    if ds_bytes(g) <= budget:
        return g.Bk
    return max(4, _fit_chunk(g, budget))


def _fit_chunk(g: Geometry, budget: int) -> int:
    for chunk in range(g.Bk // 4 * 4, 3, -4):
        if ds_working_bytes(g, chunk) <= budget:
            return chunk
    return 4


def ds_working_bytes(g: Geometry, chunk: int) -> int:
    """Device bytes the head's backward working set holds for dS at `chunk` key samples per chunk:
    the whole tiled dS (chunk == Bk, materialised by the forward), or one chunk's dS plus the
    recompute path's dQ slabs."""
    if chunk >= g.Bk:
        return ds_bytes(g)
    nkb = g.Nk_pad // 32
    per = (g.R_pad // 32) * _rup(chunk * nkb, 4) * 2048
    nchunks = -(-g.Bk // chunk)
    splits = _gemm_splits(g.R_pad // 128, chunk * nkb, g.R_pad)
    return per + nchunks * splits * g.R_pad * D * 4


def recompute_backward(g: Geometry, Qb, Kb, temp, kind, diag_off, argmax, dclip, qw, gdiag, coef, need_q, need_k,
                       chunk, stream, ds_buf=None):
    """dQ / dK / dL-dtemp partials WITHOUT a forward-written dS: per chunk of `chunk` key samples,
    triad_pairsim_dS recomputes S for those keys and writes that chunk's full dS (clamp + max +
    diagonal terms, weighted by coef), dK rows of those keys come from one tile GEMM (complete:
    a key's gradient only involves its own dS columns), and dQ accumulates the chunks' fp32 partial
    sums (tile_gemm_slabs), reduced once at the end. Peak dS memory = one chunk.
    Returns (dQ [R_pad][512] bf16 | None, dK [CT*32][512] bf16 | None, dt_part fp64)."""
    dev = Qb.device
    nkb = g.Nk_pad // 32
    CT = _rup(g.C_pad // 32, 4)
    nchunks = -(-g.Bk // chunk)
    CT_c = _rup(chunk * nkb, 4)
    n_ds = (g.R_pad // 32) * CT_c * 1024
    dS = ds_buf if ds_buf is not None and ds_buf.numel() >= n_ds else \
        torch.empty(n_ds, dtype=torch.bfloat16, device=dev)
    dQ = dK = slabs = None
    splits = 1
    if need_q:
        if nchunks == 1:
            dQ = torch.empty(g.R_pad, D, dtype=torch.bfloat16, device=dev)
        else:
            splits = _gemm_splits(g.R_pad // 128, chunk * nkb, g.R_pad)
            slabs = torch.empty(nchunks * splits, g.R_pad, D, dtype=torch.float32, device=dev)
    Qp = None
    if need_k:
        dK = torch.empty(CT * 32, D, dtype=torch.bfloat16, device=dev)
        Qp = pack_b(Qb, g.R_pad // 32, 1, stream)   # once, for every chunk's dK
    parts = []
    for c in range(nchunks):
        j0 = c * chunk
        nc = min(chunk, g.Bk - j0)
        gc = Geometry(g.Bq, g.Nq, nc, g.Nk_eff)
        ctc = _rup(nc * nkb, 4)
        Kc = Kb[j0 * g.Nk_pad:]
        dclip_c = dclip[:, j0:j0 + nc].contiguous() if nchunks > 1 else dclip
        dt_c = torch.empty(call("triad_pairsim_nparts", g.R_pad, nc), dtype=torch.float64, device=dev)
        call("triad_pairsim_dS", ptr(Qb), ptr(Kc), g.R, g.R_pad, g.Nq, g.Bq, nc, g.Nk_pad, g.Nk_eff, D,
             ptr(temp), CLAMP_LO[kind], 1, diag_off - j0, ptr(argmax[j0:]), ptr(dclip_c), ptr(qw), ptr(gdiag),
             ptr(coef), ptr(dS), ctc, ptr(dt_c), stream,
             meta=dict(kind=kind, flops=0.0, recompute_flops=2.0 * g.R * nc * g.Nk_eff * D))
        parts.append(dt_c)
        fl = 2.0 * g.R * nc * g.Nk_eff * D
        if need_q:
            if nchunks == 1:
                tile_gemm(dS, ctc, 0, Kc, g.R_pad, nc * nkb, temp, dQ, stream,
                          meta=dict(kind=kind, flops=fl, what="dQ"))
            else:
                Kp = pack_b(Kc, nc * nkb, 0, stream)
                tile_gemm_slabs(dS, ctc, 0, Kp, g.R_pad, nc * nkb, splits, slabs[c * splits], stream,
                                meta=dict(kind=kind, flops=fl, what="dQ"))
        if need_k:
            tile_gemm(dS, ctc, 1, Qb, ctc * 32, g.R_pad // 32, temp, dK[j0 * g.Nk_pad:], stream,
                      meta=dict(kind=kind, flops=fl, what="dK"), Bp=Qp)
    if need_q and nchunks > 1:
        dQ = torch.empty(g.R_pad, D, dtype=torch.bfloat16, device=dev)
        call("triad_sum_slabs", ptr(slabs), nchunks * splits, g.R_pad * D, ptr(temp), 1, ptr(dQ), stream)
    return dQ, dK, torch.cat(parts) if len(parts) > 1 else parts[0]


class _Head:
    """Per-head state of one forward (geometry, packed operands, outputs of the similarity
    forward) shared by the single-head and the fused AV+TV autograd functions."""
    pass


def _head_begin(q, k, temperature, kind, q_mask, group, ds_budget, need_grad):
    """Checks, operand packing (keys all-gathered in global mode) and the buffers of the
    similarity forward of one head."""
    _check_device(q, k, temperature, q_mask)
    Bq, Nq, dq = q.shape
    Bl, Nk, dk = k.shape
    if dq != D or dk != D:
        raise TriadError(f"feature dim must be {D}")
    if Bq != Bl:
        raise TriadError("query and key batches must match")
    W, rank = (1, 0)
    if group is not None:
        from . import dist as tdist
        W, rank = tdist.world_rank(group)
    Bg = Bq * W
    if Bg < 2:
        # the reference takes max() of the empty off-diagonal set and raises (model.py:447/565)
        raise TriadError("batch size must be >= 2 (no negatives for B == 1)")
    h = _Head()
    h.kind, h.group, h.W, h.rank, h.Nk, h.Bg = kind, group, W, rank, Nk, Bg
    h.g = g = Geometry(Bq, Nq, Bg, Nk)
    dev = q.device
    h.Qb = pack_queries(q, g)
    if W == 1:
        h.Kb = pack_keys(k, g)
    else:
        gl = Geometry(Bq, Nq, Bq, Nk)
        h.Kb = tdist.gather_keys(pack_keys(k, gl)[:gl.C_pad], g.C_alloc, group)
    h.temp = temperature.detach().reshape(1).to(torch.float32).contiguous()
    h.nparts = call("triad_pairsim_nparts", g.R_pad, g.Bk)
    h.rowmax = torch.empty(g.Bk, g.R_pad, dtype=torch.float32, device=dev)
    h.argmax = torch.empty(g.Bk, g.R_pad, dtype=torch.int32, device=dev)
    h.nn_part = torch.empty(h.nparts, dtype=torch.float64, device=dev)
    h.diagS = torch.empty(g.Bq, g.Nq, g.Nk_pad, dtype=torch.float32, device=dev)
    h.CT = _rup(g.C_pad // 32, 4)
    budget = _default_budget(dev) if ds_budget is None else int(ds_budget)
    h.chunk = ds_chunk_samples(g, budget)
    # materialise the unit dS in the forward only when it fits the budget; otherwise the
    # backward recomputes it chunk by chunk (recompute_backward)
    write_ds = need_grad and h.chunk == g.Bk
    h.dS = torch.empty((g.R_pad // 32) * h.CT * 1024, dtype=torch.bfloat16, device=dev) if write_ds else None
    h.st_part = torch.empty(h.nparts, dtype=torch.float64, device=dev) if write_ds else None
    h.q_dtype, h.k_dtype, h.t_dtype = q.dtype, k.dtype, temperature.dtype
    # kept keys per sample when k comes straight from patch_dropout (zero rows after them; host
    # int32): the pair forward may then leave out each sample's all-zero last key tile (_compact)
    kc = getattr(k, KEPT_ROWS_ATTR, None) if W == 1 and ZERO_TILE_SKIP else None
    h.kept = kc if (isinstance(kc, torch.Tensor) and kc.device.type == "cpu" and tuple(kc.shape) == (g.Bk,)) else None
    h.Kc = h.ktiles = h.kmap = None
    h.nct = g.C_pad // 32   # stored key tiles (all of them unless _compact)
    return h


@functools.lru_cache(maxsize=64)
def _fwd_keys_per_workgroup(R_pad, Bk):
    """Key samples per forward workgroup: pairsim.hip grid_for's choice (the decomposition
    triad_pairsim_nparts reports), restated so the host knows when compact key tiles apply."""
    xb = R_pad // ROWS_PER_WG
    best, ys = 1e30, 1
    for y in range(1, Bk + 1):
        j = -(-Bk // y)
        ya = -(-Bk // j)
        c = ((xb * ya + 255) // 256) * (j + 0.3)
        if c < best - 1e-9:
            best, ys = c, ya
    jpw = -(-Bk // ys)
    assert xb * (-(-Bk // jpw)) == call("triad_pairsim_nparts", R_pad, Bk)
    return jpw


_STAGE = [None] * 16   # (persistent pinned int32 buffer, event after its last copy), round robin
_STAGE_NEXT = [0]


def _stage_h2d(arr, dev):
    """int32 numpy array -> device tensor (async) through a ring of persistent pinned slots (grow-only,
    allocated once per slot: no per-call trip through the caching host allocator, which may
    synchronise); a slot is refilled only after the event recorded behind its previous copy has
    completed, so a copy the stream has not run yet never reads a refilled buffer."""
    a = np.ascontiguousarray(arr, dtype=np.int32).reshape(-1)
    i = _STAGE_NEXT[0]
    _STAGE_NEXT[0] = (i + 1) % len(_STAGE)
    prev = _STAGE[i]
    if prev is not None:
        prev[1].synchronize()
    buf = prev[0] if prev is not None and prev[0].numel() >= a.size else \
        torch.empty(max(4096, 1 << (max(1, a.size) - 1).bit_length()), dtype=torch.int32, pin_memory=True)
    buf.numpy()[:a.size] = a
    out = buf[:a.size].to(dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    _STAGE[i] = (buf, ev)
    return out


def compact_tables(kept, nkb, Nk):
    """Host tables of the compact key-tile layout (see _compact) for per-sample kept counts:
    cb (Bk + 1 int32, triad_pairsim_problem.k_tiles: sample j's stored tiles are cb[j] ..
    cb[j + 1] - 1), tidx (int64, the padded tile index j nkb + kb of each stored tile, in order) and
    kmap ([Bk][Nk] int32: the compact key row of key (j, k), -1 in a left-out tile). None when no
    sample leaves its last tile out."""
    kept = np.asarray(kept)
    tiles = np.where(kept <= 32 * (nkb - 1), nkb - 1, nkb).astype(np.int64)
    if (tiles == nkb).all():
        return None
    Bk = kept.shape[0]
    cb = np.zeros(Bk + 1, dtype=np.int32)
    cb[1:] = np.cumsum(tiles)
    nct = int(cb[-1])
    tidx = (np.repeat(np.arange(Bk) * nkb - cb[:-1], tiles) + np.arange(nct)).astype(np.int64)
    # dK row of each (sample, key < Nk) in the stored layout, -1 in a left-out tile (zero gradient)
    key = np.arange(Nk)[None, :]
    kmap = np.where(key < 32 * tiles[:, None], 32 * cb[:-1, None].astype(np.int64) + key, -1).astype(np.int32)
    return cb, tidx, kmap


def _compact(h):
    """Compact key tiles for a training head whose keys come from patch_dropout: every sample
    whose kept keys all lie before its last 32-key tile leaves that all-zero tile out of K and of
    the tiled dS (triad_pairsim_problem.k_tiles); the forward applies its S == 0 in closed form,
    dQ / dK / the dS patch run over the stored tiles only and dK's rows go back to the padded layout
    (zeros for the left-out keys: their gradient is padding, model.py:301-302). Skipped when the
    forward's workgroups hold more than 64 key samples (its per-workgroup skip mask) or nothing is
    left out."""
    g = h.g
    nkb = g.Nk_pad // 32
    if h.kept is None or h.dS is None or nkb < 2 or _fwd_keys_per_workgroup(g.R_pad, g.Bk) > 64:
        return
    tabs = compact_tables(h.kept.numpy(), nkb, h.Nk)
    if tabs is None:
        return
    cb, tidx, kmap = tabs
    nct = int(cb[-1])
    dev = h.Kb.device
    # the three tables in ONE host-to-device copy from a staging slot held until the copy has run
    nb = g.Bk + 1
    tables = _stage_h2d(np.concatenate([cb, kmap.reshape(-1), tidx.astype(np.int32)]), dev)
    h.ktiles = tables[:nb]
    h.kmap = tables[nb:nb + kmap.size].view(1, -1)
    h.nct = nct
    kc = torch.empty(_rup(nct * 32, 128), D, dtype=torch.bfloat16, device=dev)
    torch.index_select(h.Kb[:g.C_pad].view(g.Bk * nkb, 32 * D), 0, tables[nb + kmap.size:],
                       out=kc[:nct * 32].view(nct, 32 * D))
    kc[nct * 32:].zero_()
    h.Kc = kc
    h.CT = _rup(nct, 4)
    h.dS = torch.empty((g.R_pad // 32) * h.CT * 1024, dtype=torch.bfloat16, device=dev)
    if h.CT > nct:   # dK's last row panel reads the tail tiles: zeros, not stale memory
        h.dS.view(g.R_pad // 32, h.CT, 1024)[:, nct:].zero_()


def _fwd_meta(h):
    g = h.g
    return dict(kind=h.kind, flops=2.0 * g.R * g.Bk * g.Nk_eff * D, grid=h.nparts * 512,
                # algorithmic bytes: the feature operands + rowmax / argmax; the
                # tiled unit-dS stream the training forward also writes is NOT algorithmic
                # (bench.py reports it, from PMC, as traffic): 2 KB per stored 32 x 32 tile, i.e.
                # over the compacted key tiles when _compact left some out (h.nct of them)
                bytes=2.0 * D * (g.R + g.Bk * g.Nk_eff) + 8.0 * g.Bk * g.R,
                ds_bytes=(2048.0 * (g.R_pad // 32) * h.nct if h.dS is not None else 0.0))


def _head_launch(h, st):
    g = h.g
    call("triad_pairsim_fwd", ptr(h.Qb), ptr(h.Kb), g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, D,
         ptr(h.temp), CLAMP_LO[h.kind], 1, h.rank * g.Bq, ptr(h.rowmax), ptr(h.argmax), ptr(h.nn_part),
         ptr(h.diagS), ptr(h.dS), h.CT, ptr(h.st_part), None, st, meta=_fwd_meta(h))


def _problem(h, padded_keys=False):
    """The head's forward problem; padded_keys: with the full padded K and no k_tiles (the
    diagonal-S launch, triad_pairsim_diag)."""
    g = h.g
    compact = h.Kc is not None and not padded_keys
    return _lib.PairsimProblem(ptr(h.Qb), ptr(h.Kc if compact else h.Kb), g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad,
                               g.Nk_eff, ptr(h.temp), CLAMP_LO[h.kind], 1, h.rank * g.Bq, ptr(h.rowmax),
                               ptr(h.argmax), ptr(h.nn_part), ptr(h.diagS), ptr(h.dS), h.CT, ptr(h.st_part),
                               ptr(h.ktiles) if compact else None)


def _heads_launch(hs, st):
    """Every head's similarity forward in ONE launch (triad_pairsim_fwd_multi), then the heads'
    diagonal S blocks (triad_pairsim_diag over the padded keys) -- issued apart so the bench's live
    timing of the forward launch covers that kernel alone. (Round 6 built the diagonal S into the
    training forward's epilogue: the forward took 0.10 ms longer than the 0.125 ms kernel it saved,
    same box alternated, profiles/r06_diag_in_fwd_ab.log; not kept.)"""
    arr = (_lib.PairsimProblem * len(hs))(*[_problem(h, padded_keys=True) for h in hs])
    fwd = (_lib.PairsimProblem * len(hs))(*[_problem(h) for h in hs])
    for p in fwd:
        p.diag = 0
    ms = [_fwd_meta(h) for h in hs]
    meta = dict(kind=-1, what="+".join("AV" if h.kind == AV else "TV" for h in hs),
                flops=sum(m["flops"] for m in ms), bytes=sum(m["bytes"] for m in ms),
                ds_bytes=sum(m["ds_bytes"] for m in ms), grid=sum(h.nparts for h in hs) * 512)
    call("triad_pairsim_fwd_multi", fwd, len(hs), st, meta=meta)
    call("triad_pairsim_diag", arr, len(hs), st)


def _head_end(h, q_mask, thr, w_sparse, st):
    """Clip reduction, diagonal regularisers and the loss head after the similarity forward.
    Returns (losses[4], stats, clip_full); keeps what the backward needs on h."""
    g, kind, W, rank, Bg = h.g, h.kind, h.W, h.rank, h.Bg
    dev = h.Qb.device
    clip = torch.empty(g.Bq, g.Bk, dtype=torch.float32, device=dev)
    h.qw = torch.empty(g.R, dtype=torch.float32, device=dev)
    qm = None if q_mask is None else q_mask.to(torch.float32).contiguous()
    call("triad_clip_reduce", ptr(h.rowmax), g.R_pad, g.Nq, g.Bq, g.Bk, ptr(qm), ptr(clip), ptr(h.qw), st)
    dg_part = torch.empty(g.Bq, dtype=torch.float64, device=dev)
    h.dgt_part = torch.empty(g.Bq, dtype=torch.float64, device=dev)
    h.gdiag = torch.empty_like(h.diagS)
    if kind == AV:
        cnt = float(Bg * (g.Nq - 1) * g.Nk_eff)
        call("triad_diag_smooth", ptr(h.diagS), g.Bq, g.Nq, g.Nk_pad, g.Nk_eff, cnt, ptr(dg_part), ptr(h.gdiag),
             ptr(h.dgt_part), st)
    else:
        cnt = float(Bg * g.Nk_eff)
        call("triad_diag_sparsity", ptr(h.diagS), g.Bq, g.Nq, g.Nk_pad, g.Nk_eff, float(thr), cnt,
             ptr(dg_part), ptr(h.gdiag), ptr(h.dgt_part), st)
    h.n_el = float(Bg) * Bg * g.Nq * g.Nk_eff
    h.w_sparse = float(w_sparse)
    if W == 1:
        clip_full, nn_in, n_nn, dg_in, n_dg = clip, h.nn_part, h.nparts, dg_part, g.Bq
    else:
        from . import dist as tdist
        clip_full = tdist.gather_rows(clip, h.group)
        sums = tdist.allreduce_sum(torch.stack([h.nn_part.sum(), dg_part.sum()]), h.group)
        nn_in, n_nn, dg_in, n_dg = sums[0:1], 1, sums[1:2], 1
    out = torch.empty(13, dtype=torch.float32, device=dev)
    dclip = torch.empty(Bg, Bg, dtype=torch.float32, device=dev)
    lse = torch.empty(2 * Bg, dtype=torch.float32, device=dev)
    call("triad_losshead", ptr(clip_full), Bg, kind, ptr(h.temp), ptr(nn_in), n_nn, h.n_el, ptr(dg_in), n_dg,
         cnt, float(w_sparse), ptr(out), ptr(dclip), ptr(lse), st)
    h.dclip = dclip[rank * g.Bq:(rank + 1) * g.Bq].contiguous() if W > 1 else dclip
    return out[:4].clone(), out[4:].clone(), clip_full


_SAVED = ("Qb", "Kb", "argmax", "rowmax", "dclip", "qw", "gdiag", "temp", "dS", "st_part", "dgt_part", "Kc", "ktiles",
          "kmap")


def _head_saved(h):
    return [getattr(h, n) for n in _SAVED]


def _head_light(h):
    """h without its tensors (those travel through ctx.save_for_backward)."""
    c = _Head()
    for n in ("g", "kind", "W", "rank", "Nk", "n_el", "w_sparse", "nparts", "CT", "chunk", "group", "q_dtype",
              "k_dtype", "t_dtype", "nct"):
        setattr(c, n, getattr(h, n))
    return c


def _head_backward(h, saved, needs, g_total, g_ce, g_reg, g_aux):
    """(gq, gk, gt) of one head; needs = (q, k, temperature) input-gradient flags."""
    if g_total is None and g_ce is None and g_reg is None and g_aux is None:
        return None, None, None
    Qb, Kb, argmax, rowmax, dclip, qw, gdiag, temp, dS, st_part, dgt_part, Kc, ktiles, kmap = saved
    g, kind, W, rank, CT = h.g, h.kind, h.W, h.rank, h.CT
    dev = Qb.device
    st = stream_ptr(dev)
    f32 = torch.float32
    zero = torch.zeros((), dtype=f32, device=dev)
    gt_, gc_, gr_, ga_ = [zero if x is None else x.to(f32) for x in (g_total, g_ce, g_reg, g_aux)]
    c_ce = gt_ + gc_
    c_reg = gt_ + gr_
    c_nn = c_reg * (0.15 * 2.0 / h.n_el)
    if kind == AV:
        c_diag = 0.01 * (c_reg + ga_)   # reg = ... + 0.01*l_smooth; aux = 0.01*l_smooth
        c_cal = 20.0 * c_reg
    else:
        c_diag = h.w_sparse * c_reg + ga_  # reg = ... + w*sparsity; aux = sparsity
        c_cal = torch.zeros_like(c_reg)
    has_cal = 1 if (kind == AV and rank == 0) else 0   # the l_cal term is counted once
    fast = g_total is not None and g_ce is None and g_reg is None and g_aux is None and dS is not None
    gq = gk = gt = None
    if fast:
        # dS = c_nn * (unit l_nonneg grad [written by the forward] + ratio_max * max term
        #               + ratio_diag * diagonal term); the ratios are host constants here. The
        # forward stores the unit gradient divided by su = |temp| (1 at temp == 0), the patch adds
        # its terms divided by su (reading temp on the device) and alpha carries su.
        ratio_max = h.n_el / 0.3
        ratio_diag = (0.01 if kind == AV else h.w_sparse) * h.n_el / 0.3
        nmp = 1024
        max_part = torch.empty(nmp, dtype=torch.float64, device=dev)
        call("triad_dS_patch_tiles", ptr(dS), CT, g.R, g.R_pad, g.Nq, g.Bq, g.Bk, g.Nk_pad, g.Nk_eff, rank * g.Bq,
             ptr(argmax), ptr(rowmax), ptr(dclip), ptr(qw), float(ratio_max), ptr(gdiag), float(ratio_diag),
             ptr(max_part), nmp, ptr(temp), ptr(ktiles), st)
        su = torch.where(temp != 0, temp.abs(), torch.ones_like(temp))
        alpha = (temp * c_nn * su).reshape(1).contiguous()
        w = torch.stack([c_nn, c_ce / temp[0], c_diag / temp[0], c_cal]).contiguous()
        parts = (st_part, h.nparts, max_part, nmp, dgt_part, g.Bq)
    else:
        # recompute form: any mix of upstream gradients, or a dS over the memory budget
        coef = torch.stack([c_ce, c_nn, c_diag, c_cal]).contiguous()
        dQ, dK, dt_part = recompute_backward(g, Qb, Kb, temp, kind, rank * g.Bq, argmax, dclip, qw, gdiag, coef,
                                             needs[0], needs[1], h.chunk, st, ds_buf=dS)
        w = torch.stack([torch.ones_like(c_ce), zero, zero, c_cal]).contiguous()
        parts = (dt_part, dt_part.numel(), None, 0, None, 0)
        if dQ is not None:
            gq = dQ[:g.R].view(g.Bq, g.Nq, D).to(h.q_dtype)
    if fast and needs[0]:
        dQ = torch.empty(g.R_pad, D, dtype=torch.bfloat16, device=dev)
        tile_gemm(dS, CT, 0, Kb if Kc is None else Kc, g.R_pad, h.nct, alpha, dQ, st,
                  meta=dict(kind=kind, flops=2.0 * g.R * g.Bk * g.Nk_eff * D, what="dQ"))
        gq = dQ[:g.R].view(g.Bq, g.Nq, D).to(h.q_dtype)
    if needs[1]:
        if fast:
            Mk = CT * 32
            dK = torch.empty(Mk, D, dtype=torch.bfloat16, device=dev)
            tile_gemm(dS, CT, 1, Qb, Mk, g.R_pad // 32, alpha, dK, st,
                      meta=dict(kind=kind, flops=2.0 * g.R * g.Bk * g.Nk_eff * D, what="dK"))
        Nk_pad = g.Nk_pad
        if W > 1:
            from . import dist as tdist
            dK = tdist.reduce_scatter_rows(dK, g.Bq * Nk_pad, h.group)  # this rank's keys, all queries
        if fast and kmap is not None:   # stored key tiles -> (B, Nk, 512) in one gather (left-out keys: zero)
            gk = gather_rows(dK.view(1, Mk, D), kmap).view(g.Bq, h.Nk, D).to(h.k_dtype)
        else:
            gk = dK[:g.Bq * Nk_pad].view(g.Bq, Nk_pad, D)[:, :h.Nk].to(h.k_dtype)
    if needs[2]:
        dt = torch.empty(1, dtype=f32, device=dev)
        p0, n0, p1, n1, p2, n2 = parts
        call("triad_dtemp_finalize", ptr(p0), n0, ptr(p1), n1, ptr(p2), n2, ptr(temp), ptr(w), has_cal,
             ptr(dt), st)
        gt = dt.reshape(()).to(h.t_dtype)
    return gq, gk, gt


class _ContrastiveHead(torch.autograd.Function):
    """Outputs: total, contrastive, reg, aux (0.01*l_smooth for AV, sparsity for TV), stats[9], clip.

    group=None: local head (the reference loss over this process's batch).
    group=<process group>: global negatives (SURVEY §8e Mode G, triad_amd.dist): keys are
    all-gathered, this rank computes its query rows of the B_g x B_g clip matrix, and the
    loss head runs on the gathered clip on every rank (identical loss = reference at B_g).

    Backward: when only `total` is differentiated (every training step) the forward has
    already written the unit l_nonneg gradient into the tiled dS buffer, so the backward
    only patches in the max / diagonal terms and runs the two GEMMs (no recompute of S).
    Any other mix of upstream gradients recomputes dS (triad_pairsim_dS).
    """

    @staticmethod
    def forward(ctx, q, k, temperature, kind, q_mask, thr, w_sparse, group, ds_budget):
        need_grad = any(ctx.needs_input_grad[:3])  # (forward itself runs under no_grad)
        h = _head_begin(q, k, temperature, kind, q_mask, group, ds_budget, need_grad)
        st = stream_ptr(q.device)
        _head_launch(h, st)
        losses, stats, clip_full = _head_end(h, q_mask, thr, w_sparse, st)
        if need_grad:
            ctx.save_for_backward(*_head_saved(h))
        ctx.head = _head_light(h)
        ctx.mark_non_differentiable(stats, clip_full)
        ctx.set_materialize_grads(False)
        return losses[0], losses[1], losses[2], losses[3], stats, clip_full

    @staticmethod
    def backward(ctx, g_total, g_ce, g_reg, g_aux, g_stats, g_clip):
        if g_total is None and g_ce is None and g_reg is None and g_aux is None:
            return (None,) * 9
        gq, gk, gt = _head_backward(ctx.head, ctx.saved_tensors, ctx.needs_input_grad[:3], g_total, g_ce, g_reg,
                                    g_aux)
        return gq, gk, gt, None, None, None, None, None, None


class _ContrastiveHeadPair(torch.autograd.Function):
    """The tri-modal step's AV and TV heads with ONE similarity-forward launch over both
    (triad_pairsim_fwd_multi; BASELINE c3's fused similarity kernel over the pair losses -- the
    reference has no audio-text loss). Everything else per head exactly as _ContrastiveHead;
    the shared temperature's gradient is the sum of the two heads'.
    Outputs: AV (total, ce, reg, aux, stats, clip) then TV (the same six)."""

    @staticmethod
    def forward(ctx, qa, ka, qt, kt, temperature, qt_mask, thr, w_sparse, group, ds_budget):
        nig = ctx.needs_input_grad
        need_grad = any(nig[:5])
        # ONE dS budget for the pair: AV takes what it needs of it, TV what AV leaves (at least
        # its minimum chunk) -- not a full budget each
        budget = _default_budget(qa.device) if ds_budget is None else int(ds_budget)
        ha = _head_begin(qa, ka, temperature, AV, None, group, budget, need_grad)
        used = ds_working_bytes(ha.g, ha.chunk) if need_grad else 0
        ht = _head_begin(qt, kt, temperature, TV, qt_mask, group, max(0, budget - used), need_grad)
        st = stream_ptr(qa.device)
        if ha.dS is not None and ht.dS is not None:   # one training launch: compact key tiles apply
            _compact(ha)
            _compact(ht)
        if (ha.dS is None) == (ht.dS is None):
            _heads_launch([ha, ht], st)
        else:  # one head over the dS budget: the multi launch needs one mode for both
            _head_launch(ha, st)
            _head_launch(ht, st)
        la, sa, ca = _head_end(ha, None, 0.0, 0.0, st)
        lt, stt, ct = _head_end(ht, qt_mask, thr, w_sparse, st)
        if need_grad:
            ctx.save_for_backward(*_head_saved(ha), *_head_saved(ht))
        ctx.heads = (_head_light(ha), _head_light(ht))
        ctx.mark_non_differentiable(sa, ca, stt, ct)
        ctx.set_materialize_grads(False)
        return la[0], la[1], la[2], la[3], sa, ca, lt[0], lt[1], lt[2], lt[3], stt, ct

    @staticmethod
    def backward(ctx, a_total, a_ce, a_reg, a_aux, _sa, _ca, t_total, t_ce, t_reg, t_aux, _st, _ct):
        nig = ctx.needs_input_grad
        saved = ctx.saved_tensors
        n = len(_SAVED)
        ha, ht = ctx.heads
        gqa, gka, gta = _head_backward(ha, saved[:n], (nig[0], nig[1], nig[4]), a_total, a_ce, a_reg, a_aux)
        gqt, gkt, gtt = _head_backward(ht, saved[n:], (nig[2], nig[3], nig[4]), t_total, t_ce, t_reg, t_aux)
        gt = gta if gtt is None else (gtt if gta is None else gta + gtt)
        return gqa, gka, gqt, gkt, gt, None, None, None, None, None


def contrastive_head(kind, q, k, temperature, q_mask=None, threshold=0.0, sparsity_weight=0.0, group=None,
                     ds_budget=None):
    """Fused similarity + aggregation + InfoNCE + regularisers.

    kind AV: q = audio feats (B,Na,512), k = visual feats (B,Nv,512) (model.py:470-472)
    kind TV: q = text feats (B,Nt,512) with q_mask (B,Nt), k = visual feats (model.py:593)
    group: process group for global negatives (every rank must pass k with the same Nv).
    Returns (losses, stats[9], clip[B_g,B_g]); losses = (total, contrastive, reg, aux) 0-dim tensors.
    In global mode the gradients w.r.t. q, k, temperature are this rank's share of the
    full-loss gradient: sum them over ranks (the trainer's Mode-G all-reduce does).
    ds_budget: bytes of tiled dS the training forward may materialise (default: a quarter of the
    device's HBM, at most 64 GiB); above it the backward recomputes S in key-sample chunks of at
    most that size (recompute_backward). The c4 per-rank shape (256 x 2048 samples) needs 47 GB.
    """
    total, ce, reg, aux, stats, clip = _ContrastiveHead.apply(q, k, temperature, kind, q_mask, threshold,
                                                              sparsity_weight, group, ds_budget)
    return (total, ce, reg, aux), stats, clip


def contrastive_heads_av_tv(audio, visual_av, text, visual_tv, temperature, text_mask, threshold=0.0,
                            sparsity_weight=0.0, group=None, ds_budget=None):
    """Both heads of the tri-modal step with one similarity-forward launch: equal to
    contrastive_head(AV, audio, visual_av, ...) and contrastive_head(TV, text, visual_tv, ...).
    Returns ((losses, stats, clip) of AV, (losses, stats, clip) of TV)."""
    o = _ContrastiveHeadPair.apply(audio, visual_av, text, visual_tv, temperature, text_mask, threshold,
                                   sparsity_weight, group, ds_budget)
    return ((o[0], o[1], o[2], o[3]), o[4], o[5]), ((o[6], o[7], o[8], o[9]), o[10], o[11])


def gather_rows(src: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """out[b][t] = src[b][idx[b][t]] (idx -1 -> zero row); src (B, N, D) contiguous."""
    _check_device(src, idx)
    B, N = src.shape[0], src.shape[1]
    M = idx.shape[1]
    row_bytes = src[0, 0].numel() * src.element_size()
    out = torch.empty((B, M) + tuple(src.shape[2:]), dtype=src.dtype, device=src.device)
    # keep the (possibly temporary) operands referenced across the launch: a temporary freed
    # while the argument list is built could hand its block to the next temporary
    srcc = src.contiguous()
    idxc = idx.to(torch.int32).contiguous()
    call("triad_gather_rows", ptr(srcc), N, ptr(idxc), B, M, row_bytes, ptr(out), stream_ptr(src.device))
    return out


def l2_normalize(x: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """F.normalize(x, dim=-1) for bf16 rows (model.py:363-364)."""
    _check_device(x)
    xc = x.to(torch.bfloat16).contiguous()
    y = torch.empty_like(xc)
    rows = xc.numel() // xc.shape[-1]
    call("triad_l2norm_rows", ptr(xc), rows, xc.shape[-1], eps, ptr(y), stream_ptr(x.device))
    return y


def l2_normalize_f32(x: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """F.normalize(x, dim=-1) in fp32 (the reference's fp32 retrieval embeddings, retrieval.py:93-94)."""
    _check_device(x)
    xc = x.to(torch.float32).contiguous()
    y = torch.empty_like(xc)
    rows = xc.numel() // xc.shape[-1]
    call("triad_l2norm_rows_f32", ptr(xc), rows, xc.shape[-1], eps, ptr(y), stream_ptr(x.device))
    return y


# ----------------------------------------------------------------------------------------
# Projection head: proj2(LN(proj1(h))) (model.py:32-34,68 / 81-83,116 / 253-255,326)
# ----------------------------------------------------------------------------------------
def _pad_rows(x: torch.Tensor, rows: int) -> torch.Tensor:
    if x.shape[0] == rows:
        return x.contiguous()
    out = torch.empty((rows,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    out[:x.shape[0]].copy_(x)
    out[x.shape[0]:].zero_()
    return out


def _splitk(Kd, mn_tiles):
    """Split-K factor of the projection-head weight gradients (128 x 128 tiles): one round of
    workgroups over the 256 CUs, >= 512 token rows per split (so the 8,192-row text head also
    fills the chip: 16 x 16 workgroups for dW2). Measured (round-2 A/B,
    profiles/r02_dw_proj_forms.log): fewer, longer splits beat two rounds once the slab
    reduction is counted -- dW2 at 65,536 rows 66 us (16 splits) vs 78 us (32), dW1 86 vs 96 us;
    the 256 x 256 four-wave form is no faster at its best split."""
    want = max(1, 256 // mn_tiles)
    return max(1, min(want, Kd // 512))


def _dw_plan(Mp, N):
    """(form, splits) of a projection-head weight gradient [512][N] over Mp token rows. Long
    token lists: 32 splits with each split's workgroups on one XCD (gemm.hip tile_split, form
    flag 8) -- 128 x 128 tiles for dW2 (N = 512), the eight-wave 256 x 256 tile for dW1 (N = 768):
    visual 65,536 rows dW2 65.9 -> 54.6 us, dW1 86.4 -> 74.2; audio 50,944 rows dW2 56.1 -> 44.9,
    dW1 69.1 -> 63.6 (GEMM + slab reduction, profiles/r04_dw_xcd_ab.log; bit-identical to the
    default placement at equal form / splits). Short lists (the 8,192-row text head) keep _splitk's
    one round of 128 x 128 workgroups (faster there). The 256 x 256 tile's split count fills the
    256 CUs with whole XCD groups: (256 // tiles) rounded down to a multiple of 8 -- 40 splits x 6
    tiles = 240 workgroups for the 768-wide dW1 (32 left 64 CUs idle), 32 x 8 for 1,024 wide."""
    if Mp >= 32768 and N % 256 == 0:
        if N == D:
            return 1 | 8, 32
        tiles = (D // 256) * (N // 256)
        return 4 | 8, max(8, int(os.environ.get("TRIAD_DW1_SPLITS", (256 // tiles) // 8 * 8)))
    return 0, _splitk(Mp, (D // 128) * (N // 128))


def _rows_view(h):
    """(tensor, M, H, lda, n_per, bstride) addressing h's token rows in place when h is a bf16
    [..., N, H] tensor whose rows are contiguous within each leading index (e.g. the ViT's patch
    tokens sliced behind its CLS / register tokens); otherwise a contiguous bf16 copy."""
    H = h.shape[-1]
    if h.dtype == torch.bfloat16 and h.dim() >= 2 and h.stride(-1) == 1 and h.data_ptr() % 16 == 0:
        N = h.shape[-2]
        lead = h.shape[:-2]
        lda = h.stride(-2)
        if lda % 8 == 0 and lda >= H:
            if len(lead) == 0:
                return h, N, H, lda, max(N, 1), 0
            if len(lead) == 1 and h.stride(0) % 8 == 0:
                return h, lead[0] * N, H, lda, N, h.stride(0)
    hb = h.to(torch.bfloat16).reshape(-1, H).contiguous()
    return hb, hb.shape[0], H, H, hb.shape[0], 0


def _head_weight_grads(w_refs, dyp, ln, dy1, hb, M, Mp, H, w1d, w2d):
    """(dW2, dW1) of a projection head: dW2 = dy^T ln, dW1 = dy1^T h on the split-K GEMM
    (_dw_plan), bf16 straight from the slab reduction for bf16 model weights. On the head's own
    stream by default; with TRIAD_HEAD_DW_SIDE=1 bf16 weights at their first use in the backward pass
    go to the backbone weight-gradient side stream (linear.on_side_stream) -- measured no faster, and
    there they share the CUs of the audio backbone's backward GEMMs (HEAD_DW_SIDE_STREAM below)."""
    from . import linear as _lin

    def run():
        st = stream_ptr(dyp.device)
        bf, f32 = torch.bfloat16, torch.float32
        (f2, sp2), (f1, sp1) = _dw_plan(Mp, D), _dw_plan(Mp, H)
        slabs = torch.empty(max(sp2 * D * D, sp1 * D * H), dtype=f32, device=dyp.device)
        o2, o1 = int(w2d == bf), int(w1d == bf)
        dw2 = torch.empty(D, D, dtype=bf if o2 else f32, device=dyp.device)
        call("triad_gemm_bf16_splitk_form", ptr(dyp), D, 0, ptr(ln), D, 0, D, D, Mp, sp2, None, ptr(slabs), ptr(dw2),
             o2, f2, st, meta=dict(tag=f"proj-dW2x{M}", flops=2.0 * M * D * D))
        dw1 = torch.empty(D, H, dtype=bf if o1 else f32, device=dyp.device)
        call("triad_gemm_bf16_splitk_form", ptr(dy1), D, 0, ptr(hb), H, 0, D, H, Mp, sp1, None, ptr(slabs), ptr(dw1),
             o1, f1, st, meta=dict(tag=f"proj-dW1x{M}", flops=2.0 * M * D * H))
        return dw2, dw1

    if dyp.is_cuda and HEAD_DW_SIDE_STREAM and _lin.side_stream_ok(*w_refs):
        return _lin.on_side_stream(run, (dyp, ln, dy1, hb))
    return run()


# The projection heads' weight gradients run in order on the head's own stream (default) or on the
# backbone dW side stream (TRIAD_HEAD_DW_SIDE=1, round 5's form). Same box, alternated, bench step
# (profiles/r06_head_dw_side_ab.log): throughput equal (1938.7 / 1936.8 side vs 1940.7 / 1936.7 own
# stream), the heads' summed launch time 2.72-2.76 -> 2.33-2.35 ms per step: on the side stream the
# visual / audio dW launches ran 40-52 us alone but 132-153 us (median) overlapped 75-81 % of their
# time by HuBERT's backward GEMMs on the audio stream (profiles/r06_head_dw_trace_side_stream.txt,
# tools/head_dw_trace.py) -- they shared CUs rather than filling idle ones.
HEAD_DW_SIDE_STREAM = os.environ.get("TRIAD_HEAD_DW_SIDE", "0") == "1"


class _ProjectionHeadRows(torch.autograd.Function):
    """The projection head on row-panel GEMMs (rowgemm.hip): a workgroup owns 128 token rows x all
    512 columns, so the forward is ONE kernel (triad_projhead_fwd: projection1, the LayerNorm in its
    epilogue -- y1, row mean / rstd, ln -- and projection2 from the LN'd panel kept in LDS) and the
    LayerNorm backward runs in the epilogue of projection2's input-gradient GEMM
    (triad_projhead_ln_bwd: dy1 and the dgamma / dbeta / db1 column partials); dh is the tiled GEMM,
    the weight gradients the split-K GEMM. Numerics as autocast: bf16 GEMM outputs with the bias added before the one
    rounding, the LayerNorm and its backward in fp32 over the bf16 y1 / dln."""

    @staticmethod
    def forward(ctx, h, w1, b1, gamma, beta, w2, b2, eps):
        _check_device(h, w1)
        H = h.shape[-1]
        if w1.shape != (D, H) or w2.shape != (D, D):
            raise TriadError("projection head expects Linear(H->512), Linear(512->512)")
        dev = h.device
        st = stream_ptr(dev)
        bf = torch.bfloat16
        lead = h.shape[:-1]
        hv, M, _, lda, n_per, bstride = _rows_view(h)
        P = call("triad_rowpanel_count", M)
        Mp = P * 128
        w1b = w1.detach().to(bf).contiguous()
        w2b = w2.detach().to(bf).contiguous()
        b1b, b2b = b1.detach().to(bf).contiguous(), b2.detach().to(bf).contiguous()   # as autocast adds them
        g32 = gamma.detach().to(torch.float32).contiguous()
        be32 = beta.detach().to(torch.float32).contiguous()
        w1p = torch.empty(H * D, dtype=bf, device=dev)
        w2p = torch.empty(D * D, dtype=bf, device=dev)
        call("triad_wpack2", ptr(w1b), H, ptr(w1p), ptr(w2b), D, ptr(w2p), st, meta=dict(tag="proj-wpack", flops=0.0))
        y1 = torch.empty(Mp, D, dtype=bf, device=dev)
        ln = torch.empty(Mp, D, dtype=bf, device=dev)
        mean = torch.empty(Mp, dtype=torch.float32, device=dev)
        rstd = torch.empty(Mp, dtype=torch.float32, device=dev)
        y = torch.empty(Mp, D, dtype=bf, device=dev)
        # the whole forward in one kernel: GEMM1 + LayerNorm epilogue, the LN'd panel kept in LDS as
        # projection2's A operand (tagged as the two GEMMs' flops together)
        call("triad_projhead_fwd", ptr(hv), M, H, lda, n_per, bstride, ptr(w1p), ptr(b1b), ptr(g32), ptr(be32),
             float(eps), ptr(w2p), ptr(b2b), ptr(y1), ptr(ln), ptr(mean), ptr(rstd), ptr(y), st,
             meta=dict(tag=f"proj-fwdx{M}", flops=2.0 * M * D * (H + D)))
        ctx.save_for_backward(h if hv is h else hv, w1b, w2b, g32, y1, ln, mean, rstd)
        ctx.shape = (lead, H, M, Mp, hv is h)
        ctx.dtypes = (h.dtype, w1.dtype, b1.dtype, gamma.dtype, beta.dtype, w2.dtype, b2.dtype)
        ctx.w_refs = (w1, w2)
        return y[:M].view(*lead, D)

    @staticmethod
    def backward(ctx, dy):
        hs, w1b, w2b, g32, y1, ln, mean, rstd = ctx.saved_tensors
        lead, H, M, Mp, in_place = ctx.shape
        dev = dy.device
        st = stream_ptr(dev)
        f32, bf = torch.float32, torch.bfloat16
        hd, w1d, b1d, gd, bd, w2d, b2d = ctx.dtypes
        dyp = _pad_rows(dy.reshape(M, D).to(bf), Mp)
        w2p = pack_b(w2b, D // 32, 1, st)     # Bt = W2: dln = dy W2
        P = Mp // 128
        dy1 = torch.empty(Mp, D, dtype=bf, device=dev)
        part = torch.empty(P, 3, D, dtype=f32, device=dev)
        call("triad_projhead_ln_bwd", ptr(dyp), M, ptr(w2p), ptr(y1), ptr(mean), ptr(rstd), ptr(g32), ptr(dy1),
             ptr(part), st, meta=dict(tag=f"proj-dX2x{M}", flops=2.0 * M * D * D))
        cols = torch.empty(3, D, dtype=f32, device=dev)
        call("triad_sum_slabs", ptr(part), P, 3 * D, None, 0, ptr(cols), st, meta=dict(tag="proj-cols", flops=0.0))
        dh = hipgemm.mm(dy1, w1b, meta=dict(tag=f"proj-dX1x{M}", flops=2.0 * M * D * H))[:M]
        db2 = bias_grad(dyp, bf if b2d == bf else f32, meta=dict(tag="proj-bias", flops=0.0))
        hb = _pad_rows(hs.to(bf).reshape(M, H), Mp) if in_place or Mp > M else hs
        dw2, dw1 = _head_weight_grads(ctx.w_refs, dyp, ln, dy1, hb, M, Mp, H, w1d, w2d)
        return (dh.view(*lead, H).to(hd), dw1.to(w1d), cols[2].to(b1d), cols[0].to(gd), cols[1].to(bd), dw2.to(w2d),
                db2.to(b2d), None)


class _ProjectionHeadPasses(torch.autograd.Function):
    """The projection head as autocast runs it (model.py:68/116/326), as separate passes:
    projection1 / projection2 and their input gradients on the tiled HIP GEMM (gemm.py:
    256 x 256 / 256 x 128 forms, bias in the epilogue before the one bf16 rounding -- F.linear
    under autocast), the LayerNorm and its backward as single HIP row passes (triad_ln_fwd /
    triad_ln_bwd3, dgamma / dbeta / db1 column partials in the same pass), the weight gradients on
    the split-K HIP GEMM (2-4x hipBLASLt on these contraction-over-tokens shapes,
    profiles/r02_projhead_kernels.log)."""

    @staticmethod
    def forward(ctx, h, w1, b1, gamma, beta, w2, b2, eps):
        _check_device(h, w1)
        lead, H = h.shape[:-1], h.shape[-1]
        M = h.numel() // H
        if w1.shape != (D, H) or w2.shape != (D, D):
            raise TriadError("projection head expects Linear(H->512), Linear(512->512)")
        dev = h.device
        st = stream_ptr(dev)
        Mp = _rup(max(M, 1), 128)
        bf = torch.bfloat16
        hb = _pad_rows(h.to(bf).reshape(M, H), Mp)
        w1b = w1.detach().to(bf).contiguous()
        w2b = w2.detach().to(bf).contiguous()
        b1b, b2b = b1.detach().to(bf), b2.detach().to(bf)
        g32 = gamma.detach().to(torch.float32).contiguous()
        be32 = beta.detach().to(torch.float32).contiguous()
        fl1, fl2 = 2.0 * M * H * D, 2.0 * M * D * D
        y1 = hipgemm.linear(hb, w1b, b1b, meta=dict(tag=f"proj-fwd1x{M}", flops=fl1))
        ln = torch.empty(Mp, D, dtype=bf, device=dev)
        mean = torch.empty(Mp, dtype=torch.float32, device=dev)
        rstd = torch.empty(Mp, dtype=torch.float32, device=dev)
        call("triad_ln_fwd", ptr(y1), Mp, ptr(g32), ptr(be32), float(eps), ptr(ln), ptr(mean), ptr(rstd), st,
             meta=dict(tag=f"proj-ln{M}", flops=0.0))
        y = hipgemm.linear(ln, w2b, b2b, meta=dict(tag=f"proj-fwd2x{M}", flops=fl2))[:M]
        ctx.save_for_backward(hb, w1b, w2b, g32, y1, ln, mean, rstd)
        ctx.shape = (lead, H, M, Mp)
        ctx.dtypes = (h.dtype, w1.dtype, b1.dtype, gamma.dtype, beta.dtype, w2.dtype, b2.dtype)
        ctx.w_refs = (w1, w2)
        return y.view(*lead, D)

    @staticmethod
    def backward(ctx, dy):
        hb, w1b, w2b, g32, y1, ln, mean, rstd = ctx.saved_tensors
        lead, H, M, Mp = ctx.shape
        dev = dy.device
        st = stream_ptr(dev)
        f32 = torch.float32
        dyp = _pad_rows(dy.reshape(M, D).to(torch.bfloat16), Mp)
        dln = hipgemm.mm(dyp, w2b, meta=dict(tag=f"proj-dX2x{M}", flops=2.0 * M * D * D))
        dy1 = torch.empty(Mp, D, dtype=torch.bfloat16, device=dev)
        if Mp > M:
            dy1[M:].zero_()
        nb = max(1, min(1024, (M + 3) // 4))
        part = torch.empty(nb, 3, D, dtype=f32, device=dev)
        call("triad_ln_bwd3", ptr(dln), ptr(y1), ptr(mean), ptr(rstd), ptr(g32), M, ptr(dy1), ptr(part), nb, st,
             meta=dict(tag=f"proj-lnbwd{M}", flops=0.0))
        cols = torch.empty(3, D, dtype=f32, device=dev)
        call("triad_sum_slabs", ptr(part), nb, 3 * D, None, 0, ptr(cols), st, meta=dict(tag="proj-cols", flops=0.0))
        dh = hipgemm.mm(dy1, w1b, meta=dict(tag=f"proj-dX1x{M}", flops=2.0 * M * D * H))[:M]
        hd, w1d, b1d, gd, bd, w2d, b2d = ctx.dtypes
        # bf16 model weights (the trainer's shadowed Linear parameters): the gradients come out in
        # bf16 straight from the reductions, as autocast's bf16 GEMM / bias gradients do
        # (by LDS-DMA like every column sum of the step: the audio / text heads' backward runs on
        # the concurrent backbone streams)
        db2 = bias_grad(dyp, torch.bfloat16 if b2d == torch.bfloat16 else f32, meta=dict(tag="proj-bias", flops=0.0))
        dw2, dw1 = _head_weight_grads(ctx.w_refs, dyp, ln, dy1, hb, M, Mp, H, w1d, w2d)
        return (dh.view(*lead, H).to(hd), dw1.to(w1d), cols[2].to(b1d), cols[0].to(gd), cols[1].to(bd), dw2.to(w2d),
                db2.to(b2d), None)


# Forms: "rows" (row-panel GEMMs with the LayerNorm and its backward in the GEMM epilogues,
# _ProjectionHeadRows) and "passes" (tiled GEMMs + LayerNorm row passes, _ProjectionHeadPasses).
PROJHEAD_FORM = os.environ.get("TRIAD_PROJHEAD_FORM", "passes")


def projection_head(h, proj1: torch.nn.Linear, layer_norm: torch.nn.LayerNorm, proj2: torch.nn.Linear, form=None):
    """HIP projection head; returns bf16 (B, N, 512) like the autocast reference (model.py:68/116/326)."""
    fn = {"passes": _ProjectionHeadPasses, "rows": _ProjectionHeadRows}[form or PROJHEAD_FORM]
    return fn.apply(h, proj1.weight, proj1.bias, layer_norm.weight, layer_norm.bias, proj2.weight,
                    proj2.bias, layer_norm.eps)


# ----------------------------------------------------------------------------------------
# HuBERT processor normalisation (model.py:56-62) on the device
# ----------------------------------------------------------------------------------------
def global_znorm(x: torch.Tensor, eps: float = 1e-7) -> torch.Tensor:
    _check_device(x)
    xf = x.to(torch.float32).contiguous()
    y = torch.empty_like(xf)
    nb = int(max(1, min(1024, xf.numel() // 4096)))
    part = torch.empty(2 * nb, dtype=torch.float64, device=x.device)
    call("triad_global_znorm", ptr(xf), xf.numel(), float(eps), ptr(y), ptr(part), nb, stream_ptr(x.device))
    return y


# ----------------------------------------------------------------------------------------
# Patch dropout compaction (model.py:268-308)
# ----------------------------------------------------------------------------------------
class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx, inv_idx):
        ctx.save_for_backward(inv_idx)
        return gather_rows(x, idx)

    @staticmethod
    def backward(ctx, g):
        (inv_idx,) = ctx.saved_tensors
        return gather_rows(g.contiguous(), inv_idx), None, None


def dropout_indices(keep_mask: torch.Tensor, n_out: Optional[int] = None):
    """Host-side compaction plan from a (B, N) keep mask: idx[b][t] = t-th kept token of
    sample b (-1 pads to the longest kept length, or to n_out), inv[b][n] = its slot or -1."""
    keep = keep_mask.detach().to("cpu", torch.bool)
    B, N = keep.shape
    counts = keep.sum(1)
    if n_out is None:
        n_out = int(counts.max()) if B else 0
    elif B and int(counts.max()) > n_out:
        raise TriadError("n_out is shorter than the longest kept sample")
    pos = torch.cumsum(keep.to(torch.int32), dim=1) - 1
    inv = torch.where(keep, pos, torch.full_like(pos, -1)).to(torch.int32)
    idx = torch.full((B, max(n_out, 1)), -1, dtype=torch.int32)
    b_ix, n_ix = keep.nonzero(as_tuple=True)
    idx[b_ix, pos[b_ix, n_ix].long()] = n_ix.to(torch.int32)
    return idx[:, :n_out], inv, n_out


# attribute of patch_dropout's output: its kept-row count per sample (host int32); rows after it
# are zero, which the pair forward exploits (_compact); a copy or view of the tensor does not
# carry it
KEPT_ROWS_ATTR = "_triad_kept_rows"
# TRIAD_ZERO_TILE_SKIP=0: store and multiply the all-zero key tiles too (A/B)
ZERO_TILE_SKIP = os.environ.get("TRIAD_ZERO_TILE_SKIP", "1") != "0"


def patch_dropout(x: torch.Tensor, keep_mask: torch.Tensor, n_out: Optional[int] = None) -> torch.Tensor:
    """(B, N, D) -> (B, max_b kept_b, D): kept tokens in order, zero padded (model.py:282-307).
    n_out overrides the padded length (global negatives pad to the global maximum).
    keep_mask is a HOST (B, N) bool tensor: the padded length and the compaction plan are host
    values, so a device mask would cost a device->host synchronisation every step; it is refused
    rather than silently synchronised (the model draws its masks on the host, draw_keep_mask)."""
    _check_device(x)
    if keep_mask.is_cuda:
        raise TriadError("patch_dropout: keep_mask must be a host tensor (the compaction plan is built on the "
                         "host; a device mask would synchronise the device every step) -- pass keep_mask.cpu()")
    idx, inv, n_out = dropout_indices(keep_mask, n_out)
    idx_d = _lib.h2d(idx.contiguous(), x.device)
    inv_d = _lib.h2d(inv.contiguous(), x.device)
    out = _GatherRows.apply(x.contiguous(), idx_d, inv_d)
    setattr(out, KEPT_ROWS_ATTR, keep_mask.detach().to(torch.bool).sum(1).to(torch.int32))
    return out


# ----------------------------------------------------------------------------------------
# Inference similarity maps (model.py:355-368) and the materialising debug path
# ----------------------------------------------------------------------------------------
def similarity_maps(f1: torch.Tensor, f2: torch.Tensor, temperature: torch.Tensor) -> torch.Tensor:
    """normalize(f1) . normalize(f2)^T * temperature per sample, (B,N1,N2) fp32 (inference,
    model.py:355-368): ONE launch over all B samples, the L2 normalisation in its prologue and the
    temperature in its epilogue (triad_similarity_maps)."""
    _check_device(f1, f2)
    if f1.dim() == 2:
        f1 = f1.unsqueeze(0)
    if f2.dim() == 2:
        f2 = f2.unsqueeze(0)
    if f1.shape[0] != f2.shape[0] or f1.shape[-1] != f2.shape[-1]:
        raise TriadError(f"similarity_maps: {tuple(f1.shape)} vs {tuple(f2.shape)}")
    B, N1, Dd = f1.shape
    N2 = f2.shape[1]
    a = f1.to(torch.bfloat16).contiguous()
    b = f2.to(torch.bfloat16).contiguous()
    if _rup(Dd, 32) > 512:
        raise TriadError(f"similarity_maps: feature width {Dd} > 512 (the kernel's LDS tiles)")
    if Dd % 32:   # zero-padded features (norms and dots unchanged)
        a = torch.nn.functional.pad(a, (0, _rup(Dd, 32) - Dd))
        b = torch.nn.functional.pad(b, (0, _rup(Dd, 32) - Dd))
    t = temperature.detach().reshape(1).to(torch.float32).contiguous()
    out = torch.empty(B, N1, N2, dtype=torch.float32, device=f1.device)
    call("triad_similarity_maps", ptr(a), ptr(b), B, N1, N2, a.shape[-1], ptr(t), 1e-12, ptr(out),
         stream_ptr(f1.device), meta=dict(tag="simmap", flops=2.0 * B * N1 * N2 * Dd))
    return out
