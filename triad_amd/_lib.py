"""ctypes binding of libtriad_hip.so (the C ABI declared in include/triad_hip.h).

The product path has exactly one implementation: the HIP kernels in this
library. If the library is missing or the process has no HIP device, every op
raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.join(_HERE, "libtriad_hip.so")
# A/B experiments only: load a variant build of the same library (tools/build_variants.py);
# the default is the in-tree build above, which must match the sources (see load())
LIB_PATH = os.environ.get("TRIAD_LIB_VARIANT", DEFAULT_LIB)

vp, i32, u32, i64, f32, f64 = C.c_void_p, C.c_int, C.c_uint, C.c_longlong, C.c_float, C.c_double

# name -> argtypes (restype is always int status). Keep in sync with include/triad_hip.h.
SIGNATURES = {
    "triad_pairsim_nparts": [i32, i32],
    "triad_pairsim_fwd": [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, f32, i32, i32, vp, vp, vp, vp, vp,
                          i64, vp, vp, vp],
    "triad_pairsim_fwd_multi": [vp, i32, vp],
    "triad_pairsim_diag": [vp, i32, vp],
    "triad_clip_reduce": [vp, i32, i32, i32, i32, vp, vp, vp, vp],
    "triad_diag_smooth": [vp, i32, i32, i32, i32, f64, vp, vp, vp, vp],
    "triad_diag_sparsity": [vp, i32, i32, i32, i32, f32, f64, vp, vp, vp, vp],
    "triad_losshead": [vp, i32, i32, vp, vp, i32, f64, vp, i32, f64, f32, vp, vp, vp, vp],
    "triad_pairsim_dS": [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, f32, i32, i32, vp, vp, vp, vp, vp,
                         vp, i64, vp, vp],
    "triad_dS_patch": [vp, i64, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, f32, vp, f32, vp, i32, vp,
                       vp],
    "triad_dS_patch_tiles": [vp, i64, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, f32, vp, f32, vp, i32,
                             vp, vp, vp],
    "triad_dtemp_finalize": [vp, i32, vp, i32, vp, i32, vp, vp, i32, vp, vp],
    "triad_tile_gemm": [vp, i64, i32, vp, i32, i32, vp, i32, vp, vp, vp],
    "triad_tile_gemm_slabs": [vp, i64, i32, vp, i32, i32, i32, vp, vp],
    "triad_bfrag_pack16": [vp, i32, i32, vp, vp],
    "triad_tile_gemm_packed16": [vp, i64, i32, vp, i32, i32, vp, i32, vp, vp, vp],
    "triad_tile_gemm_packed16_slabs": [vp, i64, i32, vp, i32, i32, i32, vp, vp],
    "triad_gemm_bf16": [vp, i64, i32, vp, i64, i32, i32, i32, i32, vp, vp, i64, i32, vp],
    "triad_gemm_bf16_bias": [vp, i64, i32, vp, i64, i32, i32, i32, i32, vp, vp, i64, vp],
    "triad_gemm_bf16_bias_bf16": [vp, i64, i32, vp, i64, i32, i32, i32, i32, vp, vp, i64, vp],
    "triad_gemm_bf16_splitk": [vp, i64, i32, vp, i64, i32, i32, i32, i32, i32, vp, vp, vp, i32, vp],
    "triad_gemm_bf16_splitk_form": [vp, i64, i32, vp, i64, i32, i32, i32, i32, i32, vp, vp, vp, i32, i32, vp],
    "triad_wpack": [vp, i32, vp, vp],
    "triad_wpack2": [vp, i32, vp, vp, i32, vp, vp],
    "triad_projhead_fwd": [vp, i64, i32, i64, i64, i64, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp, vp],
    "triad_similarity_maps": [vp, vp, i32, i32, i32, i32, vp, f32, vp, vp],
    "triad_rowpanel_count": [i64],
    "triad_projhead_ln_fwd": [vp, i64, i32, i64, i64, i64, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp],
    "triad_rowgemm_bias": [vp, i64, i32, i64, vp, vp, vp, vp],
    "triad_projhead_ln_bwd": [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp],
    "triad_ln_fwd": [vp, i32, vp, vp, f32, vp, vp, vp, vp],
    "triad_ln_bwd3": [vp, vp, vp, vp, vp, i32, vp, vp, i32, vp],
    "triad_sum_slabs": [vp, i32, i64, vp, i32, vp, vp],
    "triad_colsum_splits": [i64, i32],
    "triad_colsum": [vp, i64, i32, i64, vp, f32, i32, vp, vp],
    "triad_colsum_dma_splits": [i64, i32],
    "triad_colsum_dma": [vp, i64, i32, i64, vp, f32, i32, vp, vp],
    "triad_global_znorm": [vp, i64, f32, vp, vp, i32, vp],
    "triad_grad_sumsq": [vp, vp, i32, vp, vp],
    "triad_adamw_step": [vp, vp, vp, vp, vp, i32, vp, vp, f32, f32, f32, f32, f32, vp, vp],
    "triad_gather_grads": [vp, i32, vp, i32, vp],
    "triad_gather_rows": [vp, i64, vp, i32, i32, i32, vp, vp],
    "triad_l2norm_rows": [vp, i32, i32, f32, vp, vp],
    "triad_l2norm_rows_f32": [vp, i32, i32, f32, vp, vp],
    "triad_retrieval_maxmean_f32": [vp, vp, i32, i32, vp, vp, i32, i32, i32, f32, vp, vp],
    "triad_chgn_workspace_bytes": [i32, i32, i32],
    "triad_chgn_gelu_fwd": [vp, i32, i32, i32, i32, vp, vp, f32, vp, vp, vp, vp, vp],
    "triad_chgn_gelu_bwd": [vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "triad_gemm_bf16_form": [vp, i64, i32, vp, i64, i32, i32, i32, i32, vp, vp, i64, i32, i32, vp],
    "triad_conv0_dw_workspace_bytes": [i32, i32, i32],
    "triad_conv0_dw": [vp, i64, vp, i32, i32, i32, i32, vp, vp, vp],
    "triad_c0gn_fwd": [vp, i64, vp, i32, i32, i32, i32, vp, vp, f32, vp, vp, vp, vp, vp, vp],
    "triad_posconv": [vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
    "triad_posconv_dw_part_bytes": [i32, i32, i32],
    "triad_posconv_dw": [vp, vp, i32, i32, i32, i32, i32, i32, vp, vp],
    "triad_rows_nt": [vp, i64, i32, i32, vp, i32, vp, vp],
    "triad_lora_update": [vp, i64, i32, i32, vp, vp, vp],
    "triad_dropaddln_fwd": [vp, vp, vp, vp, f32, i32, i32, f32, u32, vp, vp, vp, vp, vp],
    "triad_dropaddln_bwd_blocks": [i32],
    "triad_dropaddln_bwd": [vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, u32, vp, vp, vp, vp],
    "triad_gelu_table_bytes": [],
    "triad_gelu_table": [vp, vp],
    "triad_geludrop_fwd": [vp, i64, f32, u32, vp, vp, vp],
    "triad_geludrop_bwd": [vp, vp, i64, f32, u32, vp, vp, vp],
    "triad_dropout_keep": [i64, f32, u32, vp, vp],
    "triad_addln_fwd": [vp, vp, vp, vp, vp, f32, i32, i32, vp, vp, i32, vp, vp, vp],
    "triad_addln_bwd": [vp, i32, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp, vp],
    "triad_lora_tn_blocks": [i32],
    "triad_lora_tn": [vp, i64, i32, i32, vp, vp, vp, f32, vp, vp, vp],
    "triad_attn_dropmask": [i32, i32, i32, f32, u32, vp, vp, vp],
    "triad_attn_fwd_dropout": [vp, i64, i64, vp, i64, i64, vp, i64, i64, i32, i32, i32, i32, f32, vp, f32, vp, i64,
                               i64, vp, vp],
    "triad_attn_bwd_dropout": [vp, i64, i64, vp, i64, i64, vp, i64, i64, vp, i64, i64, vp, i64, i64, vp, i32, i32,
                               i32, i32, f32, vp, vp, f32, vp, i64, i64, vp, i64, i64, vp, i64, i64, vp, vp],
    "triad_attn_fwd": [vp, i64, i64, vp, i64, i64, vp, i64, i64, i32, i32, i32, i32, f32, vp, i64, i64, vp, vp],
    "triad_attn_bwd": [vp, i64, i64, vp, i64, i64, vp, i64, i64, vp, i64, i64, vp, i64, i64, vp, i32, i32, i32,
                       i32, f32, vp, i64, i64, vp, i64, i64, vp, i64, i64, vp, vp],
    "triad_dense_nparts": [i64],
    "triad_dense_rowmax": [vp, i32, i32, i32, i32, i32, vp, vp, vp],
    "triad_nonneg_fwd": [vp, i64, f32, vp, vp],
    "triad_nonneg_bwd": [vp, i64, f32, f32, vp, vp, vp],
    "triad_sims_bwd_pack": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, vp, i64, vp, vp],
    "triad_sum_parts": [vp, i32, f64, vp, vp],
}
# entry points returning a value rather than a status
RESTYPES = {"triad_pairsim_nparts": C.c_int, "triad_chgn_workspace_bytes": C.c_longlong,
            "triad_conv0_dw_workspace_bytes": C.c_longlong, "triad_gelu_table_bytes": C.c_longlong,
            "triad_posconv_dw_part_bytes": C.c_longlong,
            "triad_lora_tn_blocks": C.c_int, "triad_dropaddln_bwd_blocks": C.c_int,
            "triad_colsum_splits": C.c_int, "triad_colsum_dma_splits": C.c_int, "triad_dense_nparts": C.c_int,
            "triad_rowpanel_count": C.c_int}

# Entry points that serve ONLY the backbones' layers (frontend.py, postln.py, vit.py, attention.py):
# not part of the hot path. Every other launching entry point is hot-path work and is
# timed by bench.py (hot_path_entry_points), so a kernel added or renamed on the hot path is timed
# by default; tests/test_cpu_host.py checks that no head module calls a name listed here.
# Shared entry points (the GEMMs, column and slab sums) are hot-path ones whose backbone launches
# carry meta=dict(backbone=True) and are reported apart.
BACKBONE_ENTRY_POINTS = frozenset({
    "triad_chgn_gelu_fwd", "triad_chgn_gelu_bwd", "triad_gemm_bf16_form", "triad_conv0_dw", "triad_c0gn_fwd",
    "triad_posconv", "triad_posconv_dw", "triad_gemm_bf16_splitk", "triad_rows_nt", "triad_lora_update",
    "triad_dropaddln_fwd", "triad_dropaddln_bwd", "triad_gelu_table", "triad_geludrop_fwd", "triad_geludrop_bwd",
    "triad_dropout_keep", "triad_addln_fwd", "triad_addln_bwd", "triad_lora_tn", "triad_attn_dropmask",
    "triad_attn_fwd_dropout", "triad_attn_bwd_dropout", "triad_attn_fwd", "triad_attn_bwd"})


def hot_path_entry_points():
    """Every entry point that launches work (not a size / count query) and is not backbone-only."""
    return tuple(n for n in SIGNATURES if n not in RESTYPES and n not in BACKBONE_ENTRY_POINTS)



class PairsimProblem(C.Structure):
    """struct triad_pairsim_problem (include/triad_hip.h)."""
    _fields_ = [("Q", vp), ("K", vp), ("R", i32), ("R_pad", i32), ("Nq", i32), ("Bq", i32), ("Bk", i32),
                ("Nk_pad", i32), ("Nk_eff", i32), ("temp", vp), ("clamp_lo", f32), ("diag", i32), ("diag_off", i32),
                ("rowmax", vp), ("argmax", vp), ("nn_part", vp), ("diagS", vp), ("dS", vp), ("CT", i64),
                ("st_part", vp), ("k_tiles", vp)]


_lock = threading.Lock()
_lib = None


class TriadError(RuntimeError):
    pass


def load():
    """Load the HIP library (raises if it was not built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise TriadError(f"{LIB_PATH} not found: build it with `python -m triad_amd.build` "
                                 "(or __graft_entry__.build()); there is no CPU fallback")
            if LIB_PATH == DEFAULT_LIB:
                _check_fresh()
            lib = C.CDLL(LIB_PATH)
            for name, args in SIGNATURES.items():
                if LIB_PATH != DEFAULT_LIB and not hasattr(lib, name):
                    continue   # an A/B variant built from older sources: only what it has
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = RESTYPES.get(name, C.c_int)
            _lib = lib
    return _lib


def _check_fresh():
    """Refuse a library built from other sources than the ones in the tree (a stale prebuilt
    .so must not pass tests against edited kernels): build.py stamps the source hash."""
    from . import build
    stamp = DEFAULT_LIB + ".srchash"
    have = open(stamp).read().strip() if os.path.exists(stamp) else None
    if have != build.source_hash():
        raise TriadError(f"{DEFAULT_LIB} is stale (built from different sources than triad_amd/csrc + "
                         "include): rebuild with `python -m triad_amd.build`")


# Optional live timing of launches: {entry point name: [(start_event, end_event, meta), ...]}.
# Enabled by bench.py over its timed region; events are recorded on the current HIP stream,
# which is the stream every entry point is launched on.
TIMERS = None
# Step watchdog (triad_amd.watchdog, armed by bench.py): notes each entry point launched per stream.
WATCH = None


def _isolate(name):
    """Diagnostics (tools/stream_repeat.py --configs): TRIAD_ISOLATE = comma-separated name
    prefixes of entry points to run ALONE on the device -- a device-wide synchronisation before
    and after the launch, so no kernel of another stream shares its CUs. Unset in
    every product run."""
    spec = os.environ.get("TRIAD_ISOLATE")
    return bool(spec) and name not in RESTYPES and any(name.startswith(p) for p in spec.split(",") if p)


def call(name, *args, meta=None):
    """Invoke an entry point; non-zero status -> TriadError (RuntimeError).
    meta: per-launch metadata (e.g. algorithmic FLOPs) recorded with the timing when enabled."""
    if _isolate(name):
        import torch
        torch.cuda.synchronize()
        try:
            rc = getattr(load(), name)(*args)
        finally:
            torch.cuda.synchronize()
    elif TIMERS is not None and name in TIMERS:
        import torch
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(load(), name)(*args)
        e1.record()
        TIMERS[name].append((e0, e1, meta))
    else:
        rc = getattr(load(), name)(*args)
    if WATCH is not None and name not in RESTYPES:
        WATCH.note(name)   # event after the launch: completed <=> this entry point's kernels are done
    if name not in RESTYPES and rc != 0:
        what = "invalid argument/shape" if rc == 1001 else f"hipError_t {rc}"
        raise TriadError(f"{name} failed: {what}")
    return rc


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def h2d(t, device):
    """Host tensor -> device tensor without a host synchronisation: staged through pinned
    memory (the caching host allocator keeps the block alive until the async copy is done).
    A pageable copy would block the host until the device queue drained."""
    import torch
    device = torch.device(device)
    if device.type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


def stream_ptr(device=None):
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
