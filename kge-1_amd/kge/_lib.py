"""ctypes binding of libkgescore.so (the gfx950 HIP engine, C ABI in include/kgescore.h).

There is deliberately no fallback: if the library is missing, or a tensor is not on a
ROCm device, the call raises.  Tensors are passed as raw device pointers with explicit
leading dimensions; launches go on PyTorch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
#: KGE_LIBRARY points development scripts at another build of the same ABI (the dev library
#: with the kge_dev_* probes, kge-1_amd/csrc `make dev`); unset, the in-tree product library.
LIB_PATH = os.environ.get("KGE_LIBRARY") or os.path.join(_HERE, "libkgescore.so")

# enums (kgescore.h)
COMPLEX, DISTMULT, RESCAL, TRANSE, ROTATE, CP, SIMPLE = range(7)


def query_width(model: int, d_e: int) -> int:
    """Columns of the prepared query rows: CP contracts half an entity row (cp.py:17-19)."""
    return d_e // 2 if model == CP else d_e
DIR_SP, DIR_PO = 0, 1
PREC_FP32, PREC_BF16X3 = 0, 1
DIST_L1, DIST_L2, DIST_ROT_L1, DIST_ROT_L2 = range(4)
TIE = {"rounded_mean_rank": 0, "best_rank": 1, "worst_rank": 2}
PRECISIONS = {"fp32": PREC_FP32, "bf16x3": PREC_BF16X3}

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float

SIGNATURES = {
    "kge_version": ([], _I),
    "kge_error_string": ([_I], ctypes.c_char_p),
    "kge_prep_query": ([_I, _I, _P, _I64, _P, _P, _I64, _P, _I64, _I, _I, _P, _I64, _P], _I),
    "kge_prep_query_split": ([_I, _I, _P, _I64, _P, _P, _I64, _P, _I64, _I, _I, _P, _I64, _P, _P, _I64, _P], _I),
    "kge_prep_query_bwd": ([_I, _I, _P, _I64, _P, _P, _I64, _P, _I64, _I, _I, _P, _I64, _P, _I64,
                            _P, _I64, _P], _I),
    "kge_score_dot": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _I, _P], _I),
    "kge_split_rows": ([_P, _I64, _I64, _I, _P, _P, _I64, _P], _I),
    "kge_score_dot_split": ([_P, _P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _P], _I),
    "kge_score_dot_bwd_q": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _I, _I, _P], _I),
    "kge_score_dot_bwd_q_ws_size": ([_I64, _I64, _I, _I], _I64),
    "kge_score_dot_bwd_q_ws": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _I, _I, _P, _I64, _P], _I),
    "kge_score_dot_bwd_q_noalloc": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _I, _P], _I),
    "kge_score_dot_bwd_t": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _I, _P], _I),
    "kge_adagrad_step": ([_P, _P, _P, _I64, ctypes.c_float, ctypes.c_float, ctypes.c_float, _I, _P], _I),
    "kge_adagrad_step_multi": ([_I, _P, _P, _P, _P, _P, ctypes.c_float, ctypes.c_float, _I, _P], _I),
    "kge_lp_rows": ([_P, _I64, _P, _I64, _I, _I, _P, _P], _I),
    "kge_lp_rows_bwd": ([_P, _I64, _P, _I64, _I, _I, _P, _F, _P, _I64, _P], _I),
    "kge_score_dot_bwd_t_ex": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _I, _I, _P], _I),
    "kge_score_dist": ([_I, _F, _P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _P], _I),
    "kge_score_dist_bwd": ([_I, _F, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _P,
                            _I64, _P], _I),
    "kge_score_dist_bwd_weighted": ([_I, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _P, _I64, _P], _I),
    "kge_score_spo": ([_I, _F, _P, _I64, _P, _P, _I64, _P, _P, _I64, _I, _I, _P, _P], _I),
    "kge_score_spo_bwd": ([_I, _F, _P, _I64, _P, _P, _I64, _P, _P, _I64, _I, _I, _P, _P, _I64, _P,
                           _I64, _P], _I),
    "kge_rank_counts": ([_P, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P], _I),
    "kge_rank_hist": ([_P, _P, _I64, _I, _P, _P, _I64, _P], _I),
    "kge_softmax_xent": ([_P, _I64, _I64, _I64, _P, _F, _P, _P, _I64, _P], _I),
    "kge_softmax_kl": ([_P, _I64, _I64, _I64, _P, _P, _F, _F, _P, _P, _I64, _P], _I),
    "kge_score_cand": ([_I, _F, _I, _P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I, _P, _I64, _P], _I),
    "kge_score_cand_bwd": ([_I, _F, _I, _P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I, _P, _I64, _P, _I64, _P,
                            _I64, _P, _I64, _P], _I),
    "kge_score_cand_ordered": ([_I, _F, _I, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I, _P, _I64, _P], _I),
    "kge_score_cand_bwd_q_ordered": ([_I, _F, _I, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I, _P, _I64,
                                      _P, _I64, _P, _I64, _P], _I),
    "kge_score_cand_bwd_ent": ([_I, _F, _I, _P, _I64, _P, _I64, _P, _I64, _I64, _I, _P, _P, _I64, _P, _I64, _P,
                                _I64, _P, _I64, _P], _I),
    "kge_bucket_scatter": ([_P, _I64, _P, _P, _P], _I),
    "kge_bucket_count": ([_P, _I64, _I64, _P, _P], _I),
    "kge_sort_rows": ([_P, _I64, _I64, _I64, _I64, _P, _P, _P], _I),
    "kge_group_sorted_rows": ([_P, _P, _I64, _I64, _I64, _P, _P, _P], _I),
    "kge_stage_i64": ([_P, _P, _I64, _P], _I),
    "kge_rank_hist_multi": ([_P, _P, _I64, _I64, _I, _P, _P, _I64, _P], _I),
    "kge_rank_metrics": ([_P, _I64, _I64, _I64, _I, _P, _P], _I),
    "kge_rank_rows": ([_P, _I64, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P,
                       _I64, _I64, _P, _I64, _P, _I64, _I, _F, _P, _P], _I),
    "kge_row_norm_max": ([_P, _I64, _I64, _I, _P, _P], _I),
    "kge_score_dot_split_rank": ([_P, _P, _I64, _P, _I64, _I64, _I64, _I64, _I, _P, _P, _P, _P, _P, _I64, _P, _I64,
                                  _P], _I),
    "kge_rank_codes_ld": ([_I64], _I64),
    "kge_rank_band": ([_P, _I64, _I64, _I, _F, _P, _P, _P], _I),
    "kge_rank_rows_codes": ([_P, _I64, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I,
                             _P, _P, _I64, _I64, _P, _I64, _P, _I64, _I, _F, _P, _P], _I),
    "kge_softmax_planes_max_columns": ([], _I64),
    "kge_softmax_xent_planes": ([_P, _I64, _I64, _I64, _I64, _P, _F, _P, _P], _I),
    "kge_softmax_kl_planes": ([_P, _I64, _I64, _I64, _I64, _P, _P, _F, _F, _P, _P], _I),
    "kge_score_dot_bwd_q_planes_ws_size": ([_I64, _I64, _I], _I64),
    "kge_score_dot_bwd_q_planes": ([_P, _P, _I64, _P, _I64, _I64, _I64, _I, _P, _I64, _I, _P, _P, _I64, _P], _I),
    "kge_score_dot_bwd_t_planes": ([_P, _P, _I64, _P, _P, _I64, _I64, _I64, _I, _P, _I64, _I, _P, _P], _I),
    "kge_loss_sums": ([_P, _I64, _I64, _P, _F, _P, _P, _P], _I),
    "kge_bce_planes": ([_P, _I64, _I64, _I64, _I64, _P, _P, _F, _F, _F, _P, _P], _I),
    "kge_ns_loss": ([_I, _P, _I64, _I64, _I64, _F, _F, _P, _P, _I64, _P], _I),
    "kge_prep_query_split2": ([_I, _I, _I, _I64, _P, _P, _I64, _P, _P, _I64, _P, _I64, _I, _I, _P, _I64, _P, _P, _I64,
                               _P], _I),
    "kge_prep_query_split2_band": ([_I, _I, _I, _I64, _P, _I64, _P, _P, _I64, _P, _I64, _I, _I, _P, _I64, _P, _P, _I64,
                                    _F, _P, _P, _P], _I),
    "kge_prep_query_bwd2": ([_I, _I, _I, _I64, _P, _P, _I64, _P, _P, _I64, _P, _I64, _I, _I, _P, _I64, _P, _I64, _P,
                             _I64, _P], _I),
    "kge_softmax_row_stats": ([_P, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P], _I),
    "kge_softmax_grad": ([_P, _I64, _I64, _I64, _I64, _P, _P, _F, _P, _I64, _P], _I),
    "kge_softmax_grad_planes": ([_P, _I64, _I64, _I64, _I64, _I64, _P, _P, _F, _P, _I64, _P], _I),
    "kge_grad_planes_chunks": ([_I64], _I64),
    "kge_bce_grad_planes": ([_P, _I64, _I64, _I64, _I64, _I64, _P, _F, _F, _P, _I64, _P, _P], _I),
}

_lib: Optional[ctypes.CDLL] = None


class EngineError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load libkgescore.so once; raise loudly if it is missing (no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(
                f"libkgescore.so not found at {LIB_PATH}; build it with "
                "`make -C kge-1_amd/csrc` (or __graft_entry__.build()). The MI355X "
                "scoring engine has no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = args
            fn.restype = res
        _lib = handle
    return _lib


def _check(status: int, what: str):
    if status != 0:
        msg = lib().kge_error_string(status).decode()
        if status in (1001, 1004):
            raise ValueError(f"{what}: {msg}")
        raise EngineError(f"{what} failed ({status}): {msg}")


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def stream() -> int:
    """The current HIP stream of the current device as a raw handle.  (The private accessors
    skip the Stream object torch.cuda.current_stream() builds: ~1 us instead of ~11 us per
    call, with about seven calls per eager training step.)"""
    if _raw_stream is not None and _cur_device is not None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream().cuda_stream


def require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise EngineError(
                "kge-1_amd scores on the MI355X (gfx950) HIP engine only; got a tensor on "
                f"{t.device}. Set job.device to a ROCm device ('cuda' / 'cuda:N').")


def rows(t: torch.Tensor) -> int:
    """Leading dimension (elements) of a row-major 2-D fp32 tensor with unit col stride."""
    if t.dtype != torch.float32:
        raise ValueError(f"expected float32, got {t.dtype}")
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("expected a 2-D tensor with contiguous rows")
    return t.stride(0)


#: KGE_CHECK_INDEX=1 validates every index vector against its table on the host side
#: (one device reduction + sync per call: debugging / tests; the kernels trust indexes).
CHECK_INDEX = os.environ.get("KGE_CHECK_INDEX", "0") == "1"


def idx64(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if t is None:
        return None
    if t.dtype == torch.int64 and t.dim() == 1 and t.is_contiguous():
        return t
    t = t.reshape(-1)
    if t.dtype != torch.int64:
        t = t.long()
    return t.contiguous()


def check_index(idx: Optional[torch.Tensor], num_rows: int, what: str):
    # (skipped while a HIP graph is being recorded: the check syncs; the recorded step's
    # indexes were checked by the eager warm-up steps of the same shapes)
    if CHECK_INDEX and idx is not None and idx.numel() > 0 and not torch.cuda.is_current_stream_capturing():
        lo, hi = int(idx.min()), int(idx.max())
        if lo < 0 or hi >= num_rows:
            raise IndexError(f"{what}: index out of range [{lo}, {hi}] for {num_rows} rows")


# ------------------------------------------------------------------ thin wrappers


def prep_query(model, direction, ent, eidx, rel, ridx, n, d_e, d_r, out=None):
    require_device(ent, rel)
    eidx, ridx = idx64(eidx), idx64(ridx)
    check_index(eidx, ent.shape[0], "entity index")
    check_index(ridx, rel.shape[0], "relation index")
    q = out if out is not None else torch.empty(n, query_width(model, d_e), device=ent.device, dtype=torch.float32)
    _check(lib().kge_prep_query(model, direction, ptr(ent), rows(ent), ptr(eidx), ptr(rel), rows(rel),
                                ptr(ridx), n, d_e, d_r, ptr(q), rows(q), stream()), "kge_prep_query")
    return q


def prep_query_split(model, direction, ent, eidx, rel, ridx, n, d_e, d_r, want_fp32=True, out=None, eidx_base=0):
    """Query rows as fp32 (optional) plus bf16 hi / lo planes [n, round32(width)] in one pass
    (into out = (q or None, hi, lo) when given).  eidx_base: the id of ent's first row -- eidx
    then holds GLOBAL row ids of a table of which ent is the slice starting at that row (a
    rank's shard), all of them inside the slice; saves the caller a subtraction kernel."""
    require_device(ent, rel)
    eidx, ridx = idx64(eidx), idx64(ridx)
    if eidx_base and CHECK_INDEX and eidx is not None and not torch.cuda.is_current_stream_capturing():
        check_index(eidx - eidx_base, ent.shape[0], "entity index")
    elif not eidx_base:
        check_index(eidx, ent.shape[0], "entity index")
    check_index(ridx, rel.shape[0], "relation index")
    qw = query_width(model, d_e)
    if out is not None:
        q, hi, lo = out
        ldp = hi.stride(0)
    else:
        ldp = (qw + 31) // 32 * 32
        q = torch.empty(n, qw, device=ent.device, dtype=torch.float32) if want_fp32 else None
        hi = torch.empty(n, ldp, device=ent.device, dtype=torch.bfloat16)
        lo = torch.empty_like(hi)
    ld_ent = rows(ent)
    # the kernel addresses row eidx[i] as ent + eidx[i] * ld: shift the base by eidx_base rows
    _check(lib().kge_prep_query_split(model, direction, ptr(ent) - 4 * ld_ent * int(eidx_base), ld_ent, ptr(eidx),
                                      ptr(rel), rows(rel), ptr(ridx), n, d_e, d_r, ptr(q),
                                      rows(q) if q is not None else 0, ptr(hi), ptr(lo), ldp, stream()),
           "kge_prep_query_split")
    return q, hi, lo


def prep_query_packed(model, direction, ent, eidx, rel, ridx, eidx_base=0):
    """The bf16 hi / lo planes of the query rows packed per row, [n, 2 ldp] = [hi | lo] with
    ldp = round32(width): what score_dot_packed reads, in one buffer (the row-sharded path
    exchanges it between GPUs).  eidx_base as in prep_query_split.  A lean wrapper: this sits on
    the per-step host path of the multi-GPU scoring loop."""
    d_e = ent.shape[1]
    n = eidx.numel()
    ldp = (query_width(model, d_e) + 31) // 32 * 32
    packed = torch.empty(n, 2 * ldp, device=ent.device, dtype=torch.bfloat16)
    if CHECK_INDEX:
        require_device(ent, rel, eidx, ridx)
        check_index(eidx - eidx_base, ent.shape[0], "entity index")
        check_index(ridx, rel.shape[0], "relation index")
    eidx, ridx = idx64(eidx), idx64(ridx)
    ld_ent = rows(ent)
    base = packed.data_ptr()
    _check(lib().kge_prep_query_split(model, direction, ent.data_ptr() - 4 * ld_ent * int(eidx_base), ld_ent,
                                      eidx.data_ptr(), rel.data_ptr(), rows(rel), ridx.data_ptr(), n, d_e,
                                      rel.shape[1], None, 0, base, base + 2 * ldp, 2 * ldp, stream()),
           "kge_prep_query_split")
    return packed


def score_dot_packed(packed, t, d, out=None):
    """kge_score_dot_split on planes packed [hi | lo] per row (prep_query_packed)."""
    n = packed.shape[0]
    ldp = packed.shape[1] // 2
    m = t.shape[0]
    s = out if out is not None else torch.empty(n, m, device=t.device, dtype=torch.float32)
    base = packed.data_ptr()
    _check(lib().kge_score_dot_split(base, base + 2 * ldp, packed.stride(0), t.data_ptr(), rows(t), None, n, m, d,
                                     s.data_ptr(), rows(s), stream()), "kge_score_dot_split")
    return s


def prep_query_split2(model, dir_a, dir_b, n_a, n_a_dev, ent, eidx, rel, ridx, d_e, d_r, out):
    """kge_prep_query_split2: the stacked query rows of two batches (rows [0, n_a) in direction
    dir_a, the rest in dir_b; n_a_dev: the split point as an int64 device scalar) into
    out = (q or None, hi, lo)."""
    require_device(ent, rel)
    eidx, ridx = idx64(eidx), idx64(ridx)
    check_index(eidx, ent.shape[0], "entity index")
    check_index(ridx, rel.shape[0], "relation index")
    q, hi, lo = out
    _check(lib().kge_prep_query_split2(model, dir_a, dir_b, int(n_a), ptr(n_a_dev), ptr(ent), rows(ent), ptr(eidx),
                                       ptr(rel), rows(rel), ptr(ridx), eidx.numel(), d_e, d_r, ptr(q),
                                       rows(q) if q is not None else 0, ptr(hi), ptr(lo), hi.stride(0), stream()),
           "kge_prep_query_split2")
    return q, hi, lo


def prep_query_split2_band(model, dir_a, dir_b, n_a, ent, eidx, rel, ridx, d_e, d_r, out, band_rel, t_norm_max):
    """kge_prep_query_split2_band: prep_query_split2 into out = (q, hi, lo) plus the rows' refinement
    bands band_rel * |q_i| * t_norm_max[0] from the same launch.  Returns (q, hi, lo, band)."""
    require_device(ent, rel)
    eidx, ridx = idx64(eidx), idx64(ridx)
    check_index(eidx, ent.shape[0], "entity index")
    check_index(ridx, rel.shape[0], "relation index")
    q, hi, lo = out
    band = torch.empty(eidx.numel(), device=ent.device, dtype=torch.float32)
    _check(lib().kge_prep_query_split2_band(model, dir_a, dir_b, int(n_a), ptr(ent), rows(ent), ptr(eidx), ptr(rel),
                                            rows(rel), ptr(ridx), eidx.numel(), d_e, d_r, ptr(q), rows(q), ptr(hi),
                                            ptr(lo), hi.stride(0), float(band_rel), ptr(t_norm_max), ptr(band),
                                            stream()), "kge_prep_query_split2_band")
    return q, hi, lo, band


def prep_query_bwd2(model, dir_a, dir_b, n_a, n_a_dev, ent, eidx, rel, ridx, d_e, d_r, dq, d_ent, d_rel):
    eidx, ridx = idx64(eidx), idx64(ridx)
    _check(lib().kge_prep_query_bwd2(
        model, dir_a, dir_b, int(n_a), ptr(n_a_dev), ptr(ent), rows(ent), ptr(eidx), ptr(rel), rows(rel), ptr(ridx),
        eidx.numel(), d_e, d_r, ptr(dq), rows(dq), ptr(d_ent), rows(d_ent) if d_ent is not None else 0, ptr(d_rel),
        rows(d_rel) if d_rel is not None else 0, stream()), "kge_prep_query_bwd2")


def split_ok(d, t, precision):
    """Whether the production split-plane bf16x3 contraction applies to table t."""
    return precision == PREC_BF16X3 and d % 4 == 0 and rows(t) % 4 == 0 and t.data_ptr() % 16 == 0


def prep_query_bwd(model, direction, ent, eidx, rel, ridx, n, d_e, d_r, dq, d_ent, d_rel):
    eidx, ridx = idx64(eidx), idx64(ridx)
    _check(lib().kge_prep_query_bwd(
        model, direction, ptr(ent), rows(ent), ptr(eidx), ptr(rel), rows(rel), ptr(ridx), n, d_e, d_r,
        ptr(dq), rows(dq), ptr(d_ent), rows(d_ent) if d_ent is not None else 0, ptr(d_rel),
        rows(d_rel) if d_rel is not None else 0, stream()), "kge_prep_query_bwd")


def score_dot(q, t, tidx, precision, out=None):
    require_device(q, t)
    tidx = idx64(tidx)
    check_index(tidx, t.shape[0], "candidate index")
    n, d = q.shape
    m = tidx.numel() if tidx is not None else t.shape[0]
    s = out if out is not None else torch.empty(n, m, device=q.device, dtype=torch.float32)
    _check(lib().kge_score_dot(ptr(q), rows(q), ptr(t), rows(t), ptr(tidx), n, m, d, ptr(s), rows(s),
                               precision, stream()), "kge_score_dot")
    return s


def split_rows(x):
    """fp32 rows -> bf16 (hi, lo) planes, ld rounded up to a multiple of 32 (zero padded)."""
    n, d = x.shape
    ldo = (d + 31) // 32 * 32
    hi = torch.empty(n, ldo, device=x.device, dtype=torch.bfloat16)
    lo = torch.empty_like(hi)
    _check(lib().kge_split_rows(ptr(x), rows(x), n, d, ptr(hi), ptr(lo), ldo, stream()), "kge_split_rows")
    return hi, lo


def split_rows_into(x, hi, lo):
    """split_rows into given bf16 planes (same shape and row stride, ld >= d, zeroed past d by the
    caller or by the kernel's own padding up to its ld argument)."""
    n, d = x.shape
    if hi.shape != lo.shape or hi.stride(0) != lo.stride(0) or hi.shape[0] != n or hi.shape[1] < d:
        raise ValueError("split_rows_into: planes must be [n, ld >= d] with equal row strides")
    _check(lib().kge_split_rows(ptr(x), rows(x), n, d, ptr(hi), ptr(lo), hi.stride(0), stream()), "kge_split_rows")
    return hi, lo


def score_dot_split(q_hi, q_lo, t, tidx, d, out=None):
    """Production bf16x3 contraction on pre-split query planes."""
    require_device(q_hi, t)
    tidx = idx64(tidx)
    check_index(tidx, t.shape[0], "candidate index")
    n = q_hi.shape[0]
    m = tidx.numel() if tidx is not None else t.shape[0]
    s = out if out is not None else torch.empty(n, m, device=t.device, dtype=torch.float32)
    _check(lib().kge_score_dot_split(ptr(q_hi), ptr(q_lo), q_hi.stride(0), ptr(t), rows(t), ptr(tidx), n, m, d,
                                     ptr(s), rows(s), stream()), "kge_score_dot_split")
    return s


def contract(q, t, tidx, precision, out=None):
    """S = Q . T[tidx]^T on the engine: bf16x3 via split planes when the layout allows
    (d % 4 == 0, 16-B aligned rows), otherwise the generic kernel."""
    d = q.shape[1]
    if split_ok(d, t, precision):
        hi, lo = split_rows(q)
        return score_dot_split(hi, lo, t, tidx, d, out=out)
    return score_dot(q, t, tidx, precision, out=out)


def score_dot_bwd_q(g, t, tidx, precision, dq=None, accumulate=False):
    tidx = idx64(tidx)
    n, m = g.shape
    d = t.shape[1]
    if dq is None:
        dq = torch.empty(n, d, device=g.device, dtype=torch.float32)
        accumulate = False
    # split-K partial slabs summed in a fixed order instead of float atomics (bf16x3)
    ws_n = lib().kge_score_dot_bwd_q_ws_size(n, m, d, precision)
    ws = torch.empty(ws_n, device=g.device, dtype=torch.float32) if ws_n > 0 else None
    _check(lib().kge_score_dot_bwd_q_ws(ptr(g), rows(g), ptr(t), rows(t), ptr(tidx), n, m, d, ptr(dq),
                                        rows(dq), int(accumulate), precision, ptr(ws), ws_n, stream()),
           "kge_score_dot_bwd_q")
    return dq


def score_dot_bwd_q_noalloc(g, t, tidx, dq, accumulate=False):
    """dq (+)= g . t[tidx] (bf16x3) through the entry point that allocates nothing: the split-K
    partial slabs live in the library's static device scratch (kge_score_dot_bwd_q_noalloc).
    dq is caller-provided; calls that overlap on one GPU race on the scratch."""
    tidx = idx64(tidx)
    n, m = g.shape
    d = t.shape[1]
    _check(lib().kge_score_dot_bwd_q_noalloc(ptr(g), rows(g), ptr(t), rows(t), ptr(tidx), n, m, d, ptr(dq),
                                             rows(dq), int(accumulate), stream()), "kge_score_dot_bwd_q_noalloc")
    return dq


def score_dot_bwd_t(g, q, tidx, dt, precision, accumulate=True):
    """dt (+)= g^T . q (rows scattered through tidx); accumulate=False overwrites dt."""
    tidx = idx64(tidx)
    n, m = g.shape
    d = q.shape[1]
    _check(lib().kge_score_dot_bwd_t_ex(ptr(g), rows(g), ptr(q), rows(q), ptr(tidx), n, m, d, ptr(dt),
                                        rows(dt), int(accumulate), precision, stream()), "kge_score_dot_bwd_t_ex")
    return dt


def score_dist(kind, sign, q, t, tidx, out=None):
    require_device(q, t)
    tidx = idx64(tidx)
    n, d = q.shape
    m = tidx.numel() if tidx is not None else t.shape[0]
    s = out if out is not None else torch.empty(n, m, device=q.device, dtype=torch.float32)
    _check(lib().kge_score_dist(kind, sign, ptr(q), rows(q), ptr(t), rows(t), ptr(tidx), n, m, d, ptr(s),
                                rows(s), stream()), "kge_score_dist")
    return s


def score_dist_bwd(kind, sign, g, q, t, tidx, dq, dt):
    """dq += , dt += the gradients of sign * dist(q, t rows) for dL/dS = g.  The L2 kinds need
    g / dist per pair: where the layout allows, the distances are recomputed by the forward
    kernel into an [n, m] block, the pair weights formed there, and the owner-computes kernels
    take them (kge_score_dist_bwd_weighted); otherwise the generic kernel recomputes them per
    tile."""
    tidx = idx64(tidx)
    n, m = g.shape
    d = q.shape[1]
    if (kind in (DIST_L2, DIST_ROT_L2) and n > 0 and m > 0 and (d // 2 if kind == DIST_ROT_L2 else d) % 4 == 0
            and rows(q) % 4 == 0 and rows(t) % 4 == 0 and ptr(q) % 16 == 0 and ptr(t) % 16 == 0):
        dist = score_dist(kind, 1.0, q, t, tidx)
        w = torch.where(dist > 0, g * sign / dist, torch.zeros((), device=g.device, dtype=g.dtype))
        _check(lib().kge_score_dist_bwd_weighted(kind, ptr(w), rows(w), ptr(q), rows(q), ptr(t), rows(t), ptr(tidx),
                                                 n, m, d, ptr(dq), rows(dq) if dq is not None else 0, ptr(dt),
                                                 rows(dt) if dt is not None else 0, stream()),
               "kge_score_dist_bwd_weighted")
        return
    _check(lib().kge_score_dist_bwd(kind, sign, ptr(g), rows(g), ptr(q), rows(q), ptr(t), rows(t), ptr(tidx),
                                    n, m, d, ptr(dq), rows(dq) if dq is not None else 0, ptr(dt),
                                    rows(dt) if dt is not None else 0, stream()), "kge_score_dist_bwd")


def score_spo(model, l_norm, ent, sidx, rel, pidx, oidx, d_e, d_r, out=None):
    require_device(ent, rel)
    sidx, pidx, oidx = idx64(sidx), idx64(pidx), idx64(oidx)
    check_index(sidx, ent.shape[0], "subject index")
    check_index(oidx, ent.shape[0], "object index")
    check_index(pidx, rel.shape[0], "relation index")
    n = sidx.numel()
    o = out if out is not None else torch.empty(n, device=ent.device, dtype=torch.float32)
    _check(lib().kge_score_spo(model, float(l_norm), ptr(ent), rows(ent), ptr(sidx), ptr(rel), rows(rel),
                               ptr(pidx), ptr(oidx), n, d_e, d_r, ptr(o), stream()), "kge_score_spo")
    return o


def score_spo_bwd(model, l_norm, ent, sidx, rel, pidx, oidx, d_e, d_r, g, d_ent, d_rel):
    sidx, pidx, oidx = idx64(sidx), idx64(pidx), idx64(oidx)
    n = sidx.numel()
    _check(lib().kge_score_spo_bwd(
        model, float(l_norm), ptr(ent), rows(ent), ptr(sidx), ptr(rel), rows(rel), ptr(pidx), ptr(oidx), n,
        d_e, d_r, ptr(g), ptr(d_ent), rows(d_ent) if d_ent is not None else 0, ptr(d_rel),
        rows(d_rel) if d_rel is not None else 0, stream()), "kge_score_spo_bwd")


def rank_counts(s, c0, true_idx, true_score, f_ptr, f_col, t_ptr, t_col, greater, ties):
    n, m = s.shape
    true_idx = idx64(true_idx)
    true_score = true_score.reshape(-1).float().contiguous()
    f_ptr, f_col, t_ptr, t_col = (idx64(x) for x in (f_ptr, f_col, t_ptr, t_col))
    if not (greater.is_contiguous() and ties.is_contiguous() and greater.dtype == torch.int64):
        raise ValueError("greater / ties must be contiguous int64")
    _check(lib().kge_rank_counts(ptr(s), rows(s), n, m, c0, ptr(true_idx), ptr(true_score), ptr(f_ptr),
                                 ptr(f_col), ptr(t_ptr), ptr(t_col), ptr(greater), ptr(ties), stream()),
           "kge_rank_counts")


def rank_hist_multi(greater, ties, rows_per_hist, tie_handling, ranks, hists):
    """kge_rank_hist_multi: row i of greater / ties counts into hists[i // rows_per_hist]."""
    greater, ties = greater.contiguous(), ties.contiguous()
    n = greater.numel()
    if hists.dim() != 2 or not hists.is_contiguous() or n > hists.shape[0] * rows_per_hist:
        raise ValueError("rank_hist_multi: hists must be a contiguous [k, hist_len] tensor covering every row")
    _check(lib().kge_rank_hist_multi(ptr(greater), ptr(ties), n, rows_per_hist, TIE[tie_handling], ptr(ranks),
                                     ptr(hists), hists.shape[1], stream()), "kge_rank_hist_multi")


def _i64c(t, what):
    if t is not None and (t.dtype != torch.int64 or not t.is_contiguous()):
        raise ValueError(f"rank_rows: {what} must be a contiguous int64 tensor")
    return t


def rank_codes_ld(m: int) -> int:
    """Words per row of the code block of score_dot_split_rank for m columns."""
    return (m + 255) // 256 * 16


def rank_band(q, band_rel, t_norm_max):
    """kge_rank_band: the per-row refinement bands band_rel * |q_i| * t_norm_max of fp32 rows q."""
    n, d = q.shape
    band = torch.empty(n, device=q.device, dtype=torch.float32)
    _check(lib().kge_rank_band(ptr(q), rows(q), n, d, float(band_rel), ptr(t_norm_max), ptr(band), stream()),
           "kge_rank_band")
    return band


def score_dot_split_rank(q_hi, q_lo, t, d, n_a, part_a, part_b, band, c0, codes=None):
    """kge_score_dot_split_rank: the contraction of score_dot_split whose epilogue compares every
    score with its row's true score and writes 2-bit codes [n, rank_codes_ld(m)] (int32 words)
    instead of scores.  t: the fp32 rows of columns c0 .. c0 + len(t) of the entity axis;
    part = (true_idx, true_score) of rows [0, n_a) and of the rest (part_b None: one batch)."""
    require_device(q_hi, t)
    n, m = q_hi.shape[0], t.shape[0]
    n_b = n - n_a
    if part_b is None:
        part_b = (None, None)
        if n_b:
            raise ValueError("score_dot_split_rank: rows beyond n_a need part_b")
    args = []
    for (true_idx, true_score), k in ((part_a, n_a), (part_b, n_b)):
        if k and (true_score.dtype != torch.float32 or not true_score.is_contiguous() or true_score.numel() < k
                  or _i64c(true_idx, "true_idx").numel() < k):
            raise ValueError("score_dot_split_rank: true scores (contiguous float32) and columns (int64) per row")
        args += [ptr(true_score), ptr(true_idx)]
    if band.dtype != torch.float32 or not band.is_contiguous() or band.numel() < n:
        raise ValueError("score_dot_split_rank: band is contiguous float32 [n]")
    ldc = rank_codes_ld(m)
    if codes is None:
        codes = torch.empty(n, ldc, device=t.device, dtype=torch.int32)
    elif codes.dtype != torch.int32 or codes.shape[0] < n or codes.stride(0) < ldc or codes.stride(1) != 1:
        raise ValueError("score_dot_split_rank: codes must be int32 [n, >= rank_codes_ld(m)]")
    _check(lib().kge_score_dot_split_rank(ptr(q_hi), ptr(q_lo), q_hi.stride(0), ptr(t), rows(t), n_a, n_b, m, d,
                                          *args, ptr(band), int(c0), ptr(codes), codes.stride(0), stream()),
           "kge_score_dot_split_rank")
    return codes


def rank_rows(s, n_a, c0, part_a, part_b, f_col, t_col, greater, ties, accumulate, tie_handling=None, ranks=None,
              hists=None, rows_per_hist=0, refine=None, codes=None, m=None):
    """kge_rank_rows: one ranking launch for the stacked score block s [n_a + n_b, m] -- or, with
    codes (and m columns; s None), kge_rank_rows_codes on the code block of score_dot_split_rank.
    part = (true_idx, true_score, f_ptr, t_ptr) of each batch (part_b None: one batch);
    tie_handling (a name) also writes ranks / hists [k, hist_len]; refine = (q, t_rows,
    band_rel, t_norm_max) rescoring near-ties exactly.  Nothing is copied: every tensor
    must already have the kernel's layout."""
    if codes is not None:
        if s is not None or m is None or codes.dtype != torch.int32 or codes.stride(1) != 1:
            raise ValueError("rank_rows: codes are an int32 [n, ldc] block and come with m, without scores")
        n = codes.shape[0]
    else:
        n, m = s.shape
    n_b = n - n_a
    if part_b is None:
        part_b = (None, None, None, None)
        if n_b:
            raise ValueError("rank_rows: rows beyond n_a need part_b")
    args = []
    for true_idx, true_score, f_ptr, t_ptr in (part_a, part_b):
        if true_score is not None and (true_score.dtype != torch.float32 or not true_score.is_contiguous()):
            raise ValueError("rank_rows: true scores must be contiguous float32")
        args += [ptr(_i64c(true_idx, "true_idx")), ptr(true_score), ptr(_i64c(f_ptr, "f_ptr")),
                 ptr(_i64c(t_ptr, "t_ptr"))]
    if not (greater.is_contiguous() and ties.is_contiguous() and greater.dtype == torch.int64
            and ties.dtype == torch.int64):
        raise ValueError("rank_rows: greater / ties must be contiguous int64")
    nrank = 1 + (part_a[2] is not None) + (part_a[3] is not None)
    if greater.numel() < nrank * n or ties.numel() < nrank * n:
        raise ValueError("rank_rows: greater / ties hold [rankings, rows] counts")
    tie = -1 if tie_handling is None else TIE[tie_handling]
    hist_len = 0
    if hists is not None:
        if hists.dim() != 2 or not hists.is_contiguous() or hists.dtype != torch.float32 \
                or rows_per_hist <= 0 or nrank * n > hists.shape[0] * rows_per_hist:
            raise ValueError("rank_rows: hists must be a contiguous float32 [k, hist_len] covering every row")
        hist_len = hists.shape[1]
    if ranks is not None and (_i64c(ranks, "ranks").numel() < nrank * n):
        raise ValueError("rank_rows: ranks holds [rankings, rows]")
    q = t_rows = tmax = None
    band, d = 0.0, 0
    if refine is not None:
        q, t_rows, band, tmax = refine
        d = q.shape[1]
        if q.shape[0] != n or t_rows.shape[0] != m or t_rows.shape[1] != d:
            raise ValueError("rank_rows: refinement operands do not match the score block")
    fn, src, ld = ((lib().kge_rank_rows, s, rows(s)) if codes is None
                   else (lib().kge_rank_rows_codes, codes, codes.stride(0)))
    _check(fn(ptr(src), ld, n_a, n_b, m, c0, *args, ptr(_i64c(f_col, "f_col")),
              ptr(_i64c(t_col, "t_col")), ptr(greater), ptr(ties), int(accumulate), tie, ptr(ranks),
              ptr(hists), hist_len, rows_per_hist, ptr(q), rows(q) if q is not None else 0,
              ptr(t_rows), rows(t_rows) if t_rows is not None else 0, d, float(band), ptr(tmax),
              stream()), "kge_rank_rows")


def row_norm_max(t):
    """Device scalar max_j |t_j|_2 (kge_row_norm_max)."""
    out = torch.empty(1, device=t.device, dtype=torch.float32)
    _check(lib().kge_row_norm_max(ptr(t), rows(t), t.shape[0], t.shape[1], ptr(out), stream()), "kge_row_norm_max")
    return out


def rank_hist(greater, ties, tie_handling, ranks, hist):
    greater, ties = greater.contiguous(), ties.contiguous()
    n = greater.numel()
    _check(lib().kge_rank_hist(ptr(greater), ptr(ties), n, TIE[tie_handling], ptr(ranks), ptr(hist),
                               hist.numel() if hist is not None else 0, stream()), "kge_rank_hist")


def softmax_xent(s, labels, scale, g=None, loss=None):
    """Per-row softmax cross entropy of score rows S[:, :m] (a possibly padded view) against
    index labels; optionally G = scale * (softmax - onehot) into g (g may be s: in place).
    Returns loss [n] (unscaled per-row losses)."""
    require_device(s)
    labels = idx64(labels)
    n, m = s.shape
    check_index(labels, m, "label")
    if loss is None:
        loss = torch.empty(n, device=s.device, dtype=torch.float32)
    _check(lib().kge_softmax_xent(ptr(s), rows(s), n, m, ptr(labels), float(scale), ptr(loss), ptr(g),
                                  rows(g) if g is not None else 0, stream()), "kge_softmax_xent")
    return loss


def score_cand(model, l_norm, direction, q, ent, cand, out=None):
    """out[i, c] = score(q_i, ent[cand[i, c]]) with score_spo semantics (kge_score_cand)."""
    require_device(q, ent, cand)
    cand = cand if (cand.dtype == torch.int64 and cand.dim() == 2 and cand.stride(1) == 1) else \
        cand.long().contiguous()
    check_index(cand, ent.shape[0], "candidate index")
    n, k = cand.shape
    d = q.shape[1]
    o = out if out is not None else torch.empty(n, k, device=q.device, dtype=torch.float32)
    _check(lib().kge_score_cand(model, float(l_norm), direction, ptr(q), rows(q), ptr(ent), rows(ent), ptr(cand),
                                cand.stride(0), n, k, d, ptr(o), rows(o), stream()), "kge_score_cand")
    return o


def sort_rows(x, id_bound=0):
    """kge_sort_rows: (ids of every row ascending, the positions they came from) of an int64
    [n, k <= 8192] matrix of non-negative ids -- torch.sort(x, 1, stable=True) in one launch.
    id_bound: an exclusive upper bound of the ids when the caller knows one (32-bit keys below
    2^21: faster), 0 otherwise."""
    require_device(x)
    if x.dtype != torch.int64 or x.dim() != 2 or x.stride(1) != 1 or x.shape[1] > 8192:
        raise ValueError("sort_rows: an int64 [n, k <= 8192] matrix with unit column stride")
    n, k = x.shape
    srt, col = torch.empty(n, k, dtype=torch.int64, device=x.device), torch.empty(n, k, dtype=torch.int64,
                                                                                  device=x.device)
    _check(lib().kge_sort_rows(ptr(x), x.stride(0) if n > 1 else k, n, k, int(id_bound), ptr(srt), ptr(col), stream()),
           "kge_sort_rows")
    return srt, col


def score_cand_ordered(model, l_norm, direction, q, ent, cand, col, out=None):
    """kge_score_cand_ordered: out[i, col[i, c]] = score(q_i, ent[cand[i, c]]) -- the candidate
    lists in the caller's order (ascending per row: table rows shared through the XCDs' L2),
    col[i, :] the permutation back to the output columns (contiguous int64 [n, k] both)."""
    require_device(q, ent, cand, col)
    if cand.dtype != torch.int64 or col.dtype != torch.int64 or not cand.is_contiguous() or not col.is_contiguous() \
            or cand.shape != col.shape or cand.dim() != 2:
        raise ValueError("score_cand_ordered: cand and col are contiguous int64 [n, k]")
    check_index(cand, ent.shape[0], "candidate index")
    n, k = cand.shape
    d = q.shape[1]
    o = out if out is not None else torch.empty(n, k, device=q.device, dtype=torch.float32)
    _check(lib().kge_score_cand_ordered(model, float(l_norm), direction, ptr(q), rows(q), ptr(ent), rows(ent),
                                        ptr(cand), k, ptr(col), k, n, k, d, ptr(o), rows(o), stream()),
           "kge_score_cand_ordered")
    return o


def score_cand_bwd_q_ordered(model, l_norm, direction, q, ent, cand, col, s, g, dq) -> bool:
    """kge_score_cand_bwd_q_ordered (dq only).  False when the layout is not served."""
    n, k = cand.shape
    rc = lib().kge_score_cand_bwd_q_ordered(model, float(l_norm), direction, ptr(q), rows(q), ptr(ent), rows(ent),
                                            ptr(cand), k, ptr(col), k, n, k, q.shape[1], ptr(s),
                                            rows(s) if s is not None else 0, ptr(g), rows(g), ptr(dq), rows(dq),
                                            stream())
    if rc == 1002:  # KGE_ERR_ALIGN
        return False
    _check(rc, "kge_score_cand_bwd_q_ordered")
    return True


def score_cand_bwd(model, l_norm, direction, q, ent, cand, s, g, dq, d_ent):
    cand = cand if (cand.dtype == torch.int64 and cand.dim() == 2 and cand.stride(1) == 1) else \
        cand.long().contiguous()
    n, k = cand.shape
    d = q.shape[1]
    _check(lib().kge_score_cand_bwd(model, float(l_norm), direction, ptr(q), rows(q), ptr(ent), rows(ent),
                                    ptr(cand), cand.stride(0), n, k, d, ptr(s), rows(s) if s is not None else 0,
                                    ptr(g), rows(g), ptr(dq), rows(dq) if dq is not None else 0, ptr(d_ent),
                                    rows(d_ent) if d_ent is not None else 0, stream()), "kge_score_cand_bwd")


def group_sorted_rows(srt, col, num_buckets):
    """kge_group_sorted_rows: (order, seg_ptr) of the pairs of sorted candidate lists grouped by
    candidate id (srt, col from sort_rows; at most 4096 rows)."""
    n, k = srt.shape
    seg_ptr = torch.empty(num_buckets + 1, dtype=torch.int64, device=srt.device)
    order = torch.empty(n * k, dtype=torch.int64, device=srt.device)
    _check(lib().kge_group_sorted_rows(ptr(srt), ptr(col), n, k, num_buckets, ptr(seg_ptr), ptr(order), stream()),
           "kge_group_sorted_rows")
    return order, seg_ptr


def score_cand_bwd_ent(model, l_norm, direction, q, ent, cand, s, g, d_ent, sorted_lists=None) -> bool:
    """d_ent += d(sum g * scores)/d ent without fp32 atomics: the n*k pairs are grouped by
    entity with a counting sort -- one group slot per entity, fixed size, no host sync -- and
    each entity row is reduced once.  sorted_lists: (srt, col) of sort_rows(cand) when the
    caller has them (the grouping is then one launch, kge_group_sorted_rows; otherwise
    kge_bucket_count, an exclusive scan and kge_bucket_scatter).
    Returns False (nothing done) when the layout is not supported."""
    unit = q.shape[1] // 2 if model == ROTATE else q.shape[1]
    if unit % 4 or unit > 2048 or rows(q) % 4 or rows(ent) % 4 or rows(d_ent) % 4 or q.data_ptr() % 16 \
            or ent.data_ptr() % 16 or d_ent.data_ptr() % 16:
        return False
    cand = cand.long().contiguous()
    n, k = cand.shape
    flat = cand.reshape(-1)
    E = ent.shape[0]
    if sorted_lists is not None and sorted_lists[0].numel() and n <= 4096:
        order, seg_ptr = group_sorted_rows(sorted_lists[0], sorted_lists[1], E)
    else:
        seg_ptr = torch.zeros(E + 1, dtype=torch.int64, device=cand.device)
        _check(lib().kge_bucket_count(ptr(flat), flat.numel(), E, ptr(seg_ptr[1:]), stream()), "kge_bucket_count")
        seg_ptr.cumsum_(0)
        cursor = seg_ptr[:-1].clone()
        order = torch.empty_like(flat)
        _check(lib().kge_bucket_scatter(ptr(flat), flat.numel(), ptr(cursor), ptr(order), stream()),
               "kge_bucket_scatter")
    _check(lib().kge_score_cand_bwd_ent(model, float(l_norm), direction, ptr(q), rows(q), ptr(ent), rows(ent),
                                        ptr(cand), n, k, q.shape[1], ptr(order), ptr(seg_ptr), ent.shape[0], ptr(s),
                                        rows(s) if s is not None else 0, ptr(g), rows(g), ptr(d_ent), rows(d_ent),
                                        stream()), "kge_score_cand_bwd_ent")
    return True


def softmax_row_stats(s, c0, labels):
    """(row max, row sum exp(x - max), target score or 0) over the column slice s = columns
    [c0, c0 + m) of score rows; labels are global column ids."""
    require_device(s)
    labels = idx64(labels)
    n, m = s.shape
    mx = torch.empty(n, device=s.device, dtype=torch.float32)
    sm = torch.empty_like(mx)
    tg = torch.empty_like(mx) if labels is not None else None
    _check(lib().kge_softmax_row_stats(ptr(s), rows(s), n, m, int(c0), ptr(labels), ptr(mx), ptr(sm), ptr(tg),
                                       stream()), "kge_softmax_row_stats")
    return mx, sm, tg


def softmax_grad(s, c0, labels, lse, scale, g):
    """g = scale * (exp(s - lse[:, None]) - onehot(labels - c0)) on the column slice."""
    labels = idx64(labels)
    lse = lse.contiguous()
    n, m = s.shape
    _check(lib().kge_softmax_grad(ptr(s), rows(s), n, m, int(c0), ptr(labels), ptr(lse), float(scale), ptr(g),
                                  rows(g), stream()), "kge_softmax_grad")
    return g


def softmax_grad_planes(s, c0, labels, lse, scale):
    """softmax_grad with the gradient as bf16 hi / lo planes in a buffer of its own (any row
    length): GradPlanes for score_dot_bwd_q_planes / _t_planes."""
    labels = idx64(labels)
    lse = lse.contiguous()
    n, m = s.shape
    n_pad, ld = planes_layout(n, m)
    buf = torch.empty(n_pad, ld, device=s.device, dtype=torch.float32)
    _check(lib().kge_softmax_grad_planes(ptr(s), rows(s), n, n_pad, m, int(c0), ptr(labels), ptr(lse), float(scale),
                                         ptr(buf), ld, stream()), "kge_softmax_grad_planes")
    return GradPlanes(buf, n, m)


def bce_grad_planes(s, c0, labels, offset, scale):
    """Binary cross entropy with logits on s + offset against the one-hot rows whose hot column is
    labels[i] - c0 (when it lies in this block): returns (sum of the block's losses as a 0-dim
    float64 tensor, unscaled; GradPlanes of G = scale * (sigmoid(s + offset) - y)) -- the row-shard
    form of the bce loss (kge_bce_grad_planes; any row length)."""
    labels = idx64(labels)
    n, m = s.shape
    n_pad, ld = planes_layout(n, m)
    buf = torch.empty(n_pad, ld, device=s.device, dtype=torch.float32)
    chunks = int(lib().kge_grad_planes_chunks(ld))
    part = torch.empty(n, chunks, device=s.device, dtype=torch.float32)
    _check(lib().kge_bce_grad_planes(ptr(s), rows(s), n, n_pad, m, int(c0), ptr(labels), float(offset), float(scale),
                                     ptr(buf), ld, ptr(part), stream()), "kge_bce_grad_planes")
    return part.sum(dtype=torch.float64), GradPlanes(buf, n, m)


def softmax_kl(s, l_ptr, l_col, smoothing, scale, g=None, loss=None):
    """Per-row KL(t || softmax(S[:, :m])) for CSR positive lists (l_ptr [n+1], l_col) with
    label smoothing; optionally G = scale * (T softmax - t) into g (g may be s).  Returns the
    per-row losses [n] (unscaled)."""
    require_device(s)
    l_ptr, l_col = idx64(l_ptr), idx64(l_col)
    n, m = s.shape
    if l_ptr.numel() != n + 1:
        raise ValueError(f"l_ptr has {l_ptr.numel()} entries, expected {n + 1}")
    check_index(l_col, m, "label column")
    if loss is None:
        loss = torch.empty(n, device=s.device, dtype=torch.float32)
    _check(lib().kge_softmax_kl(ptr(s), rows(s), n, m, ptr(l_ptr), ptr(l_col), float(smoothing), float(scale),
                                ptr(loss), ptr(g), rows(g) if g is not None else 0, stream()), "kge_softmax_kl")
    return loss


# ---- the fused loss with its gradient as bf16 planes, and the GEMMs that read them


class GradPlanes:
    """dL/dS of a fused loss as bf16 hi / lo planes living in the score buffer itself
    (kge_softmax_*_planes): buf is the fp32 [n_pad, ld] buffer the scores were written to."""

    def __init__(self, buf: torch.Tensor, n: int, m: int):
        self.buf, self.n, self.m = buf, n, m
        self.n_pad, self.ld = buf.shape
        flat = buf.view(torch.bfloat16)  # [n_pad, 2 ld]: hi plane | lo plane per row
        self.hi, self.lo = flat[:, :self.ld], flat[:, self.ld:]
        self.ldgp = 2 * self.ld


def planes_layout(n: int, m: int):
    """(rows, leading dimension) of the score buffer when its gradient is to be left as
    planes: rows padded to the GEMMs' K stage (32), columns to 32."""
    return (n + 31) // 32 * 32, (m + 31) // 32 * 32


def planes_ok(m: int) -> bool:
    return 4 <= m <= lib().kge_softmax_planes_max_columns()


def softmax_planes(buf, n, m, labels, l_ptr, smoothing, scale, loss_kind="kl", offset=0.0) -> tuple:
    """Per-row losses [n] of the scores in buf[:n, :m]; the buffer is left holding the
    gradient planes (GradPlanes).  l_ptr None: index labels (cross entropy), else CSR positives.
    loss_kind "bce": binary cross entropy with logits on scores + offset instead (kge_bce_planes)."""
    require_device(buf)
    labels, l_ptr = idx64(labels), idx64(l_ptr)
    n_pad, ld = buf.shape
    if l_ptr is None:
        check_index(labels, m, "label")
    else:
        if l_ptr.numel() != n + 1:
            raise ValueError(f"l_ptr has {l_ptr.numel()} entries, expected {n + 1}")
        check_index(labels, m, "label column")
    loss = torch.empty(n, device=buf.device, dtype=torch.float32)
    if loss_kind == "bce":
        _check(lib().kge_bce_planes(ptr(buf), ld, n, n_pad, m, ptr(l_ptr), ptr(labels), float(smoothing),
                                    float(offset), float(scale), ptr(loss), stream()), "kge_bce_planes")
    elif loss_kind != "kl":
        raise ValueError(f"softmax_planes: unknown loss kind {loss_kind!r}")
    elif l_ptr is None:
        _check(lib().kge_softmax_xent_planes(ptr(buf), ld, n, n_pad, m, ptr(labels), float(scale), ptr(loss),
                                             stream()), "kge_softmax_xent_planes")
    else:
        _check(lib().kge_softmax_kl_planes(ptr(buf), ld, n, n_pad, m, ptr(l_ptr), ptr(labels), float(smoothing),
                                           float(scale), ptr(loss), stream()), "kge_softmax_kl_planes")
    return loss, GradPlanes(buf, n, m)


NS_MARGIN, NS_BCE = 0, 1


def ns_loss(kind, s, arg, scale):
    """kge_ns_loss on a [n, k] block (column 0 the positive): (per-row losses [n], g [n, k])."""
    require_device(s)
    n, k = s.shape
    loss = torch.empty(n, device=s.device, dtype=torch.float32)
    g = torch.empty(n, k, device=s.device, dtype=torch.float32)
    _check(lib().kge_ns_loss(int(kind), ptr(s), rows(s), n, k, float(arg), float(scale), ptr(loss), ptr(g), rows(g),
                             stream()), "kge_ns_loss")
    return loss, g


def loss_sums(loss_rows, n_first, scale, n_first_dev=None):
    """(total [0-dim], parts [2]) = scale * sums of the per-row losses, split at row n_first
    (or at the int64 device scalar n_first_dev)."""
    parts = torch.empty(2, device=loss_rows.device, dtype=torch.float32)
    total = torch.empty((), device=loss_rows.device, dtype=torch.float32)
    _check(lib().kge_loss_sums(ptr(loss_rows), loss_rows.numel(), int(n_first), ptr(n_first_dev), float(scale),
                               ptr(parts), ptr(total), stream()), "kge_loss_sums")
    return total, parts


def rank_metrics(hists: torch.Tensor, kmax: int) -> torch.Tensor:
    """kge_rank_metrics: [K, 3 + kmax] float64 rows (count, sum of ranks, sum of reciprocal ranks,
    hits@1..kmax) of K fp32 rank histograms [K, E]."""
    require_device(hists)
    if hists.dtype != torch.float32 or hists.dim() != 2 or hists.stride(1) != 1:
        hists = hists.float().contiguous()
    k, e = hists.shape
    out = torch.empty(k, 3 + kmax, device=hists.device, dtype=torch.float64)
    _check(lib().kge_rank_metrics(ptr(hists), hists.stride(0), k, e, int(kmax), ptr(out), stream()), "kge_rank_metrics")
    return out


def adjacent_or_cat(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """cat((a, b)) of two 1-D tensors -- without a copy when b already follows a in memory
    (rows of one index block)."""
    if (a.dtype == b.dtype and a.is_contiguous() and b.is_contiguous()
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
            and b.storage_offset() == a.storage_offset() + a.numel()):
        return a.as_strided((a.numel() + b.numel(),), (1,))
    return torch.cat((a, b))


def score_dot_bwd_q_planes(gp: GradPlanes, t, gscale=None, dq=None, accumulate=False):
    """dq (+)= gscale * G . t from gradient planes (kge_score_dot_bwd_q_planes)."""
    n, m, d = gp.n, gp.m, t.shape[1]
    if dq is None:
        dq = torch.empty(n, d, device=t.device, dtype=torch.float32)
        accumulate = False
    ws_n = lib().kge_score_dot_bwd_q_planes_ws_size(n, m, d)
    ws = torch.empty(ws_n, device=t.device, dtype=torch.float32)
    _check(lib().kge_score_dot_bwd_q_planes(ptr(gp.hi), ptr(gp.lo), gp.ldgp, ptr(t), rows(t), n, m, d, ptr(dq),
                                            rows(dq), int(accumulate), ptr(gscale), ptr(ws), ws_n, stream()),
           "kge_score_dot_bwd_q_planes")
    return dq


def score_dot_bwd_t_planes(gp: GradPlanes, q_hi, q_lo, dt, gscale=None, accumulate=False):
    """dt (+)= gscale * G^T . Q from gradient planes and query planes whose rows
    [n, n_pad) are zero (kge_score_dot_bwd_t_planes)."""
    if q_hi.shape[0] < gp.n_pad or q_lo.shape[0] < gp.n_pad or q_hi.stride(0) != q_lo.stride(0):
        raise ValueError("query planes must hold n_pad rows (zero past n) with equal row strides")
    _check(lib().kge_score_dot_bwd_t_planes(ptr(gp.hi), ptr(gp.lo), gp.ldgp, ptr(q_hi), ptr(q_lo), q_hi.stride(0),
                                            gp.n_pad, gp.m, dt.shape[1], ptr(dt), rows(dt), int(accumulate),
                                            ptr(gscale), stream()), "kge_score_dot_bwd_t_planes")
    return dt


def stage_i64(src_pinned, dst):
    """dst[:] = src_pinned (int64, host-pinned) by a kernel on the current stream (kge_stage_i64)."""
    if not (src_pinned.is_pinned() and dst.is_cuda and src_pinned.dtype == dst.dtype == torch.int64
            and src_pinned.is_contiguous() and dst.is_contiguous() and src_pinned.numel() == dst.numel()):
        raise ValueError("stage_i64: needs a contiguous pinned int64 source and a same-size CUDA int64 target")
    _check(lib().kge_stage_i64(ptr(src_pinned), ptr(dst), dst.numel(), stream()), "kge_stage_i64")


def lp_rows(w, idx, p):
    """row_sums[i] = sum_k |w[idx[i], k]|^p for p in 1 .. 4 (kge_lp_rows)."""
    require_device(w)
    idx = idx64(idx).reshape(-1)
    check_index(idx, w.shape[0], "penalty index")
    out = torch.empty(idx.numel(), device=w.device, dtype=torch.float32)
    _check(lib().kge_lp_rows(ptr(w), rows(w), ptr(idx), idx.numel(), w.shape[1], int(p), ptr(out), stream()),
           "kge_lp_rows")
    return out


def lp_rows_bwd(w, idx, p, gscale, coeff, dw):
    """dw[idx[i], :] += gscale * coeff * d|x|^p/dx at w[idx[i], :] (kge_lp_rows_bwd); gscale: a 0-dim /
    1-element fp32 device tensor or None."""
    idx = idx64(idx).reshape(-1)
    _check(lib().kge_lp_rows_bwd(ptr(w), rows(w), ptr(idx), idx.numel(), w.shape[1], int(p), ptr(gscale),
                                 float(coeff), ptr(dw), rows(dw), stream()), "kge_lp_rows_bwd")
    return dw


ADAGRAD_MULTI_MAX = 8


def adagrad_step_multi(items, eps, weight_decay, maximize):
    """One fused Adagrad step on several tensors in a single launch (kge_adagrad_step_multi).
    items: up to ADAGRAD_MULTI_MAX tuples (param, grad, state_sum, minus_clr) of contiguous fp32
    CUDA tensors."""
    k = len(items)
    if k == 0:
        return
    if k > ADAGRAD_MULTI_MAX:
        raise ValueError(f"at most {ADAGRAD_MULTI_MAX} tensors per launch")
    arr_p = (ctypes.c_void_p * k)(*[ptr(p) for p, _, _, _ in items])
    arr_g = (ctypes.c_void_p * k)(*[ptr(g) for _, g, _, _ in items])
    arr_s = (ctypes.c_void_p * k)(*[ptr(s) for _, _, s, _ in items])
    arr_n = (ctypes.c_int64 * k)(*[p.numel() for p, _, _, _ in items])
    arr_c = (ctypes.c_float * k)(*[float(c) for _, _, _, c in items])
    _check(lib().kge_adagrad_step_multi(k, arr_p, arr_g, arr_s, arr_n, arr_c, float(eps), float(weight_decay),
                                        int(bool(maximize)), stream()), "kge_adagrad_step_multi")


def adagrad_step(param, grad, state_sum, minus_clr, eps, weight_decay, maximize):
    """One fused Adagrad step in place on contiguous fp32 CUDA tensors (kge_adagrad_step)."""
    _check(lib().kge_adagrad_step(ptr(param), ptr(grad), ptr(state_sum), param.numel(), float(minus_clr),
                                  float(eps), float(weight_decay), int(bool(maximize)), stream()), "kge_adagrad_step")
