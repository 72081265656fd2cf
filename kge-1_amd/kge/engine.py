"""Autograd wrappers around libkgescore (the gfx950 HIP engine).

Two scoring ops cover every in-scope scorer:

* ``score_all``  -- prep + contraction against every row of a candidate table:
  the ``sp_`` / ``_po`` combines of RelationalScorer.score_emb (kge_model.py:120-182),
  fused with the LookupEmbedder gather when row indexes are given.  Bilinear models
  contract on MFMA (kge_score_dot), distance models on the VALU (kge_score_dist).
* ``score_spo``  -- row-wise triple scores (combine="spo").

Backward passes are the engine's backward kernels; when the query table and the
candidate table are the same tensor (the entity table), both gradient contributions are
accumulated into ONE dense buffer, the layout torch's embedding_dense_backward produces.
"""
from __future__ import annotations

import contextlib
import threading
from typing import Optional

import torch

from . import _lib as L

BILINEAR = (L.COMPLEX, L.DISTMULT, L.RESCAL, L.CP, L.SIMPLE)


def window(kind: int, direction: int, t: torch.Tensor) -> torch.Tensor:
    """The columns of the candidate rows a query contracts with (a view): CP scores
    subjects with the first half of an entity row and objects with the second (cp.py:17-19),
    so sp_ reads t[:, d/2:] and _po t[:, :d/2]; every other model the whole row."""
    if kind == L.CP:
        h = t.shape[1] // 2
        return t[:, h:] if direction == L.DIR_SP else t[:, :h]
    return t

#: When set to a list, every all-entities contraction launch appends a pair of HIP events
#: recorded on the launching stream right before / after it (bench.py's kernel timing).
KERNEL_EVENTS = None


def _timed(fn, *args, **kwargs):
    if KERNEL_EVENTS is None:
        return fn(*args, **kwargs)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    out = fn(*args, **kwargs)
    b.record()
    KERNEL_EVENTS.append((a, b))
    return out


class BatchStreams:
    """Round-robin HIP streams for batches that do not depend on one another (scoring and
    evaluation batches; never the steps of a training run).

    One all-entities contraction seldom fills the chip to the end: its tiles come in rounds of
    one per CU and the last round is partial, and the small launches around it (query
    preparation, true scores, rank counting) wait behind it on the same stream.  With the next
    batch on another stream its preparation and first tiles run on the CUs the previous batch
    has already left.  All streams have the default priority.

        with BatchStreams(device, 2) as bs:
            for i, batch in enumerate(batches):
                with bs.batch(i):
                    scores = model.score_sp(s, p)      # launched on stream i % 2

    Entering makes every stream wait for the caller's current stream, leaving makes the
    caller's stream wait for all of them.  A tensor made inside ``batch(i)`` belongs to that
    stream: use it there, or after the block has been left (and call ``record_stream`` on it
    if it is then freed while another stream may still read it).  ``count`` <= 1 or a CPU
    device: every batch stays on the caller's stream."""

    def __init__(self, device, count: int):
        self.device = torch.device(device)
        self.streams = []
        if count > 1 and self.device.type == "cuda":
            self.streams = [torch.cuda.Stream(device=self.device) for _ in range(count)]

    def __enter__(self):
        if self.streams:
            cur = self._caller = torch.cuda.current_stream(self.device)
            for st in self.streams:
                st.wait_stream(cur)
            self._turns = [_StreamTurn(st, cur) for st in self.streams]
        return self

    def __exit__(self, *exc):
        if self.streams:
            cur = torch.cuda.current_stream(self.device)
            for st in self.streams:
                cur.wait_stream(st)
            self._turns = None
        return False

    def batch(self, i: int):
        if not self.streams:
            return contextlib.nullcontext()
        turns = getattr(self, "_turns", None)
        if turns is None:  # used without the outer `with`: torch's own (slower) stream context
            return torch.cuda.stream(self.streams[i % len(self.streams)])
        return turns[i % len(turns)]


class _StreamTurn:
    """Makes one stream of a BatchStreams current for a block and the caller's stream current
    again afterwards: two set_stream calls, where torch.cuda.stream() also looks the current
    stream and device up on every entry (about 10 us per batch)."""

    __slots__ = ("stream", "caller")

    def __init__(self, stream, caller):
        self.stream, self.caller = stream, caller

    def __enter__(self):
        torch.cuda.set_stream(self.stream)
        return self.stream

    def __exit__(self, *exc):
        torch.cuda.set_stream(self.caller)
        return False


def dist_kind(kind: int, l_norm: float):
    """(kernel distance kind, sign) for TransE (-dist, transe.py:16-21) and RotatE
    (+dist, a quirk of the reference, rotate.py:28-60)."""
    if l_norm not in (1.0, 2.0):
        raise ValueError(f"l_norm={l_norm} not supported (1 or 2)")
    if kind == L.TRANSE:
        return (L.DIST_L1 if l_norm == 1.0 else L.DIST_L2), -1.0
    if kind == L.ROTATE:
        return (L.DIST_ROT_L1 if l_norm == 1.0 else L.DIST_ROT_L2), 1.0
    raise ValueError(kind)


def _rows(x: torch.Tensor) -> torch.Tensor:
    if x.dim() != 2 or x.stride(1) != 1:
        x = x.contiguous()
    return x


def _scores_forward(ctx, kind, direction, precision, l_norm, ent, eidx, rel, ridx, tab, tidx, out=None):
    """Query preparation + all-candidates scores (into ``out`` when given).  Returns
    (S, Q) with Q kept for the backward pass (empty when no gradient is needed)."""
    n = eidx.numel() if eidx is not None else ent.shape[0]
    d_e, d_r = ent.shape[1], rel.shape[1]
    if tab.shape[1] != d_e:
        raise ValueError(f"candidate dim {tab.shape[1]} != entity dim {d_e}")
    qw, tab_w = L.query_width(kind, d_e), window(kind, direction, tab)
    if kind in BILINEAR and L.split_ok(qw, tab_w, precision):
        # one pass emits Q (kept for backward only when a gradient is needed) and its
        # bf16 hi / lo planes for the split contraction
        need_q = any(ctx.needs_input_grad[i] for i in (4, 6, 8))
        q, q_hi, q_lo = L.prep_query_split(kind, direction, ent, eidx, rel, ridx, n, d_e, d_r, need_q)
        s = _timed(L.score_dot_split, q_hi, q_lo, tab_w, tidx, qw, out=out)
        if q is None:
            q = q_hi.new_empty(0)
    elif kind in BILINEAR:
        q = L.prep_query(kind, direction, ent, eidx, rel, ridx, n, d_e, d_r)
        s = _timed(L.contract, q, tab_w, tidx, precision, out=out)
    else:
        q = L.prep_query(kind, direction, ent, eidx, rel, ridx, n, d_e, d_r)
        dk, sign = dist_kind(kind, l_norm)
        s = _timed(L.score_dist, dk, sign, q, tab, tidx, out=out)
    ctx.meta = (kind, direction, precision, l_norm, n, d_e, d_r, ent is tab)
    return s, q


def _scores_backward(ctx, g, ent, eidx, rel, ridx, tab, tidx, q, gscale=None):
    """Gradients of the scores w.r.t. (ent, rel, tab) for dL/dS = gscale * g (gscale: an
    optional 0-dim device tensor, folded into the small operands instead of g)."""
    kind, direction, precision, l_norm, n, d_e, d_r, same = ctx.meta
    need_ent, need_rel, need_tab = ctx.needs_input_grad[4], ctx.needs_input_grad[6], ctx.needs_input_grad[8]
    d_tab = torch.zeros_like(tab) if (need_tab or (same and need_ent)) else None
    d_ent = d_tab if same else (torch.zeros_like(ent) if need_ent else None)
    d_rel = torch.zeros_like(rel) if need_rel else None
    dq = torch.zeros_like(q) if (need_ent or need_rel) else None
    if kind in BILINEAR:
        if dq is not None:
            L.score_dot_bwd_q(g, window(kind, direction, tab), tidx, precision, dq=dq, accumulate=False)
            if gscale is not None:
                dq.mul_(gscale)
        if d_tab is not None:
            L.score_dot_bwd_t(g, q if gscale is None else q * gscale, tidx, window(kind, direction, d_tab),
                              precision)
    else:
        dk, sign = dist_kind(kind, l_norm)
        L.score_dist_bwd(dk, sign, g if gscale is None else g * gscale, q, tab, tidx, dq, d_tab)
    if dq is not None:
        L.prep_query_bwd(kind, direction, ent, eidx, rel, ridx, n, d_e, d_r, dq, d_ent, d_rel)
    return None if same else d_ent, d_rel, d_tab


class _ScoreAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kind, direction, precision, l_norm, ent, eidx, rel, ridx, tab, tidx):
        ent, rel, tab = _rows(ent), _rows(rel), _rows(tab)
        s, q = _scores_forward(ctx, kind, direction, precision, l_norm, ent, eidx, rel, ridx, tab, tidx)
        ctx.save_for_backward(ent, eidx, rel, ridx, tab, tidx, q)
        return s

    @staticmethod
    def backward(ctx, g):
        ent, eidx, rel, ridx, tab, tidx, q = ctx.saved_tensors
        d_ent, d_rel, d_tab = _scores_backward(ctx, _rows(g), ent, eidx, rel, ridx, tab, tidx, q)
        return None, None, None, None, d_ent, None, d_rel, None, d_tab, None


class _ScoreXent(torch.autograd.Function):
    """scale * sum_i CE(S[i, :], labels[i]) with the all-candidates scores S never leaving
    the engine: S is written into a buffer whose rows are padded to 16 B, the loss kernel
    turns it in place into G = scale * (softmax(S) - onehot), and backward feeds G to the
    contraction's backward GEMMs (whose loads vectorise on the padded rows)."""

    @staticmethod
    def forward(ctx, kind, direction, precision, l_norm, ent, eidx, rel, ridx, tab, tidx, labels, l_ptr, smoothing,
                scale):
        ent, rel, tab = _rows(ent), _rows(rel), _rows(tab)
        n = eidx.numel() if eidx is not None else ent.shape[0]
        m = tidx.numel() if tidx is not None else tab.shape[0]
        buf = torch.empty(n, (m + 3) // 4 * 4, device=tab.device, dtype=torch.float32)
        s, q = _scores_forward(ctx, kind, direction, precision, l_norm, ent, eidx, rel, ridx, tab, tidx,
                               out=buf[:, :m])
        if l_ptr is None:  # index labels (1vsAll)
            loss_rows = L.softmax_xent(s, labels, scale, g=s)
        else:  # CSR positive lists (KvsAll)
            loss_rows = L.softmax_kl(s, l_ptr, labels, smoothing, scale, g=s)
        ctx.save_for_backward(ent, eidx, rel, ridx, tab, tidx, q, s)
        return loss_rows.sum() * scale

    @staticmethod
    def backward(ctx, gl):
        ent, eidx, rel, ridx, tab, tidx, q, g = ctx.saved_tensors
        d_ent, d_rel, d_tab = _scores_backward(ctx, g, ent, eidx, rel, ridx, tab, tidx, q, gscale=gl)
        return None, None, None, None, d_ent, None, d_rel, None, d_tab, None, None, None, None, None


class _FusedLoss(threading.local):
    """Which loss the fused passes of this thread compute: "kl" (softmax cross entropy / KL, the
    default) or "bce" (binary cross entropy with logits on scores + offset)."""
    kind = "kl"
    offset = 0.0


_LOSS = _FusedLoss()


@contextlib.contextmanager
def fused_loss_kind(kind: str, offset: float = 0.0):
    """Inside, the fused losses (score_all_xent and its relatives) compute ``kind`` instead of the
    softmax loss.  "bce" is served by the plane-fed pass only: where that does not apply the
    fused entry points return None and the caller scores and applies the loss unfused."""
    if kind not in ("kl", "bce"):
        raise ValueError(f"fused loss kind {kind!r}")
    prev = (_LOSS.kind, _LOSS.offset)
    _LOSS.kind, _LOSS.offset = kind, float(offset)
    try:
        yield
    finally:
        _LOSS.kind, _LOSS.offset = prev


class StackedQueries:
    """Two query batches stacked by rows: rows [0, n_a) are direction dir_a queries, rows
    [n_a, n) direction dir_b queries; eidx / ridx index all n rows.  n_a_dev (an int64 device
    scalar) overrides n_a on the device, so that a recorded step serves batches whose split
    differs (the host then only knows n)."""

    def __init__(self, dir_a, dir_b, eidx, ridx, n_a, n_a_dev=None):
        self.dir_a, self.dir_b, self.eidx, self.ridx, self.n_a, self.n_a_dev = dir_a, dir_b, eidx, ridx, n_a, n_a_dev

    @staticmethod
    def of(parts):
        """From one or two (direction, eidx, ridx) batches (no copy when the index vectors of
        the second already follow the first's in memory)."""
        if len(parts) == 1:
            d, e, r = parts[0]
            return StackedQueries(d, d, L.idx64(e), L.idx64(r), e.numel())
        (da, ea, ra), (db, eb, rb) = parts
        ea, ra, eb, rb = L.idx64(ea), L.idx64(ra), L.idx64(eb), L.idx64(rb)
        return StackedQueries(da, db, L.adjacent_or_cat(ea, eb), L.adjacent_or_cat(ra, rb), ea.numel())


class _ScoreXentPlanes(torch.autograd.Function):
    """The fused loss of one or two stacked query batches against every row of the entity table
    with its gradient kept as bf16 hi / lo PLANES (bf16x3 precision): ONE preparation launch
    writes the queries of both parts straight into one block of hi / lo planes, one
    contraction writes the scores, the loss kernel turns them in place into the planes of
    G = scale * dloss/dS, and the backward GEMMs read G and Q from those planes by LDS-DMA
    (kge_score_dot_bwd_q_planes / _t_planes): no fp32 copy of Q, no split per tile, dT written
    (not accumulated).  Returns (total, parts): total = scale * sum of all rows' losses carries
    the gradient; parts = scale * (sum of the first batch's rows, sum of the second's) is
    detached (for reporting).

    tab: the candidate rows when they are not the table the queries are gathered from (e.g.
    a dropout copy of the entity table, queries built from dropped rows); None: ent itself,
    whose gradient then collects both the candidates' and the queries' contributions."""

    @staticmethod
    def forward(ctx, kind, ent, rel, sq, labels, l_ptr, smoothing, scale, tab=None):
        ent, rel = _rows(ent), _rows(rel)
        cand = ent if tab is None else _rows(tab)
        n, m = sq.eidx.numel(), cand.shape[0]
        d_e, d_r = ent.shape[1], rel.shape[1]
        qw, tab_w = L.query_width(kind, d_e), window(kind, sq.dir_a, cand)
        n_pad, ld = L.planes_layout(n, m)
        buf = torch.empty(n_pad, ld, device=ent.device, dtype=torch.float32)
        ldp = (qw + 31) // 32 * 32
        hi = torch.empty(n_pad, ldp, device=ent.device, dtype=torch.bfloat16)
        lo = torch.empty_like(hi)
        if n_pad > n:  # K padding of the dT GEMM
            hi[n:].zero_()
            lo[n:].zero_()
        L.prep_query_split2(kind, sq.dir_a, sq.dir_b, sq.n_a, sq.n_a_dev, ent, sq.eidx, rel, sq.ridx, d_e, d_r,
                            out=(None, hi[:n], lo[:n]))
        _timed(L.score_dot_split, hi[:n], lo[:n], tab_w, None, qw, out=buf[:n, :m])
        loss_rows, _ = L.softmax_planes(buf, n, m, labels, l_ptr, smoothing, scale, _LOSS.kind, _LOSS.offset)
        ctx.meta = (kind, n, m, d_e, d_r, sq.dir_a, sq.dir_b, sq.n_a, sq.n_a_dev is not None, tab is None)
        ctx.save_for_backward(ent, rel, hi, lo, buf, sq.eidx, sq.ridx,
                              sq.n_a_dev if sq.n_a_dev is not None else sq.eidx.new_empty(0), cand)
        total, per_part = L.loss_sums(loss_rows, sq.n_a, scale, sq.n_a_dev)  # one launch, fixed order
        ctx.mark_non_differentiable(per_part)
        ctx.set_materialize_grads(False)  # no zero tensor for the detached parts' gradient
        return total, per_part

    @staticmethod
    def backward(ctx, g_total, _g_parts):
        if g_total is None:
            return (None,) * 9
        kind, n, m, d_e, d_r, dir_a, dir_b, n_a, has_dev, same = ctx.meta
        ent, rel, hi, lo, buf, eidx, ridx, n_a_dev, cand = ctx.saved_tensors
        gl = g_total.reshape(1).float().contiguous()  # read by the kernels from device memory
        gp = L.GradPlanes(buf, n, m)
        tab_w = window(kind, dir_a, cand)
        dq = L.score_dot_bwd_q_planes(gp, tab_w, gscale=gl)
        if tab_w.shape[1] == d_e:  # the GEMM covers every column: write, do not accumulate
            d_cand = torch.empty_like(cand)
            L.score_dot_bwd_t_planes(gp, hi, lo, d_cand, gscale=gl, accumulate=False)
        else:  # CP: the contraction sees one half of the entity rows
            d_cand = torch.zeros_like(cand)
            L.score_dot_bwd_t_planes(gp, hi, lo, window(kind, dir_a, d_cand), gscale=gl, accumulate=False)
        d_ent = d_cand if same else torch.zeros_like(ent)
        d_rel = torch.zeros_like(rel)
        L.prep_query_bwd2(kind, dir_a, dir_b, n_a, n_a_dev if has_dev else None, ent, eidx, rel, ridx, d_e, d_r, dq,
                          d_ent, d_rel)
        return (None, d_ent if ctx.needs_input_grad[1] else None, d_rel if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None if same or not ctx.needs_input_grad[8] else d_cand)


_ARANGE = {}
_ZEROS_I64 = {}


def _zeros_i64(n: int, device) -> torch.Tensor:
    """n int64 zeros on the device, kept and shared (read-only: the label vector "column 0")."""
    key = (n, str(device))
    if key not in _ZEROS_I64:
        if torch.cuda.is_current_stream_capturing():
            return torch.zeros(n, dtype=torch.int64, device=device)  # recorded with the step
        _ZEROS_I64[key] = torch.zeros(n, dtype=torch.int64, device=device)
    return _ZEROS_I64[key]


def _arange(n: int, device) -> torch.Tensor:
    """0 .. n-1 as int64 on the device, kept (a recorded step must not re-create it per replay)."""
    key = (n, str(device))
    if key not in _ARANGE:
        if torch.cuda.is_current_stream_capturing():
            return torch.arange(n, device=device, dtype=torch.int64)  # recorded with the step
        _ARANGE[key] = torch.arange(n, device=device, dtype=torch.int64)
    return _ARANGE[key]


def _planes_applicable(kind, precision, ent, direction) -> bool:
    """Whether the plane-fed fused loss serves this scorer: bf16x3, a bilinear model, layouts
    the split contraction and the DMA-staged GEMMs take, rows the loss kernel holds in registers."""
    if kind not in BILINEAR or precision != L.PREC_BF16X3 or ent.dim() != 2 or ent.stride(1) != 1:
        return False
    qw, tab_w = L.query_width(kind, ent.shape[1]), window(kind, direction, ent)
    return (L.split_ok(qw, tab_w, precision) and L.planes_ok(ent.shape[0]) and ent.shape[1] % 4 == 0
            and qw % 8 == 0 and ent.data_ptr() % 16 == 0)


def score_all_xent(kind: int, direction: int, precision: int, l_norm: float, ent: torch.Tensor,
                   eidx: Optional[torch.Tensor], rel: torch.Tensor, ridx: Optional[torch.Tensor],
                   tab: torch.Tensor, tidx: Optional[torch.Tensor], labels: torch.Tensor,
                   scale: float, l_ptr: Optional[torch.Tensor] = None, smoothing: float = 0.0) -> torch.Tensor:
    """scale * sum_i loss_i(score_all(...)[i, :]) fused with its gradient; a 0-dim tensor that
    backpropagates into ent / rel / tab.
      l_ptr None: labels[i] is the index of row i's target, loss_i = CrossEntropy -- the
                  1vsAll objective (kge/util/loss.py:192-208; kge/job/train.py:1042,1052);
      otherwise : labels[l_ptr[i]:l_ptr[i+1]] are row i's positives, loss_i = KL against
                  the smoothed, L1-normalised label row -- the KvsAll objective
                  (kge/util/loss.py:209-213; kge/job/train.py:715-721, 744-751)."""
    L.require_device(ent, rel, tab)
    if tab is ent and tidx is None and eidx is not None and _planes_applicable(kind, precision, ent, direction):
        total, _ = _ScoreXentPlanes.apply(kind, ent, rel, StackedQueries.of([(direction, eidx, ridx)]),
                                          L.idx64(labels), L.idx64(l_ptr), float(smoothing), float(scale))
        return total
    if (tab is not ent and tidx is None and eidx is None and ridx is None and ent.dim() == 2 and rel.dim() == 2
            and ent.shape[0] == rel.shape[0] and ent.shape[1] == tab.shape[1]
            and ent.dtype == rel.dtype == torch.float32
            and _planes_applicable(kind, precision, tab, direction)):
        # query rows given as tensors (one entity row and one relation row per query, e.g. after
        # dropout) against their own candidate table: the same plane-fed pass, rows taken in order
        rows = _arange(ent.shape[0], ent.device)
        total, _ = _ScoreXentPlanes.apply(kind, ent, rel, StackedQueries.of([(direction, rows, rows)]),
                                          L.idx64(labels), L.idx64(l_ptr), float(smoothing), float(scale), tab)
        return total
    if _LOSS.kind != "kl":
        return None  # only the plane-fed pass computes the other losses
    return _ScoreXent.apply(kind, direction, precision, float(l_norm), ent, L.idx64(eidx), rel, L.idx64(ridx),
                            tab, L.idx64(tidx), L.idx64(labels), L.idx64(l_ptr), float(smoothing), float(scale))


class _ScoreXent2(torch.autograd.Function):
    """Two query batches against the same table in ONE engine pass (the sp_ and _po halves of
    a 1vsAll / KvsAll step): the query rows of both are prepared into one [n_a + n_b, d]
    block, scored by one contraction, turned into G by one loss launch, and the backward
    runs one dQ GEMM and one dT GEMM over the stacked block.  dT = G^T Q over the
    concatenated K = n_a + n_b is written, not accumulated (no zero fill, no read), and the
    table gradient leaves as a single tensor (no autograd accumulation of two halves)."""

    @staticmethod
    def forward(ctx, kind, precision, ent, rel, dir_a, eidx_a, ridx_a, lab_a, lptr_a, dir_b, eidx_b, ridx_b,
                lab_b, lptr_b, smoothing, scale):
        ent, rel = _rows(ent), _rows(rel)
        n_a, n_b = eidx_a.numel(), eidx_b.numel()
        n, m = n_a + n_b, ent.shape[0]
        d_e, d_r = ent.shape[1], rel.shape[1]
        qw, tab_w = L.query_width(kind, d_e), window(kind, dir_a, ent)
        need = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        buf = torch.empty(n, (m + 3) // 4 * 4, device=ent.device, dtype=torch.float32)
        s = buf[:, :m]
        q = torch.empty(n, qw, device=ent.device, dtype=torch.float32) if need else None
        parts = ((dir_a, eidx_a, ridx_a, 0, n_a), (dir_b, eidx_b, ridx_b, n_a, n))
        if L.split_ok(qw, tab_w, precision):
            ldp = (qw + 31) // 32 * 32
            hi = torch.empty(n, ldp, device=ent.device, dtype=torch.bfloat16)
            lo = torch.empty_like(hi)
            for dr, ei, ri, r0, r1 in parts:
                L.prep_query_split(kind, dr, ent, ei, rel, ri, r1 - r0, d_e, d_r,
                                   out=(q[r0:r1] if need else None, hi[r0:r1], lo[r0:r1]))
            _timed(L.score_dot_split, hi, lo, tab_w, None, qw, out=s)
        else:
            if q is None:
                q = torch.empty(n, qw, device=ent.device, dtype=torch.float32)
            for dr, ei, ri, r0, r1 in parts:
                L.prep_query(kind, dr, ent, ei, rel, ri, r1 - r0, d_e, d_r, out=q[r0:r1])
            _timed(L.contract, q, tab_w, None, precision, out=s)
        if lptr_a is None:  # index labels (1vsAll)
            loss_rows = L.softmax_xent(s, torch.cat((lab_a, lab_b)), scale, g=s)
        else:  # CSR positives (KvsAll)
            l_ptr = torch.cat((lptr_a[:-1], lptr_b + lptr_a[-1]))
            loss_rows = L.softmax_kl(s, l_ptr, torch.cat((lab_a, lab_b)), smoothing, scale, g=s)
        ctx.meta = (kind, precision, n_a, n, d_e, d_r, dir_a, dir_b)
        ctx.save_for_backward(ent, rel, eidx_a, ridx_a, eidx_b, ridx_b, q if q is not None else s.new_empty(0), s)
        if 2 * n_a == n:  # equal parts (1vsAll): one reduction for both sums
            per_part = loss_rows.view(2, n_a).sum(1) * scale
        else:
            per_part = torch.stack((loss_rows[:n_a].sum(), loss_rows[n_a:].sum())) * scale
        total = per_part.sum()
        ctx.mark_non_differentiable(per_part)
        return total, per_part

    @staticmethod
    def backward(ctx, gl, _g_parts):
        kind, precision, n_a, n, d_e, d_r, dir_a, dir_b = ctx.meta
        ent, rel, eidx_a, ridx_a, eidx_b, ridx_b, q, g = ctx.saved_tensors
        tab_w = window(kind, dir_a, ent)
        # dL/dS = gl * G: the scalar is folded into the [n, d] operands
        dq = L.score_dot_bwd_q(g, tab_w, None, precision)
        dq.mul_(gl)
        q_s = q * gl
        if tab_w.shape[1] == d_e:  # the GEMM covers every column: write, do not accumulate
            d_ent = torch.empty_like(ent)
            L.score_dot_bwd_t(g, q_s, None, d_ent, precision, accumulate=False)
        else:
            d_ent = torch.zeros_like(ent)
            L.score_dot_bwd_t(g, q_s, None, window(kind, dir_a, d_ent), precision)
        d_rel = torch.zeros_like(rel)
        L.prep_query_bwd(kind, dir_a, ent, eidx_a, rel, ridx_a, n_a, d_e, d_r, dq[:n_a], d_ent, d_rel)
        L.prep_query_bwd(kind, dir_b, ent, eidx_b, rel, ridx_b, n - n_a, d_e, d_r, dq[n_a:], d_ent, d_rel)
        return (None, None, d_ent if ctx.needs_input_grad[2] else None, d_rel if ctx.needs_input_grad[3] else None,
                None, None, None, None, None, None, None, None, None, None, None, None)


def score_all_xent2(kind: int, precision: int, ent: torch.Tensor, rel: torch.Tensor, part_a, part_b, scale: float,
                    smoothing: float = 0.0):
    """Two query batches scored against every row of ent in ONE engine pass (the sp_ and _po
    halves of a 1vsAll / KvsAll step).  Returns (total, parts): total = scale * sum of both
    parts' per-row losses, a 0-dim tensor that backpropagates into ent / rel; parts = the two
    parts' shares of it, detached (for reporting).  part = (direction, eidx, ridx, labels,
    l_ptr) with the label conventions of score_all_xent (both parts index labels, or both
    CSR).  None when the batches cannot share one contraction (distance models; CP queries
    of different directions contract different halves of the rows) -- the caller runs them
    separately."""
    dir_a, eidx_a, ridx_a, lab_a, lptr_a = part_a
    dir_b, eidx_b, ridx_b, lab_b, lptr_b = part_b
    if kind not in BILINEAR or (kind == L.CP and dir_a != dir_b) or (lptr_a is None) != (lptr_b is None):
        return None
    L.require_device(ent, rel)
    if _planes_applicable(kind, precision, ent, dir_a):
        lab = L.adjacent_or_cat(L.idx64(lab_a), L.idx64(lab_b))
        l_ptr = None
        if lptr_a is not None:
            lptr_a, lptr_b = L.idx64(lptr_a), L.idx64(lptr_b)
            l_ptr = torch.cat((lptr_a[:-1], lptr_b + lptr_a[-1]))
        return _ScoreXentPlanes.apply(kind, ent, rel, StackedQueries.of([(dir_a, eidx_a, ridx_a), (dir_b, eidx_b, ridx_b)]),
                                      lab, l_ptr, float(smoothing), float(scale))
    if _LOSS.kind != "kl":
        return None
    return _ScoreXent2.apply(kind, precision, ent, rel, dir_a, L.idx64(eidx_a), L.idx64(ridx_a), L.idx64(lab_a),
                             L.idx64(lptr_a), dir_b, L.idx64(eidx_b), L.idx64(ridx_b), L.idx64(lab_b),
                             L.idx64(lptr_b), float(smoothing), float(scale))


def stacked_xent_applicable(kind: int, precision: int, ent: torch.Tensor, dir_a: int, dir_b: int) -> bool:
    """Whether score_all_xent_stacked serves this scorer / precision / table layout."""
    return (kind in BILINEAR and not (kind == L.CP and dir_a != dir_b)
            and _planes_applicable(kind, precision, _rows(ent), dir_a))


def score_all_xent_stacked(kind: int, precision: int, ent: torch.Tensor, rel: torch.Tensor, dir_a: int, dir_b: int,
                           eidx: torch.Tensor, ridx: torch.Tensor, n_a_dev: torch.Tensor, labels: torch.Tensor,
                           l_ptr: Optional[torch.Tensor], scale: float, smoothing: float = 0.0):
    """score_all_xent2 for query rows that are already stacked (rows [0, n_a) direction dir_a, the
    rest dir_b) with n_a an int64 device scalar -- nothing here depends on its value on the host,
    so the launches can be recorded once and replayed for batches whose split differs.  Served by
    the plane-fed path only: None when it does not apply to this scorer / precision / layout."""
    L.require_device(ent, rel, eidx, ridx, n_a_dev)
    if not stacked_xent_applicable(kind, precision, ent, dir_a, dir_b):
        return None
    sq = StackedQueries(dir_a, dir_b, L.idx64(eidx), L.idx64(ridx), 0, L.idx64(n_a_dev))
    return _ScoreXentPlanes.apply(kind, ent, rel, sq, L.idx64(labels), L.idx64(l_ptr), float(smoothing), float(scale))


def score_all(kind: int, direction: int, precision: int, l_norm: float, ent: torch.Tensor,
              eidx: Optional[torch.Tensor], rel: torch.Tensor, ridx: Optional[torch.Tensor],
              tab: torch.Tensor, tidx: Optional[torch.Tensor] = None) -> torch.Tensor:
    """S[i, j] = score of query i (prep(ent[eidx[i]], rel[ridx[i]])) against candidate
    tab[tidx[j]] (all rows of tab when tidx is None)."""
    L.require_device(ent, rel, tab)
    return _ScoreAll.apply(kind, direction, precision, float(l_norm), ent, L.idx64(eidx), rel,
                           L.idx64(ridx), tab, L.idx64(tidx))


class _NoGradCtx:
    """Stands in for an autograd context where no gradient is taken."""
    needs_input_grad = (False,) * 16
    meta = None


@torch.no_grad()
def score_parts(kind: int, precision: int, l_norm: float, ent: torch.Tensor, rel: torch.Tensor, parts,
                tidx: Optional[torch.Tensor] = None, want_q: bool = False, out: Optional[torch.Tensor] = None):
    """Several query batches against the same candidates, stacked by rows, without gradient
    (evaluation): parts = [(direction, eidx, ridx), ...]; returns (S, Q) with S [sum n_k, m]
    a view of a buffer whose rows are padded to 16 B (or ``out``, e.g. column blocks of a
    wider buffer) and Q the fp32 query rows [sum n_k, width] when want_q (None when the
    parts' queries do not share one layout).  Bilinear models whose parts contract the same
    columns run ONE query preparation block and ONE contraction; other models score the
    parts into their row blocks one by one."""
    L.require_device(ent, rel)
    ent, rel = _rows(ent), _rows(rel)
    tidx = L.idx64(tidx)
    parts = [(d, L.idx64(e), L.idx64(r)) for d, e, r in parts]
    sizes = [e.numel() for _, e, _ in parts]
    n = sum(sizes)
    m = tidx.numel() if tidx is not None else ent.shape[0]
    d_e, d_r = ent.shape[1], rel.shape[1]
    if out is None:
        out = torch.empty(n, (m + 3) // 4 * 4, device=ent.device, dtype=torch.float32)[:, :m]
    qw = L.query_width(kind, d_e)
    same_window = kind != L.CP or len({d for d, _, _ in parts}) == 1
    q = None
    if kind in BILINEAR and same_window:
        tab_w = window(kind, parts[0][0], ent)
        split = L.split_ok(qw, tab_w, precision)
        if want_q or not split:
            q = torch.empty(n, qw, device=ent.device, dtype=torch.float32)
        if split:
            ldp = (qw + 31) // 32 * 32
            hi = torch.empty(n, ldp, device=ent.device, dtype=torch.bfloat16)
            lo = torch.empty_like(hi)
            if len(parts) <= 2:  # one preparation launch for the stacked block
                sq = StackedQueries.of(parts)
                L.prep_query_split2(kind, sq.dir_a, sq.dir_b, sq.n_a, None, ent, sq.eidx, rel, sq.ridx, d_e, d_r,
                                    out=(q if want_q else None, hi, lo))
            else:
                r0 = 0
                for (dr, ei, ri), k in zip(parts, sizes):
                    L.prep_query_split(kind, dr, ent, ei, rel, ri, k, d_e, d_r,
                                       out=(q[r0:r0 + k] if want_q else None, hi[r0:r0 + k], lo[r0:r0 + k]))
                    r0 += k
            _timed(L.score_dot_split, hi, lo, tab_w, tidx, qw, out=out)
        else:
            r0 = 0
            for (dr, ei, ri), k in zip(parts, sizes):
                L.prep_query(kind, dr, ent, ei, rel, ri, k, d_e, d_r, out=q[r0:r0 + k])
                r0 += k
            _timed(L.contract, q, tab_w, tidx, precision, out=out)
        return out, (q if want_q else None)
    r0 = 0
    for (dr, ei, ri), k in zip(parts, sizes):
        _scores_forward(_NoGradCtx(), kind, dr, precision, l_norm, ent, ei, rel, ri, ent, tidx, out=out[r0:r0 + k])
        r0 += k
    return out, None


def rank_codes_applicable(kind: int, precision: int, ent: torch.Tensor) -> bool:
    """Whether rank_parts serves this scorer / table: a bilinear model whose queries contract
    with whole entity rows, on the split bf16x3 contraction."""
    ent = _rows(ent)
    return (kind in (L.COMPLEX, L.DISTMULT, L.RESCAL, L.SIMPLE) and ent.dim() == 2 and ent.stride(1) == 1
            and L.split_ok(L.query_width(kind, ent.shape[1]), ent, precision))


@torch.no_grad()
def rank_parts(kind: int, ent: torch.Tensor, rel: torch.Tensor, parts, true_parts, c0: int, c1: int, band_rel,
               t_norm_max, tab: Optional[torch.Tensor] = None):
    """The evaluation contraction with the ranking fused in (kge_score_dot_split_rank): the
    stacked query batches parts = [(direction, eidx, ridx), ...] (one or two) against entity rows
    [c0, c1), each score compared with its row's true score in the contraction's epilogue;
    true_parts = [(true_idx, true_score), ...] per batch.  band_rel None: plain comparison of
    the bf16x3 scores; else entries within band_rel |q_i| t_norm_max of the true score are marked
    for exact rescoring.  tab: the candidate rows when they are not rows [c0, c1) of ``ent`` -- a
    row-sharded job builds its queries from gathered rows (``ent``) and ranks them against its
    shard (``tab``, whose first row is entity c0).  Returns (codes [n, ldc] int32, fp32 query rows
    or None, n_a)."""
    L.require_device(ent, rel)
    ent, rel = _rows(ent), _rows(rel)
    parts = [(d, L.idx64(e), L.idx64(r)) for d, e, r in parts]
    n = sum(e.numel() for _, e, _ in parts)
    d_e, d_r = ent.shape[1], rel.shape[1]
    qw = L.query_width(kind, d_e)
    refine = band_rel is not None
    q = torch.empty(n, qw, device=ent.device, dtype=torch.float32) if refine else None
    ldp = (qw + 31) // 32 * 32
    hi = torch.empty(n, ldp, device=ent.device, dtype=torch.bfloat16)
    lo = torch.empty_like(hi)
    sq = StackedQueries.of(parts)
    if refine:  # the bands come out of the preparation launch
        _, _, _, band = L.prep_query_split2_band(kind, sq.dir_a, sq.dir_b, sq.n_a, ent, sq.eidx, rel, sq.ridx, d_e, d_r,
                                                 (q, hi, lo), band_rel, t_norm_max)
    else:
        L.prep_query_split2(kind, sq.dir_a, sq.dir_b, sq.n_a, None, ent, sq.eidx, rel, sq.ridx, d_e, d_r,
                            out=(q, hi, lo))
        band = torch.full((n,), -1.0, device=ent.device, dtype=torch.float32)
    codes = _timed(L.score_dot_split_rank, hi, lo, ent[c0:c1] if tab is None else _rows(tab), qw, sq.n_a, true_parts[0],
                   true_parts[1] if len(true_parts) > 1 else None, band, c0)
    return codes, q, sq.n_a


class _ScoreSpo(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kind, l_norm, ent, sidx, rel, pidx, oidx):
        ent, rel = _rows(ent), _rows(rel)
        d_e, d_r = ent.shape[1], rel.shape[1]
        out = L.score_spo(kind, l_norm, ent, sidx, rel, pidx, oidx, d_e, d_r)
        ctx.meta = (kind, l_norm, d_e, d_r)
        ctx.save_for_backward(ent, sidx, rel, pidx, oidx)
        return out

    @staticmethod
    def backward(ctx, g):
        kind, l_norm, d_e, d_r = ctx.meta
        ent, sidx, rel, pidx, oidx = ctx.saved_tensors
        d_ent = torch.zeros_like(ent) if ctx.needs_input_grad[2] else None
        d_rel = torch.zeros_like(rel) if ctx.needs_input_grad[4] else None
        if d_ent is not None or d_rel is not None:
            L.score_spo_bwd(kind, l_norm, ent, sidx, rel, pidx, oidx, d_e, d_r, g.contiguous(), d_ent, d_rel)
        return None, None, d_ent, None, d_rel, None, None


def score_spo(kind: int, l_norm: float, ent, sidx, rel, pidx, oidx) -> torch.Tensor:
    L.require_device(ent, rel)
    if not torch.is_grad_enabled() or not (ent.requires_grad or rel.requires_grad):
        # evaluation: no autograd node to build (about 10 us of host time per call)
        ent, rel = _rows(ent), _rows(rel)
        return L.score_spo(kind, float(l_norm), ent, L.idx64(sidx), rel, L.idx64(pidx), L.idx64(oidx), ent.shape[1],
                           rel.shape[1])
    return _ScoreSpo.apply(kind, float(l_norm), ent, L.idx64(sidx), rel, L.idx64(pidx), L.idx64(oidx))


def _cand_order(cand: torch.Tensor, n_rows: int):
    """(sorted candidate lists, their output columns) when ordering pays, else None.  Workgroup i
    of the candidate kernels gathers the table rows of query i's list; with every list ascending,
    the workgroups resident on an XCD sweep the table together and a row fetched for one query is
    found in that XCD's L2 by the others (measured at 512 x 1,025 candidates over 14,541 rows of
    4 KB: 78 % L2 hits instead of 10 %, forward 268 -> 190 us, dq 262 -> 149 us).  That needs
    rows that several of an XCD's queries use: (n / 8) * k uses of n_rows rows."""
    n, k = cand.shape
    # (inside a recorded step the lists are always ordered: the other grouping of the d_ent pass
    # goes through a library scan, whose memset nodes do not belong in a HIP graph)
    recording = cand.is_cuda and torch.cuda.is_current_stream_capturing() and n <= 4096 and k <= 8192
    if (k < 32 or n * k < 16 * n_rows) and not recording:
        return None
    return L.sort_rows(cand, n_rows) if k <= 8192 else tuple(torch.sort(cand, 1))


class _ScoreCand(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kind, direction, l_norm, ent, eidx, rel, ridx, cand):
        ent, rel = _rows(ent), _rows(rel)
        n = eidx.numel()
        d_e, d_r = ent.shape[1], rel.shape[1]
        q = L.prep_query(kind, direction, ent, eidx, rel, ridx, n, d_e, d_r)
        ent_w = window(kind, direction, ent)
        order = _cand_order(cand, ent.shape[0])
        if order is None:
            s = L.score_cand(kind, l_norm, direction, q, ent_w, cand)
            order = (cand.new_empty(0), cand.new_empty(0))
        else:
            s = L.score_cand_ordered(kind, l_norm, direction, q, ent_w, *order)
        ctx.meta = (kind, direction, l_norm, n, d_e, d_r)
        ctx.save_for_backward(ent, eidx, rel, ridx, cand, q, s, *order)
        return s

    @staticmethod
    def backward(ctx, g):
        kind, direction, l_norm, n, d_e, d_r = ctx.meta
        ent, eidx, rel, ridx, cand, q, s, srt, col = ctx.saved_tensors
        need_ent, need_rel = ctx.needs_input_grad[3], ctx.needs_input_grad[5]
        # Inside a training job's step (in_place_row_gradients) a dense gradient that an earlier
        # backward of the step left in .grad -- the other corrupted slot's -- takes this one's rows
        # where it stands: every kernel below accumulates, so neither a zero fill of a table-sized
        # buffer nor autograd's sum of two of them is needed.
        from .model.embedder.lookup_embedder import _in_place_ok

        def held(t):  # the dense gradient a leaf table already holds, if this backward may add to it
            g_t = t.grad if t.is_leaf and t.requires_grad else None
            return g_t if g_t is not None and g_t.is_contiguous() and _in_place_ok(g_t, t, torch.float32) else None

        ent_in_place = need_ent and held(ent) is not None
        rel_in_place = need_rel and held(rel) is not None
        d_ent = ent.grad if ent_in_place else (torch.zeros_like(ent) if need_ent else None)
        d_rel = rel.grad if rel_in_place else (torch.zeros_like(rel) if need_rel else None)
        dq = torch.empty_like(q) if (need_ent or need_rel) else None
        g = _rows(g.float())
        # candidate rows repeat across queries: grouped per entity (sort) instead of atomics
        ent_w = window(kind, direction, ent)
        d_ent_w = window(kind, direction, d_ent) if d_ent is not None else None
        ent_done = d_ent is not None and L.score_cand_bwd_ent(kind, l_norm, direction, q, ent_w, cand, s, g,
                                                              d_ent_w, sorted_lists=(srt, col))
        if not (dq is not None and srt.numel() and (ent_done or d_ent is None)
                and L.score_cand_bwd_q_ordered(kind, l_norm, direction, q, ent_w, srt, col, s, g, dq)):
            L.score_cand_bwd(kind, l_norm, direction, q, ent_w, cand, s, g, dq, None if ent_done else d_ent_w)
        if dq is not None:
            L.prep_query_bwd(kind, direction, ent, eidx, rel, ridx, n, d_e, d_r, dq, d_ent, d_rel)
        return (None, None, None, None if ent_in_place else d_ent, None, None if rel_in_place else d_rel, None, None)


def score_cand(kind: int, direction: int, l_norm: float, ent: torch.Tensor, eidx: torch.Tensor, rel: torch.Tensor,
               ridx: torch.Tensor, cand: torch.Tensor) -> torch.Tensor:
    """[n, k] scores of query i = prep(ent[eidx[i]], rel[ridx[i]]) against its own candidates
    ent[cand[i, :]] -- KgeModel.score_spo of the n * k triples that complete each query with
    a candidate (the negative-sampling "triple" scoring, kge/job/train.py:868-892) without
    materialising them."""
    L.require_device(ent, rel, cand)
    return _ScoreCand.apply(kind, direction, float(l_norm), ent, L.idx64(eidx), rel, L.idx64(ridx),
                            cand.long() if cand.dtype != torch.int64 else cand)


class _XentColumn0(torch.autograd.Function):
    """scale * sum_i CE(scores[i, :], label 0): the negative-sampling loss of a [n, 1 + N] score
    block whose column 0 is the positive -- KLDivWithSoftmaxKgeLoss on the one-hot label matrix
    (loss.py:192-213: the normalised labels stay one-hot, so KL == CE), one engine kernel for
    loss and gradient instead of torch's log_softmax / normalize / kl_div chain."""

    @staticmethod
    def forward(ctx, scores, scale):
        s = _rows(scores.float())
        n = s.shape[0]
        labels = _zeros_i64(n, s.device)  # kept: no fill kernel per call
        g = torch.empty_like(s)
        loss_rows = L.softmax_xent(s, labels, scale, g=g)
        ctx.save_for_backward(g)
        return loss_rows.sum() * scale

    @staticmethod
    def backward(ctx, grad):
        (g,) = ctx.saved_tensors
        return g * grad, None


def xent_column0(scores: torch.Tensor, scale: float) -> torch.Tensor:
    L.require_device(scores)
    return _XentColumn0.apply(scores, float(scale))


class _NsLossColumn0(torch.autograd.Function):
    """scale * sum_i loss_i of a [n, 1 + N] negative-sampling score block whose column 0 is the
    positive, for the margin-ranking loss (loss.py:227-250) and for bce (loss.py:137-158), one
    engine kernel for loss and gradient (kge_ns_loss) instead of torch's index / repeat chains."""

    @staticmethod
    def forward(ctx, scores, kind, arg, scale):
        s = _rows(scores.float())
        loss_rows, g = L.ns_loss(kind, s, arg, scale)
        ctx.save_for_backward(g)
        return loss_rows.sum() * scale

    @staticmethod
    def backward(ctx, grad):
        (g,) = ctx.saved_tensors
        return g * grad, None, None, None


def ns_loss_column0(scores: torch.Tensor, kind: str, arg: float, scale: float) -> torch.Tensor:
    """kind "margin_ranking" (arg = the margin) or "bce" (arg = the offset added to the scores)."""
    L.require_device(scores)
    return _NsLossColumn0.apply(scores, {"margin_ranking": L.NS_MARGIN, "bce": L.NS_BCE}[kind], float(arg),
                                float(scale))


def score_spo_emb(kind: int, l_norm: float, s_emb, p_emb, o_emb) -> torch.Tensor:
    """combine="spo" on embedding rows: s, o stacked into one table."""
    n = p_emb.shape[0]
    so = torch.cat((s_emb, o_emb), 0)
    ar = torch.arange(n, device=p_emb.device)
    return score_spo(kind, l_norm, so, ar, p_emb, ar, ar + n)
