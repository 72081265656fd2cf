"""Entity-table row sharding over the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  GPU k owns
entity rows [k*ceil(E/W), (k+1)*ceil(E/W)) -- exactly the reference's
``entity_ranking.chunk_size`` decomposition (entity_ranking.py:153-216), whose per-chunk
rank/tie counts sum exactly.  The relation table is replicated.

Data path of one all-entities scoring step for a global batch of W*B queries (each rank
contributes B):
  1. all_gather of the (entity, relation) query indexes       -- W*B*16 bytes
  2. the owner of each query entity row computes the query vector q = prep(e, r), the
     others contribute zeros; all_reduce(SUM) of Q [W*B, d]     -- W*B*d*4 bytes
     (x + 0 + ... + 0 == x exactly, so every rank holds bit-identical Q)
  3. local contraction against the rank's shard: S_k [W*B, E_k] on the engine.
Entity ranking then needs only an all_reduce(SUM) of the int64 greater/tie counts
(rank_counts over the local shard) -- no score ever crosses the link.  The
"all-gather of per-shard top-k" in the north star is ``topk``: per-shard top-k (score,
global id), all_gather, merge.

The compute ops are injected (``ops``) so the exchange logic is testable with the gloo
backend on CPU (tests/test_sharded_gloo.py); the default ops are the HIP engine.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist


# ---- collectives.  RCCL ("nccl") moves device memory directly.  gloo is given CPU tensors
# only: device tensors are staged through host memory with synchronous copies (rehearsing
# several ranks on one GPU; gloo collectives on device tensors are not used).


def _staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_reduce(t: torch.Tensor, op=None, group=None):
    op = dist.ReduceOp.SUM if op is None else op
    if _staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t


def all_gather(outs, t: torch.Tensor, group=None):
    if _staged(t, group):
        hs = [torch.empty(o.shape, dtype=o.dtype) for o in outs]
        dist.all_gather(hs, t.cpu(), group=group)
        for o, h in zip(outs, hs):
            o.copy_(h)
    else:
        dist.all_gather(outs, t, group=group)
    return outs


def all_gather_into_tensor(out: torch.Tensor, t: torch.Tensor, group=None, async_op: bool = False):
    """Returns a work handle when async_op (None when the call completed synchronously)."""
    if _staged(t, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, t.cpu(), group=group)
        out.copy_(h)
        return None
    return dist.all_gather_into_tensor(out, t, group=group, async_op=async_op)


def reduce_scatter_tensor(out: torch.Tensor, t: torch.Tensor, group=None):
    """out = this rank's block of the sum over ranks of t ([W * len(out), ...], rank-major blocks).
    RCCL: one reduce_scatter.  gloo has no reduce_scatter: the rehearsal path all-reduces a host
    copy and keeps the rank's block (same result, more bytes)."""
    if dist.get_backend(group) == "gloo":
        h = t.cpu() if t.is_cuda else t.clone()
        dist.all_reduce(h, group=group)
        r, n = dist.get_rank(group), out.shape[0]
        out.copy_(h[r * n:(r + 1) * n])
    else:
        dist.reduce_scatter_tensor(out, t, group=group)
    return out


class ExchangePlan:
    """Where every query row of a global batch lives during the owner-major exchange.

    The m query rows (every rank holds the same index batch) are grouped by the rank that owns
    their entity row; rank w contributes its c_w rows in one all_gather of cap = max_w c_w rows
    per rank (equal block sizes: one plain all-gather), so row i of the batch sits at
    ``slot[i] = owner_i * cap + (its position among owner_i's rows)`` of the gathered
    [W * cap, d] block.  The same layout carries the partial query gradients back: one
    reduce_scatter hands every owner the summed gradients of its own rows.  Built on the host
    from the batch's entity ids (numpy, no device sync) and uploaded as one int64 vector."""

    def __init__(self, e_ids, per: int, world: int, rank: int, device):
        import numpy as np

        e = np.asarray(e_ids, dtype=np.int64).reshape(-1)
        m = e.shape[0]
        owner = e // per if m else e
        counts = np.bincount(owner, minlength=world)[:world] if m else np.zeros(world, np.int64)
        order = np.argsort(owner, kind="stable")
        starts = np.zeros(world + 1, np.int64)
        np.cumsum(counts, out=starts[1:])
        self.cap = int(max(1, counts.max() if m else 1))
        slot = np.empty(m, np.int64)
        slot[order] = owner[order] * self.cap + (np.arange(m, dtype=np.int64) - starts[owner[order]])
        mine = order[starts[rank]:starts[rank + 1]]  # this rank's rows, ascending batch position
        self.count = int(mine.shape[0])
        self.m = m
        packed = torch.from_numpy(np.concatenate([slot, mine]))
        if torch.device(device).type == "cuda":
            packed = packed.pin_memory().to(device, non_blocking=True)
        self.slot, self.mine = packed[:m], packed[m:]
        self.mine_host = mine


def bce_grad_block(s, c0, labels, offset, scale, g):
    """train.loss bce on one shard's block of a 1vsAll batch, in torch ops (small blocks, and the CPU
    ops of the gloo tests): g = scale * (sigmoid(s + offset) - y) with y one-hot at column
    labels[i] - c0 when that falls into the block; returns the block's unscaled loss sum,
    sum_ij softplus(x_ij) - y_ij x_ij (loss.py:137-158), as a 0-dim float64 tensor."""
    x = s + offset if offset != 0.0 else s
    m = s.shape[1]
    col = labels - c0
    inside = (col >= 0) & (col < m)
    colc = col.clamp(0, m - 1).unsqueeze(1)
    hot = torch.gather(x, 1, colc).squeeze(1)
    loss = torch.nn.functional.softplus(x).double().sum() - torch.where(inside, hot, torch.zeros_like(hot)).double().sum()
    out = torch.sigmoid(x) * scale
    out.scatter_add_(1, colc, torch.where(inside, -scale, 0.0).to(out.dtype).unsqueeze(1))
    g.copy_(out)
    return loss


class EngineOps:
    """Default compute: libkgescore."""

    def __init__(self, kind: int, precision: int, l_norm: float = 1.0):
        from . import _lib

        self.L = _lib
        self.kind = kind
        self.precision = precision
        self.l_norm = l_norm

    def prep(self, direction, ent, eidx, rel, ridx):
        n = eidx.numel()
        return self.L.prep_query(self.kind, direction, ent, eidx, rel, ridx, n, ent.shape[1], rel.shape[1])

    def score(self, q, tab, out=None):
        from .engine import BILINEAR, dist_kind

        if self.kind in BILINEAR:
            return self.L.contract(q, tab, None, self.precision, out=out)
        dk, sign = dist_kind(self.kind, self.l_norm)
        return self.L.score_dist(dk, sign, q, tab, None, out=out)

    # ---- query rows as bf16 hi / lo planes packed [hi | lo] per row: what the split contraction
    # reads, in ONE buffer to exchange (the same bytes as the fp32 rows, and no split pass after)
    def planes_ok(self, ent, direction) -> bool:
        from .engine import BILINEAR, window

        qw = self.L.query_width(self.kind, ent.shape[1])
        return (self.kind in BILINEAR and ent.dim() == 2 and ent.stride(1) == 1
                and self.L.split_ok(qw, window(self.kind, direction, ent), self.precision))

    def prep_planes(self, direction, ent, eidx, rel, ridx, eidx_base=0):
        """eidx: global row ids of the table whose rows [eidx_base, eidx_base + len(ent)) ent holds."""
        return self.L.prep_query_packed(self.kind, direction, ent, eidx, rel, ridx, eidx_base)

    def score_planes(self, packed, tab, out=None):
        return self.L.score_dot_packed(packed, tab, tab.shape[1], out=out)

    # ---- vocab-parallel 1vsAll training on gradient planes: the shard's slice of G leaves the
    # loss kernel as bf16 hi / lo planes and the backward GEMMs read G and the query rows by
    # LDS-DMA (no per-tile split of fp32 operands)
    def train_planes_ok(self, ent, direction) -> bool:
        from .engine import BILINEAR, window

        if self.kind not in BILINEAR or self.precision != self.L.PREC_BF16X3 or ent.dim() != 2 or ent.stride(1) != 1:
            return False
        qw, tab_w = self.L.query_width(self.kind, ent.shape[1]), window(self.kind, direction, ent)
        return (self.L.split_ok(qw, tab_w, self.precision) and ent.shape[1] % 4 == 0 and qw % 8 == 0
                and ent.data_ptr() % 16 == 0 and tab_w.shape[1] == qw)

    def split_padded(self, q):
        """bf16 hi / lo planes of the query rows, padded with zero rows to the GEMMs' K stage."""
        n, d = q.shape
        n_pad = (n + 31) // 32 * 32
        ld = (d + 31) // 32 * 32
        hi = torch.empty(n_pad, ld, device=q.device, dtype=torch.bfloat16)
        lo = torch.empty_like(hi)
        if n_pad > n:
            hi[n:].zero_()
            lo[n:].zero_()
        self.L.split_rows_into(q, hi[:n], lo[:n])
        return hi, lo

    def score_split(self, hi, lo, n, tab, out=None):
        return self.L.score_dot_split(hi[:n], lo[:n], tab, None, tab.shape[1], out=out)

    def softmax_grad_planes(self, s, c0, labels, lse, scale):
        return self.L.softmax_grad_planes(s, c0, labels, lse, scale)

    def score_bwd_planes(self, gp, hi, lo, tab, d_tab, dq=None):
        """Returns dq = G . tab (written, into dq when given); d_tab += G^T . Q."""
        dq = self.L.score_dot_bwd_q_planes(gp, tab, dq=dq)
        self.L.score_dot_bwd_t_planes(gp, hi, lo, d_tab, accumulate=True)
        return dq

    def bce_grad_planes(self, s, c0, labels, offset, scale):
        """(unscaled loss sum of this shard's block, gradient planes) of train.loss bce."""
        return self.L.bce_grad_planes(s, c0, labels, offset, scale)

    def bce_grad(self, s, c0, labels, offset, scale, g):
        return bce_grad_block(s, c0, labels, offset, scale, g)

    def row_stats(self, s, c0, labels):
        return self.L.softmax_row_stats(s, c0, labels)

    def softmax_grad(self, s, c0, labels, lse, scale, g):
        return self.L.softmax_grad(s, c0, labels, lse, scale, g)

    def score_bwd(self, g, q, tab, dq, d_tab):
        """dq = d/dq <g, S(q, tab)> (written), d_tab += d/dtab <g, S>."""
        from .engine import BILINEAR, dist_kind

        if self.kind in BILINEAR:
            self.L.score_dot_bwd_q(g, tab, None, self.precision, dq=dq, accumulate=False)
            self.L.score_dot_bwd_t(g, q, None, d_tab, self.precision)
        else:
            dq.zero_()
            dk, sign = dist_kind(self.kind, self.l_norm)
            self.L.score_dist_bwd(dk, sign, g, q, tab, None, dq, d_tab)

    def prep_bwd(self, direction, ent, eidx, rel, ridx, dq, d_ent, d_rel):
        n = eidx.numel()
        self.L.prep_query_bwd(self.kind, direction, ent, eidx, rel, ridx, n, ent.shape[1], rel.shape[1], dq, d_ent,
                              d_rel)

    def spo(self, ent_s, rel, p, ent_o):
        n = p.numel()
        ar = torch.arange(n, device=rel.device)
        so = torch.cat((ent_s, ent_o), 0)
        return self.L.score_spo(self.kind, self.l_norm, so, ar, rel, p, ar + n, so.shape[1], rel.shape[1])

    def spo_stacked(self, rows, rel, p, swap=False):
        """spo on a block that already holds the n subject rows followed by the n object rows
        (swap: scored as (o, p, s), the reciprocal model's second direction): no copy, cached indexes."""
        from .engine import _arange

        n = p.numel()
        ar = _arange(2 * n, rows.device)
        a, b = (ar[n:], ar[:n]) if swap else (ar[:n], ar[n:])
        return self.L.score_spo(self.kind, self.l_norm, rows, a, rel, p, b, rows.shape[1], rel.shape[1])

    def rank_counts(self, s, c0, true_idx, true_score, fp, fc, tp, tc, greater, ties):
        self.L.rank_counts(s, c0, true_idx, true_score, fp, fc, tp, tc, greater, ties)

    def rank_hist_multi(self, greater, ties, rows_per_hist, tie_handling, ranks, hists):
        self.L.rank_hist_multi(greater, ties, rows_per_hist, tie_handling, ranks, hists)

    def rank_rows(self, s, n_a, c0, part_a, part_b, f_col, t_col, greater, ties, refine=None, codes=None, m=None):
        """Adds the stacked block's counts over columns [c0, c0 + m) (kge_rank_rows on a score
        block s, or kge_rank_rows_codes on the code block of rank_codes)."""
        self.L.rank_rows(s, n_a, c0, part_a, part_b, f_col, t_col, greater, ties, accumulate=True, refine=refine,
                         codes=codes, m=m)

    def rank_codes(self, q, tab, n_a, true_a, true_b, refinement, c0):
        """The stacked fp32 query rows q against the rows of tab (columns c0 .. of the entity
        axis) with the ranking fused into the contraction (kge_score_dot_split_rank): 2-bit codes
        instead of a score block, or None when this scorer / layout is not served."""
        from .engine import rank_codes_applicable

        if not rank_codes_applicable(self.kind, self.precision, tab) or q.shape[1] != tab.shape[1]:
            return None
        hi, lo = self.L.split_rows(q)
        if refinement is not None:
            band = self.L.rank_band(q, refinement[0], refinement[1])
        else:
            band = torch.full((q.shape[0],), -1.0, device=q.device, dtype=torch.float32)
        return self.L.score_dot_split_rank(hi, lo, tab, q.shape[1], n_a, true_a, true_b, band, c0)

    def rank_codes_rows(self, rows, rel, p_a, p_b, dir_b, tab, n_a, true_a, true_b, refinement, c0):
        """rank_codes with the query preparation folded in: the stacked queries (direction 0 from
        rows[:n_a] with relations p_a, direction dir_b from rows[n_a:] with p_b) are prepared
        straight into bf16 planes by ONE launch (engine.rank_parts), no fp32 stack / split pass.
        Returns (codes, fp32 query rows or None) or None when not served."""
        from . import engine

        if not engine.rank_codes_applicable(self.kind, self.precision, tab) or rows.shape[1] != tab.shape[1]:
            return None
        ar = engine._arange(rows.shape[0], rows.device)
        codes, q, _ = engine.rank_parts(
            self.kind, rows, rel, [(0, ar[:n_a], p_a), (dir_b, ar[n_a:], p_b)], [true_a, true_b], c0,
            c0 + tab.shape[0], refinement[0] if refinement is not None else None,
            refinement[1] if refinement is not None else None, tab=tab)
        return codes, q

    def refinement(self, ent):
        """(band relative to |q_i| max_j |t_j|, device scalar max_j |t_j| over ``ent``) when the
        near-tie rescoring of kge_rank_rows applies to scores contracted against ``ent`` -- a
        bf16x3 contraction of fp32 query rows with whole, float4-readable entity rows -- else
        None: the caller then ranks exact-fp32 scores."""
        from .job.entity_ranking import refine_band

        if (self.precision != self.L.PREC_BF16X3
                or self.kind not in (self.L.COMPLEX, self.L.DISTMULT, self.L.RESCAL, self.L.SIMPLE)
                or ent.dim() != 2 or ent.stride(1) != 1 or ent.shape[1] % 4 or ent.stride(0) % 4
                or ent.data_ptr() % 16 or ent.shape[0] == 0):
            return None
        return refine_band(ent.shape[1]), self.L.row_norm_max(ent)


def sharding_enabled(config) -> bool:
    """Whether jobs run entity-row-sharded: engine.row_sharded "auto" shards whenever a
    torch.distributed world larger than one process exists (one process per GPU, as torchrun
    starts them); "on" demands an initialised process group and shards over it whatever its
    size (a world of one is the degenerate single-shard case); "off" never shards."""
    mode = config.check("engine.row_sharded", ["auto", "on", "off"])
    if mode == "off":
        return False
    ready = dist.is_available() and dist.is_initialized()
    if mode == "on":
        if not ready:
            raise RuntimeError("engine.row_sharded is 'on' but torch.distributed is not initialised "
                               "(start one process per GPU with torchrun)")
        return True
    return ready and dist.get_world_size() > 1


def engine_ops_for(model):
    """EngineOps of a KgeModel's scorer (its engine kernel kind, precision and norm)."""
    scorer = model.get_scorer()
    if scorer.engine_kind is None:
        raise NotImplementedError(f"{type(scorer).__name__} has no engine kernels: row sharding is not available")
    return EngineOps(scorer.engine_kind, scorer.precision(), scorer.l_norm())


def shard_bounds(num_entities: int, world: int, rank: int):
    per = math.ceil(num_entities / world)
    lo = min(num_entities, rank * per)
    return lo, min(num_entities, lo + per)


class _Ticket:
    """An exchange in flight (submit_queries_local): the collective's work handle (None once
    waited for, or when it completed synchronously), the gathered rows, this rank's rows (kept
    alive until the gather has read them), the query direction and whether the rows are packed
    bf16 planes."""
    __slots__ = ("work", "q_all", "q_local", "direction", "planes")

    def __init__(self, work, q_all, q_local, direction, planes):
        self.work, self.q_all, self.q_local, self.direction, self.planes = work, q_all, q_local, direction, planes


class RowShardedScorer:
    #: smallest [n, E_k] score block whose training gradient is kept as bf16 planes
    PLANES_MIN_ELEMS = 1 << 25
    #: the same for train.loss bce (whose fp32 gradient is formed by torch ops: 0.95 ms per step at
    #: 2,048 x 14,541 against 0.53 ms through the planes)
    BCE_PLANES_MIN_ELEMS = 1 << 20

    def __init__(self, ent_shard: torch.Tensor, lo: int, hi: int, num_entities: int, rel: torch.Tensor, ops,
                 group=None):
        self.ent = ent_shard
        self.lo, self.hi = lo, hi
        self.E = num_entities
        self.rel = rel
        self.ops = ops
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    # ---------------------------------------------------------------- helpers
    def _win(self, direction: int, t: torch.Tensor) -> torch.Tensor:
        """Entity-row columns the queries of this direction contract with (CP: a half)."""
        from .engine import window

        kind = getattr(self.ops, "kind", None)
        return t if kind is None else window(kind, direction, t)

    def _all_gather_1d(self, x: torch.Tensor) -> torch.Tensor:
        out = [torch.empty_like(x) for _ in range(self.world)]
        all_gather(out, x.contiguous(), group=self.group)
        return torch.cat(out)

    def _owned_rows(self, ids: torch.Tensor):
        owned = (ids >= self.lo) & (ids < self.hi)
        local = (ids - self.lo).clamp(0, max(0, self.hi - self.lo - 1))
        return owned, local

    def gather_rows(self, ids: torch.Tensor) -> torch.Tensor:
        """Full entity rows for global ids (every rank gets bit-identical rows)."""
        owned, local = self._owned_rows(ids)
        rows = self.ent[local]
        rows = torch.where(owned[:, None], rows, torch.zeros_like(rows))
        all_reduce(rows, group=self.group)
        return rows

    def queries(self, e: torch.Tensor, p: torch.Tensor, direction: int):
        """Steps 1-2: global index exchange + owner-computed query rows (all_reduce)."""
        e_all = self._all_gather_1d(e)
        p_all = self._all_gather_1d(p)
        owned, local = self._owned_rows(e_all)
        q = self.ops.prep(direction, self.ent, local, self.rel, p_all)
        q = torch.where(owned[:, None], q, torch.zeros_like(q))
        all_reduce(q, group=self.group)
        return q, e_all, p_all

    # ---------------------------------------------------------------- scoring
    def score_sp(self, s: torch.Tensor, p: torch.Tensor, direction: int = 0) -> torch.Tensor:
        """Local shard of the global score matrix: [W*B, hi - lo]."""
        q, _, _ = self.queries(s, p, direction)
        return self.ops.score(q, self._win(direction, self.ent))

    def queries_local(self, e: torch.Tensor, p: torch.Tensor, direction: int = 0) -> torch.Tensor:
        """Shard-affine batches (a loader that routes each query to the rank owning its
        entity row, e.g. 1vsAll sp_ queries by subject): every rank computes its own B
        query rows and one all_gather hands all W*B rows to every rank -- half the link
        traffic of the owner-computes all_reduce in ``queries``."""
        owned, local = self._owned_rows(e)
        if not bool(owned.all()):
            raise ValueError("queries_local needs every query entity in this rank's shard")
        q = self.ops.prep(direction, self.ent, local, self.rel, p)
        out = torch.empty((self.world * q.shape[0], q.shape[1]), dtype=q.dtype, device=q.device)
        all_gather_into_tensor(out, q.contiguous(), group=self.group)
        return out

    def score_sp_local(self, s: torch.Tensor, p: torch.Tensor, direction: int = 0) -> torch.Tensor:
        """score_sp for shard-affine batches: [W*B, hi - lo] local slice of the scores."""
        return self.ops.score(self.queries_local(s, p, direction), self._win(direction, self.ent))

    def submit_queries_local(self, e: torch.Tensor, p: torch.Tensor, direction: int = 0):
        """Start the exchange of a shard-affine batch (queries_local) without waiting for it:
        the query rows are prepared on the current stream and their all_gather is issued
        asynchronously (RCCL runs it on its own stream), so the caller can score the previous
        batch meanwhile.  Returns a ticket for ``score_submitted``.

        e, p may hold SEVERAL batches back to back (k B queries): one preparation launch and
        one collective then serve k scoring steps -- fewer, larger collectives: the per-call
        host cost of the collective is paid once per k steps (``score_submitted(ticket, part)``
        scores the gathered rows in k blocks)."""
        # shard-affine by contract: every query entity is one of this rank's rows
        planes = getattr(self.ops, "planes_ok", None) is not None and self.ops.planes_ok(self.ent, direction)
        if planes:  # bf16 hi / lo planes, packed per row: no split pass on the receiving side
            q = self.ops.prep_planes(direction, self.ent, e, self.rel, p, eidx_base=self.lo)
        else:
            q = self.ops.prep(direction, self.ent, e - self.lo, self.rel, p).contiguous()
        out = torch.empty((self.world * q.shape[0], q.shape[1]), dtype=q.dtype, device=q.device)
        work = all_gather_into_tensor(out, q, group=self.group, async_op=True)
        return _Ticket(work, out, q, direction, planes)

    def score_submitted(self, ticket, part=None) -> torch.Tensor:
        """Local slice [W*B, hi - lo] of the scores of a batch started by submit_queries_local.

        part = (x, k): only the x-th of k equal blocks of the gathered rows, for a ticket of k
        batches per rank.  The gathered rows are rank-major (rank 0's k B rows, then rank 1's,
        ...), so block x holds W B consecutive rows: the queries of ranks and local batches
        (w, j) with x W <= w k + j < (x + 1) W.  Over x = 0 .. k-1 every submitted query is
        scored exactly once; which step scores it is the only difference to k single-batch
        tickets."""
        if ticket.work is not None:
            ticket.work.wait()  # the current stream waits for the gather; the host does not block
            ticket.work = None
        q_all = ticket.q_all
        if part is not None:
            x, k = part
            if q_all.shape[0] % k or not 0 <= x < k:
                raise ValueError(f"part {part} of {q_all.shape[0]} gathered rows")
            rows = q_all.shape[0] // k
            q_all = q_all[x * rows:(x + 1) * rows]
        if ticket.planes:
            return self.ops.score_planes(q_all, self._win(ticket.direction, self.ent))
        return self.ops.score(q_all, self._win(ticket.direction, self.ent))

    def topk(self, scores_local: torch.Tensor, k: int):
        """All-gather of per-shard top-k (score, global entity id), merged on every rank."""
        kk = min(k, scores_local.shape[1])
        v, i = torch.topk(scores_local, kk, dim=1)
        i = i + self.lo
        if kk < k:  # pad so every rank contributes the same shape
            pad = k - kk
            v = torch.cat([v, torch.full((v.shape[0], pad), -math.inf, device=v.device)], 1)
            i = torch.cat([i, torch.full((i.shape[0], pad), -1, device=i.device, dtype=i.dtype)], 1)
        vs = [torch.empty_like(v) for _ in range(self.world)]
        is_ = [torch.empty_like(i) for _ in range(self.world)]
        all_gather(vs, v.contiguous(), group=self.group)
        all_gather(is_, i.contiguous(), group=self.group)
        V, I = torch.cat(vs, 1), torch.cat(is_, 1)
        tv, ti = torch.topk(V, k, dim=1)
        return tv, torch.gather(I, 1, ti)

    # ---------------------------------------------------------------- training
    def train_1vsall_grads(self, s: torch.Tensor, p: torch.Tensor, o: torch.Tensor):
        """Vocab-parallel 1vsAll: every rank passes its
        own B triples; the global batch is the W*B gathered triples and the objective is
        the reference's  sum over (sp_, _po) of CE(scores, target) / (W*B)
        (train.py:1032-1062 with batch W*B).  Per direction:
          all_gather triples -> owner-computed Q (all_reduce) -> local logits [W*B, E_k]
          -> local (max, sumexp, target) -> all_reduce MAX / SUM / SUM (3 x W*B floats)
          -> lse -> local G_k = scale (softmax - onehot) in place of the logits
          -> dQ = sum_k G_k E_k (all_reduce, W*B x d) ; dE_k = G_k^T Q stays local
          -> prep backward for the queries this rank owns.
        The relation gradient is all_reduced once (each query's at its owner).
        Returns (loss as a float, d_ent for this rank's shard, d_rel) -- identical loss on
        every rank."""
        tr = torch.stack([s, p, o], 1)
        loss, d_ent, d_rel = self.train_1vsall_global(self._all_gather_1d(tr.reshape(-1)).view(-1, 3))
        return float(loss), d_ent, d_rel

    #: largest stacked [2 n, E_k] logits block (elements) scored in one pass; above it the two
    #: directions run one after the other (half the live score memory)
    STACK_MAX_ELEMS = 1 << 34

    def train_1vsall_global(self, tr_all: torch.Tensor, host_triples=None, loss=("kl", 0.0)):
        """train_1vsall_grads for a global batch [n, 3] that every rank already holds
        identically (the index batch is tiny, so a job hands every rank the whole batch
        instead of gathering slices).  host_triples: the same batch in host memory (a job's
        loader has it there); without it the batch is read back from the device once.

        Collectives per step (4 when both directions share one contraction, else 5):
          1. all_gather of the owner-computed query rows of BOTH directions, owner-major
             (ExchangePlan) -- each row travels once, from its owner;
          2. all_gather of the per-shard softmax statistics (max, sum-exp, target logit) as one
             [3, m] block per rank; every rank forms the global max, the rescaled sum and the
             target in the same fixed order, so lse is bit-identical everywhere;
          3. reduce_scatter of the partial dQ = G_k . E_k in the same owner-major layout: every
             owner receives the summed gradients of its own query rows only;
          4. all_reduce of the relation gradient (each query's at its owner).
        dE_k = G_k^T . Q stays local with the shard.

        loss = ("bce", offset): train.loss bce (loss.py:137-158, reduction "sum", on scores + offset
        against the one-hot rows) instead of the softmax cross entropy.  Binary cross entropy
        couples no columns, so collective 2 is not needed: every shard turns its logits into its
        slice of G = scale (sigmoid - y) by itself, and one all_reduce of a scalar gives the loss
        every rank reports."""
        loss_kind, loss_offset = loss
        if loss_kind not in ("kl", "bce"):
            raise ValueError(f"row-sharded 1vsAll loss {loss_kind!r} (kl or bce)")
        n = tr_all.shape[0]
        scale = 1.0 / n
        E_k = self.hi - self.lo
        dev = self.ent.device
        d_ent = torch.zeros_like(self.ent)
        d_rel = torch.zeros_like(self.rel)
        loss = torch.zeros((), device=dev, dtype=torch.float64)
        if n == 0:
            return loss, d_ent, d_rel
        dirs = ((0, 0, 2), (1, 2, 0))  # (direction, entity column, label column): sp_ then _po
        # stacked query order: the n sp_ rows, then the n _po rows
        e_all = torch.cat([tr_all[:, 0], tr_all[:, 2]])
        p_all = torch.cat([tr_all[:, 1], tr_all[:, 1]])
        labels = torch.cat([tr_all[:, 2], tr_all[:, 0]])
        host = host_triples if host_triples is not None else tr_all.cpu()
        host = host.numpy() if torch.is_tensor(host) else host
        per = max(1, math.ceil(self.E / self.world))
        import numpy as np

        plan = ExchangePlan(np.concatenate([host[:, 0], host[:, 2]]), per, self.world, self.rank, dev)
        cap, c_me = plan.cap, plan.count
        n0 = int((plan.mine_host < n).sum())  # this rank's sp_ rows come first (stable order)
        mine = plan.mine
        e_mine, p_mine = e_all[mine] - self.lo, p_all[mine]
        # ---- 1. owner-computed query rows, one all_gather
        q_mine = None
        for direction, a, b in ((0, 0, n0), (1, n0, c_me)):
            if b > a:
                part = self.ops.prep(direction, self.ent, e_mine[a:b], self.rel, p_mine[a:b])
                if q_mine is None:
                    q_mine = torch.empty(cap, part.shape[1], device=dev, dtype=part.dtype)
                q_mine[a:b] = part
        if q_mine is None:  # this rank owns none of the batch's query entities
            q_mine = torch.empty(cap, self._win(0, self.ent).shape[1], device=dev, dtype=self.ent.dtype)
        if c_me < cap:
            q_mine[c_me:].zero_()
        q_pad = torch.empty(self.world * cap, q_mine.shape[1], device=dev, dtype=q_mine.dtype)
        all_gather_into_tensor(q_pad, q_mine, group=self.group)
        q = q_pad.index_select(0, plan.slot)  # [2 n, d] in stacked order, identical on every rank
        del q_pad
        same_window = self._win(0, self.ent).data_ptr() == self._win(1, self.ent).data_ptr() and \
            self._win(0, self.ent).shape == self._win(1, self.ent).shape
        if same_window and 2 * n * E_k <= self.STACK_MAX_ELEMS:
            groups = [(0, 0, 2 * n)]  # (direction of the window, first row, last row)
        else:
            groups = [(0, 0, n), (1, n, 2 * n)]
        dq = torch.empty_like(q)
        for direction, r0, r1 in groups:
            m = r1 - r0
            qg, lab = q[r0:r1], labels[r0:r1]
            buf = torch.empty(m, (E_k + 3) // 4 * 4, device=dev, dtype=torch.float32)
            tab_w = self._win(direction, self.ent)
            # gradient planes pay off once the GEMMs dominate the step (a few more launches and
            # one more [m, E_k] buffer: at 1,024 x 14,541 the fp32 path is 10 % faster, at
            # 1,024 x 574,311 the planes are 16 % faster)
            # (bce has no fused fp32-gradient kernel: its fp32 path is a dozen elementwise torch
            # passes over the block, so the one-pass planes kernel takes over much earlier)
            min_elems = self.PLANES_MIN_ELEMS if loss_kind == "kl" else min(self.PLANES_MIN_ELEMS, self.BCE_PLANES_MIN_ELEMS)
            planes = (m * E_k >= min_elems and getattr(self.ops, "train_planes_ok", None) is not None
                      and self.ops.train_planes_ok(self.ent, direction))
            if planes:
                q_hi, q_lo = self.ops.split_padded(qg)
                logits = self.ops.score_split(q_hi, q_lo, m, tab_w, out=buf[:, :E_k])
            else:
                logits = self.ops.score(qg, tab_w, out=buf[:, :E_k])
            if loss_kind == "bce":  # elementwise: the shard's slice of G and of the loss, no exchange
                if planes:
                    part, gp = self.ops.bce_grad_planes(logits, self.lo, lab, loss_offset, scale)
                    del logits, buf
                    self.ops.score_bwd_planes(gp, q_hi, q_lo, tab_w, self._win(direction, d_ent), dq=dq[r0:r1])
                    del gp
                else:
                    part = self.ops.bce_grad(logits, self.lo, lab, loss_offset, scale, logits)
                    self.ops.score_bwd(logits, qg, tab_w, dq[r0:r1], self._win(direction, d_ent))
                    del logits, buf
                loss += part * scale
                continue
            # ---- 2. softmax statistics of every shard, one all_gather
            mx, sm, tg = self.ops.row_stats(logits, self.lo, lab)
            st = torch.stack([mx, sm, tg])
            st_all = torch.empty(self.world, 3, m, device=dev, dtype=st.dtype)
            all_gather_into_tensor(st_all.view(self.world * 3, m), st, group=self.group)
            mx_w, sm_w, tg_w = st_all[:, 0], st_all[:, 1], st_all[:, 2]
            M = mx_w.max(0).values
            z = torch.where(mx_w == -math.inf, torch.zeros_like(sm_w), sm_w * torch.exp(mx_w - M)).sum(0)
            lse = M + torch.log(z)
            loss += ((lse - tg_w.sum(0)).double().sum() * scale)
            if planes:
                gp = self.ops.softmax_grad_planes(logits, self.lo, lab, lse, scale)
                del logits, buf
                self.ops.score_bwd_planes(gp, q_hi, q_lo, tab_w, self._win(direction, d_ent), dq=dq[r0:r1])
                del gp
            else:
                g = self.ops.softmax_grad(logits, self.lo, lab, lse, scale, logits)
                self.ops.score_bwd(g, qg, tab_w, dq[r0:r1], self._win(direction, d_ent))
                del g, logits, buf
        # ---- 3. partial query gradients back to the owners, one reduce_scatter
        dq_pad = torch.zeros(self.world * cap, dq.shape[1], device=dev, dtype=dq.dtype)
        dq_pad.index_copy_(0, plan.slot, dq)
        dq_mine = torch.empty(cap, dq.shape[1], device=dev, dtype=dq.dtype)
        reduce_scatter_tensor(dq_mine, dq_pad, group=self.group)
        del dq_pad
        for direction, a, b in ((0, 0, n0), (1, n0, c_me)):
            if b > a:
                self.ops.prep_bwd(direction, self.ent, e_mine[a:b], self.rel, p_mine[a:b], dq_mine[a:b].contiguous(),
                                  d_ent, d_rel)
        # ---- 4. the replicated relation table's gradient
        all_reduce(d_rel, group=self.group)
        self.collectives_last_step = 3 + len(groups)
        if loss_kind == "bce":  # the shards' loss shares (the kl loss is formed from gathered statistics)
            loss = loss.reshape(1)
            all_reduce(loss, group=self.group)
            loss = loss.reshape(())
            self.collectives_last_step = 4
        return loss, d_ent, d_rel  # loss: a 0-dim float64 tensor on the table's device (no host sync)

    # ---------------------------------------------------------------- eval
    def rank_counts(self, s, p, o, f_sp, f_po, t_sp=None, t_po=None, p_inverse=None):
        """Global greater/tie counts of the true o (sp_) and s (_po) for a batch that
        every rank holds identically (s, p, o [B]); CSR filter lists as in
        EntityRankingJob.  Returns greater/ties [2 directions, 2 (greater, ties), 3 rankings x B]
        summed over shards with one all_reduce.  p_inverse: the relation ids p + R of a
        reciprocal-relations model, whose (?, p, o) side is scored as (o, p + R, ?) -- both
        its queries and its true score (reciprocal_relations_model.py:57-74)."""
        B = s.numel()
        rows = self.gather_rows(torch.cat([s, o]))  # full s rows then o rows, on every rank
        ar = torch.arange(B, device=s.device)
        true_o = self.ops.spo(rows[:B], self.rel, p, rows[B:])
        if p_inverse is None:
            sides = ((ar, 0, p, o, true_o, f_sp, t_sp), (ar + B, 1, p, s, true_o, f_po, t_po))
        else:
            true_s = self.ops.spo(rows[B:], self.rel, p_inverse, rows[:B])
            sides = ((ar, 0, p, o, true_o, f_sp, t_sp), (ar + B, 0, p_inverse, s, true_s, f_po, t_po))
        counts = torch.zeros(2, 2, 3 * B, dtype=torch.int64, device=s.device)
        for di, (eidx, direction, rel_ids, tgt, true, f, t) in enumerate(sides):
            q = self.ops.prep(direction, rows, eidx, self.rel, rel_ids)
            sc = self.ops.score(q, self._win(direction, self.ent))
            self.ops.rank_counts(sc, self.lo, tgt, true, f[0], f[1], t[0] if t is not None else None,
                                 t[1] if t is not None else None, counts[di, 0], counts[di, 1])
        all_reduce(counts, group=self.group)
        return counts

    def rank_block(self, s, p, o, f_ptrs, f_col, t_ptrs=None, t_col=None, p_inverse=None, refinement=None):
        """rank_counts as ONE stacked pass per batch: the (s, p, ?) rows on top of the (?, p, o)
        rows, one contraction against the shard, one ranking launch over it (ops.rank_rows,
        columns offset by this shard's first row) and one all_reduce of the counts.  f_ptrs /
        t_ptrs: the (sp, po) CSR pointer vectors of the batch into the combined column arrays
        f_col / t_col (EntityRankingJob._stack_csr).  refinement: ops.refinement(self.ent) --
        near-ties of the true score inside this shard are rescored exactly, so bf16x3 scores give
        the counts of exactly computed ones (the band is per shard: |q_i| max |t_j| over ITS
        rows; no exchange).  Returns [2 (greater, ties), rankings x 2 B] global counts, or None
        when the two directions contract with different entity-row windows (the caller then
        takes rank_counts)."""
        if not self.rank_block_applies(p_inverse is not None):
            return None
        rows = self.gather_rows(torch.cat([s, o]))  # full s rows then o rows, on every rank
        counts = self.rank_block_local(rows, s, p, o, f_ptrs, f_col, t_ptrs, t_col, p_inverse, refinement)
        all_reduce(counts, group=self.group)
        return counts

    def rank_block_applies(self, two_sided: bool) -> bool:
        """Whether both directions contract with the same entity-row window (one stacked pass)."""
        wa, wb = self._win(0, self.ent), self._win(0 if two_sided else 1, self.ent)
        return wa.data_ptr() == wb.data_ptr() and wa.shape == wb.shape

    def rank_block_local(self, rows, s, p, o, f_ptrs, f_col, t_ptrs=None, t_col=None, p_inverse=None, refinement=None):
        """The local part of rank_block: this shard's counts [2, rankings x 2 B] of one batch, NOT
        yet summed over the shards.  rows: the full entity rows of the batch's subjects followed
        by its objects ([2 B, d], identical on every rank: gather_rows) -- a caller that gathers
        the rows of several batches in one exchange and sums the counts of several batches in one
        all_reduce pays two collectives per GROUP of batches instead of two per batch."""
        B = s.numel()
        dir_b = 1 if p_inverse is None else 0
        wa = self._win(0, self.ent)
        dev = s.device
        stacked = getattr(self.ops, "spo_stacked", None)
        if stacked is not None and rows.is_contiguous():
            true_o = stacked(rows, self.rel, p).view(-1).float().contiguous()
            true_s = true_o if p_inverse is None else stacked(rows, self.rel, p_inverse, swap=True).view(-1).float().contiguous()
        else:
            true_o = self.ops.spo(rows[:B], self.rel, p, rows[B:]).view(-1).float().contiguous()
            true_s = true_o if p_inverse is None else self.ops.spo(rows[B:], self.rel, p_inverse, rows[:B]).view(-1).float().contiguous()
        rel_b = p if p_inverse is None else p_inverse
        E_k = self.hi - self.lo
        nrank = 1 + (f_ptrs is not None) + (t_ptrs is not None)
        counts = torch.zeros(2, nrank * 2 * B, dtype=torch.int64, device=dev)
        o, s = o.contiguous(), s.contiguous()
        part_a = (o, true_o, f_ptrs[0] if f_ptrs is not None else None, t_ptrs[0] if t_ptrs is not None else None)
        part_b = (s, true_s, f_ptrs[1] if f_ptrs is not None else None, t_ptrs[1] if t_ptrs is not None else None)
        codes = q = None
        fused_rows = getattr(self.ops, "rank_codes_rows", None)
        if fused_rows is not None:  # queries prepared straight into planes, ranking fused into the contraction
            got = fused_rows(rows, self.rel, p, rel_b, dir_b, wa, B, (o, true_o), (s, true_s), refinement, self.lo)
            if got is not None:
                codes, q = got
        if codes is None:
            ar = torch.arange(B, device=dev)
            q = torch.cat([self.ops.prep(0, rows, ar, self.rel, p), self.ops.prep(dir_b, rows, ar + B, self.rel, rel_b)])
            fused = getattr(self.ops, "rank_codes", None)
            codes = fused(q, wa, B, (o, true_o), (s, true_s), refinement, self.lo) if fused is not None else None
        refine = (q, self.ent, refinement[0], refinement[1]) if refinement is not None else None
        if codes is not None:  # the scores are compared inside the contraction: no score block
            self.ops.rank_rows(None, B, self.lo, part_a, part_b, f_col, t_col, counts[0], counts[1], refine=refine,
                               codes=codes, m=E_k)
        else:
            buf = torch.empty(2 * B, (E_k + 3) // 4 * 4, device=dev, dtype=torch.float32)
            scores = self.ops.score(q, wa, out=buf[:, :E_k])
            self.ops.rank_rows(scores, B, self.lo, part_a, part_b, f_col, t_col, counts[0], counts[1], refine=refine)
        return counts

    def all_gather_table(self) -> torch.Tensor:
        """The full [E, d] entity table assembled from every rank's shard (checkpoints, or
        handing a sharded-trained model to unsharded code)."""
        per = math.ceil(self.E / self.world)
        mine = torch.zeros(per, self.ent.shape[1], dtype=self.ent.dtype, device=self.ent.device)
        mine[:self.hi - self.lo] = self.ent
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        all_gather(parts, mine, group=self.group)
        return torch.cat(parts)[:self.E]
