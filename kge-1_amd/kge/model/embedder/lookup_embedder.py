"""LookupEmbedder: one stored fp32 row per object (lookup_embedder.py:13-158).

The table is an ``nn.Embedding`` so checkpoints keep the reference's state_dict keys
(``_entity_embedder._embeddings.weight``).  On the fused scoring path the table is not
gathered here at all: KgeModel hands the weight to the engine, whose prep kernel gathers
the query rows and whose contraction streams the whole table (no embed_all copy).
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn.functional
from torch import Tensor

from ..kge_model import KgeEmbedder


import contextlib
import threading


class _InPlaceState:
    """Process-wide, not thread-local: the backward of a CUDA graph runs on autograd's device
    thread, which a flag local to the calling thread never reaches."""

    def __init__(self):
        self.depth = 0
        self.lock = threading.Lock()

    @property
    def on(self) -> bool:
        return self.depth > 0


_state = _InPlaceState()


@contextlib.contextmanager
def in_place_row_gradients():
    """While active (process-wide: see _InPlaceState), the backward of embed(), of the recorded Lp
    penalty and of the candidate scores adds its rows straight into a dense ``weight.grad`` that an
    earlier backward of the same step has left, and hands autograd no gradient of its own.  That is
    only right when the caller wants the gradients ACCUMULATED in ``.grad`` -- a training job
    around its own ``backward()`` calls, with no other thread differentiating through the same
    tables meanwhile.  Outside it the Functions return the dense gradient like any other op, so
    ``torch.autograd.grad``, gradient hooks and accumulation wrappers see it."""
    with _state.lock:
        _state.depth += 1
    try:
        yield
    finally:
        with _state.lock:
            _state.depth -= 1


def _in_place_ok(held, weight, dtype) -> bool:
    return (_state.on and held is not None and not held.is_sparse and held.dtype == dtype
            and held.shape == weight.shape and not torch.is_grad_enabled())


class _Rows(torch.autograd.Function):
    """weight[indexes] whose backward is one scatter-add (index_add_) -- a few microseconds on
    the device, against the sort-based embedding_dense_backward of nn.Embedding (~60 us per call
    whatever the table's size).  Inside ``in_place_row_gradients()``, when the table already holds
    a dense gradient (an earlier backward of the step left it), the rows are added into it where
    it stands; otherwise into a zero tensor that autograd then takes as the gradient.  Same
    values; rows that occur several times sum their gradients by atomic adds."""

    @staticmethod
    def forward(ctx, weight, indexes):
        ctx.save_for_backward(weight, indexes)
        return weight.index_select(0, indexes.reshape(-1)).view(*indexes.shape, weight.shape[1])

    @staticmethod
    def backward(ctx, g):
        weight, indexes = ctx.saved_tensors
        g = g.reshape(-1, g.shape[-1])
        idx = indexes.reshape(-1)
        held = weight.grad
        if _in_place_ok(held, weight, g.dtype):
            held.index_add_(0, idx, g)
            return None, None
        d_weight = torch.zeros(weight.shape[0], g.shape[1], device=g.device, dtype=g.dtype)
        d_weight.index_add_(0, idx, g)
        return d_weight, None


class _LpOccurrences(torch.autograd.Function):
    """coeff * sum over the occurrences i of sum_k |weight[indexes[i], k]|^p on the engine
    (kge_lp_rows / kge_lp_rows_bwd): a launch and a row-sum forward, one launch backward,
    instead of a dozen elementwise kernels each way."""

    @staticmethod
    def forward(ctx, weight, indexes, p, coeff):
        from ... import _lib

        ctx.save_for_backward(weight, indexes)
        ctx.p, ctx.coeff = p, coeff
        return _lib.lp_rows(weight, indexes, p).sum() * coeff

    @staticmethod
    def backward(ctx, g):
        from ... import _lib

        weight, indexes = ctx.saved_tensors
        gs = g.reshape(1).float().contiguous()
        held = weight.grad
        if _in_place_ok(held, weight, torch.float32) and held.stride(1) == 1:
            # the loss backward has left the table's dense gradient: the touched rows are added
            # into it where it stands (no table-sized zero tensor, no table-sized add)
            _lib.lp_rows_bwd(weight, indexes, ctx.p, gs, ctx.coeff, held)
            return None, None, None, None
        d_weight = torch.zeros_like(weight)
        _lib.lp_rows_bwd(weight, indexes, ctx.p, gs, ctx.coeff, d_weight)
        return d_weight, None, None, None


class LookupEmbedder(KgeEmbedder):
    def __init__(self, config, dataset, configuration_key: str, vocab_size: int, init_for_load_only=False):
        super().__init__(config, dataset, configuration_key, init_for_load_only=init_for_load_only)
        self.normalize_p = self.get_option("normalize.p")
        self.normalize_with_grad = self.get_option("normalize.with_grad")
        self.regularize = self.check_option("regularize", ["", "lp"])
        self.sparse = self.get_option("sparse")
        self.vocab_size = vocab_size
        self._embeddings = torch.nn.Embedding(self.vocab_size, self.dim, sparse=self.sparse)
        if not init_for_load_only:
            self._init_embeddings(self._embeddings.weight.data)
        dropout = self.get_option("dropout")
        if dropout < 0:
            dropout = 0.0
        self.dropout = torch.nn.Dropout(dropout)
        #: (lo, hi) while this process holds only rows [lo, hi) of the table (a row-sharded job:
        #: kge.sharded); the weight is then [hi - lo, dim] and nothing here can embed an id
        self.shard = None

    # ---- row sharding (kge.sharded): the table's rows split over the processes of a job
    def shard_rows(self, lo: int, hi: int) -> torch.nn.Parameter:
        """Keep only rows [lo, hi): the weight becomes a [hi - lo, dim] parameter of its own
        storage (the full table is released) that the sharded job scores and trains.  embed /
        embed_all / penalty and the fused scoring path refuse to run until ``unshard``."""
        if self.shard is not None:
            raise RuntimeError(f"{self.configuration_key}: already holds rows {self.shard} only")
        w = self._embeddings.weight
        return self.install_rows(torch.nn.Parameter(w.data[lo:hi].clone(), requires_grad=w.requires_grad), lo, hi)

    def install_rows(self, param: torch.nn.Parameter, lo: int, hi: int) -> torch.nn.Parameter:
        if param.shape != (hi - lo, self.dim):
            raise ValueError(f"rows [{lo}, {hi}) of a {self.dim}-wide table, got {tuple(param.shape)}")
        self._embeddings.weight = param
        self.shard = (lo, hi)
        return param

    def unshard(self, full: Tensor):
        """Install the whole [vocab_size, dim] table again (assembled from every process's rows)."""
        if tuple(full.shape) != (self.vocab_size, self.dim):
            raise ValueError(f"expected the whole [{self.vocab_size}, {self.dim}] table, got {tuple(full.shape)}")
        self._embeddings.weight = torch.nn.Parameter(full)
        self.shard = None

    def _whole(self):
        if self.shard is not None:
            raise RuntimeError(f"{self.configuration_key}: this process holds rows [{self.shard[0]}, {self.shard[1]}) "
                               f"of the table only (row-sharded job); score through kge.sharded.RowShardedScorer or "
                               f"call the job's sync_model() first")

    def prepare_job(self, job, **kwargs):
        super().prepare_job(job, **kwargs)
        if self.normalize_p > 0:  # lookup_embedder.py:58-75

            def normalize_embeddings(job):
                if self.normalize_with_grad:
                    self._embeddings.weight = torch.nn.functional.normalize(
                        self._embeddings.weight, p=self.normalize_p, dim=-1)
                else:
                    with torch.no_grad():
                        self._embeddings.weight = torch.nn.Parameter(torch.nn.functional.normalize(
                            self._embeddings.weight, p=self.normalize_p, dim=-1))

            job.pre_batch_hooks.append(normalize_embeddings)

    def is_plain(self) -> bool:
        """True when embed(i) == weight[i] exactly (no dropout in training mode)."""
        return not (self.dropout.p > 0 and self.training)

    def weight_for_scoring(self) -> Tensor:
        self._whole()
        return self._embeddings.weight

    def embed(self, indexes: Tensor) -> Tensor:
        self._whole()
        w = self._embeddings.weight
        if w.is_cuda and not self.sparse:
            return self._postprocess(_Rows.apply(w, indexes.long()))
        return self._postprocess(self._embeddings(indexes.long()))

    def embed_all(self) -> Tensor:
        # identical values and gradient to weight[arange(V)] (lookup_embedder.py:102-107)
        self._whole()
        return self._postprocess(self._embeddings.weight)

    def _postprocess(self, embeddings: Tensor) -> Tensor:
        if self.dropout.p > 0:
            embeddings = self.dropout(embeddings)
        return embeddings

    def _embeddings_all(self) -> Tensor:
        return self._embeddings.weight

    def penalty_active(self) -> bool:
        """Whether penalty() returns a term (lp regularisation with a non-zero weight)."""
        return self.regularize != "" and self.get_option("regularize_weight") != 0.0

    def penalty_weighted(self) -> bool:
        """Whether the penalty weights each row by its frequency among the batch's indexes."""
        return self.penalty_active() and bool(self.get_option("regularize_args.weighted"))

    def lp_term(self, weight: Tensor, indexes: Tensor, count: int) -> Tensor:
        """The Lp term of penalty() (lookup_embedder.py:112-158) over ``weight`` in place of the
        embedder's whole table: w / p * sum |weight|^p, or, frequency-weighted, over the rows
        ``indexes`` of ``weight`` (each as often as it occurs) divided by ``count``.  A
        row-sharded table sums this over its shards: rank k passes its rows, the batch's
        indexes that fall into them, and the batch's full index count."""
        p = self.get_option("regularize_args.p") if self.has_option("regularize_args.p") else 2
        w = self.get_option("regularize_weight")
        if not self.get_option("regularize_args.weighted"):
            return (w / p * weight.norm(p=p) ** p).sum()
        unique_indexes, counts = torch.unique(indexes, return_counts=True)
        rows = weight[unique_indexes]
        if p % 2 == 1:
            rows = torch.abs(rows)
        return (w / p * (rows ** p * counts.float().view(-1, 1))).sum() / count

    def penalty(self, **kwargs) -> List:
        """Lp regularisation (lookup_embedder.py:112-158).

        While a HIP graph is being recorded the weighted form sums over the OCCURRENCES of the
        indexes instead of over unique indexes times their counts: the same sum (a row that
        occurs c times contributes c equal terms) without torch.unique, whose output shape
        depends on the data and cannot be recorded."""
        result = super().penalty(**kwargs)
        if self.regularize == "" or self.get_option("regularize_weight") == 0.0:
            return result
        self._whole()
        p = self.get_option("regularize_args.p") if self.has_option("regularize_args.p") else 2
        w = self.get_option("regularize_weight")
        if not self.get_option("regularize_args.weighted"):
            params = self._embeddings_all()
            result += [(f"{self.configuration_key}.L{p}_penalty", (w / p * params.norm(p=p) ** p).sum())]
        elif kwargs["indexes"].is_cuda and torch.cuda.is_current_stream_capturing():
            indexes = kwargs["indexes"]
            weight = self._embeddings.weight
            if p in (1, 2, 3, 4) and weight.dtype == torch.float32 and weight.stride(1) == 1:
                value = _LpOccurrences.apply(weight, indexes, int(p), w / p / len(indexes))
            else:
                params = weight.index_select(0, indexes)
                if p % 2 == 1:
                    params = torch.abs(params)
                value = (w / p * params ** p).sum() / len(indexes)
            result += [(f"{self.configuration_key}.L{p}_penalty", value)]
        else:
            unique_indexes, counts = torch.unique(kwargs["indexes"], return_counts=True)
            params = self._embeddings(unique_indexes)
            if p % 2 == 1:
                params = torch.abs(params)
            result += [(f"{self.configuration_key}.L{p}_penalty",
                        (w / p * (params ** p * counts.float().view(-1, 1))).sum() / len(kwargs["indexes"]))]
        return result
