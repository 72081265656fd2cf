"""TrainingJobNegativeSampling (kge/job/train.py:759-999) on the engine.

Per batch and corrupted slot, each positive (s, p, o) is scored together with its N
negatives -- a [B, 1 + N] score matrix whose column 0 is the positive -- and the configured
loss is applied with labels[:, 0] = 1.  Implementations (negative_sampling.implementation):

* ``triple`` -- the reference scores B * (1 + N) materialised triples with score_spo
  (train.py:868-892).  Here the s / o slots go through KgeModel.score_sp_cand /
  score_po_cand: the fused candidate-gather kernel kge_score_cand, same per-triple
  semantics, no triple tensor.  The p slot (and models without the fused path) fall back to
  score_spo on expanded triples -- itself an engine kernel (kge_score_spo).
* ``all``   -- score_sp / score_po against every entity, then pick (train.py:893-930).
* ``batch`` -- score against the chunk's unique targets, then pick (train.py:931-968).

Negatives are drawn on the device (kge/util/sampler.py), so the step has no host work
beyond its one loss read-back.
"""
from __future__ import annotations

import math
import time

import torch

from ..util.sampler import KgeSampler, KgeUniformSampler, O, P, S
from .train import TrainingJob, _GraphStep


class _NSGraphStep(_GraphStep):
    """The negative-sampling step as a recorded graph (engine.graph_step): the batch's B triples are
    the recorded index block; the negatives are drawn inside the recording (torch's generator
    advances with every replay), scored, and the loss, both backward passes and the optimizer
    step follow -- some 50 launches that otherwise cost more host time than device time at the
    usual handful of negatives.  Batches that bring their own negatives, and partial batches,
    run eagerly."""

    def _capacity(self) -> int:
        return 3 * self.job.batch_size

    def _block(self, batch):
        triples = batch["triples"]
        if "negative_samples" in batch or triples.dim() != 2 or tuple(triples.shape) != (self.job.batch_size, 3):
            return None
        # column-major: the recorded [B, 3] view below then has contiguous columns, which the scoring
        # calls take as they are (a row-major block costs a copy kernel per column and slot)
        return triples.long().t().reshape(-1)

    def _recorded_batch(self):
        return {"triples": self.static.view(3, self.job.batch_size).t()}

    def _penalty_batch(self):
        return self._recorded_batch()


class TrainingJobNegativeSampling(TrainingJob):
    def __init__(self, config, dataset, parent_job=None, model=None):
        super().__init__(config, dataset, parent_job, model=model)
        self._sampler = KgeSampler.create(config, "negative_sampling", dataset, self.device)
        impl = config.get("negative_sampling.implementation")
        if impl not in ("triple", "all", "batch", "auto"):
            raise ValueError(f"negative_sampling.implementation={impl}")
        if impl == "auto":
            # The reference picks by cost (train.py:762-771): "batch" for shared or more than 30
            # negatives, else "triple"; the implementations score the same (triple, candidate)
            # pairs.  On the engine the per-query candidate kernel (kge_score_cand) beats scoring
            # the chunk's unique candidates at any count unless the negatives are shared (C4: 2.3
            # against 7 ms per step), so "triple" it is whenever that kernel serves the model.
            if self._sampler.shared:
                impl = "batch"
            elif self.model._lookup_tables() is not None:
                impl = "triple"
            else:
                impl = "batch" if max(self._sampler.num_samples) > 30 else "triple"
        self._implementation = impl
        self._max_chunk_size = config.get("negative_sampling.chunk_size")
        self.type_str = "negative_sampling"
        from ..util.loss import BCEWithLogitsKgeLoss, KLDivWithSoftmaxKgeLoss, MarginRankingKgeLoss

        #: The loss of a [chunk, 1 + N] block whose column 0 is the positive as ONE engine kernel
        #: (loss + gradient) instead of torch's loss chain: "kl" on the one-hot label matrix is the
        #: cross entropy against column 0 (engine.xent_column0); "margin_ranking" and "bce" (sum)
        #: run kge_ns_loss (engine.ns_loss_column0).  None: kge.util.loss on the score block.
        self._fused_loss = None
        if bool(config.get("engine.fused_loss")) and str(self.device).startswith("cuda"):
            if type(self.loss) is KLDivWithSoftmaxKgeLoss:
                self._fused_loss = ("kl", 0.0)
            elif type(self.loss) is MarginRankingKgeLoss:
                self._fused_loss = ("margin_ranking", float(self.loss._loss.margin))
            elif type(self.loss) is BCEWithLogitsKgeLoss and not self.loss._mean:
                self._fused_loss = ("bce", float(self.loss._offset))

    def _prepare(self):
        super()._prepare()
        self._replicas_only()
        self.num_examples = self.dataset.split(self.train_split).size(0)
        # The step is recorded when nothing in it needs the host: negatives drawn by torch.randint
        # (no filtering rounds, no shared sample), scored by the candidate kernels, the loss fused.
        opt = self.optimizer
        sampler = self._sampler
        self._graph_step = None
        if (self.config.get("engine.graph_step") and torch.device(self.device).type == "cuda"
                and self._fused_loss is not None and self._implementation == "triple"
                and type(sampler) is KgeUniformSampler and not sampler.shared and not any(sampler.filter_positives)
                and sampler.num_samples[P] == 0
                and self.batch_size <= 4096 and 1 + max(sampler.num_samples) <= 8192  # engine._cand_order
                and hasattr(opt, "graph_safe") and opt.graph_safe() and not self.pre_batch_hooks
                and self._penalties_recordable(weighted_ok=True)
                and self.model._lookup_tables() is not None):
            self._graph_step = _NSGraphStep(self)

    def _collate(self, example_ids):
        return {"triples": self.dataset.split(self.train_split)[example_ids, :].long()}

    # --------------------------------------------------------------------- scoring
    def _scores(self, triples: torch.Tensor, slot: int, neg: torch.Tensor) -> torch.Tensor:
        """[chunk, 1 + N] scores, column 0 the positive."""
        cand = torch.cat((triples[:, slot:slot + 1], neg), 1)
        n, k = cand.shape
        if self._implementation == "triple":
            out = None
            if slot == O:
                out = self.model.score_sp_cand(triples[:, S], triples[:, P], cand)
            elif slot == S:
                out = self.model.score_po_cand(triples[:, P], triples[:, O], cand)
            if out is not None:
                return out
            t = triples.repeat(1, k).view(-1, 3)
            t[:, slot] = cand.reshape(-1)
            direction = "s" if slot == S else ("o" if slot == O else "p")
            return self.model.score_spo(t[:, S], t[:, P], t[:, O], direction=direction).view(n, k)
        if self._implementation == "all":
            if slot == S:
                allsc = self.model.score_po(triples[:, P], triples[:, O])
            elif slot == P:
                allsc = self.model.score_so(triples[:, S], triples[:, O])
            else:
                allsc = self.model.score_sp(triples[:, S], triples[:, P])
            return torch.gather(allsc, 1, cand)
        # batch
        uniq, col = torch.unique(cand.reshape(-1), return_inverse=True)
        if slot == S:
            allsc = self.model.score_po(triples[:, P], triples[:, O], uniq)
        elif slot == P:
            allsc = self.model.score_so(triples[:, S], triples[:, O], uniq)
        else:
            allsc = self.model.score_sp(triples[:, S], triples[:, P], uniq)
        return torch.gather(allsc, 1, col.view(n, k))

    def _process_batch(self, batch_index, batch) -> TrainingJob._ProcessBatchResult:
        prepare = -time.time()
        triples = batch["triples"].to(self.device, non_blocking=True)
        bs = len(triples)
        if "negative_samples" in batch:  # drawn by the caller (the reference's collate output)
            negs = [ns.to(self.device).long() if self._sampler.num_samples[slot] > 0 else None
                    for slot, ns in zip((S, P, O), batch["negative_samples"])]
        else:
            negs = [self._sampler.sample(triples, slot) if self._sampler.num_samples[slot] > 0 else None
                    for slot in (S, P, O)]
        prepare += time.time()
        fwd = bwd = 0.0
        total = None
        chunk = self._max_chunk_size if self._max_chunk_size > 0 else bs
        labels = None
        for c in range(math.ceil(bs / chunk)):
            lo, hi = c * chunk, min(bs, (c + 1) * chunk)
            tr = triples[lo:hi]
            for slot in (S, P, O):
                ns = self._sampler.num_samples[slot]
                if ns <= 0:
                    continue
                fwd -= time.time()
                scores = self._scores(tr, slot, negs[slot][lo:hi])
                fused = self._fused_loss is not None and scores.is_cuda
                if not fused and (labels is None or labels.shape != (hi - lo, 1 + ns)):
                    labels = torch.zeros(hi - lo, 1 + ns, device=self.device)  # only kge.util.loss reads them
                    labels[:, 0] = 1.0
                if fused:
                    from .. import engine

                    kind, arg = self._fused_loss
                    loss = (engine.xent_column0(scores, 1.0 / bs) if kind == "kl"
                            else engine.ns_loss_column0(scores, kind, arg, 1.0 / bs))
                else:
                    loss = self.loss(scores, labels, num_negatives=ns) / bs
                fwd += time.time()
                bwd -= time.time()
                self._backward(loss)
                bwd += time.time()
                total = loss.detach() if total is None else total + loss.detach()
        if total is None:
            total = torch.zeros((), device=self.device)
        return TrainingJob._ProcessBatchResult(total.detach(), bs, prepare, fwd, bwd)
