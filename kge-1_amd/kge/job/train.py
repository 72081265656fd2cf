"""Training jobs that drive the scoring hot path: TrainingJob1vsAll (train.py:1002-1062)
and TrainingJobKvsAll (train.py:493-756) over the TrainingJob epoch loop (train.py:45-490).

Per batch they call KgeModel.score_sp / score_po exactly as the reference does; the
engine runs the fused gather + contraction forward and the MFMA backward.  Difference
from the reference, by design: the per-direction ``loss.item()`` host syncs are
replaced by an asynchronous copy of each batch loss that the epoch loop reads one batch
later, so the host never drains the device queue inside the epoch.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Any, Dict, Optional

import numpy as np
import torch

from .. import _lib
from ..model.kge_model import KgeModel
from ..util.loss import BCEWithLogitsKgeLoss, KgeLoss, KLDivWithSoftmaxKgeLoss
from ..util.optimizer import KgeLRScheduler, KgeOptimizer
from .job import Job

S, P, O = 0, 1, 2


class TrainingJob(Job):
    @dataclass
    class _ProcessBatchResult:
        loss: Any  # float, or a 0-dim device tensor read by the epoch loop one batch later
        size: int
        prepare_time: float
        forward_time: float
        backward_time: float

        @property
        def avg_loss(self) -> float:
            return float(self.loss)

    def __init__(self, config, dataset, parent_job=None, model=None):
        super().__init__(config, dataset, parent_job)
        self.model: KgeModel = model if model is not None else KgeModel.create(config, dataset)
        self.optimizer = KgeOptimizer.create(config, self.model)
        self.kge_lr_scheduler = KgeLRScheduler(config, self.optimizer)
        self.loss = KgeLoss.create(config)
        self.abort_on_nan: bool = config.get("train.abort_on_nan")
        self.batch_size: int = config.get("train.batch_size")
        self.train_split = config.get("train.split")
        self.epoch = 0
        self.loader = None
        self.num_examples = None
        self.type_str: Optional[str] = None
        self.pre_batch_hooks = []
        self.post_batch_trace_hooks = []
        self.post_epoch_trace_hooks = []
        self.post_epoch_hooks = []
        self.post_valid_hooks = []
        self.valid_job = None
        self.valid_trace = []
        self.best_state = None
        self.generator = torch.Generator()
        seed = config.get("random_seed.torch")
        if seed >= 0:
            self.generator.manual_seed(seed)
        self.model.train()

    @staticmethod
    def create(config, dataset, parent_job=None, model=None) -> "TrainingJob":
        t = config.get("train.type")
        if t == "KvsAll":
            return TrainingJobKvsAll(config, dataset, parent_job, model=model)
        if t == "1vsAll":
            return TrainingJob1vsAll(config, dataset, parent_job, model=model)
        if t == "negative_sampling":
            from .negative_sampling import TrainingJobNegativeSampling

            return TrainingJobNegativeSampling(config, dataset, parent_job, model=model)
        raise ValueError("train.type")

    def _prepare(self):
        self.model.prepare_job(self)

    def _replicas_only(self):
        """For the training types without a row-sharded step (KvsAll, negative sampling; the
        vocab-parallel step serves 1vsAll): engine.row_sharded "on" is refused, and under "auto"
        in a world of several processes every process trains its own replica, which is said once."""
        from ..sharded import sharding_enabled

        if not sharding_enabled(self.config):
            return
        if self.config.get("engine.row_sharded") == "on":
            raise NotImplementedError(f"engine.row_sharded: on -- the {self.type_str} training job does not shard "
                                      f"the entity table (1vsAll training and entity ranking do)")
        self.config.log(f"{self.type_str} training does not shard the entity table: every process of this "
                        f"torch.distributed world trains a replica of its own (engine.row_sharded: auto)")

    def _run(self):
        """The epoch loop of train.py:136-250: train an epoch, validate every valid.every
        epochs (EvaluationJob on valid.split sharing this model), step the LR scheduler
        (metric-based schedulers on the validation metric), stop early when the metric has
        not improved for valid.early_stopping.patience validations or misses its minimum
        threshold.  Checkpoint files are outside the scoring path: the best epoch is kept in
        memory (self.best_state) instead of being written.  In a row-sharded job every rank
        keeps ITS rows of that epoch's entity table (all ranks decide on the same, all-reduced
        validation metric, so the copies belong to one epoch); best_state_full() assembles them.
        Returns the epoch traces."""
        cfg = self.config
        metric_name = cfg.get("valid.metric")
        patience = cfg.get("valid.early_stopping.patience")
        traces = []
        while True:
            if self.valid_trace and self.valid_trace[-1]["epoch"] == self.epoch:
                best = max(range(len(self.valid_trace)), key=lambda i: self.valid_trace[i][metric_name])
                if best == len(self.valid_trace) - 1:
                    self.best_state = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
                if patience > 0 and len(self.valid_trace) > patience and best < len(self.valid_trace) - patience:
                    cfg.log(f"Stopping early ({metric_name} did not improve over best result in the last "
                            f"{patience} validation runs).")
                    break
                if (self.epoch > cfg.get("valid.early_stopping.min_threshold.epochs")
                        and self.valid_trace[best][metric_name]
                        < cfg.get("valid.early_stopping.min_threshold.metric_value")):
                    cfg.log(f"Stopping early ({metric_name} did not achieve min treshold after {self.epoch} epochs")
                    break
            if self.epoch >= cfg.get("train.max_epochs"):
                break
            self.epoch += 1
            trace = self.run_epoch()
            traces.append(trace)
            for f in self.post_epoch_hooks:
                f(self, trace)
            every = cfg.get("valid.every")
            if every > 0 and self.epoch % every == 0:
                vtrace = self._validate()
                self.valid_trace.append(vtrace)
                for f in self.post_valid_hooks:
                    f(self, vtrace)
                self.kge_lr_scheduler.step(vtrace[metric_name])
            else:
                self.kge_lr_scheduler.step()
        self.sync_model()
        return traces

    def best_state_full(self):
        """self.best_state with whole tables on every rank (a collective in a row-sharded job)."""
        sharded = getattr(self, "_sharded", None)
        if sharded is None or self.best_state is None:
            return self.best_state
        return sharded.full_state(self.best_state)

    def sync_model(self):
        """Make the model's tables complete on every rank: a row-sharded job all-gathers its
        entity-row shards (a collective: every rank calls it); otherwise nothing to do."""
        sharded = getattr(self, "_sharded", None)
        if sharded is not None:
            sharded.sync_model()

    def _validate(self) -> Dict[str, Any]:
        """Run the validation job (created on first use, train.py:77-84) on this model."""
        if self.valid_job is None:
            from .entity_ranking import EvaluationJob

            valid_conf = self.config.clone()
            valid_conf.set("job.type", "eval")
            if self.config.get("valid.split") != "":
                valid_conf.set("eval.split", self.config.get("valid.split"))
            self.valid_job = EvaluationJob.create(valid_conf, self.dataset, parent_job=self, model=self.model)
            if getattr(self, "sharded_ops", None) is not None:
                self.valid_job.sharded_ops = self.sharded_ops
        self.valid_job.epoch = self.epoch
        return self.valid_job.run()

    def _batches(self):
        perm = torch.randperm(self.num_examples, generator=self.generator)
        sharded = getattr(self, "_sharded", None)
        if sharded is not None:  # every rank steps through the same global batches
            perm = sharded.broadcast(perm)
        for b in range(0, self.num_examples, self.batch_size):
            yield perm[b:b + self.batch_size]

    def run_epoch(self) -> Dict[str, Any]:
        """One pass over the training examples (train.py:295-429)."""
        if not self._is_prepared:
            self._prepare()
            self._is_prepared = True
        sum_loss = 0.0
        sum_penalty = 0.0
        epoch_time = -time.time()
        fwd = bwd = prep = opt_t = 0.0
        n_batches = 0
        pending = None  # (host copy of a batch loss, its event, batch size, host copy of the penalty)

        def settle(p):
            nonlocal sum_loss, sum_penalty
            buf, ev, size, pen = p
            if ev is not None:
                ev.synchronize()
            v = float(buf)
            pen = float(pen)
            sum_loss += v * size
            sum_penalty += pen
            if self.abort_on_nan and math.isnan(v + pen):
                raise FloatingPointError("Cost became nan, aborting training job")

        def host_copy(x):
            """A 0-dim device tensor on its way to pinned host memory (stream-ordered, not waited
            for); anything else as it is."""
            if torch.is_tensor(x) and x.is_cuda:
                buf = torch.empty((), dtype=x.dtype, pin_memory=True)
                buf.copy_(x.detach(), non_blocking=True)
                return buf, True
            return x, False

        for batch_index, example_ids in enumerate(self._batches()):
            for f in self.pre_batch_hooks:
                f(self)
            batch = self._collate(example_ids)
            res, penalty, t_opt = self.train_step(batch_index, batch)
            opt_t += t_opt
            # The batch loss and penalty are read one batch late (async copies + an event): the
            # host queues batch b + 1 while the device still runs batch b, instead of draining the
            # queue every batch as loss.item() / penalty.item() would (the reference's per-batch
            # syncs).  A NaN aborts one optimizer step later than in the reference.
            loss_h, a = host_copy(res.loss)
            pen_h, b = host_copy(penalty)
            ev = None
            if a or b:
                ev = torch.cuda.Event()
                ev.record()
            cur = (loss_h, ev, res.size, pen_h)
            if pending is not None:
                settle(pending)
            pending = cur
            prep += res.prepare_time
            fwd += res.forward_time
            bwd += res.backward_time
            n_batches += 1
        if pending is not None:
            settle(pending)
        epoch_time += time.time()
        trace = dict(type=self.type_str, scope="epoch", epoch=self.epoch, split=self.train_split,
                     batches=n_batches, size=self.num_examples,
                     lr=[group["lr"] for group in self.optimizer.param_groups],
                     avg_loss=sum_loss / max(1, self.num_examples),
                     avg_penalty=sum_penalty / max(1, n_batches),
                     avg_cost=sum_loss / max(1, self.num_examples) + sum_penalty / max(1, n_batches),
                     epoch_time=epoch_time, prepare_time=prep,
                     forward_time=fwd, backward_time=bwd, optimizer_time=opt_t, event="epoch_completed")
        for f in self.post_epoch_trace_hooks:
            f(self, trace)
        return trace

    def _collate(self, example_ids):
        raise NotImplementedError

    def _backward(self, value: torch.Tensor):
        """value.backward() for a 0-dim loss with a PERSISTENT seed gradient: autograd otherwise
        makes ones_like(value) per call, a fill kernel that a recorded step replays every time."""
        one = getattr(self, "_seed_one", None)
        if one is None or one.device != value.device or one.dtype != value.dtype:
            one = self._seed_one = torch.ones((), device=value.device, dtype=value.dtype)
        value.backward(one)

    def _fused_loss_kind(self):
        """(kind, offset) of the loss the engine fuses into the scoring pass for this job --
        ("kl", 0.0) for train.loss kl (softmax cross entropy / KL), ("bce", loss_arg) for
        train.loss bce (sum reduction; loss.py:137-158) -- or None: engine.fused_loss is off or
        the loss is computed by kge.util.loss on the score matrix."""
        if not self.config.get("engine.fused_loss"):
            return None
        if isinstance(self.loss, KLDivWithSoftmaxKgeLoss):
            return ("kl", 0.0)
        if type(self.loss) is BCEWithLogitsKgeLoss and not self.loss._mean:
            return ("bce", float(self.loss._offset))
        return None

    def process_batch(self, batch_index, batch) -> "TrainingJob._ProcessBatchResult":
        kind = self._fused_loss_kind()
        if kind is None or kind[0] == "kl":
            return self._process_batch(batch_index, batch)
        from .. import engine

        with engine.fused_loss_kind(*kind):  # the fused passes inside compute this loss
            return self._process_batch(batch_index, batch)

    def train_step(self, batch_index, batch):
        """One optimizer step on one batch -- zero_grad, forward/backward (process_batch),
        penalty backward, optimizer.step: the body of the reference's batch loop
        (train.py:309-429).  Returns (result, penalty, optimizer seconds).  Replayed from a
        recorded HIP graph when the job has one for this batch (engine.graph_step)."""
        from ..model.embedder.lookup_embedder import in_place_row_gradients

        # the step's backward calls accumulate into .grad: lookups may add their rows in place
        with in_place_row_gradients():
            graph = getattr(self, "_graph_step", None)
            if graph is not None:
                res = graph.run(batch_index, batch)
                if res is not None:
                    return res, graph.penalty if graph.penalty is not None else 0.0, 0.0
            self.optimizer.zero_grad()
            res = self.process_batch(batch_index, batch)
            penalty = self._penalty_backward(batch_index, batch)
        t0 = time.time()
        self.optimizer.step()
        return res, penalty, time.time() - t0

    def _penalty_backward(self, batch_index, batch):
        """The penalty terms of the batch (train.py:320-337): backward on each, and their sum as a
        0-dim tensor (0.0 when nothing regularises) -- not read on the host here."""
        total = None
        for _, pv in self.model.penalty(epoch=self.epoch, batch_index=batch_index, batch=batch):
            self._backward(pv) if pv.dim() == 0 else pv.backward()
            total = pv.detach() if total is None else pv.detach() + total
        return 0.0 if total is None else total

    def _penalties_recordable(self, weighted_ok: bool) -> bool:
        """Whether the model's penalty terms can be part of a recorded step: none at all, or Lp
        terms of lookup embedders (frequency-weighted ones only when the recorded batch carries
        its triples)."""
        from ..model.embedder.lookup_embedder import LookupEmbedder

        m = self.model
        for e in (m.get_s_embedder(), m.get_p_embedder(), m.get_o_embedder()):
            if not getattr(e, "penalty_active", lambda: True)():
                continue
            if not isinstance(e, LookupEmbedder) or (e.penalty_weighted() and not weighted_ok):
                return False
        return True


class _TripleColumns:
    """A batch's triples as KgeModel.penalty reads them -- ``.to(device)``, then the index columns
    ``[:, S]``, ``[:, P]``, ``[:, O]`` -- served from three contiguous device vectors: a recorded
    step neither stacks them into a [B, 3] tensor nor copies its strided columns out again."""

    def __init__(self, s, p, o):
        self._cols = (s, p, o)

    def to(self, *args, **kwargs):
        return self

    def __len__(self):
        return len(self._cols[0])

    def __getitem__(self, key):
        rows, col = key
        if rows != slice(None) or not isinstance(col, int):
            raise IndexError("only whole columns [:, S | P | O] of the recorded triples are served")
        return self._cols[col]


class _GraphStep:
    """A training step recorded once as a HIP graph and replayed per batch (engine.graph_step).

    The step's device work is fixed for a full batch: one fused scoring / softmax pass over
    the stacked (s, p, ?) and (?, p, o) queries, its backward GEMMs and prep backward, the
    fused Adagrad kernels -- a dozen launches plus autograd bookkeeping on the host, which costs
    as long as the device work itself.  Two full batches run eagerly first (kernel
    attributes, optimizer state, allocator warm-up); the third is recorded (recording runs
    nothing) and replayed, and every later full batch is copied into the recorded index
    buffer and replayed.  The optimizer's host-side step counters are advanced per replay.
    A partial last batch, or any step the recording cannot take, runs eagerly.  Like any
    recorded graph it assumes the parameters and optimizer state stay where they are
    (in-place updates such as load_state_dict are fine; re-creating the tensors is not:
    call disable() or build a new job).

    Subclasses say what a batch's index block is: _block(batch) -> a flat int64 host tensor
    (None: this batch runs eagerly) that is uploaded into the first len(block) elements of the
    recorded device buffer of _capacity() elements, and _recorded_batch() -> the batch dict (views
    of that buffer) the job's process_batch is recorded with."""

    WARMUP = 2

    def __init__(self, job: "TrainingJob"):
        self.job = job
        self.graph = None
        self.static = None  # recorded flat int64 device index buffer
        self.pinned = []  # two pinned host staging buffers (+ their copy events) for the batch
        self.turn = 0
        self.loss = None  # recorded 0-dim loss
        self.penalty = None  # recorded 0-dim sum of the penalty terms (None: nothing regularises)
        self.stepped = []
        self.warm = 0
        self.disabled = False
        self.error = None  # why recording was abandoned, if it was
        self.hyper = None  # the optimizer's (lr, weight decay, eps) per group at recording time

    def disable(self):
        self.disabled = True
        self.graph = None

    def _hyper(self):
        return [(g["lr"], g.get("weight_decay"), g.get("eps")) for g in self.job.optimizer.param_groups]

    # ---- what a batch looks like (1vsAll: the [5, B] index block of TrainingJob1vsAll.INDEX_BLOCK)
    def _capacity(self) -> int:
        return len(TrainingJob1vsAll.INDEX_BLOCK) * self.job.batch_size

    def _block(self, batch):
        triples = batch["triples"]
        if triples.dim() != 2 or triples.shape[0] != self.job.batch_size:
            return None
        return triples.long()[:, list(TrainingJob1vsAll.INDEX_BLOCK)].t().reshape(-1)

    def _recorded_batch(self):
        return {"cols": self.static.view(len(TrainingJob1vsAll.INDEX_BLOCK), self.job.batch_size)}

    def _penalty_batch(self):
        """The batch the penalty terms are recorded with: the triples as columns of the block."""
        cols = self._recorded_batch()["cols"]
        s_row, o_row, p_row = (TrainingJob1vsAll.INDEX_BLOCK.index(c) for c in (S, O, P))
        # built on first use: only weighted penalties read the triples, and the stack is a kernel
        # that would otherwise be recorded into every step
        return {"triples": _TripleColumns(cols[s_row], cols[p_row], cols[o_row])}

    # ---- the step
    def run(self, batch_index, batch):
        job = self.job
        if self.disabled:
            return None
        if self.graph is None and self.warm < self.WARMUP:
            self.warm += 1
            return None  # the caller runs this batch eagerly
        if self.graph is not None and self._hyper() != self.hyper:
            # the learning rate is an argument of the recorded optimizer kernel: after an lr
            # scheduler (or anyone else) changed it, this batch is recorded anew
            self.graph = None
        t = -time.time()
        block = self._block(batch)
        if block is None or block.numel() > self._capacity():
            return None
        if self.graph is None:
            if not self._record(batch_index, block):
                return None
            # recording counted this step in the optimizer state already
        else:
            self._upload(block)
            job.optimizer.advance_steps(self.stepped)
        self.graph.replay()
        t += time.time()
        return TrainingJob._ProcessBatchResult(self._loss_of(block), job.batch_size, 0.0, t, 0.0)

    def _upload(self, block):
        """The batch's index block into the recorded device buffer, in stream order.  A copy from
        pageable memory would block the host until the device drains: staged through pinned memory
        (two buffers: the read of batch b - 1 may still be pending) and uploaded by a kernel."""
        n = block.numel()
        if not self.pinned:
            self.pinned = [[torch.empty(self._capacity(), dtype=torch.int64, pin_memory=True), None]
                           for _ in range(2)]
        slot = self.pinned[self.turn]
        self.turn ^= 1
        if slot[1] is not None:
            slot[1].synchronize()
        slot[0][:n].copy_(block)
        _lib.stage_i64(slot[0][:n], self.static[:n])  # a kernel, not a DMA copy, on this stream
        slot[1] = torch.cuda.Event()
        slot[1].record()

    def _loss_of(self, block):
        """The loss the step reports, from what the recording returned."""
        return self.loss

    def _pool(self):
        """The memory pool the recording allocates from (None: one of its own)."""
        return None

    def _record(self, batch_index, block) -> bool:
        job = self.job
        opt = job.optimizer
        steps = {p: st["step"].clone() for p, st in opt.state.items() if "step" in st}
        host = torch.zeros(self._capacity(), dtype=torch.int64)
        host[:block.numel()] = block
        if self.static is None:
            self.static = host.to(job.device)
        else:  # recorded again (another learning rate, another variant of the step): the same buffer
            self.static.copy_(host)
        opt.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, pool=self._pool()):
                res = job.process_batch(batch_index, self._recorded_batch())
                pen = job._penalty_backward(batch_index, self._penalty_batch())
                opt.step()
        except Exception as e:  # not recordable: this and every later batch run eagerly
            for p, s in steps.items():
                opt.state[p]["step"] = s
            opt.zero_grad(set_to_none=True)
            import traceback

            self.error = f"{type(e).__name__}: {e}\n{traceback.format_exc()}"
            job.config.log(f"engine.graph_step disabled: {self.error}")
            self.disable()
            return False
        if not torch.is_tensor(res.loss):
            self.error = "the recorded step returned a host loss"
            self.disable()
            return False
        self.graph = g
        self.hyper = self._hyper()
        self.loss = res.loss
        self.penalty = pen if torch.is_tensor(pen) else None
        self.stepped = [p for grp in opt.param_groups for p in grp["params"] if p.grad is not None]
        return True


class _KvsAllGraphStep(_GraphStep):
    """The KvsAll step as a recorded graph.  A batch is B query rows -- the (s, p, ?) queries
    stacked on the (?, p, o) queries, their split point differing from batch to batch -- with
    their positives as a CSR of varying length, so the recorded buffer is
        [entity index (B) | relation index (B) | label pointer (B + 1) | split point (1) | label columns (cap)]
    and the recorded kernels read the split point from it (kge_prep_query_split2, kge_loss_sums).
    A batch whose positives exceed the capacity (or a partial batch) runs eagerly."""

    def __init__(self, job):
        super().__init__(job)
        B = job.batch_size
        labels = sum(len(ix.values) for ix in job.query_indexes)
        mean = labels / max(1, job.num_examples)
        cap = 8192
        while cap < 2 * mean * B:
            cap *= 2
        self.cap = cap

    def _capacity(self) -> int:
        return 3 * self.job.batch_size + 2 + self.cap

    def _block(self, batch):
        ex = batch["examples"]
        if len(ex) != self.job.batch_size:
            return None
        return self.job._stacked_block(ex.numpy())

    def _recorded_batch(self):
        B = self.job.batch_size
        st = self.static
        return {"stacked": (st[:B], st[B:2 * B], st[2 * B:3 * B + 1], st[3 * B + 1:3 * B + 2], st[3 * B + 2:])}

    def _penalty_batch(self):
        return {}  # unweighted terms only (TrainingJobKvsAll._prepare): no indexes needed

    def _loss_of(self, block):
        # the recording returns both query types' losses; the reference reports the last query
        # type that has examples in the batch, which the host knows from the split point
        B = self.job.batch_size
        two = len(self.job._part_spec) == 2 and int(block[3 * B + 1]) < B
        return self.loss[1 if two else 0]


class _KvsAllSplitGraphStep(_KvsAllGraphStep):
    """The KvsAll step with dropout in the embedders: its two query types are scored one after the
    other (each against its own dropped copy of the entity table), so the shapes of a step depend
    on where the batch splits into (s, p, ?) and (?, p, o) queries.  ONE RECORDING PER SPLIT POINT:
    the split of a shuffled batch is binomial, a few dozen values occur at all, and every recording
    reads the same index buffer and allocates from one shared pool (a step's intermediates are dead
    when it ends; its loss is copied to the host before the next replay is issued).  Beyond
    MAX_GRAPHS different splits a batch runs eagerly."""

    MAX_GRAPHS = 160

    def __init__(self, job):
        super().__init__(job)
        self.graphs = {}  # split point -> (graph, loss, penalty, parameters it steps)
        self.n_first = 0
        self._shared_pool = None

    def disable(self):
        super().disable()
        self.graphs = {}

    def _pool(self):
        if self._shared_pool is None:
            self._shared_pool = torch.cuda.graph_pool_handle()
        return self._shared_pool

    def _recorded_batch(self):
        B = self.job.batch_size
        st = self.static
        return {"split": (st[:B], st[B:2 * B], st[2 * B:3 * B + 1], st[3 * B + 2:], self.n_first)}

    def _loss_of(self, block):
        return self.loss

    def run(self, batch_index, batch):
        job = self.job
        if self.disabled:
            return None
        if self.warm < self.WARMUP:
            self.warm += 1
            return None
        if self.graphs and self._hyper() != self.hyper:
            self.graphs = {}  # another learning rate: every split is recorded anew
        t = -time.time()
        block = self._block(batch)
        if block is None or block.numel() > self._capacity():
            return None
        B = job.batch_size
        n_first = int(block[3 * B + 1])
        entry = self.graphs.get(n_first)
        if entry is None:
            if len(self.graphs) >= self.MAX_GRAPHS:
                return None
            self.n_first = n_first
            self.graph = None
            if not self._record(batch_index, block):
                return None
            entry = self.graphs[n_first] = (self.graph, self.loss, self.penalty, self.stepped)
        else:
            self._upload(block)
            job.optimizer.advance_steps(entry[3])
        self.graph, self.loss, self.penalty, self.stepped = entry
        self.graph.replay()
        t += time.time()
        return TrainingJob._ProcessBatchResult(self.loss, B, 0.0, t, 0.0)


class TrainingJob1vsAll(TrainingJob):
    """Each (s, p, o) scores (s, p, ?) and (?, p, o) against all entities; CE loss."""

    #: triple columns of the rows of a batch's device index block: s, o, s, p, p
    INDEX_BLOCK = (S, O, S, P, P)

    def __init__(self, config, dataset, parent_job=None, model=None):
        super().__init__(config, dataset, parent_job, model=model)
        self.type_str = "1vsAll"
        self._graph_step = None
        self._sharded = None
        #: compute ops of the row-sharded path; None: the engine (kge.sharded.EngineOps).
        #: Tests inject CPU ops here to run the exchange logic over gloo.
        self.sharded_ops = None

    def _prepare(self):
        super()._prepare()
        self.num_examples = self.dataset.split(self.train_split).size(0)
        from ..sharded import sharding_enabled

        if sharding_enabled(self.config):
            self._sharded = ShardedTraining1vsAll(self)
            return
        opt = self.optimizer
        self._graph_step = None  # decided anew by every _prepare
        if (self.config.get("engine.graph_step") and self._fused_loss_kind() is not None
                and torch.device(self.device).type == "cuda"
                and hasattr(opt, "graph_safe") and opt.graph_safe()
                and not self.pre_batch_hooks  # e.g. the embedding normaliser re-creates the weights
                and self._penalties_recordable(weighted_ok=True)
                # plain lookups, or lookups with dropout (torch's dropout is recorded with the
                # step: every replay draws new masks)
                and (self.model._lookup_tables() is not None or self.model._lookup_embedders_with_dropout())):
            self._graph_step = _GraphStep(self)

    def _collate(self, example_ids):
        return {"triples": self.dataset.split(self.train_split)[example_ids, :].long()}

    def _penalty_backward(self, batch_index, batch):
        if self._sharded is not None:
            return self._sharded.penalty_backward(batch)
        return super()._penalty_backward(batch_index, batch)

    def _process_batch(self, batch_index, batch) -> TrainingJob._ProcessBatchResult:
        """train.py:1032-1062: sp then po, each loss / B followed by backward.  With
        engine.fused_loss and the kl loss, scoring + cross entropy + its gradient of both
        directions run as one engine op (KgeModel.score_sp_po_xent; per direction with
        score_sp_xent / score_po_xent when the scorer cannot share one contraction)."""
        if self._sharded is not None:
            return self._sharded.process_batch(batch)
        t = -time.time()
        if "cols" in batch:  # the [5, B] device index block (the replayed step stages it this way)
            cols = batch["cols"]
        else:
            triples = batch["triples"].to(self.device, non_blocking=True)
            cols = triples.t()[list(self.INDEX_BLOCK)].contiguous()
        # Rows s, o, s, p, p: the stacked queries of the fused step read ONE contiguous vector each
        # for their entity indexes (s | o), their labels (o | s) and their relation indexes (p | p)
        s_, o_, s2_, p_, p2_ = cols[0], cols[1], cols[2], cols[3], cols[4]
        bs = cols.shape[1]
        t += time.time()
        fused = self._fused_loss_kind() is not None
        fwd = -time.time()
        both = None
        if fused:
            both = self.model.score_xent_parts(self.model.xent_part_sp(s_, p_, o_),
                                               self.model.xent_part_po(p2_, o_, s2_), 1.0 / bs)
        if both is not None:  # sp_ and _po in one engine pass; one backward (same gradient sum)
            total, _ = both
            fwd += time.time()
            bwd = -time.time()
            self._backward(total)  # a persistent seed gradient: no fill kernel per step
            bwd += time.time()
            return TrainingJob._ProcessBatchResult(total.detach(), bs, t, fwd, bwd)
        loss_sp = self.model.score_sp_xent(s_, p_, o_, 1.0 / bs) if fused else None
        if loss_sp is None:
            scores_sp = self.model.score_sp(s_, p_)
            loss_sp = self.loss(scores_sp, o_) / bs
            del scores_sp
        fwd += time.time()
        bwd = -time.time()
        loss_sp.backward()
        bwd += time.time()
        fwd -= time.time()
        loss_po = self.model.score_po_xent(p_, o_, s_, 1.0 / bs) if fused else None
        if loss_po is None:
            scores_po = self.model.score_po(p_, o_)
            loss_po = self.loss(scores_po, s_) / bs
            del scores_po
        fwd += time.time()
        bwd -= time.time()
        loss_po.backward()
        bwd += time.time()
        return TrainingJob._ProcessBatchResult(loss_sp.detach() + loss_po.detach(), bs, t, fwd, bwd)


class ShardedTraining1vsAll:
    """TrainingJob1vsAll over an entity table row-sharded across the processes of a
    torch.distributed world (one per GPU; kge.sharded.RowShardedScorer.train_1vsall_global):
    vocab-parallel softmax cross entropy (train.loss kl) or per-shard binary cross entropy (bce), no
    score or gradient matrix on the link.

    Every rank steps through the same global batches (the batch order is broadcast from
    rank 0) and HOLDS only rows [lo, hi) of the entity table: the model's entity embedder is
    cut down to them (LookupEmbedder.shard_rows), so the parameter, its gradient and its
    optimizer state are [hi - lo, d] -- at the Wikidata5M shape on 8 GPUs 1.18 GB each instead
    of 9.4 GB.  The whole table exists only where ``sync_model`` assembles it (an all-gather:
    at the end of training, for checkpoints or unsharded scoring).  The relation table is
    replicated: every rank applies the same all-reduced gradient.  The objective and its
    gradients equal the unsharded job's (train.py:1032-1062)."""

    def __init__(self, job: "TrainingJob1vsAll"):
        import torch.distributed as dist

        from ..sharded import RowShardedScorer, engine_ops_for, shard_bounds

        if isinstance(job.loss, KLDivWithSoftmaxKgeLoss):
            self.loss = ("kl", 0.0)
        elif type(job.loss) is BCEWithLogitsKgeLoss and not job.loss._mean:
            self.loss = ("bce", float(job.loss._offset))  # elementwise: no statistics cross the shards
        else:
            raise NotImplementedError("row-sharded 1vsAll training supports train.loss kl and bce")
        if job.model._lookup_tables() is None and job.sharded_ops is None:
            raise NotImplementedError("row-sharded training needs plain lookup embedders and an engine scorer")
        self.job = job
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.embedder = job.model.get_s_embedder()
        if self.embedder is not job.model.get_o_embedder():
            raise NotImplementedError("row-sharded training needs one entity embedder for subjects and objects")
        rel_w = job.model.get_p_embedder()._embeddings.weight
        E = self.embedder.vocab_size
        self.lo, self.hi = shard_bounds(E, self.world, self.rank)
        # the model keeps this rank's rows only; they are the live, trained copy
        self.ent_param = self.embedder.shard_rows(self.lo, self.hi)
        self.rel_param = rel_w
        ops = job.sharded_ops if job.sharded_ops is not None else engine_ops_for(job.model)
        self.scorer = RowShardedScorer(self.ent_param.data, self.lo, self.hi, E, rel_w.data, ops)
        job.optimizer = KgeOptimizer.create(job.config, params=[self.ent_param, self.rel_param])
        job.kge_lr_scheduler = KgeLRScheduler(job.config, job.optimizer)

    def reshard(self):
        """After sync_model put the whole table into the model: hand the model this rank's rows
        again (the parameter the optimizer holds; it has been the live copy all along) and drop
        the assembled table."""
        if self.embedder.shard is None:
            self.embedder.install_rows(self.ent_param, self.lo, self.hi)

    def broadcast(self, cpu_tensor: torch.Tensor) -> torch.Tensor:
        """rank 0's value of a CPU tensor on every rank (staged through the job's device when
        the backend moves device memory only)."""
        import torch.distributed as dist

        if dist.get_backend() == "gloo":
            t = cpu_tensor.clone()
            dist.broadcast(t, src=0)
            return t
        t = cpu_tensor.to(self.job.device)
        dist.broadcast(t, src=0)
        return t.cpu()

    def process_batch(self, batch) -> "TrainingJob._ProcessBatchResult":
        t = -time.time()
        self.reshard()
        host = batch["triples"].long()
        triples = host.to(self.job.device)
        t += time.time()
        fwd = -time.time()
        loss, d_ent, d_rel = self.scorer.train_1vsall_global(triples, host_triples=host if not host.is_cuda else None,
                                                             loss=self.loss)
        fwd += time.time()
        self.ent_param.grad = d_ent
        self.rel_param.grad = d_rel
        return TrainingJob._ProcessBatchResult(loss, len(triples), t, fwd, 0.0)

    def penalty_backward(self, batch):
        """The embedders' Lp penalty terms of the batch (kge_model.py:588-605,
        lookup_embedder.py:112-158) on the row-sharded table: each rank differentiates the
        entity terms over ITS rows -- its share of the whole-table norm, or the subjects and
        objects of the global batch that fall into its shard, divided by the batch's full
        index count -- and every rank the replicated relation term.  Returns the value the
        unsharded job reports: the ranks' entity parts summed, plus the relation term."""
        from ..sharded import all_reduce

        model = self.job.model
        ent_e, rel_e = model.get_s_embedder(), model.get_p_embedder()
        if not (ent_e.penalty_active() or rel_e.penalty_active()):
            return 0.0
        triples = batch["triples"].to(self.job.device).long()
        local = torch.zeros((), device=triples.device)
        replicated = torch.zeros((), device=triples.device)
        with torch.enable_grad():
            for emb, param, cols in ((ent_e, self.ent_param, (S, O)), (rel_e, self.rel_param, (P,))):
                if not emb.penalty_active():
                    continue
                for col in cols:
                    idx = triples[:, col]
                    if param is self.ent_param:
                        idx = idx[(idx >= self.lo) & (idx < self.hi)] - self.lo
                    value = emb.lp_term(param, idx, len(triples))
                    value.backward()  # adds to the gradient process_batch left on the parameter
                    if param is self.ent_param:
                        local += value.detach()
                    else:
                        replicated += value.detach()
        return all_reduce(local) + replicated

    def sync_model(self):
        """All-gather the shards into the whole entity table and install it in the model (before
        unsharded scoring, or to save the model): the one place the whole table exists.  The next
        training batch drops it again (reshard)."""
        self.embedder.unshard(self.gather_rows(self.ent_param.data))

    def gather_rows(self, shard_rows: torch.Tensor) -> torch.Tensor:
        """The whole [E, d] table from every rank's [hi - lo, d] rows (a collective)."""
        from ..sharded import RowShardedScorer

        sc = self.scorer
        return RowShardedScorer(shard_rows, sc.lo, sc.hi, sc.E, sc.rel, sc.ops, sc.group).all_gather_table()

    def full_state(self, state: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """A state_dict taken while the model held this rank's rows only (TrainingJob.best_state)
        with the entity table assembled from every rank's copy -- a collective: every rank calls
        it with its own state."""
        key = next(n for n, p in self.job.model.named_parameters() if p is self.embedder._embeddings.weight)
        out = dict(state)
        if tuple(out[key].shape) == (self.hi - self.lo, self.embedder.dim):
            out[key] = self.gather_rows(out[key].to(self.ent_param.device))
        return out


class TrainingJobKvsAll(TrainingJob):
    """Queries (s, p, ?) / (?, p, o) with all their training answers as a label matrix
    (train.py:493-756); KL loss on log_softmax of the scores."""

    def __init__(self, config, dataset, parent_job=None, model=None):
        super().__init__(config, dataset, parent_job, model=model)
        self.label_smoothing = config.get("KvsAll.label_smoothing")
        if self.label_smoothing < 0:
            self.label_smoothing = 0.0
        elif 0 < self.label_smoothing <= 1.0 / dataset.num_entities():
            self.label_smoothing = 1.0 / dataset.num_entities()
        self.type_str = "KvsAll"
        self._graph_step = None

    def _prepare(self):
        super()._prepare()
        self._replicas_only()
        self.query_types = [k for k, v in self.config.get("KvsAll.query_types").items() if v]
        self.query_indexes = []
        self.query_last_example = []
        self.num_examples = 0
        index_of = {"sp_": "sp_to_o", "s_o": "so_to_p", "_po": "po_to_s"}  # train.py:568-577
        for qt in self.query_types:
            idx = self.dataset.index(f"{self.train_split}_{index_of[qt]}")
            self.query_indexes.append(idx)
            self.num_examples += len(idx)
            self.query_last_example.append(self.num_examples)
        # How the model scores each query type, as (engine direction, key column of the entity
        # index, key column of the relation index, offset added to the relation index): asked of
        # the model itself (a reciprocal-relations model answers (?, p, o) as (o, p + R, ?)).
        # (s, ?, o) queries score relations (KgeModel.score_so): outside the engine's all-entities
        # passes, they run per query type through the scorer's generic path.
        entity_targets = "s_o" not in self.query_types
        self._part_spec = []
        for qt in self.query_types:
            k0, k1 = torch.tensor([0]), torch.tensor([1])
            if qt == "s_o":
                self._part_spec.append(None)
                continue
            if qt == "sp_":  # keys (s, p)
                d, e, r, _, _ = self.model.xent_part_sp(k0, k1, None)
            else:  # keys (p, o)
                d, e, r, _, _ = self.model.xent_part_po(k0, k1, None)
            e_col = 0 if int(e[0]) == 0 else 1
            self._part_spec.append((d, e_col, 1 - e_col, int(r[0]) - (1 - e_col)))
        from ..sharded import sharding_enabled

        opt = self.optimizer
        self._graph_step = None  # decided anew by every _prepare
        if (self.config.get("engine.graph_step") and self._fused_loss_kind() is not None
                and 1 <= len(self.query_types) <= 2 and entity_targets
                and torch.device(self.device).type == "cuda"
                and hasattr(opt, "graph_safe") and opt.graph_safe()
                and not self.pre_batch_hooks
                and not sharding_enabled(self.config)
                and self._penalties_recordable(weighted_ok=False)):  # its triples vary in number
            if self._stacked_applicable():
                self._graph_step = _KvsAllGraphStep(self)
            elif self._split_applicable():
                self._graph_step = _KvsAllSplitGraphStep(self)

    def _split_applicable(self) -> bool:
        """Whether the step can be recorded per split point (_KvsAllSplitGraphStep): lookup
        embedders whose only addition is dropout (the fused loss in its embedding-row form)."""
        from ..model.reciprocal_relations_model import ReciprocalRelationsModel

        m = self.model
        return (not isinstance(m, ReciprocalRelationsModel) and m._lookup_tables() is None
                and m._lookup_embedders_with_dropout() and self._fused_loss_kind()[0] == "kl")

    def _process_split(self, split, bs):
        """The recorded step's body when the query types are scored one after the other (dropout):
        rows [0, n_first) of the device block of _stacked_block are the first query type's, the
        rest the second's; n_first is a host integer (one recording per value)."""
        eidx, ridx, l_ptr, l_col, n_first = split
        spans = [(0, 0, n_first)] if len(self._part_spec) == 1 else [(0, 0, n_first), (1, n_first, bs)]
        fwd = bwd = 0.0
        total = None
        for qi, a, b in spans:
            if b <= a:
                continue
            fwd -= time.time()
            # (the label pointer keeps its absolute positions into l_col)
            loss = self.model._xent_dropout(eidx[a:b], ridx[a:b], self._part_spec[qi][0], l_col, 1.0 / bs,
                                            l_ptr[a:b + 1], self.label_smoothing)
            fwd += time.time()
            bwd -= time.time()
            loss.backward()
            bwd += time.time()
            total = loss.detach()  # the reference keeps the last query type's value
        return TrainingJob._ProcessBatchResult(total, bs, 0.0, fwd, bwd)

    def _stacked_applicable(self) -> bool:
        """Whether the recorded step's engine pass (KgeModel.score_xent_stacked) serves this model."""
        from .. import _lib, engine

        tabs = self.model._lookup_tables()
        scorer = self.model.get_scorer()
        if tabs is None or scorer.engine_kind is None:
            return False
        dirs = [(_lib.DIR_SP if spec[0] == "sp_" else _lib.DIR_PO) for spec in self._part_spec]
        return engine.stacked_xent_applicable(scorer.engine_kind, scorer.precision(), tabs[0].detach(), dirs[0],
                                              dirs[-1])

    def _stacked_block(self, ex: np.ndarray):
        """The batch as ONE flat int64 block for the recorded step (_KvsAllGraphStep): stacked
        entity indexes [B], relation indexes [B], label pointer [B + 1], the number of rows of
        the first query type [1], label columns [nnz] -- the first query type's rows first."""
        e_parts, r_parts, len_parts, col_parts = [], [], [], []
        start = 0
        n_first = 0
        for qi, (_, e_col, r_col, r_off) in enumerate(self._part_spec):
            end = self.query_last_example[qi]
            sel = ex[(ex >= start) & (ex < end)] - start
            start = end
            ix = self.query_indexes[qi]
            keys = ix.keys[sel]
            lo = ix.offsets[sel]
            lens = ix.offsets[sel + 1] - lo
            tot = int(lens.sum())
            ends = np.cumsum(lens)
            pos = np.arange(tot, dtype=np.int64) - np.repeat(ends - lens, lens) + np.repeat(lo, lens)
            e_parts.append(keys[:, e_col])
            r_parts.append(keys[:, r_col] + r_off)
            len_parts.append(lens)
            col_parts.append(ix.values[pos])
            if qi == 0:
                n_first = len(sel)
        n = len(ex)
        if len(self._part_spec) == 1:
            n_first = n
        l_ptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(np.concatenate(len_parts), out=l_ptr[1:])
        block = np.concatenate(e_parts + r_parts + [l_ptr, np.asarray([n_first], dtype=np.int64)] + col_parts)
        return torch.from_numpy(block.astype(np.int64, copy=False))

    def _process_stacked(self, stacked, bs):
        """The recorded step's body: both query types from the device block of _stacked_block."""
        eidx, ridx, l_ptr, n_first, l_col = stacked
        dirs = [spec[0] for spec in self._part_spec]
        fwd = -time.time()
        losses = self.model.score_xent_stacked(dirs[0], dirs[-1], eidx, ridx, n_first, l_col, l_ptr, 1.0 / bs,
                                               self.label_smoothing)
        fwd += time.time()
        if losses is None:
            raise RuntimeError("the scorer cannot run both query types in one engine pass")
        total, per_type = losses
        bwd = -time.time()
        self._backward(total)
        bwd += time.time()
        # both query types' losses: the caller picks the one the reference would report
        return TrainingJob._ProcessBatchResult(per_type, bs, 0.0, fwd, bwd)

    def _collate(self, example_ids):
        batch = {"examples": example_ids}
        if self._weighted_penalty():
            batch["triples"] = self._batch_triples(example_ids.numpy())
        return batch

    def _weighted_penalty(self) -> bool:
        """Whether a penalty term weights embeddings by their frequency in the batch's triples."""
        m = self.model
        return any(getattr(e, "penalty_weighted", lambda: False)()
                   for e in (m.get_s_embedder(), m.get_p_embedder(), m.get_o_embedder()))

    def _batch_triples(self, ex: np.ndarray) -> torch.Tensor:
        """All true triples of the batch, one per (query, label) in batch order (train.py:625-674):
        what weighted penalties count index frequencies on."""
        qt_of = np.searchsorted(np.asarray(self.query_last_example), ex, side="right")
        starts = np.concatenate(([0], np.asarray(self.query_last_example[:-1], dtype=np.int64)))
        lens = np.zeros(len(ex), dtype=np.int64)
        for qi, ix in enumerate(self.query_indexes):
            sel = np.nonzero(qt_of == qi)[0]
            local = ex[sel] - starts[qi]
            lens[sel] = ix.offsets[local + 1] - ix.offsets[local]
        first = np.zeros(len(ex) + 1, dtype=np.int64)
        np.cumsum(lens, out=first[1:])
        triples = np.zeros((int(first[-1]), 3), dtype=np.int64)
        for qi, (qt, ix) in enumerate(zip(self.query_types, self.query_indexes)):
            sel = np.nonzero(qt_of == qi)[0]
            if len(sel) == 0:
                continue
            local = ex[sel] - starts[qi]
            n = lens[sel]
            rows = np.repeat(first[sel], n) + np.arange(int(n.sum()), dtype=np.int64) - np.repeat(np.cumsum(n) - n, n)
            pos = np.repeat(ix.offsets[local], n) + np.arange(int(n.sum()), dtype=np.int64) - np.repeat(
                np.cumsum(n) - n, n)
            k1_col, k2_col, target_col = {"sp_": (S, P, O), "s_o": (S, O, P), "_po": (P, O, S)}[qt]
            triples[rows, k1_col] = np.repeat(ix.keys[local, 0], n)
            triples[rows, k2_col] = np.repeat(ix.keys[local, 1], n)
            triples[rows, target_col] = ix.values[pos]
        return torch.from_numpy(triples)

    def _queries(self, qi, sel):
        """(query pairs [n, 2], label CSR pointer [n + 1], label columns) of the selected
        examples of query type qi, on the device.  Built on the host from the index (numpy)
        and shipped in ONE pinned non-blocking copy: no device sync (a device-side build
        needs the label count on the host, i.e. a sync that drains the queue every batch)."""
        ix = self.query_indexes[qi]
        q = ix.keys[sel].astype(np.int64, copy=False)
        lo = ix.offsets[sel].astype(np.int64, copy=False)
        lens = ix.offsets[sel + 1].astype(np.int64, copy=False) - lo
        l_ptr = np.zeros(len(sel) + 1, dtype=np.int64)
        np.cumsum(lens, out=l_ptr[1:])
        pos = np.arange(l_ptr[-1], dtype=np.int64) - np.repeat(l_ptr[:-1], lens) + np.repeat(lo, lens)
        l_col = ix.values[pos].astype(np.int64, copy=False)
        n = len(sel)
        host = torch.from_numpy(np.concatenate((q.reshape(-1), l_ptr, l_col)))
        if torch.device(self.device).type == "cuda":
            host = host.pin_memory()
        dev = host.to(self.device, non_blocking=True)
        return dev[:2 * n].view(n, 2), dev[2 * n:3 * n + 1], dev[3 * n + 1:]

    def _process_batch(self, batch_index, batch) -> TrainingJob._ProcessBatchResult:
        if "stacked" in batch:
            return self._process_stacked(batch["stacked"], self.batch_size)
        if "split" in batch:
            return self._process_split(batch["split"], self.batch_size)
        t = -time.time()
        ex = batch["examples"].numpy()
        bs = len(ex)
        E = self.dataset.num_entities()
        t += time.time()
        fwd = bwd = 0.0
        total = None
        fused = self._fused_loss_kind() is not None
        if fused and len(self.query_types) == 2 and "s_o" not in self.query_types:
            res = self._process_batch_fused2(ex, bs)
            if res is not None:
                return res
        start = 0
        for qi, qt in enumerate(self.query_types):
            end = self.query_last_example[qi]
            sel = ex[(ex >= start) & (ex < end)] - start
            start = end
            if len(sel) == 0:
                continue
            t -= time.time()
            q, l_ptr, l_col = self._queries(qi, sel)
            loss = None
            if fused and qt != "s_o":
                # positives as a CSR (no dense label matrix); KL + gradient in the engine
                t += time.time()
                fwd -= time.time()
                fn = self.model.score_sp_kl if qt == "sp_" else self.model.score_po_kl
                loss = fn(q[:, 0], q[:, 1], l_ptr, l_col, self.label_smoothing, 1.0 / bs)
                fwd += time.time()
                t -= time.time()
            if loss is None:
                width = self.dataset.num_relations() if qt == "s_o" else E
                labels = torch.zeros(len(sel), width, device=self.device)
                rows = torch.repeat_interleave(torch.arange(len(sel), device=self.device), l_ptr[1:] - l_ptr[:-1])
                labels[rows, l_col] = 1.0
                if self.label_smoothing > 0.0 and qt != "s_o":  # entity targets only (train.py:715-721)
                    labels = (1.0 - self.label_smoothing) * labels + 1.0 / E
                t += time.time()
                fwd -= time.time()
                if qt == "sp_":
                    scores = self.model.score_sp(q[:, 0], q[:, 1])
                elif qt == "s_o":
                    scores = self.model.score_so(q[:, 0], q[:, 1])
                else:
                    scores = self.model.score_po(q[:, 0], q[:, 1])
                loss = self.loss(scores, labels) / bs
                fwd += time.time()
            else:
                t += time.time()
            bwd -= time.time()
            loss.backward()
            bwd += time.time()
            total = loss.detach()  # reference keeps the last query type's value
        return TrainingJob._ProcessBatchResult(total if total is not None else 0.0, bs, t, fwd, bwd)

    def _process_batch_fused2(self, ex, bs):
        """Both query types of the batch in one engine pass (KgeModel.score_xent_parts):
        one contraction, one KL launch and one backward for the stacked sp_ and _po query
        rows; the reported loss is the last query type's, as in the reference.
        None when a query type has no example in this batch or the scorer cannot fuse."""
        t = -time.time()
        parts, start = [], 0
        for qi, qt in enumerate(self.query_types):
            end = self.query_last_example[qi]
            sel = ex[(ex >= start) & (ex < end)] - start
            start = end
            if len(sel) == 0:
                return None
            q, l_ptr, l_col = self._queries(qi, sel)
            part = self.model.xent_part_sp if qt == "sp_" else self.model.xent_part_po
            parts.append(part(q[:, 0], q[:, 1], l_col, l_ptr))
        t += time.time()
        fwd = -time.time()
        losses = self.model.score_xent_parts(parts[0], parts[1], 1.0 / bs, self.label_smoothing)
        fwd += time.time()
        if losses is None:
            return None
        total, per_type = losses
        bwd = -time.time()
        self._backward(total)
        bwd += time.time()
        return TrainingJob._ProcessBatchResult(per_type[1], bs, t, fwd, bwd)
