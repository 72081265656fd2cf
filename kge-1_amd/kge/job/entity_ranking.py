"""Entity-ranking evaluation (EvaluationJob eval.py:10-132, EntityRankingJob
entity_ranking.py:11-577) as an on-device pipeline.

Per batch of evaluation triples:
  1. true scores via KgeModel.score_spo (entity_ranking.py:139-140);
  2. per entity chunk, the scores of KgeModel.score_sp_po stacked by rows -- (s, p, ?)
     queries on top of (?, p, o) queries, one engine pass (entity_ranking.py:153-168);
  3. kge_rank_rows, one launch for both directions: raw / filtered / filtered-with-test
     greater & tie counts straight from the score chunk, the true entry replaced by the true
     score, filtering applied from per-query CSR lists of known answers
     (entity_ranking.py:172-216, 469-529);
  4. tie handling + rank histograms (entity_ranking.py:531-551, eval.py:148-171): in the same
     launch when one chunk covers every entity, else kge_rank_hist_multi after the last chunk.
The filter lists are built once per job from the dataset splits (vectorised numpy)
instead of the reference's per-triple Python collate (job/util.py:5-38).  Counts are sums
over chunks, which is exactly the reference's chunk_size decomposition and the
per-shard reduction of the row-sharded multi-GPU path (kge.sharded).
"""
from __future__ import annotations

import contextlib
import time
from typing import Dict, List

import numpy as np
import torch

from .. import _lib
from ..dataset import KvsAllIndex
from .job import Job

#: engine.eval_precision value: bf16x3 contraction, near-ties of the true score rescored exactly
REFINED = "bf16x3_refined"


def refine_band(d: int) -> float:
    """Refinement band of kge_rank_rows relative to |q_i| * max_j |t_j|: a bound on the error of
    the bf16x3 contraction of d-wide rows.

    Representation: every operand x is split as hi = bf16(x), lo = bf16(x - hi), both rounded to
    nearest (v_cvt_pk_bf16_f32; x - hi is exact in fp32), so |lo| <= 2^-9 (1 + 2^-9) |x| and the
    rest r = x - hi - lo has |r| <= 2^-18 |x|.  The contraction sums hi hi + hi lo + lo hi (each
    product exact in fp32); against the exact product it lacks lo_q lo_t + r_q t + (hi_q + lo_q) r_t,
    at most (1 + 2^-8 + 1 + 1 + 2^-18) 2^-18 < 0.76 * 2^-16 of |q_k t_k|.  2^-16 covers it with a
    third to spare (the band's own fp32 arithmetic needs 1e-6 of it).
    Accumulation: the 3 d products are added in fp32 (inside the MFMA and across K stages): at
    most 3 d * 2^-25 of sum_k |q_k t_k| on average partial sums.
    And sum_k |q_k t_k| <= |q| |t|.  (Measured errors on N(0, 0.1) tables at d = 512: below 2e-6
    in these units, against a band of 6.1e-5.)"""
    return 2.0 ** -16 + 3 * d * 2.0 ** -25


RANKING_SUFFIX = {"_raw": "", "_filt": "_filtered", "_filt_test": "_filtered_with_test"}


class EvaluationJob(Job):
    def __init__(self, config, dataset, parent_job=None, model=None):
        super().__init__(config, dataset, parent_job)
        self.model = model
        self.batch_size = config.get("eval.batch_size")
        max_k = min(dataset.num_entities(), max(config.get("entity_ranking.hits_at_k_s")))
        self.hits_at_k_s = [k for k in config.get("entity_ranking.hits_at_k_s") if k <= max_k]
        self.eval_split = config.get("eval.split")
        self.filter_splits = list(config.get("entity_ranking.filter_splits"))
        if self.eval_split not in self.filter_splits:
            self.filter_splits.append(self.eval_split)
        self.filter_with_test = config.get("entity_ranking.filter_with_test")
        self.epoch = -1
        self.post_epoch_trace_hooks = []

    @staticmethod
    def create(config, dataset, parent_job=None, model=None):
        if config.get("eval.type") == "entity_ranking":
            return EntityRankingJob(config, dataset, parent_job=parent_job, model=model)
        raise ValueError("eval.type")


def _csr_minus(ptr_a, col_a, ptr_b, col_b, num_entities):
    """Per-row set difference A \\ B of two CSRs with the same rows."""
    n = len(ptr_a) - 1
    ra = np.repeat(np.arange(n, dtype=np.int64), np.diff(ptr_a))
    rb = np.repeat(np.arange(n, dtype=np.int64), np.diff(ptr_b))
    keep = ~np.isin(ra * num_entities + col_a, rb * num_entities + col_b)
    col = col_a[keep]
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(ra[keep], minlength=n), out=ptr[1:])
    return ptr, col


class EntityRankingJob(EvaluationJob):
    def __init__(self, config, dataset, parent_job=None, model=None):
        super().__init__(config, dataset, parent_job, model)
        self.tie_handling = config.check(
            "entity_ranking.tie_handling", ["rounded_mean_rank", "best_rank", "worst_rank"])
        #: additional metrics per slot: "..._head" ranks the subject of (?, p, o), "..._tail" the
        #: object of (s, p, ?) (eval.py:125-146)
        self.head_and_tail = config.get("entity_ranking.metrics_per.head_and_tail")
        #: metrics per relation class and per training-frequency quartile of the ranked slot's
        #: query arguments (eval.py:174-224)
        self.per_relation_type = config.get("entity_ranking.metrics_per.relation_type")
        self.per_argument_frequency = config.get("entity_ranking.metrics_per.argument_frequency")
        #: compute ops of the row-sharded path; None: the engine (kge.sharded.EngineOps)
        self.sharded_ops = None
        self.capture_ranks = False  # keep per-query ranks in self.ranks (tests / tracing)
        self._refine = False  # set per run from engine.eval_precision
        self._streams = None  # engine.BatchStreams, made by the first run
        self._rank_weights = None  # [2, E] fp64: ranks 1..E and their fp32 reciprocals
        self._graph_state = {}  # engine.graph_eval: the recorded device pass and what it depends on
        self.ranks: Dict[str, np.ndarray] = {}

    # ---------------------------------------------------------------- preparation
    def _filter_index(self, splits: List[str]):
        key = "filter:" + "+".join(sorted(splits))
        cache = self.dataset._indexes
        if key not in cache:
            t = np.concatenate([self.dataset.split(s).numpy() for s in splits]).astype(np.int64)
            cache[key] = (KvsAllIndex(t, (0, 1), 2), KvsAllIndex(t, (1, 2), 0))
        return cache[key]

    def _prepare(self):
        self.model.prepare_job(self)
        from ..model.reciprocal_relations_model import ReciprocalRelationsModel

        self._two_sided = isinstance(self.model, ReciprocalRelationsModel)
        self.triples = self.dataset.split(self.eval_split).long()
        tri = self.triples.numpy()
        E = self.dataset.num_entities()
        # triples per launch group: eval.batch_size, raised to engine.eval_batch_size while the
        # [2B, chunk] block of a group stays below 8 GiB as fp32 scores
        chunk = self.config.get("entity_ranking.chunk_size")
        cols = E if chunk is None or chunk <= 0 else min(E, chunk)
        self._bs = max(self.batch_size, min(int(self.config.get("engine.eval_batch_size")), (1 << 30) // max(cols, 1)))
        self.use_test = "test" not in self.filter_splits and self.filter_with_test
        self.rankings = ["_raw", "_filt", "_filt_test"] if self.use_test else ["_raw", "_filt"]
        f_sp, f_po = self._filter_index(self.filter_splits)
        csr = {"sp": f_sp.csr_for(tri[:, [0, 1]]), "po": f_po.csr_for(tri[:, [1, 2]])}
        dev = self.device
        self._f = {k: (torch.from_numpy(p).to(dev), torch.from_numpy(c if len(c) else np.zeros(1, np.int64)).to(dev))
                   for k, (p, c) in csr.items()}
        self._t = None
        tcsr = None
        if self.use_test:
            t_sp, t_po = self._filter_index(["test"])
            tcsr = {"sp": _csr_minus(*t_sp.csr_for(tri[:, [0, 1]]), *csr["sp"], E),
                    "po": _csr_minus(*t_po.csr_for(tri[:, [1, 2]]), *csr["po"], E)}
            self._t = {k: (torch.from_numpy(p).to(dev),
                           torch.from_numpy(c if len(c) else np.zeros(1, np.int64)).to(dev))
                       for k, (p, c) in tcsr.items()}
        # the stacked ranking launch (kge_rank_rows) reads both directions' lists from ONE column
        # array: the (?, p, o) pointers are shifted behind the (s, p, ?) columns
        self._stacked = [self._stack_csr(csr, dev), self._stack_csr(tcsr, dev) if tcsr is not None else None]
        # per batch the index vectors [s_b | o_b] and [p_b | p_b], batch after batch: the stacked
        # (s, p, ?) / (?, p, o) queries of a batch read ONE contiguous entity-index vector and one
        # relation-index vector (no per-batch gather or concatenation)
        se, sp = [], []
        for b0 in range(0, len(self.triples), self._bs):
            t = self.triples[b0:b0 + self._bs]
            se += [t[:, 0], t[:, 2]]
            sp += [t[:, 1], t[:, 1]]
        self._stack_e = torch.cat(se).contiguous().to(dev) if se else torch.zeros(0, dtype=torch.int64, device=dev)
        self._stack_p = torch.cat(sp).contiguous().to(dev) if sp else torch.zeros(0, dtype=torch.int64, device=dev)

        self._prepare_groups(tri, dev)

    def _prepare_groups(self, tri: np.ndarray, dev):
        """Per evaluation triple and ranking direction (0: object of (s, p, ?), 1: subject of
        (?, p, o)) the group of each requested breakdown; -1 leaves the rank out of it.
        self._groups: name -> (group names, ids [2, N] on the device)."""
        from ..dataset import PERCENTILES

        self._groups = {}
        s, p, o = tri[:, 0].astype(np.int64), tri[:, 1].astype(np.int64), tri[:, 2].astype(np.int64)
        if self.per_relation_type:
            names = list(self.dataset.index("relations_per_type"))
            of_type = {k: i for i, k in enumerate(names)}
            type_of_rel = np.array([of_type[k] for k in self.dataset.index("relation_types")], np.int64)
            g = type_of_rel[p] if len(p) else p
            self._groups["relation_type"] = (names, torch.from_numpy(np.stack([g, g])).to(dev))
        if self.per_argument_frequency:
            percs = self.dataset.index("frequency_percentiles")
            names = [name for name, _, _ in PERCENTILES]

            def quartile_of(arg, num, ids):
                q = np.full(num, -1, np.int64)
                for gi, name in enumerate(names):
                    members = np.fromiter(percs[arg][name], np.int64, len(percs[arg][name]))
                    q[members] = gi
                return q[ids] if len(ids) else ids

            E, R = self.dataset.num_entities(), self.dataset.num_relations()
            none = np.full(len(p), -1, np.int64)
            gp = quartile_of("relation", R, p)
            for arg, ids in (("subject", np.stack([none, quartile_of("subject", E, s)])),
                             ("relation", np.stack([gp, gp])),
                             ("object", np.stack([quartile_of("object", E, o), none]))):
                self._groups[arg] = (names, torch.from_numpy(ids).to(dev))

    def _count_groups(self, group_hists, rk, b0, B):
        """Adds the ranks rk [ranking, direction, B] of the batch at b0 to every breakdown's
        histograms [ranking, direction, group (+ one unused slot for left-out ranks), rank]."""
        nrank = rk.shape[0]
        for name, (names, ids) in self._groups.items():
            h = group_hists[name]
            G1, E = h.shape[2], h.shape[3]
            g = ids[:, b0:b0 + B]
            g = torch.where(g < 0, G1 - 1, g)
            slot = torch.arange(nrank * 2, device=rk.device).view(nrank, 2, 1)
            idx = ((slot * G1 + g.unsqueeze(0)) * E + rk).view(-1)
            h.view(-1).index_add_(0, idx, torch.ones(idx.numel(), device=rk.device))

    @staticmethod
    def _stack_csr(csr, dev):
        (p_sp, c_sp), (p_po, c_po) = csr["sp"], csr["po"]
        col = np.concatenate([c_sp, c_po, np.zeros(1, np.int64)]).astype(np.int64)
        return (torch.from_numpy(p_sp.astype(np.int64)).to(dev),
                torch.from_numpy((p_po + len(c_sp)).astype(np.int64)).to(dev), torch.from_numpy(col).to(dev))

    # ---------------------------------------------------------------- evaluation
    @torch.no_grad()
    def _run(self) -> dict:
        """Scores with engine.eval_precision for the whole run, whatever precision training
        uses: ranks compare near-ties and the reference ranks fp32 scores, so evaluation either
        contracts in fp32 or contracts in bf16x3 and rescores every near-tie of the true score
        exactly (bf16x3_refined; kge_rank_rows)."""
        scorer = self.model.get_scorer()
        saved = scorer.precision_override
        name = self.config.check("engine.eval_precision", list(_lib.PRECISIONS) + [REFINED])
        self._refine = name == REFINED
        if self._refine:
            # models without a split contraction rank exact-fp32 scores (decided in _run_ranking)
            name = "bf16x3"
        scorer.precision_override = name
        try:
            return self._run_ranking()
        finally:
            scorer.precision_override = saved

    def _sharded_scorer(self):
        """RowShardedScorer over this rank's rows of the model's entity table when the job
        runs in a torch.distributed world (engine.row_sharded), else None."""
        from ..sharded import RowShardedScorer, engine_ops_for, shard_bounds, sharding_enabled
        import torch.distributed as dist

        if not sharding_enabled(self.config):
            return None
        world = dist.get_world_size()
        emb = self.model.get_s_embedder()
        ent = emb._embeddings.weight.detach()
        rel = self.model.get_p_embedder()._embeddings.weight.detach()
        E = self.dataset.num_entities()
        lo, hi = shard_bounds(E, world, dist.get_rank())
        ops = self.sharded_ops if self.sharded_ops is not None else engine_ops_for(self.model)
        held = getattr(emb, "shard", None)
        if held is not None:  # a row-sharded training job's model: it holds exactly these rows
            if held != (lo, hi):
                raise RuntimeError(f"the model holds entity rows {held}, this rank ranks rows {(lo, hi)}")
            return RowShardedScorer(ent, lo, hi, E, rel, ops)
        return RowShardedScorer(ent[lo:hi], lo, hi, E, rel, ops)

    def _run_ranking(self) -> dict:
        was_training = self.model.training
        self.model.eval()
        E = self.dataset.num_entities()
        dev = self.device
        nrank = len(self.rankings)
        sharded = self._sharded_scorer()
        chunk = self.config.get("entity_ranking.chunk_size")
        chunk = E if chunk is None or chunk < 0 else chunk
        hists_sharded = torch.zeros(2, nrank, E, device=dev) if sharded is not None else None
        ent_rows = None
        self._shard_refinement = None
        if sharded is not None:
            # per shard: near-ties of the true score among THIS rank's columns are rescored
            # exactly (the band is |q_i| max |t_j| over the shard's rows); where that does not
            # apply the shards rank exact-fp32 scores
            want, self._refine = self._refine, False
            if want and getattr(sharded.ops, "refinement", None) is not None:
                self._shard_refinement = sharded.ops.refinement(sharded.ent)
            if want and self._shard_refinement is None:
                self.model.get_scorer().precision_override = "fp32"
                if hasattr(sharded.ops, "precision"):
                    sharded.ops.precision = self.model.get_scorer().precision()
        if self._refine:
            # refinement needs fp32 query rows that contract with whole entity rows: the bilinear
            # lookup models except CP; every other model ranks fp32 scores
            tabs = self.model._lookup_tables()
            self._refine = tabs is not None and self.model.get_scorer().engine_kind in (
                _lib.COMPLEX, _lib.DISTMULT, _lib.RESCAL, _lib.SIMPLE)
            if self._refine:
                ent_rows = tabs[0].detach()
                # the rescoring reads the rows as float4 (kge_rank_rows): 16-B aligned rows of a
                # multiple of 4 columns; any other layout ranks fp32 scores
                self._refine = (ent_rows.dim() == 2 and ent_rows.stride(1) == 1 and ent_rows.shape[1] % 4 == 0
                                and ent_rows.stride(0) % 4 == 0 and ent_rows.data_ptr() % 16 == 0)
            if not self._refine:
                ent_rows = None
                self.model.get_scorer().precision_override = "fp32"
        # Ranking fused into the contraction (engine.fused_rank): bilinear lookup models on the split
        # bf16x3 contraction, with or without refinement; everything else ranks a score block
        self._fused_rank = False
        if sharded is None and self.config.get("engine.fused_rank"):
            from .. import engine

            tabs = self.model._lookup_tables()
            sc = self.model.get_scorer()
            if tabs is not None and engine.rank_codes_applicable(sc.engine_kind, sc.precision(), tabs[0].detach()):
                self._fused_rank = True
                if ent_rows is None:
                    ent_rows = tabs[0].detach()
        N = len(self.triples)
        if self._streams is None:
            # independent batches take turns on engine.eval_streams HIP streams; every accumulation
            # across batches (histograms, group counts) is an atomic add of exact small integers.
            # The row-sharded path stays on one stream: its collectives are ordered per process.
            from ..engine import BatchStreams

            self._streams = BatchStreams(dev, self.config.get("engine.eval_streams"))

        def device_pass(hists, ghists, ranks_out):
            """All device work of the run: adds every batch's ranks to the (zeroed) histograms."""
            tmax = _lib.row_norm_max(ent_rows) if self._refine else None  # ahead of the batches: every stream reads it
            with self._streams if sharded is None else contextlib.nullcontext():
                self._rank_batches(N, E, chunk, sharded, nrank, hists.view(nrank * 2, E), hists_sharded, ghists,
                                   ranks_out, ent_rows, tmax)

        epoch_time = -time.time()
        recorded = self._recorded_pass(device_pass, sharded, nrank, E, chunk, ent_rows) if sharded is None else None
        if recorded is not None:
            hists_d, group_hists, ranks_out = recorded
        else:
            #: [ranking, direction (tail "o", head "s"), rank] histograms
            hists_d = torch.zeros(nrank, 2, E, device=dev)
            group_hists = {name: torch.zeros(nrank, 2, len(names) + 1, E, device=dev)
                           for name, (names, _) in self._groups.items()}
            ranks_out = {f"{d}{r}": [] for d in "so" for r in self.rankings}
            device_pass(hists_d, group_hists, ranks_out)
        metrics = {}
        if hists_sharded is not None:
            hists_d += hists_sharded.permute(1, 0, 2)
        # key -> [ranking, rank] histograms in the order of the reference's hooks (eval.py:148-224);
        # counts are small integers: the fp32 sums are exact
        keyed = {"all": hists_d.sum(1)}
        if self.head_and_tail:
            keyed["head"], keyed["tail"] = hists_d[:, 1], hists_d[:, 0]
        for name, (names, _) in self._groups.items():
            h = group_hists[name]
            for gi, g in enumerate(names):
                if name == "relation_type":
                    keyed[g] = h[:, :, gi].sum(1)
                    if self.head_and_tail:
                        keyed[g + "_head"], keyed[g + "_tail"] = h[:, 1, gi], h[:, 0, gi]
                else:
                    keyed[f"{name}_{g}"] = h[:, :, gi].sum(1)
        # entity_ranking.py:376-387: per key, every ranking -- all of them in one device pass
        suffixes = [RANKING_SUFFIX[r] + ("_" + key if key != "all" else "")
                    for key in keyed for r in self.rankings]
        metrics.update(self._compute_metrics_stacked(torch.cat(list(keyed.values())), suffixes))
        # closed after the metrics (entity_ranking.py:111, 388): their device-to-host copy waits for
        # the batches, so this is the run's wall time, not the time it took to issue it
        epoch_time += time.time()
        if self.capture_ranks:
            self.ranks = {k: torch.cat(v).cpu().numpy() if v else np.zeros(0, np.int64)
                          for k, v in ranks_out.items()}
        trace = dict(type="entity_ranking", scope="epoch", split=self.eval_split,
                     filter_splits=self.filter_splits, epoch=self.epoch, batches=(N + self.batch_size - 1)
                     // self.batch_size, size=N, epoch_time=epoch_time, event="eval_completed", **metrics)
        for f in self.post_epoch_trace_hooks:
            f(self, trace)
        if was_training:
            self.model.train()
        return trace

    def _recorded_pass(self, device_pass, sharded, nrank, E, chunk, ent_rows):
        """engine.graph_eval: the device work of an evaluation run -- every batch of the split, on
        all of its streams -- recorded ONCE as a HIP graph and replayed by every later run of this
        job (a training job validates with one EntityRankingJob, epoch after epoch).  The split, the
        filter lists, the grouping and every shape are fixed per job, and the kernels read the
        model's tables through their addresses, so a replay ranks with the weights as they are then.
        The host otherwise spends as long issuing the ~100 launches of a run as the device spends
        running them.  The first run of a configuration is eager (kernel attributes, allocator),
        the second is recorded; anything the recording depends on (tables re-created, another
        precision, ranks to capture, ...) is part of its key, and a changed key starts over.
        Returns (histograms, group histograms, ranks) of this run, or None: run eagerly."""
        st = self._graph_state
        if (st.get("disabled") or not self.config.get("engine.graph_eval")
                or torch.device(self.device).type != "cuda" or torch.cuda.is_current_stream_capturing()):
            return None
        tabs = self.model._lookup_tables()
        if tabs is None or self.model.get_scorer().engine_kind is None:
            return None  # embedders / scorers outside the engine may synchronise
        stacked = [t for part in self._stacked if part is not None for t in part]
        key = (tuple((t.data_ptr(), tuple(t.shape)) for t in tabs), ent_rows.data_ptr() if ent_rows is not None else 0,
               tuple(t.data_ptr() for t in stacked), self._stack_e.data_ptr(), self._stack_p.data_ptr(),
               tuple((name, ids.data_ptr()) for name, (_, ids) in self._groups.items()),
               nrank, E, chunk, self._bs, self._refine, self._fused_rank, self._two_sided, self.tie_handling,
               self.capture_ranks, len(self._streams.streams), self.model.get_scorer().precision_override)
        if st.get("key") != key:  # first run of this configuration: eager
            st.clear()
            st["key"] = key
            return None
        if "graph" not in st:
            dev = self.device
            hists = torch.zeros(nrank, 2, E, device=dev)
            ghists = {name: torch.zeros(nrank, 2, len(names) + 1, E, device=dev)
                      for name, (names, _) in self._groups.items()}
            ranks_out = {f"{d}{r}": [] for d in "so" for r in self.rankings}
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    hists.zero_()  # fill kernels (no memset nodes)
                    for h in ghists.values():
                        h.zero_()
                    device_pass(hists, ghists, ranks_out)
            except Exception as e:  # not recordable: this job evaluates eagerly from now on
                import traceback

                st.clear()
                st["disabled"] = True
                st["error"] = f"{type(e).__name__}: {e}\n{traceback.format_exc()}"
                try:  # an invalidated capture reports its error once more at the next call
                    torch.cuda.synchronize()
                except Exception:
                    pass
                self.config.log(f"engine.graph_eval disabled: {st['error']}")
                return None
            st["graph"], st["out"] = g, (hists, ghists, ranks_out)
        st["graph"].replay()
        return st["out"]

    def _rank_batches(self, N, E, chunk, sharded, nrank, hists_flat, hists_sharded, group_hists, ranks_out,
                      ent_rows, tmax):
        """The batch loop of _run_ranking: adds every batch's ranks to the histograms."""
        dev = self.device
        if (sharded is not None and getattr(sharded.ops, "rank_rows", None) is not None
                and sharded.rank_block_applies(self._two_sided)):
            return self._rank_batches_sharded(N, sharded, nrank, hists_sharded, group_hists, ranks_out)
        for bi, b0 in enumerate(range(0, N, self._bs)):
            with (self._streams.batch(bi) if sharded is None else contextlib.nullcontext()):
                b1 = min(N, b0 + self._bs)
                B = b1 - b0
                s, o = self._stack_e[2 * b0:2 * b0 + B], self._stack_e[2 * b0 + B:2 * b0 + 2 * B]
                p, p_po = self._stack_p[2 * b0:2 * b0 + B], self._stack_p[2 * b0 + B:2 * b0 + 2 * B]
                if sharded is not None:
                    # each rank counts over its own rows; one all_reduce of the int64 counts makes
                    # them global (the reference's chunk_size decomposition, entity_ranking.py:153-216)
                    p_inv = (p + self.dataset.num_relations()) if self._two_sided else None
                    counts = None
                    if getattr(sharded.ops, "rank_rows", None) is not None:
                        # one stacked pass per batch, as in the unsharded job
                        (fp_sp, fp_po, f_col), tstack = self._stacked
                        tp = (tstack[0][b0:], tstack[1][b0:]) if tstack is not None else None
                        counts = sharded.rank_block(s, p, o, (fp_sp[b0:], fp_po[b0:]), f_col, tp,
                                                    tstack[2] if tstack is not None else None, p_inverse=p_inv,
                                                    refinement=self._shard_refinement)
                    rk = torch.empty(2, nrank, B, dtype=torch.int64, device=dev)
                    if counts is not None:  # [2, rankings x (2 B)]: ranking-major, then direction
                        c = counts.view(2, nrank, 2, B).permute(0, 2, 1, 3).contiguous()  # -> [.., direction, ranking, B]
                        per_dir = [(c[0, di].view(-1), c[1, di].view(-1)) for di in range(2)]
                    else:
                        tf = self._t
                        counts = sharded.rank_counts(
                            s, p, o, (self._f["sp"][0][b0:], self._f["sp"][1]),
                            (self._f["po"][0][b0:], self._f["po"][1]),
                            (tf["sp"][0][b0:], tf["sp"][1]) if tf is not None else None,
                            (tf["po"][0][b0:], tf["po"][1]) if tf is not None else None, p_inverse=p_inv)
                        per_dir = [(counts[di, 0, :nrank * B], counts[di, 1, :nrank * B]) for di in range(2)]
                    for di, d in enumerate("os"):
                        sharded.ops.rank_hist_multi(per_dir[di][0], per_dir[di][1], B, self.tie_handling,
                                                    rk[di].view(-1), hists_sharded[di])
                        if self.capture_ranks:
                            for ri, r in enumerate(self.rankings):
                                ranks_out[f"{d}{r}"].append(rk[di, ri])
                    if group_hists:
                        self._count_groups(group_hists, rk.permute(1, 0, 2), b0, B)
                    continue
                o_true = self.model.score_spo(s, p, o, "o").view(-1).float().contiguous()
                # score_spo(.., "s") is the same triple score unless the model scores the two
                # directions differently (reciprocal relations): skip the second launch then
                s_true = o_true if not self._two_sided else self.model.score_spo(s, p, o, "s").view(-1).float().contiguous()
                (fp_sp, fp_po, f_col), tstack = self._stacked
                tp_sp, tp_po, t_col = tstack if tstack is not None else (None, None, None)
                part_a = (o, o_true, fp_sp[b0:], tp_sp[b0:] if tp_sp is not None else None)
                part_b = (s, s_true, fp_po[b0:], tp_po[b0:] if tp_po is not None else None)
                single = chunk >= E
                counts = (torch.empty if single else torch.zeros)(2, nrank * 2 * B, dtype=torch.int64, device=dev)
                rk = torch.empty(nrank * 2 * B, dtype=torch.int64, device=dev)
                for c0 in range(0, E, chunk):
                    c1 = min(E, c0 + chunk)
                    finish = dict(accumulate=not single, tie_handling=self.tie_handling if single else None,
                                  ranks=rk if single else None, hists=hists_flat if single else None, rows_per_hist=B)
                    if self._fused_rank:
                        # the contraction compares every score with its row's true score in registers
                        # and leaves 2-bit codes: no [2B, C] score block is written or read
                        if self._refine and tmax is None:
                            tmax = _lib.row_norm_max(ent_rows)
                        fused = self.model.rank_sp_po_codes(
                            s, p, o, o_true, s_true, c0, c1, refine_band(ent_rows.shape[1]) if self._refine else None,
                            tmax, p_po=p_po)
                        if fused is None:
                            raise RuntimeError("the model stopped serving the fused ranking contraction")
                        codes, q = fused
                        refine = (q, ent_rows[c0:c1], refine_band(q.shape[1]), tmax) if self._refine else None
                        _lib.rank_rows(None, B, c0, part_a, part_b, f_col, t_col, counts[0], counts[1], codes=codes,
                                       m=c1 - c0, refine=refine, **finish)
                        del codes
                        continue
                    subset = None if single else torch.arange(c0, c1, device=dev)
                    # [2B, C]: the (s, p, ?) rows on top of the (?, p, o) rows, one engine pass
                    scores, q = self.model.score_sp_po_rows(s, p, o, subset, want_q=self._refine, p_po=p_po)
                    refine = None
                    if q is not None:
                        if tmax is None:
                            tmax = _lib.row_norm_max(ent_rows)
                        refine = (q, ent_rows[c0:c1], refine_band(q.shape[1]), tmax)
                    elif self._refine:
                        raise RuntimeError("engine.eval_precision bf16x3_refined: the engine returned no fp32 query "
                                           "rows to rescore near-ties with")
                    # a single chunk finishes the batch in the same launch: ranks + histograms
                    _lib.rank_rows(scores, B, c0, part_a, part_b, f_col, t_col, counts[0], counts[1], refine=refine,
                                   **finish)
                    del scores
                if not single:
                    _lib.rank_hist_multi(counts[0], counts[1], B, self.tie_handling, rk, hists_flat)
                rk = rk.view(nrank, 2, B)
                if group_hists:
                    self._count_groups(group_hists, rk, b0, B)
                if self.capture_ranks:
                    for di, d in enumerate("os"):
                        for ri, r in enumerate(self.rankings):
                            ranks_out[f"{d}{r}"].append(rk[ri, di])

    def _rank_batches_sharded(self, N, sharded, nrank, hists_sharded, group_hists, ranks_out):
        """The row-sharded batch loop with its exchanges GROUPED over engine.eval_exchange_group
        batches: one gather of the full rows of a group's subjects and objects (every rank holds
        the same triples), the stacked local pass per batch against this rank's rows, and one
        all_reduce of the group's counts -- 2 collectives per group instead of 2 per batch (each
        costs tens of microseconds of host time whatever it carries).  The counts sum exactly,
        so the ranks are those of the per-batch exchange (entity_ranking.py:153-216)."""
        from ..sharded import all_reduce

        G = max(1, int(self.config.get("engine.eval_exchange_group")))
        bs = self._bs
        (fp_sp, fp_po, f_col), tstack = self._stacked
        R = self.dataset.num_relations()
        for g0 in range(0, N, G * bs):
            g1 = min(N, g0 + G * bs)
            rows_g = sharded.gather_rows(self._stack_e[2 * g0:2 * g1])  # per batch: its s rows, then its o rows
            local, spans = [], []
            for b0 in range(g0, g1, bs):
                B = min(g1, b0 + bs) - b0
                s, o = self._stack_e[2 * b0:2 * b0 + B], self._stack_e[2 * b0 + B:2 * b0 + 2 * B]
                p = self._stack_p[2 * b0:2 * b0 + B]
                tp = (tstack[0][b0:], tstack[1][b0:]) if tstack is not None else None
                local.append(sharded.rank_block_local(
                    rows_g[2 * (b0 - g0):2 * (b0 - g0) + 2 * B], s, p, o, (fp_sp[b0:], fp_po[b0:]), f_col, tp,
                    tstack[2] if tstack is not None else None, p_inverse=(p + R) if self._two_sided else None,
                    refinement=self._shard_refinement))
                spans.append((b0, B))
            flat = torch.cat([c.view(-1) for c in local]) if len(local) > 1 else local[0].view(-1)
            all_reduce(flat, group=sharded.group)
            off = 0
            for (b0, B), c_loc in zip(spans, local):
                counts = flat[off:off + c_loc.numel()].view(2, nrank * 2 * B)
                off += c_loc.numel()
                # [2, rankings x (2 B)]: ranking-major, then direction -> [.., direction, ranking, B]
                c = counts.view(2, nrank, 2, B).permute(0, 2, 1, 3).contiguous()
                rk = torch.empty(2, nrank, B, dtype=torch.int64, device=self.device)
                for di, d in enumerate("os"):
                    sharded.ops.rank_hist_multi(c[0, di].view(-1), c[1, di].view(-1), B, self.tie_handling,
                                                rk[di].view(-1), hists_sharded[di])
                    if self.capture_ranks:
                        for ri, r in enumerate(self.rankings):
                            ranks_out[f"{d}{r}"].append(rk[di, ri])
                if group_hists:
                    self._count_groups(group_hists, rk.permute(1, 0, 2), b0, B)

    def _compute_metrics(self, rank_hist: torch.Tensor, suffix: str = "") -> Dict[str, float]:
        """entity_ranking.py:553-577 for one rank histogram."""
        return self._compute_metrics_stacked(rank_hist.view(1, -1), [suffix])

    def _compute_metrics_stacked(self, rank_hists: torch.Tensor, suffixes: List[str]) -> Dict[str, float]:
        """entity_ranking.py:553-577 for a stack of rank histograms [K, E] (one suffix each):
        mean rank, mean reciprocal rank and hits@k of every histogram in one launch
        (kge_rank_metrics) and ONE device-to-host copy instead of three host round trips per
        histogram (host histograms, e.g. of a CPU rehearsal, take the same sums through torch).  The operands are
        the reference's fp32 ones (counts, ranks, fp32 reciprocals, fp32 hits quotients); the two
        weighted sums accumulate in fp64, which differs from an fp32 sum only by that sum's own
        rounding."""
        E = self.dataset.num_entities()
        K = rank_hists.shape[0]
        kmax = max(self.hits_at_k_s)
        if rank_hists.is_cuda:
            table = _lib.rank_metrics(rank_hists, kmax).tolist()  # one launch, one copy
        else:
            if self._rank_weights is None or self._rank_weights.device != rank_hists.device:
                ranks = torch.arange(1, E + 1, device=rank_hists.device).float()
                self._rank_weights = torch.stack([ranks.double(), (1.0 / ranks).double()])  # fp32 values
            h64 = rank_hists.double()
            n = rank_hists.sum(1, keepdim=True)  # exact: integer counts far below 2^24
            hits = torch.cumsum(rank_hists[:, :kmax], dim=1) / n  # fp32 quotients
            table = torch.cat([n.double(), (h64 * self._rank_weights[0]).sum(1, keepdim=True),
                               (h64 * self._rank_weights[1]).sum(1, keepdim=True), hits.double()], dim=1).tolist()
        metrics = {}
        for row, suffix in zip(table, suffixes):
            cnt = row[0]
            metrics["mean_rank" + suffix] = row[1] / cnt if cnt > 0.0 else 0.0
            metrics["mean_reciprocal_rank" + suffix] = row[2] / cnt if cnt > 0.0 else 0.0
            for k in self.hits_at_k_s:
                metrics["hits_at_{}{}".format(k, suffix)] = row[3 + k - 1] if cnt > 0.0 else 0.0
        assert len(table) == K == len(suffixes)
        return metrics
