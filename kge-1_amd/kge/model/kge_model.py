"""KgeModel / RelationalScorer / KgeEmbedder: the plugin API of the scoring path.

Mirrors LibKGE's kge/model/kge_model.py (KgeBase 26-88, RelationalScorer 91-182,
KgeEmbedder 185-339, KgeModel 342-746): same class names, factories resolving
``<model>.class_name`` in ``kge.model``, same method signatures, shapes and error
behaviour.  What differs is underneath: scorers that implement ``engine_kind`` run on
libkgescore (gfx950 HIP), and KgeModel.score_sp / score_po / score_sp_po fuse the
LookupEmbedder gather into the engine call instead of materialising embed_all().
"""
from __future__ import annotations

import importlib
from typing import Any, Dict, List, Optional

import torch
from torch import Tensor

from ..config import Config, Configurable

SLOTS = [0, 1, 2]
S, P, O = SLOTS


class KgeBase(torch.nn.Module, Configurable):
    """Base class for models, scorers and embedders (kge_model.py:26-88)."""

    def __init__(self, config: Config, dataset, configuration_key=None):
        Configurable.__init__(self, config, configuration_key)
        torch.nn.Module.__init__(self)
        self.dataset = dataset
        self.meta: Dict[str, Any] = dict()

    def initialize(self, what: Tensor, initialize: str, initialize_args):
        try:
            getattr(torch.nn.init, initialize)(what, **initialize_args)
        except Exception as e:
            raise ValueError(
                "invalid initialization options: {} with args {}".format(initialize, initialize_args)) from e

    def prepare_job(self, job, **kwargs):
        pass

    def penalty(self, **kwargs) -> List[Tensor]:
        return []

    def save(self):
        return self.state_dict(), self.meta

    def load(self, savepoint):
        self.load_state_dict(savepoint[0])
        self.meta = savepoint[1]


class RelationalScorer(KgeBase):
    """Scores (s, p, o) embedding triples (kge_model.py:91-182).

    Subclasses either implement ``score_emb_spo`` (row-wise) or override ``score_emb``.
    Engine-backed scorers set ``engine_kind`` and get score_emb for "spo", "sp_", "_po"
    from libkgescore; other combines fall back to the generic row-wise expansion.
    """

    engine_kind: Optional[int] = None

    #: The reference's TransE and RESCAL scorers pass the generic "s_o" result through their
    #: own ``out.view(p_emb.size(0), -1)`` (transe.py:22-24, rescal.py:51-53): the [n_s, n_p]
    #: score matrix leaves reinterpreted (not transposed) as [n_p, n_s].  Scorers that set
    #: this flag reproduce that layout, so callers see what the reference returns.
    s_o_viewed_by_relation_count = False

    def __init__(self, config: Config, dataset, configuration_key: str):
        super().__init__(config, dataset, configuration_key)

    # --- engine parameters
    def l_norm(self) -> float:
        return 1.0

    #: set by a job for the duration of a run to score with another precision than
    #: engine.precision (EntityRankingJob applies engine.eval_precision this way)
    precision_override: Optional[str] = None

    def precision(self) -> int:
        from .. import _lib

        name = self.precision_override or self.config.get("engine.precision")
        if name not in _lib.PRECISIONS:
            raise ValueError(f"engine precision {name!r}: expected one of {sorted(_lib.PRECISIONS)}")
        return _lib.PRECISIONS[name]

    def score_emb_spo(self, s_emb: Tensor, p_emb: Tensor, o_emb: Tensor) -> Tensor:
        return self.score_emb(s_emb, p_emb, o_emb, "spo")

    def score_emb(self, s_emb: Tensor, p_emb: Tensor, o_emb: Tensor, combine: str) -> Tensor:
        """combine: "spo" -> [n, 1]; "sp_" -> [n, n_o]; "_po" -> [n, n_s]; "s_o" -> [n, n_p]
        (kge_model.py:120-182)."""
        n = p_emb.size(0)
        if self.engine_kind is not None and combine in ("spo", "sp_", "_po"):
            from .. import engine, _lib

            if combine == "spo":
                assert s_emb.size(0) == n and o_emb.size(0) == n
                out = engine.score_spo_emb(self.engine_kind, self.l_norm(), s_emb, p_emb, o_emb)
            elif combine == "sp_":
                assert s_emb.size(0) == n
                out = engine.score_all(self.engine_kind, _lib.DIR_SP, self.precision(), self.l_norm(),
                                       s_emb, None, p_emb, None, o_emb, None)
            else:
                assert o_emb.size(0) == n
                out = engine.score_all(self.engine_kind, _lib.DIR_PO, self.precision(), self.l_norm(),
                                       o_emb, None, p_emb, None, s_emb, None)
            return out.view(n, -1)

        # generic fallback: expand to row-wise triples (kge_model.py:154-178)
        if combine == "spo":
            assert s_emb.size(0) == n and o_emb.size(0) == n
            out = self.score_emb_spo(s_emb, p_emb, o_emb)
        elif combine == "sp_":
            assert s_emb.size(0) == n
            n_o = o_emb.size(0)
            out = self.score_emb_spo(s_emb.repeat_interleave(n_o, 0), p_emb.repeat_interleave(n_o, 0),
                                     o_emb.repeat((n, 1)))
        elif combine == "_po":
            assert o_emb.size(0) == n
            n_s = s_emb.size(0)
            out = self.score_emb_spo(s_emb.repeat((n, 1)), p_emb.repeat_interleave(n_s, 0),
                                     o_emb.repeat_interleave(n_s, 0))
        elif combine == "s_o":
            n = s_emb.size(0)
            assert o_emb.size(0) == n
            n_p = p_emb.size(0)
            out = self.score_emb_spo(s_emb.repeat_interleave(n_p, 0), p_emb.repeat((n, 1)),
                                     o_emb.repeat_interleave(n_p, 0))
            if self.s_o_viewed_by_relation_count:
                n = n_p
        else:
            raise ValueError('cannot handle combine="{}".format(combine)')
        return out.view(n, -1)

    # --- fused lookup path (indexes instead of embeddings)
    def score_lookup(self, ent: Tensor, rel: Tensor, e_idx: Tensor, p_idx: Tensor, direction: str,
                     cand_idx: Optional[Tensor] = None) -> Tensor:
        """Scores of queries (ent[e_idx], rel[p_idx]) in direction "sp_" / "_po" against
        ent[cand_idx] (all entities when None), gather fused into the engine."""
        from .. import engine, _lib

        d = _lib.DIR_SP if direction == "sp_" else _lib.DIR_PO
        return engine.score_all(self.engine_kind, d, self.precision(), self.l_norm(), ent, e_idx, rel, p_idx,
                                ent, cand_idx)

    def score_lookup_parts(self, ent: Tensor, rel: Tensor, parts, cand_idx: Optional[Tensor] = None,
                           want_q: bool = False, out: Optional[Tensor] = None):
        """Several query batches (direction "sp_" / "_po", e_idx, p_idx) against the same
        candidates, stacked by rows, without gradient (engine.score_parts): (S, Q)."""
        from .. import engine, _lib

        conv = [((_lib.DIR_SP if d == "sp_" else _lib.DIR_PO), e, p) for d, e, p in parts]
        return engine.score_parts(self.engine_kind, self.precision(), self.l_norm(), ent, rel, conv, cand_idx,
                                  want_q, out)

    def score_lookup_xent(self, ent: Tensor, rel: Tensor, e_idx: Tensor, p_idx: Tensor, direction: str,
                          labels: Tensor, scale: float, l_ptr: Optional[Tensor] = None,
                          smoothing: float = 0.0) -> Tensor:
        """scale * sum_i CE(score_lookup(...)[i, :], labels[i]) in one engine pass (the
        1vsAll loss of kge/job/train.py:1042,1052 fused into the scorer)."""
        from .. import engine, _lib

        d = _lib.DIR_SP if direction == "sp_" else _lib.DIR_PO
        return engine.score_all_xent(self.engine_kind, d, self.precision(), self.l_norm(), ent, e_idx, rel, p_idx,
                                     ent, None, labels, scale, l_ptr, smoothing)

    def score_emb_xent(self, e_emb: Tensor, p_emb: Tensor, cand: Tensor, direction: str, labels: Tensor,
                       scale: float, l_ptr: Optional[Tensor] = None, smoothing: float = 0.0) -> Tensor:
        """score_lookup_xent for queries given as embedding rows (one entity row and one
        relation row per query) against the candidate rows cand: what a lookup embedder with
        dropout hands over -- dropped query rows and a dropped copy of the table."""
        from .. import engine, _lib

        d = _lib.DIR_SP if direction == "sp_" else _lib.DIR_PO
        return engine.score_all_xent(self.engine_kind, d, self.precision(), self.l_norm(), e_emb, None, p_emb, None,
                                     cand, None, labels, scale, l_ptr, smoothing)

    def score_lookup_xent2(self, ent: Tensor, rel: Tensor, part_a, part_b, scale: float,
                           smoothing: float = 0.0) -> Optional[Tensor]:
        """Both halves of a training step in one engine pass: part = (direction "sp_" / "_po",
        e_idx, p_idx, labels, l_ptr).  Returns (total, [loss_a, loss_b] detached) (see
        engine.score_all_xent2), or None when this scorer cannot share one contraction between
        the parts."""
        from .. import engine, _lib

        if self.engine_kind is None:
            return None

        def conv(part):
            d, e, p, lab, lp = part
            return (_lib.DIR_SP if d == "sp_" else _lib.DIR_PO), e, p, lab, lp

        return engine.score_all_xent2(self.engine_kind, self.precision(), ent, rel, conv(part_a), conv(part_b),
                                      scale, smoothing)

    def score_lookup_xent_stacked(self, ent: Tensor, rel: Tensor, dir_a: str, dir_b: str, e_idx: Tensor,
                                  p_idx: Tensor, n_a_dev: Tensor, labels: Tensor, l_ptr: Optional[Tensor],
                                  scale: float, smoothing: float = 0.0):
        """score_lookup_xent2 on pre-stacked query rows with the split point in device memory
        (engine.score_all_xent_stacked); None when this scorer cannot fuse them."""
        from .. import engine, _lib

        if self.engine_kind is None:
            return None
        da = _lib.DIR_SP if dir_a == "sp_" else _lib.DIR_PO
        db = _lib.DIR_SP if dir_b == "sp_" else _lib.DIR_PO
        return engine.score_all_xent_stacked(self.engine_kind, self.precision(), ent, rel, da, db, e_idx, p_idx,
                                             n_a_dev, labels, l_ptr, scale, smoothing)

    def score_lookup_cand(self, ent: Tensor, rel: Tensor, e_idx: Tensor, p_idx: Tensor, direction: str,
                          cand: Tensor) -> Tensor:
        """[n, k]: query (ent[e_idx[i]], rel[p_idx[i]]) in direction "sp_" / "_po" against its
        own candidates ent[cand[i, :]] (score_spo semantics; negative sampling)."""
        from .. import engine, _lib

        d = _lib.DIR_SP if direction == "sp_" else _lib.DIR_PO
        return engine.score_cand(self.engine_kind, d, self.l_norm(), ent, e_idx, rel, p_idx, cand)

    def score_lookup_spo(self, ent: Tensor, rel: Tensor, s: Tensor, p: Tensor, o: Tensor) -> Tensor:
        from .. import engine

        return engine.score_spo(self.engine_kind, self.l_norm(), ent, s, rel, p, o)


class KgeEmbedder(KgeBase):
    """Embeds a fixed vocabulary (kge_model.py:185-339)."""

    def __init__(self, config: Config, dataset, configuration_key: str, init_for_load_only=False):
        super().__init__(config, dataset, configuration_key)
        self.embedder_type: str = self.get_option("type")
        self.dim: int = self.get_option("dim")

    def _init_embeddings(self, data: Tensor):
        initialize = self.get_option("initialize")
        try:
            initialize_args = dict(self.get_option("initialize_args." + initialize))
        except KeyError:
            initialize_args = dict(self.get_option("initialize_args"))
        if initialize == "uniform_" and "a" not in initialize_args and "b" in initialize_args:
            initialize_args["a"] = initialize_args["b"] * -1  # kge_model.py:237-240
        self.initialize(data, initialize, initialize_args)

    @staticmethod
    def create(config: Config, dataset, configuration_key: str, vocab_size: int,
               init_for_load_only=False) -> "KgeEmbedder":
        try:
            embedder_type = config.get_default(configuration_key + ".type")
            class_name = config.get(embedder_type + ".class_name")
            module = importlib.import_module("kge.model")
        except Exception as e:
            raise Exception("Can't find {}.type in config".format(configuration_key)) from e
        try:
            return getattr(module, class_name)(config, dataset, configuration_key, vocab_size,
                                               init_for_load_only=init_for_load_only)
        except (ImportError, AttributeError) as e:
            raise ValueError("Can't find class {} in 'kge.model' for embedder {}".format(
                class_name, embedder_type)) from e

    def forward(self, indexes: Tensor) -> Tensor:
        return self.embed(indexes)

    def embed(self, indexes: Tensor) -> Tensor:
        raise NotImplementedError

    def embed_all(self) -> Tensor:
        raise NotImplementedError


class KgeModel(KgeBase):
    """Entity + relation embedders and a RelationalScorer (kge_model.py:342-746)."""

    def __init__(self, config: Config, dataset, scorer, create_embedders=True, configuration_key=None,
                 init_for_load_only=False):
        super().__init__(config, dataset, configuration_key)
        if create_embedders:
            self._entity_embedder = KgeEmbedder.create(
                config, dataset, self.configuration_key + ".entity_embedder", dataset.num_entities(),
                init_for_load_only=init_for_load_only)
            self._relation_embedder = KgeEmbedder.create(
                config, dataset, self.configuration_key + ".relation_embedder", dataset.num_relations(),
                init_for_load_only=init_for_load_only)
        if isinstance(scorer, type):
            self._scorer = scorer(config=config, dataset=dataset, configuration_key=self.configuration_key)
        else:
            self._scorer = scorer

    def _init_configuration(self, config: Config, configuration_key: Optional[str]):
        Configurable._init_configuration(self, config, configuration_key)
        if not getattr(self, "model", None):
            if self.configuration_key:
                self.model: str = config.get(self.configuration_key + ".type")
            else:
                self.model: str = config.get("model")
                self.configuration_key = self.model

    @staticmethod
    def create(config: Config, dataset, configuration_key: Optional[str] = None,
               init_for_load_only=False) -> "KgeModel":
        try:
            model_name = config.get(configuration_key + ".type") if configuration_key else config.get("model")
            config._import(model_name)
            class_name = config.get(model_name + ".class_name")
            module = importlib.import_module("kge.model")
        except Exception as e:
            raise Exception("Can't find {}.type in config".format(configuration_key)) from e
        try:
            model = getattr(module, class_name)(config=config, dataset=dataset,
                                                configuration_key=configuration_key,
                                                init_for_load_only=init_for_load_only)
        except (ImportError, AttributeError) as e:
            raise ValueError("Can't find class {} in 'kge.model' for model {}".format(class_name, model_name)) from e
        model.to(config.get("job.device"))
        return model

    @staticmethod
    def create_from(checkpoint: Dict, dataset=None, use_tmp_log_folder=True, new_config: Config = None):
        """Rebuild a model from a checkpoint dict written by ``save`` (plain tensors and
        an options dict; loads with ``torch.load(weights_only=True)``)."""
        from ..dataset import Dataset

        config = Config(load_default=True)
        config.load_options(checkpoint["config"])
        if new_config is not None:
            config.load_options(new_config.options)
        if dataset is None:
            dataset = Dataset(config, None)
        model = KgeModel.create(config, dataset, init_for_load_only=True)
        model.load_state_dict(checkpoint["model"])
        model.eval()
        return model

    def prepare_job(self, job, **kwargs):
        super().prepare_job(job, **kwargs)
        self._entity_embedder.prepare_job(job, **kwargs)
        self._relation_embedder.prepare_job(job, **kwargs)

    def penalty(self, **kwargs) -> List[Tensor]:
        embs = (self.get_s_embedder(), self.get_p_embedder(), self.get_o_embedder())
        if not any(getattr(e, "penalty_active", lambda: True)() for e in embs):
            # nothing regularises (the default weight 0): skip the per-batch index upload
            # the reference does anyway (kge_model.py:588-605 moves the batch to the device)
            return super().penalty(**kwargs)
        if "batch" in kwargs and "triples" in kwargs["batch"]:
            triples = kwargs["batch"]["triples"].to(self.config.get("job.device"))
            return (super().penalty(**kwargs)
                    + self.get_s_embedder().penalty(indexes=triples[:, S], **kwargs)
                    + self.get_p_embedder().penalty(indexes=triples[:, P], **kwargs)
                    + self.get_o_embedder().penalty(indexes=triples[:, O], **kwargs))
        return (super().penalty(**kwargs) + self.get_s_embedder().penalty(**kwargs)
                + self.get_p_embedder().penalty(**kwargs) + self.get_o_embedder().penalty(**kwargs))

    def get_s_embedder(self) -> KgeEmbedder:
        return self._entity_embedder

    def get_o_embedder(self) -> KgeEmbedder:
        return self._entity_embedder

    def get_p_embedder(self) -> KgeEmbedder:
        return self._relation_embedder

    def get_scorer(self) -> RelationalScorer:
        return self._scorer

    # ----------------------------------------------------------------- fused lookup path
    def _lookup_tables(self):
        """(entity weight, relation weight) when the fused engine path applies: both
        embedders are plain lookups without dropout and the scorer is engine-backed."""
        from .embedder.lookup_embedder import LookupEmbedder

        e, r = self.get_s_embedder(), self.get_p_embedder()
        if (self._scorer.engine_kind is not None and isinstance(e, LookupEmbedder)
                and isinstance(r, LookupEmbedder) and e is self.get_o_embedder()
                and e.is_plain() and r.is_plain()):
            return e.weight_for_scoring(), r.weight_for_scoring()
        return None

    def _lookup_embedders_with_dropout(self) -> bool:
        """Whether the fused losses apply in their embedding-row form: lookup embedders (one
        shared by subjects and objects) that only add dropout, and an engine-backed scorer."""
        from .embedder.lookup_embedder import LookupEmbedder

        e, r = self.get_s_embedder(), self.get_p_embedder()
        return (self._scorer.engine_kind is not None and isinstance(e, LookupEmbedder)
                and isinstance(r, LookupEmbedder) and e is self.get_o_embedder())

    def _xent_dropout(self, e_idx, p_idx, direction, labels, scale, l_ptr=None, smoothing=0.0):
        """The fused loss with dropout in the embedders: dropped query rows and a dropped copy of
        the entity table (torch's dropout, drawn in the order score_sp / score_po draw them),
        scored and differentiated in one engine pass; autograd carries the gradients through
        the dropout masks and the lookups."""
        ent_e, rel_e = self.get_s_embedder(), self.get_p_embedder()
        if direction == "sp_":  # kge_model.py:639-659: s, p, then all objects
            e, p = ent_e.embed(e_idx), rel_e.embed(p_idx)
            cand = ent_e.embed_all()
        else:  # kge_model.py:661-682: all subjects, o, then p
            cand = ent_e.embed_all()
            e, p = ent_e.embed(e_idx), rel_e.embed(p_idx)
        return self._scorer.score_emb_xent(e, p, cand, direction, labels, scale, l_ptr, smoothing)

    # ----------------------------------------------------------------- scoring API
    def score_spo(self, s: Tensor, p: Tensor, o: Tensor, direction=None) -> Tensor:
        """Scores of triples (s_i, p_i, o_i) -> [n] (kge_model.py:620-637)."""
        tabs = self._lookup_tables()
        if tabs is not None:
            return self._scorer.score_lookup_spo(tabs[0], tabs[1], s, p, o).view(-1)
        s = self.get_s_embedder().embed(s)
        p = self.get_p_embedder().embed(p)
        o = self.get_o_embedder().embed(o)
        return self._scorer.score_emb(s, p, o, combine="spo").view(-1)

    def score_sp(self, s: Tensor, p: Tensor, o: Tensor = None) -> Tensor:
        """[n, E] (or [n, |o|]) scores of (s_i, p_i, e_j) (kge_model.py:639-659)."""
        tabs = self._lookup_tables()
        if tabs is not None:
            return self._scorer.score_lookup(tabs[0], tabs[1], s, p, "sp_", o)
        s = self.get_s_embedder().embed(s)
        p = self.get_p_embedder().embed(p)
        o = self.get_o_embedder().embed_all() if o is None else self.get_o_embedder().embed(o)
        return self._scorer.score_emb(s, p, o, combine="sp_")

    def score_po(self, p: Tensor, o: Tensor, s: Tensor = None) -> Tensor:
        """[n, E] (or [n, |s|]) scores of (e_j, p_i, o_i) (kge_model.py:661-682)."""
        tabs = self._lookup_tables()
        if tabs is not None:
            return self._scorer.score_lookup(tabs[0], tabs[1], o, p, "_po", s)
        s = self.get_s_embedder().embed_all() if s is None else self.get_s_embedder().embed(s)
        o = self.get_o_embedder().embed(o)
        p = self.get_p_embedder().embed(p)
        return self._scorer.score_emb(s, p, o, combine="_po")

    def score_sp_xent(self, s: Tensor, p: Tensor, o: Tensor, scale: float) -> Optional[Tensor]:
        """scale * sum_i CrossEntropy(score_sp(s, p)[i, :], o[i]) fused into the engine, or
        None when the fused path does not apply (non-lookup embedders, dropout, scorer
        without an engine kernel): the caller then scores and applies its loss itself."""
        tabs = self._lookup_tables()
        if tabs is None:
            return self._xent_dropout(s, p, "sp_", o, scale) if self._lookup_embedders_with_dropout() else None
        return self._scorer.score_lookup_xent(tabs[0], tabs[1], s, p, "sp_", o, scale)

    def score_po_xent(self, p: Tensor, o: Tensor, s: Tensor, scale: float) -> Optional[Tensor]:
        """scale * sum_i CrossEntropy(score_po(p, o)[i, :], s[i]) (see score_sp_xent)."""
        tabs = self._lookup_tables()
        if tabs is None:
            return self._xent_dropout(o, p, "_po", s, scale) if self._lookup_embedders_with_dropout() else None
        return self._scorer.score_lookup_xent(tabs[0], tabs[1], o, p, "_po", s, scale)

    # --- both directions of a training step in one engine pass
    def xent_part_sp(self, s: Tensor, p: Tensor, labels: Tensor, l_ptr: Optional[Tensor] = None):
        """The (s, p, ?) query batch of a fused loss: (direction, e_idx, p_idx, labels, l_ptr)."""
        return ("sp_", s, p, labels, l_ptr)

    def xent_part_po(self, p: Tensor, o: Tensor, labels: Tensor, l_ptr: Optional[Tensor] = None):
        """The (?, p, o) query batch of a fused loss."""
        return ("_po", o, p, labels, l_ptr)

    def score_xent_parts(self, part_a, part_b, scale: float, smoothing: float = 0.0) -> Optional[Tensor]:
        """(total, [loss_a, loss_b]) of two query batches (xent_part_sp / xent_part_po) in one
        engine pass: total = loss_a + loss_b carries the gradient, the pair is detached (for
        reporting); None when not fusable (the caller then runs score_*_xent / score_*_kl)."""
        tabs = self._lookup_tables()
        if tabs is None:
            return None
        return self._scorer.score_lookup_xent2(tabs[0], tabs[1], part_a, part_b, scale, smoothing)

    def score_xent_stacked(self, dir_a: str, dir_b: str, e_idx: Tensor, p_idx: Tensor, n_a_dev: Tensor, labels: Tensor,
                           l_ptr: Optional[Tensor], scale: float, smoothing: float = 0.0):
        """score_xent_parts for two query batches that are ALREADY stacked by rows (e_idx / p_idx
        index every row; rows [0, n_a) are direction dir_a ("sp_" / "_po") queries, the rest dir_b
        queries) with the split point n_a an int64 DEVICE scalar: a step recorded as a HIP graph
        serves batches whose split differs.  Labels as in score_xent_parts, stacked likewise.
        (total, [loss_a, loss_b] detached), or None when not fusable."""
        tabs = self._lookup_tables()
        if tabs is None:
            return None
        return self._scorer.score_lookup_xent_stacked(tabs[0], tabs[1], dir_a, dir_b, e_idx, p_idx, n_a_dev, labels,
                                                      l_ptr, scale, smoothing)

    def score_sp_po_xent(self, s: Tensor, p: Tensor, o: Tensor, scale: float) -> Optional[Tensor]:
        """score_sp_xent(s, p, o, scale) + score_po_xent(p, o, s, scale) in one engine pass (the two
        losses of a 1vsAll step, train.py:1041-1057) as (total, [sp part, po part] detached), or
        None."""
        return self.score_xent_parts(self.xent_part_sp(s, p, o), self.xent_part_po(p, o, s), scale)

    def score_sp_cand(self, s: Tensor, p: Tensor, cand: Tensor) -> Optional[Tensor]:
        """[n, k] = score_spo(s_i, p_i, cand[i, c]) for every candidate object, without
        building the n * k triples (negative sampling, train.py:868-892); None when the
        fused path does not apply (the caller then expands triples for score_spo)."""
        tabs = self._lookup_tables()
        if tabs is None:
            return None
        return self._scorer.score_lookup_cand(tabs[0], tabs[1], s, p, "sp_", cand)

    def score_po_cand(self, p: Tensor, o: Tensor, cand: Tensor) -> Optional[Tensor]:
        """[n, k] = score_spo(cand[i, c], p_i, o_i) for every candidate subject."""
        tabs = self._lookup_tables()
        if tabs is None:
            return None
        return self._scorer.score_lookup_cand(tabs[0], tabs[1], o, p, "_po", cand)

    def score_sp_kl(self, s: Tensor, p: Tensor, l_ptr: Tensor, l_col: Tensor, smoothing: float,
                    scale: float) -> Optional[Tensor]:
        """KvsAll: scale * sum_i KL(label row i || softmax(score_sp(s, p)[i, :])) fused into the
        engine; row i's positives are l_col[l_ptr[i]:l_ptr[i+1]].  None when not fusable."""
        tabs = self._lookup_tables()
        if tabs is None:
            if self._lookup_embedders_with_dropout():
                return self._xent_dropout(s, p, "sp_", l_col, scale, l_ptr, smoothing)
            return None
        return self._scorer.score_lookup_xent(tabs[0], tabs[1], s, p, "sp_", l_col, scale, l_ptr, smoothing)

    def score_po_kl(self, p: Tensor, o: Tensor, l_ptr: Tensor, l_col: Tensor, smoothing: float,
                    scale: float) -> Optional[Tensor]:
        """KvsAll (?, p, o) queries; see score_sp_kl."""
        tabs = self._lookup_tables()
        if tabs is None:
            if self._lookup_embedders_with_dropout():
                return self._xent_dropout(o, p, "_po", l_col, scale, l_ptr, smoothing)
            return None
        return self._scorer.score_lookup_xent(tabs[0], tabs[1], o, p, "_po", l_col, scale, l_ptr, smoothing)

    def score_so(self, s: Tensor, o: Tensor, p: Tensor = None) -> Tensor:
        """[n, R] (or [n, |p|]) scores of (s_i, r_j, o_i) (kge_model.py:684-704)."""
        s = self.get_s_embedder().embed(s)
        o = self.get_o_embedder().embed(o)
        p = self.get_p_embedder().embed_all() if p is None else self.get_p_embedder().embed(p)
        return self._scorer.score_emb(s, p, o, combine="s_o")

    def _sp_po_parts(self, s: Tensor, p: Tensor, o: Tensor, p_po: Tensor = None):
        """The two query batches of score_sp_po as (direction, e_idx, p_idx); p_po: the relation
        indexes of the (?, p, o) batch when the caller holds them as a vector of their own."""
        return [("sp_", s, p), ("_po", o, p if p_po is None else p_po)]

    def score_sp_po_rows(self, s: Tensor, p: Tensor, o: Tensor, entity_subset: Tensor = None, want_q: bool = False,
                         p_po: Tensor = None):
        """The scores of score_sp_po stacked by ROWS, without gradient: (S, Q) with S [2n, C],
        rows [0, n) = score_sp(s, p, subset), rows [n, 2n) = score_po(p, o, subset); Q the fp32
        query rows behind S (or None: not asked for / not available for this model).  One
        engine pass where the model allows it; the evaluation job ranks from this block.  p_po
        (equal to p) lets a caller whose index vectors (s | o) and (p | p_po) are contiguous in
        memory avoid their concatenation."""
        tabs = self._lookup_tables()
        if tabs is not None:
            return self._scorer.score_lookup_parts(tabs[0], tabs[1], self._sp_po_parts(s, p, o, p_po), entity_subset,
                                                   want_q)
        with torch.no_grad():
            both = self.score_sp_po(s, p, o, entity_subset)
        C = both.shape[1] // 2
        return torch.cat((both[:, :C], both[:, C:]), dim=0), None

    def rank_sp_po_codes(self, s: Tensor, p: Tensor, o: Tensor, true_o: Tensor, true_s: Tensor, c0: int, c1: int,
                         band_rel=None, t_norm_max=None, p_po: Tensor = None):
        """What the evaluation job ranks from, without the score block: the scores of
        score_sp_po_rows over entities [c0, c1) compared with each query's true score inside the
        contraction (engine.rank_parts) -- rows [0, n) the (s, p, ?) queries against true_o (true
        column o), rows [n, 2n) the (?, p, o) queries against true_s (true column s).  Returns
        (codes, fp32 query rows or None) or None when the model is not served (the caller then
        ranks score_sp_po_rows)."""
        from .. import engine, _lib

        tabs = self._lookup_tables()
        sc = self._scorer
        if tabs is None or not engine.rank_codes_applicable(sc.engine_kind, sc.precision(), tabs[0].detach()):
            return None
        parts = [((_lib.DIR_SP if d == "sp_" else _lib.DIR_PO), e, r) for d, e, r in self._sp_po_parts(s, p, o, p_po)]
        codes, q, _ = engine.rank_parts(sc.engine_kind, tabs[0].detach(), tabs[1].detach(), parts,
                                        [(o, true_o), (s, true_s)], c0, c1, band_rel, t_norm_max)
        return codes, q

    def score_sp_po(self, s: Tensor, p: Tensor, o: Tensor, entity_subset: Tensor = None) -> Tensor:
        """cat(score_sp(s,p,subset), score_po(p,o,subset)) -> [n, 2|subset|]
        (kge_model.py:706-746)."""
        tabs = self._lookup_tables()
        if tabs is not None:
            parts = self._sp_po_parts(s, p, o)
            if not (torch.is_grad_enabled() and (tabs[0].requires_grad or tabs[1].requires_grad)):
                # both halves straight into their column blocks of one buffer
                C = tabs[0].shape[0] if entity_subset is None else entity_subset.numel()
                buf = torch.empty(s.numel(), 2 * C, device=tabs[0].device, dtype=torch.float32)
                self._scorer.score_lookup_parts(tabs[0], tabs[1], parts[:1], entity_subset, out=buf[:, :C])
                self._scorer.score_lookup_parts(tabs[0], tabs[1], parts[1:], entity_subset, out=buf[:, C:])
                return buf
            sp = self._scorer.score_lookup(tabs[0], tabs[1], parts[0][1], parts[0][2], parts[0][0], entity_subset)
            po = self._scorer.score_lookup(tabs[0], tabs[1], parts[1][1], parts[1][2], parts[1][0], entity_subset)
            return torch.cat((sp, po), dim=1)
        s = self.get_s_embedder().embed(s)
        p = self.get_p_embedder().embed(p)
        o = self.get_o_embedder().embed(o)
        if self.get_s_embedder() is self.get_o_embedder():
            if entity_subset is not None:
                all_entities = self.get_s_embedder().embed(entity_subset)
            else:
                all_entities = self.get_s_embedder().embed_all()
            sp_scores = self._scorer.score_emb(s, p, all_entities, combine="sp_")
            po_scores = self._scorer.score_emb(all_entities, p, o, combine="_po")
        else:
            if entity_subset is not None:
                all_objects = self.get_o_embedder().embed(entity_subset)
                all_subjects = self.get_s_embedder().embed(entity_subset)
            else:
                all_objects = self.get_o_embedder().embed_all()
                all_subjects = self.get_s_embedder().embed_all()
            sp_scores = self._scorer.score_emb(s, p, all_objects, combine="sp_")
            po_scores = self._scorer.score_emb(all_subjects, p, o, combine="_po")
        return torch.cat((sp_scores, po_scores), dim=1)
