"""ReciprocalRelationsModel (reciprocal_relations_model.py:7-106): a base model with a
relation table of size 2R; (?, p, o) questions are answered as (o, p + R, ?), so every
all-entities query runs through the base scorer's ``sp_`` engine kernel."""
from __future__ import annotations

import torch
from torch import Tensor

from .kge_model import KgeModel


class ReciprocalRelationsModel(KgeModel):
    def __init__(self, config, dataset, configuration_key=None, init_for_load_only=False):
        self._init_configuration(config, configuration_key)
        alt_dataset = dataset.shallow_copy()
        alt_dataset._num_relations = dataset.num_relations() * 2
        base_model = KgeModel.create(config=config, dataset=alt_dataset,
                                     configuration_key=self.configuration_key + ".base_model",
                                     init_for_load_only=init_for_load_only)
        super().__init__(config=config, dataset=dataset, scorer=base_model.get_scorer(),
                         create_embedders=False, init_for_load_only=init_for_load_only)
        self._base_model = base_model
        self._entity_embedder = self._base_model.get_s_embedder()
        self._relation_embedder = self._base_model.get_p_embedder()

    def prepare_job(self, job, **kwargs):
        self._base_model.prepare_job(job, **kwargs)

    def penalty(self, **kwargs):
        return self._base_model.penalty(**kwargs)

    def score_spo(self, s: Tensor, p: Tensor, o: Tensor, direction=None) -> Tensor:
        if direction == "o":
            return super().score_spo(s, p, o, "o")
        elif direction == "s":
            return super().score_spo(o, p + self.dataset.num_relations(), s, "o")
        raise Exception("The reciprocal relations model cannot compute undirected spo scores.")

    def score_po(self, p: Tensor, o: Tensor, s: Tensor = None) -> Tensor:
        tabs = self._lookup_tables()
        p_inv = p + self.dataset.num_relations()
        if tabs is not None:
            return self._scorer.score_lookup(tabs[0], tabs[1], o, p_inv, "sp_", s)
        s = self.get_s_embedder().embed_all() if s is None else self.get_s_embedder().embed(s)
        p = self.get_p_embedder().embed(p_inv)
        o = self.get_o_embedder().embed(o)
        return self._scorer.score_emb(o, p, s, combine="sp_")

    def _xent_dropout_po(self, p, o, labels, scale, l_ptr=None, smoothing=0.0):
        """The fused loss of (?, p, o) queries with dropout in the embedders: dropped rows drawn
        in score_po's order (reciprocal_relations_model.py:67-74: all subjects, p + R, then o),
        scored as (o, p + R, ?) and differentiated in one engine pass."""
        if not self._lookup_embedders_with_dropout():
            return None
        ent_e, rel_e = self.get_s_embedder(), self.get_p_embedder()
        cand = ent_e.embed_all()
        p_inv = rel_e.embed(p + self.dataset.num_relations())
        o = self.get_o_embedder().embed(o)
        return self._scorer.score_emb_xent(o, p_inv, cand, "sp_", labels, scale, l_ptr, smoothing)

    def score_po_xent(self, p: Tensor, o: Tensor, s: Tensor, scale: float):
        tabs = self._lookup_tables()
        if tabs is None:
            return self._xent_dropout_po(p, o, s, scale)
        return self._scorer.score_lookup_xent(tabs[0], tabs[1], o, p + self.dataset.num_relations(), "sp_", s,
                                              scale)

    def xent_part_po(self, p: Tensor, o: Tensor, labels: Tensor, l_ptr=None):
        """(?, p, o) is scored as (o, p + R, ?) (reciprocal_relations_model.py:67-74)."""
        return ("sp_", o, p + self.dataset.num_relations(), labels, l_ptr)

    def score_po_cand(self, p: Tensor, o: Tensor, cand: Tensor):
        """score_spo(cand, p, o, direction="s") == score of (o, p + R, cand) as "sp_"
        (reciprocal_relations_model.py:57-65)."""
        tabs = self._lookup_tables()
        if tabs is None:
            return None
        return self._scorer.score_lookup_cand(tabs[0], tabs[1], o, p + self.dataset.num_relations(), "sp_", cand)

    def score_po_kl(self, p: Tensor, o: Tensor, l_ptr: Tensor, l_col: Tensor, smoothing: float, scale: float):
        tabs = self._lookup_tables()
        if tabs is None:
            return self._xent_dropout_po(p, o, l_col, scale, l_ptr, smoothing)
        return self._scorer.score_lookup_xent(tabs[0], tabs[1], o, p + self.dataset.num_relations(), "sp_", l_col,
                                              scale, l_ptr, smoothing)

    def score_so(self, s, o, p=None):
        raise Exception("The reciprocal relations model cannot score relations.")

    def _sp_po_parts(self, s: Tensor, p: Tensor, o: Tensor, p_po: Tensor = None):
        return [("sp_", s, p), ("sp_", o, p + self.dataset.num_relations())]

    def score_sp_po(self, s: Tensor, p: Tensor, o: Tensor, entity_subset: Tensor = None) -> Tensor:
        tabs = self._lookup_tables()
        p_inv = p + self.dataset.num_relations()
        if tabs is not None:
            return super().score_sp_po(s, p, o, entity_subset)
        s = self.get_s_embedder().embed(s)
        pi = self.get_p_embedder().embed(p_inv)
        p = self.get_p_embedder().embed(p)
        o = self.get_o_embedder().embed(o)
        ents = (self.get_s_embedder().embed(entity_subset) if entity_subset is not None
                else self.get_s_embedder().embed_all())
        sp_scores = self._scorer.score_emb(s, p, ents, combine="sp_")
        po_scores = self._scorer.score_emb(o, pi, ents, combine="sp_")
        return torch.cat((sp_scores, po_scores), dim=1)
