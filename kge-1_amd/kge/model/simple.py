"""SimplE (simple.py:7-58): an entity row is [e_h | e_t], a relation row [r_f | r_b], and
score(s, r, o) = (sum(s_h * r_f * o_t) + sum(s_t * r_b * o_h)) / 2.  Engine restatement:
one K = d contraction per direction with the halves of the query swapped and the 1/2
folded in -- sp_ = 0.5 [s_t * r_b | s_h * r_f] . [e_h | e_t]^T and
_po = 0.5 [o_t * r_f | o_h * r_b] . [e_h | e_t]^T (equal to the reference's two K = d/2
products up to fp32 rounding; exact on dyadic inputs)."""
from .. import _lib
from .kge_model import KgeModel, RelationalScorer


class SimplEScorer(RelationalScorer):
    engine_kind = _lib.SIMPLE


class SimplE(KgeModel):
    def __init__(self, config, dataset, configuration_key=None, init_for_load_only=False):
        self._init_configuration(config, configuration_key)
        if self.get_option("entity_embedder.dim") % 2 != 0:
            raise ValueError("SimplE requires embeddings of even dimensionality"
                             " (got {})".format(self.get_option("entity_embedder.dim")))
        super().__init__(config=config, dataset=dataset, scorer=SimplEScorer,
                         configuration_key=self.configuration_key, init_for_load_only=init_for_load_only)
