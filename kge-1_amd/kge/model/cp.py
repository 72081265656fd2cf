"""CP (cp.py:7-57): score(s, r, o) = sum(s_h * r * o_t), where an entity row holds a
subject half s_h = e[:d/2] and an object half o_t = e[d/2:].  Engine restatement:
sp_ = (s_h * r) . E[:, d/2:]^T and _po = (o_t * r) . E[:, :d/2]^T -- the prepared query is
d/2 wide and the all-entities contraction reads the matching half of every entity row
(a strided view of the table, no copy)."""
from .. import _lib
from .kge_model import KgeModel, RelationalScorer


class CPScorer(RelationalScorer):
    engine_kind = _lib.CP


class CP(KgeModel):
    def __init__(self, config, dataset, configuration_key=None, init_for_load_only=False):
        self._init_configuration(config, configuration_key)
        if self.get_option("entity_embedder.dim") % 2 != 0:
            raise ValueError("CP requires embeddings of even dimensionality"
                             " (got {})".format(self.get_option("entity_embedder.dim")))
        if self.get_option("relation_embedder.dim") < 0:
            self.set_option("relation_embedder.dim", self.get_option("entity_embedder.dim") // 2, log=True)
        super().__init__(config=config, dataset=dataset, scorer=CPScorer,
                         configuration_key=self.configuration_key, init_for_load_only=init_for_load_only)
