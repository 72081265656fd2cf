"""RotatE (rotate.py:11-145): score = || |s * rot(r) - o| ||_p over the d/2 complex
components, rot(r) = cos r + i sin r.  Scores are POSITIVE distances, as in the
reference.  sp_ and _po stream through the engine's VALU distance kernel
instead of materialising n x E x d/2 tensors; _po is restated as
|e * rot(r) - o| = |e - o * conj(rot(r))| (|rot| = 1)."""
from .. import _lib
from .kge_model import KgeModel, RelationalScorer


class RotatEScorer(RelationalScorer):
    engine_kind = _lib.ROTATE

    def __init__(self, config, dataset, configuration_key=None):
        super().__init__(config, dataset, configuration_key)
        self._norm = self.get_option("l_norm")

    def l_norm(self) -> float:
        return float(self._norm)


class RotatE(KgeModel):
    def __init__(self, config, dataset, configuration_key=None, init_for_load_only=False):
        self._init_configuration(config, configuration_key)
        if self.get_option("entity_embedder.dim") % 2 != 0:
            raise ValueError("RotatE requires embeddings of even dimensionality"
                             " (got {})".format(self.get_option("entity_embedder.dim")))
        if self.get_option("relation_embedder.dim") < 0:
            self.set_option("relation_embedder.dim", self.get_option("entity_embedder.dim") // 2, log=True)
        super().__init__(config=config, dataset=dataset, scorer=RotatEScorer,
                         configuration_key=self.configuration_key, init_for_load_only=init_for_load_only)
