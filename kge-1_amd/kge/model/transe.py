"""TransE (transe.py:8-43): score = -||s + r - o||_p.  sp_ / _po run on the engine's
VALU distance kernel (the reference uses torch.cdist); spo keeps F.pairwise_distance
semantics (eps 1e-6 added to the difference)."""
from .. import _lib
from .kge_model import KgeModel, RelationalScorer


class TransEScorer(RelationalScorer):
    engine_kind = _lib.TRANSE
    s_o_viewed_by_relation_count = True  # the reference reshapes "s_o" scores this way

    def __init__(self, config, dataset, configuration_key=None):
        super().__init__(config, dataset, configuration_key)
        self._norm = self.get_option("l_norm")

    def l_norm(self) -> float:
        return float(self._norm)


class TransE(KgeModel):
    def __init__(self, config, dataset, configuration_key=None, init_for_load_only=False):
        super().__init__(config=config, dataset=dataset, scorer=TransEScorer,
                         configuration_key=configuration_key, init_for_load_only=init_for_load_only)
