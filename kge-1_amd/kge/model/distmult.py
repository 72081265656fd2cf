"""DistMult (distmult.py:7-45): score(s, r, o) = sum(s * r * o); sp_ = (s * r) . E^T,
_po = (o * r) . E^T on the engine's MFMA contraction."""
from .. import _lib
from .kge_model import KgeModel, RelationalScorer


class DistMultScorer(RelationalScorer):
    engine_kind = _lib.DISTMULT


class DistMult(KgeModel):
    def __init__(self, config, dataset, configuration_key=None, init_for_load_only=False):
        super().__init__(config=config, dataset=dataset, scorer=DistMultScorer,
                         configuration_key=configuration_key, init_for_load_only=init_for_load_only)
