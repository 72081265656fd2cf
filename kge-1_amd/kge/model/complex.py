"""ComplEx (complex.py:7-63): score(s, r, o) = Re(<s, r, conj(o)>) with embeddings
stored as [re | im] halves.  Engine restatement: sp_ = cmul(s, r) . E^T and
_po = cmul(conj(r), o) . E^T, one K = d contraction (the reference's K = 2d duplicated
layout, complex.py:27-38, gives the same values up to fp32 rounding)."""
from .. import _lib
from .kge_model import KgeModel, RelationalScorer


class ComplExScorer(RelationalScorer):
    engine_kind = _lib.COMPLEX


class ComplEx(KgeModel):
    def __init__(self, config, dataset, configuration_key=None, init_for_load_only=False):
        super().__init__(config=config, dataset=dataset, scorer=ComplExScorer,
                         configuration_key=configuration_key, init_for_load_only=init_for_load_only)
