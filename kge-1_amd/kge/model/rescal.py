"""RESCAL (rescal.py:8-96): score(s, r, o) = s^T M_r o, M_r = relation row viewed as a
d x d row-major matrix.  sp_ = (s^T M_r) . E^T, _po = (M_r o) . E^T."""
from .. import _lib
from .kge_model import KgeModel, RelationalScorer


class RescalScorer(RelationalScorer):
    engine_kind = _lib.RESCAL
    s_o_viewed_by_relation_count = True  # the reference reshapes "s_o" scores this way


class Rescal(KgeModel):
    def __init__(self, config, dataset, configuration_key=None, init_for_load_only=False):
        self._init_configuration(config, configuration_key)
        rescal_set_relation_embedder_dim(config, dataset, self.configuration_key + ".relation_embedder")
        super().__init__(config=config, dataset=dataset, scorer=RescalScorer,
                         configuration_key=self.configuration_key, init_for_load_only=init_for_load_only)


def rescal_set_relation_embedder_dim(config, dataset, rel_emb_conf_key):
    """dim < 0 -> square of the entity dim (rescal.py:79-96)."""
    dim = config.get_default(rel_emb_conf_key + ".dim")
    if dim < 0:
        ent_key = rel_emb_conf_key.replace("relation_embedder", "entity_embedder")
        if ent_key == rel_emb_conf_key:
            raise ValueError("Cannot determine relation embedding size; please set manually.")
        dim = config.get_default(ent_key + ".dim") ** 2
        config.set(rel_emb_conf_key + ".dim", dim, log=True)
