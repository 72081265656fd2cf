"""Model plugins resolved by class name (KgeModel.create / KgeEmbedder.create)."""
from .kge_model import KgeBase, KgeEmbedder, KgeModel, RelationalScorer  # noqa: F401
from .embedder.lookup_embedder import LookupEmbedder  # noqa: F401
from .complex import ComplEx, ComplExScorer  # noqa: F401
from .distmult import DistMult, DistMultScorer  # noqa: F401
from .rescal import Rescal, RescalScorer  # noqa: F401
from .transe import TransE, TransEScorer  # noqa: F401
from .rotate import RotatE, RotatEScorer  # noqa: F401
from .cp import CP, CPScorer  # noqa: F401
from .simple import SimplE, SimplEScorer  # noqa: F401
from .reciprocal_relations_model import ReciprocalRelationsModel  # noqa: F401
