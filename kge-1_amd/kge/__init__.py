"""kge -- MI355X-native scoring engine for LibKGE's 1vsAll / KvsAll hot path.

Host code mirrors the reference's plugin API (kge.model.KgeModel / RelationalScorer /
KgeEmbedder); the work runs in libkgescore.so (hand-written gfx950 HIP kernels).
"""
from .config import Config, Configurable  # noqa: E402,F401
from .dataset import Dataset  # noqa: E402,F401
from .model.kge_model import KgeModel, KgeEmbedder  # noqa: E402,F401
