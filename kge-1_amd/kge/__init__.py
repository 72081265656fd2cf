"""kge -- MI355X-native scoring engine for LibKGE's 1vsAll / KvsAll hot path.

Host code mirrors the reference's plugin API (kge.model.KgeModel / RelationalScorer /
KgeEmbedder); the work runs in libkgescore.so (hand-written gfx950 HIP kernels).
"""
