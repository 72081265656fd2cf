import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kge-1_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")

# tests validate every index vector against its table before launching a kernel
os.environ.setdefault("KGE_CHECK_INDEX", "1")


def seeded_scorer_tables(seed, regime, model, E, R, d_e, d_r):
    """The tables of the larger scorer fixtures, regenerated from the numpy seed recorded in the
    fixture (tests/golden/make_golden.py stores only the reference's outputs for them)."""
    import math

    import numpy as np

    rng = np.random.default_rng(seed)
    if regime == "normal":
        ent = (rng.standard_normal((E, d_e), dtype=np.float32) * np.float32(0.1)).astype(np.float32)
        rel = (rng.standard_normal((R, d_r), dtype=np.float32) * np.float32(0.1)).astype(np.float32)
    else:
        ent = (rng.integers(-16, 17, (E, d_e)) / 8.0).astype(np.float32)
        rel = (rng.integers(-16, 17, (R, d_r)) / 8.0).astype(np.float32)
    if model == "rotate":
        rel = ((rng.random((R, d_r)) * 2 - 1) * math.pi).astype(np.float32)
    return ent, rel


def table_checksum(x):
    import numpy as np

    return [float(x.astype(np.float64).sum()), float(np.abs(x.astype(np.float64)).sum()),
            float(x[0, 0]), float(x[-1, -1])]


def load_scorer_fixture(fn):
    """A scorer fixture as a dict; fixtures that record a table seed instead of the tables get
    "ent" / "rel" regenerated (and checked against the recorded checksums)."""
    import json

    import numpy as np

    f = np.load(fn)
    d = {k: f[k] for k in f.files}
    if "ent" not in d:
        meta = json.loads(str(d["meta"]))
        ent, rel = seeded_scorer_tables(meta["table_seed"], meta["regime"], meta["model"], meta["E"], meta["R"],
                                        meta["d_e"], meta["d_r"])
        assert table_checksum(ent) == meta["ent_checksum"] and table_checksum(rel) == meta["rel_checksum"], \
            "seeded tables differ from the ones the reference was run on (numpy stream changed?)"
        d["ent"], d["rel"] = ent, rel
    return d
