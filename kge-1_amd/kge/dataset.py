"""Dataset: splits of (s, p, o) index triples plus the lookup indexes the scoring jobs
need.  Mirrors the parts of LibKGE's kge/dataset.py the path uses: ``Dataset.create``
(dataset.py:87-108), the ``.del`` triple loader (tab-separated, int32, dataset.py:168-182),
``num_entities`` / ``num_relations``, ``split`` and ``index("<split>_sp_to_o" /
"<split>_po_to_s")`` (indexing.py:8-98, 287-301).  No pickle cache (the reference's
pickles do not reload under torch >= 2.6 anyway).

``Dataset.synthetic`` builds the published dataset shapes offline (no data ships with
the reference and there is no network): FB15K-237 (14,541 / 237; 272,115 / 17,535 /
20,466), WN18RR (40,943 / 11; 86,835 / 3,034 / 3,134), Wikidata5M (4,594,485 / 822).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np
import torch

from .config import Config, Configurable

SHAPES = {
    "fb15k-237": (14541, 237, (272115, 17535, 20466)),
    "wn18rr": (40943, 11, (86835, 3034, 3134)),
    "wikidata5m": (4594485, 822, (20614279, 5163, 5133)),
    "toy": (1000, 20, (10000, 500, 500)),
}


class KvsAllIndex:
    """key (a, b) -> sorted unique values, stored as CSR over sorted unique keys."""

    def __init__(self, triples: np.ndarray, key_cols, value_col: int):
        t = np.asarray(triples, dtype=np.int64)
        k0, k1, v = t[:, key_cols[0]], t[:, key_cols[1]], t[:, value_col]
        order = np.lexsort((v, k1, k0))
        k0, k1, v = k0[order], k1[order], v[order]
        keep = np.ones(len(v), bool)
        keep[1:] = (k0[1:] != k0[:-1]) | (k1[1:] != k1[:-1]) | (v[1:] != v[:-1])
        k0, k1, v = k0[keep], k1[keep], v[keep]
        newkey = np.ones(len(v), bool)
        newkey[1:] = (k0[1:] != k0[:-1]) | (k1[1:] != k1[:-1])
        starts = np.flatnonzero(newkey)
        self.keys = np.stack([k0[starts], k1[starts]], 1)
        self.offsets = np.append(starts, len(v)).astype(np.int64)
        self.values = v
        self._lookup = None

    def __len__(self):
        return len(self.keys)

    def _dict(self):
        if self._lookup is None:
            self._lookup = {(int(a), int(b)): i for i, (a, b) in enumerate(self.keys)}
        return self._lookup

    def get(self, key, default=None):
        i = self._dict().get((int(key[0]), int(key[1])))
        if i is None:
            return default if default is not None else torch.zeros(0, dtype=torch.long)
        return torch.from_numpy(self.values[self.offsets[i]:self.offsets[i + 1]])

    __getitem__ = get

    def csr_for(self, queries: np.ndarray):
        """CSR (ptr[len(queries)+1], col) of the value lists of each query key (a, b)."""
        q = np.asarray(queries, dtype=np.int64)
        E = int(max(self.keys[:, 1].max(initial=0), q[:, 1].max(initial=0))) + 1
        kcode = self.keys[:, 0] * E + self.keys[:, 1]
        qcode = q[:, 0] * E + q[:, 1]
        pos = np.searchsorted(kcode, qcode)
        pos_c = np.minimum(pos, len(kcode) - 1) if len(kcode) else pos
        found = (len(kcode) > 0) & (kcode[pos_c] == qcode) if len(kcode) else np.zeros(len(q), bool)
        lo = np.where(found, self.offsets[pos_c] if len(kcode) else 0, 0)
        hi = np.where(found, self.offsets[pos_c + 1] if len(kcode) else 0, 0)
        lens = hi - lo
        ptr = np.zeros(len(q) + 1, np.int64)
        np.cumsum(lens, out=ptr[1:])
        total = int(ptr[-1])
        if total == 0:
            return ptr, np.zeros(0, np.int64)
        rowstart = np.repeat(lo - ptr[:-1], lens)
        col = self.values[np.arange(total, dtype=np.int64) + rowstart]
        return ptr, col


def _relation_types(train: np.ndarray, num_relations: int):
    """Relation -> "1-1" / "1-N" / "M-1" / "M-N" (indexing.py:142-179): M when a (p, o) pair of the
    relation has more than 1.5 subjects on average over the training triples, N likewise for
    objects per (s, p) pair; fp32 ratios, duplicates counted, no training triples -> "1-1"."""
    t = np.asarray(train, dtype=np.int64)
    R = num_relations
    n = np.bincount(t[:, 1], minlength=R).astype(np.float32)
    big = int(t[:, [0, 2]].max(initial=0)) + 1
    distinct_po = np.bincount(np.unique(t[:, 1] * big + t[:, 2]) // big, minlength=R).astype(np.float32)
    distinct_sp = np.bincount(np.unique(t[:, 1] * big + t[:, 0]) // big, minlength=R).astype(np.float32)
    with np.errstate(invalid="ignore", divide="ignore"):
        is_m = n / distinct_po > 1.5
        is_n = n / distinct_sp > 1.5
    return ["{}-{}".format("M" if m else "1", "N" if k else "1") for m, k in zip(is_m, is_n)]


PERCENTILES = (("25%", 0.0, 0.25), ("50%", 0.25, 0.5), ("75%", 0.5, 0.75), ("top", 0.75, 1.0))


def _frequency_percentiles(train: np.ndarray, num_entities: int, num_relations: int):
    """{"subject" | "relation" | "object": {"25%" | "50%" | "75%" | "top": set of ids}}: the ids of a
    slot ordered by training frequency (ties in id order), cut at int(fraction * count)
    (indexing.py:200-263)."""
    t = np.asarray(train, dtype=np.int64)
    out = {}
    for arg, col, num in (("subject", 0, num_entities), ("relation", 1, num_relations), ("object", 2, num_entities)):
        order = np.argsort(np.bincount(t[:, col], minlength=num), kind="stable")
        out[arg] = {name: set(order[int(b * num):int(e * num)].tolist()) for name, b, e in PERCENTILES}
    return out


class Dataset(Configurable):
    def __init__(self, config: Config, folder: Optional[str] = None):
        super().__init__(config, "dataset")
        self.folder = folder
        ne = config.get("dataset.num_entities") if config.exists("dataset.num_entities") else -1
        nr = config.get("dataset.num_relations") if config.exists("dataset.num_relations") else -1
        self._num_entities: Optional[int] = ne if ne >= 0 else None
        self._num_relations: Optional[int] = nr if nr >= 0 else None
        self._triples: Dict[str, torch.Tensor] = {}
        self._indexes: Dict[str, object] = {}

    # ------------------------------------------------------------------ creation
    @staticmethod
    def create(config: Config, preload_data: bool = True, folder: Optional[str] = None) -> "Dataset":
        name = config.get("dataset.name")
        if folder is None:
            base = os.environ.get("KGE_DATA", os.path.join(os.getcwd(), "data"))
            folder = os.path.join(base, name)
        yml = os.path.join(folder, "dataset.yaml")
        if os.path.isfile(yml):
            config.load(yml)
        ds = Dataset(config, folder)
        if preload_data:
            ds.num_entities()
            ds.num_relations()
            for split in ("train", "valid", "test"):
                try:
                    ds.split(split)
                except IOError:
                    pass
        return ds

    @staticmethod
    def synthetic(config: Config, name: str = "fb15k-237", seed: int = 0, num_entities: int = None,
                  num_relations: int = None, sizes=None) -> "Dataset":
        """Seeded synthetic dataset of a published shape: unique triples, entities drawn
        with a Zipf-like skew (so that filtering matters), exact split sizes."""
        E, R, sz = SHAPES.get(name, (None, None, None))
        E = num_entities or E
        R = num_relations or R
        sz = tuple(sizes or sz)
        total = int(sum(sz))
        rng = np.random.default_rng(seed)
        w = 1.0 / np.arange(1, E + 1) ** 0.6
        cdf = np.cumsum(w / w.sum())
        uniq = np.zeros(0, np.int64)
        while len(uniq) < total:
            n = int((total - len(uniq)) * 1.3) + 1024
            s = np.minimum(np.searchsorted(cdf, rng.random(n)), E - 1)
            o = np.minimum(np.searchsorted(cdf, rng.random(n)), E - 1)
            p = rng.integers(0, R, n)
            code = (s * R + p) * E + o
            allc = np.concatenate([uniq, code])
            _, first = np.unique(allc, return_index=True)
            uniq = allc[np.sort(first)]
        uniq = uniq[:total]
        o = uniq % E
        sp = uniq // E
        p = sp % R
        s = sp // R
        t = np.stack([s, p, o], 1).astype(np.int32)
        config.set("dataset.name", name)
        config.set("dataset.num_entities", int(E))
        config.set("dataset.num_relations", int(R))
        ds = Dataset(config, None)
        a, b = sz[0], sz[0] + sz[1]
        ds._triples = {"train": torch.from_numpy(t[:a].copy()), "valid": torch.from_numpy(t[a:b].copy()),
                       "test": torch.from_numpy(t[b:].copy())}
        return ds

    def shallow_copy(self) -> "Dataset":
        c = Dataset(self.config, self.folder)
        c._num_entities, c._num_relations = self._num_entities, self._num_relations
        c._triples = self._triples
        c._indexes = self._indexes
        return c

    # ------------------------------------------------------------------ loading
    def _file(self, key: str) -> str:
        if self.folder is None or not os.path.exists(self.folder):
            raise IOError("Dataset {} not found".format(self.config.get("dataset.name")))
        fn = os.path.join(self.folder, self.config.get(f"dataset.files.{key}.filename"))
        if not os.path.exists(fn):
            raise IOError(f"File {fn} for key {key} could not be found")
        return fn

    @staticmethod
    def load_triples_file(filename: str) -> torch.Tensor:
        """Tab-separated s, p, o (extra columns ignored) -> int32 [n, 3]."""
        data = np.loadtxt(filename, usecols=range(3), dtype=np.int32, ndmin=2, delimiter="\t")
        return torch.from_numpy(data)

    def num_entities(self) -> int:
        if self._num_entities is None:
            with open(self._file("entity_ids")) as f:
                self._num_entities = sum(1 for line in f if line.strip())
        return self._num_entities

    def num_relations(self) -> int:
        if self._num_relations is None:
            with open(self._file("relation_ids")) as f:
                self._num_relations = sum(1 for line in f if line.strip())
        return self._num_relations

    def split(self, split: str) -> torch.Tensor:
        if split not in self._triples:
            self._triples[split] = Dataset.load_triples_file(self._file(split))
        return self._triples[split]

    def index(self, key: str):
        """"<split>_sp_to_o" / "<split>_po_to_s" / "<split>_so_to_p" (indexing.py:287-301), "relation_types",
        "relations_per_type" and "frequency_percentiles" (indexing.py:142-263)."""
        if key not in self._indexes:
            if key == "relation_types":
                self._indexes[key] = _relation_types(self.split("train").numpy(), self.num_relations())
            elif key == "relations_per_type":
                per_type: Dict[str, set] = {}
                for i, k in enumerate(self.index("relation_types")):
                    per_type.setdefault(k, set()).add(i)
                self._indexes[key] = per_type
            elif key == "frequency_percentiles":
                self._indexes[key] = _frequency_percentiles(
                    self.split("train").numpy(), self.num_entities(), self.num_relations())
            elif key.endswith("_sp_to_o"):
                t = self.split(key[: -len("_sp_to_o")]).numpy()
                self._indexes[key] = KvsAllIndex(t, (0, 1), 2)
            elif key.endswith("_po_to_s"):
                t = self.split(key[: -len("_po_to_s")]).numpy()
                self._indexes[key] = KvsAllIndex(t, (1, 2), 0)
            elif key.endswith("_so_to_p"):
                t = self.split(key[: -len("_so_to_p")]).numpy()
                self._indexes[key] = KvsAllIndex(t, (0, 2), 1)
            else:
                raise KeyError(key)
        return self._indexes[key]
