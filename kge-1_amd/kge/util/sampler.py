"""Negative samplers (kge/util/sampler.py:12-315), drawing on the training device.

The reference samples on the host inside the DataLoader collate (train.py:800-818), with a
numba loop for filtering.  Here every step is a vectorised device op, so the NS step never
leaves the GPU:

* ``uniform``   -- torch.randint over the slot's vocabulary (sampler.py:191-197);
* ``frequency`` -- torch.multinomial over slot counts + symmetric prior
  (sampler.py:318-345);
* ``shared``    -- one draw per batch shared by all rows, with each row's own positive
  dropped (sampler.py:199-255);
* filtering    -- sampled positives (the training triples completing (p, o) / (s, o) / (s, p)) are
  re-drawn until none is left (sampler.py:140-171): membership is one searchsorted into a
  device copy of the slot's CSR index, globally sorted by (key, value).

Draws come from the device RNG, so samples differ from the reference's host RNG stream
(the reference itself is not reproducible across worker counts); the distribution and every
constraint above are the same.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

S, P, O = 0, 1, 2
SLOT_STR = ["s", "p", "o"]


class KgeSampler:
    def __init__(self, config, configuration_key: str, dataset, device):
        self.config = config
        self.dataset = dataset
        self.device = torch.device(device)
        get = lambda k: config.get(f"{configuration_key}.{k}")  # noqa: E731
        self.shared = bool(get("shared"))
        self.with_replacement = bool(get("with_replacement"))
        if not self.with_replacement and not self.shared:
            raise ValueError("Without replacement sampling is only supported when shared negative sampling is enabled.")
        self.num_samples = [int(get(f"num_samples.{s}")) for s in SLOT_STR]
        self.filter_positives = [bool(get(f"filtering.{s}")) for s in SLOT_STR]
        self.vocabulary_size = [dataset.num_relations() if s == P else dataset.num_entities() for s in range(3)]
        split = get("filtering.split") or config.get("train.split")
        if any(self.filter_positives) and self.shared:
            raise ValueError("Filtering is not supported when shared negative sampling is enabled.")
        # auto config: -1 copies s <-> o, p -> 0 (sampler.py:69-75)
        for slot, copy_from in ((S, O), (P, None), (O, S)):
            if self.num_samples[slot] < 0:
                if copy_from is not None and self.num_samples[copy_from] > 0:
                    self.num_samples[slot] = self.num_samples[copy_from]
                else:
                    self.num_samples[slot] = 0
        self._filter = [None, None, None]
        for slot, name in ((S, "po_to_s"), (P, "so_to_p"), (O, "sp_to_o")):
            if self.filter_positives[slot]:
                self._filter[slot] = self._device_index(dataset.index(f"{split}_{name}"))

    def _device_index(self, idx):
        """(key codes, (key rank * V + value) codes) -- both sorted -- of a KvsAllIndex."""
        k1max = int(max(idx.keys[:, 1].max(initial=0), self.dataset.num_entities(), self.dataset.num_relations())) + 1
        kcode = idx.keys[:, 0].astype(np.int64) * k1max + idx.keys[:, 1]
        lens = np.diff(idx.offsets)
        rank = np.repeat(np.arange(len(idx.keys), dtype=np.int64), lens)
        V = max(self.vocabulary_size) + 1
        vcode = rank * V + idx.values.astype(np.int64)
        return (torch.from_numpy(kcode).to(self.device), torch.from_numpy(vcode).to(self.device), k1max, V)

    @staticmethod
    def create(config, configuration_key: str, dataset, device="cuda"):
        t = config.get(configuration_key + ".sampling_type")
        if t == "uniform":
            return KgeUniformSampler(config, configuration_key, dataset, device)
        if t == "frequency":
            return KgeFrequencySampler(config, configuration_key, dataset, device)
        raise ValueError(configuration_key + ".sampling_type")

    # ------------------------------------------------------------------- sampling
    def sample(self, positive_triples: torch.Tensor, slot: int, num_samples: Optional[int] = None) -> torch.Tensor:
        """[n, num_samples] int64 negatives for `slot` of the (device) positive triples."""
        if num_samples is None:
            num_samples = self.num_samples[slot]
        if self.shared:
            neg = self._sample_shared(positive_triples, slot, num_samples)
        else:
            neg = self._sample(len(positive_triples), slot, num_samples)
        if self._filter[slot] is not None:
            neg = self._filter_and_resample(neg, slot, positive_triples)
        return neg

    def _sample(self, n: int, slot: int, num_samples: int) -> torch.Tensor:
        raise NotImplementedError

    def _sample_shared(self, positive_triples, slot, num_samples):
        raise NotImplementedError("The selected sampler does not support shared negative samples.")

    def _is_positive(self, neg: torch.Tensor, slot: int, positive_triples: torch.Tensor) -> torch.Tensor:
        kcode, vcode, k1max, V = self._filter[slot]
        ka, kb = {S: (P, O), P: (S, O), O: (S, P)}[slot]  # the slot's key columns, in index order
        a, b = positive_triples[:, ka], positive_triples[:, kb]
        q = a * k1max + b
        pos = torch.searchsorted(kcode, q).clamp_(max=max(len(kcode) - 1, 0))
        has = kcode[pos] == q if len(kcode) else torch.zeros_like(q, dtype=torch.bool)
        codes = pos[:, None] * V + neg
        j = torch.searchsorted(vcode, codes).clamp_(max=max(len(vcode) - 1, 0))
        return has[:, None] & (vcode[j] == codes)

    def _filter_and_resample(self, neg, slot, positive_triples, max_rounds: int = 1000):
        for _ in range(max_rounds):
            bad = self._is_positive(neg, slot, positive_triples)
            nbad = int(bad.sum())  # host sync per round; rounds are few (positives are sparse)
            if nbad == 0:
                return neg
            neg = neg.masked_scatter(bad, self._sample(1, slot, nbad).view(-1))
        raise RuntimeError("negative filtering did not converge (a query has almost every entity as positive?)")


class KgeUniformSampler(KgeSampler):
    def _sample(self, n, slot, num_samples):
        return torch.randint(self.vocabulary_size[slot], (n, num_samples), device=self.device)

    def _sample_shared(self, positive_triples, slot, num_samples):
        """sampler.py:199-255 on device: num_distinct + 1 WOR draws shared by the batch; in
        each row the row's positive (if drawn) -- else a random position -- is overwritten
        by the extra draw; WR sampling then up-samples the distinct columns."""
        n = len(positive_triples)
        V = self.vocabulary_size[slot]
        if self.with_replacement:
            # distribution of #distinct values in num_samples WR draws from V - 1 (as the reference)
            num_distinct = int(torch.unique(torch.randint(V - 1, (num_samples,), device=self.device)).numel())
        else:
            num_distinct = num_samples
        shared = torch.randperm(V, device=self.device)[: num_distinct + 1]
        match = shared[None, :num_distinct + 1] == positive_triples[:, slot][:, None]  # [n, nd+1]
        has = match.any(1)
        drop = torch.where(has, match.float().argmax(1),
                           torch.randint(num_distinct + 1, (n,), device=self.device))
        samples = shared[:num_distinct].repeat(n, 1)
        rows = torch.nonzero(drop != num_distinct).view(-1)
        samples[rows, drop[rows]] = shared[num_distinct]
        if num_distinct != num_samples:
            extra = torch.randint(num_distinct, (num_samples - num_distinct,), device=self.device)
            samples = torch.cat((samples, samples[:, extra]), 1)
        return samples


class KgeFrequencySampler(KgeSampler):
    """Slot frequencies in the training split + symmetric prior (sampler.py:318-345)."""

    def __init__(self, config, configuration_key, dataset, device):
        super().__init__(config, configuration_key, dataset, device)
        alpha = float(config.get(f"{configuration_key}.frequency.smoothing"))
        train = dataset.split(config.get("train.split")).long()
        self._probs = []
        for slot in range(3):
            counts = torch.bincount(train[:, slot], minlength=self.vocabulary_size[slot]).double() + alpha
            self._probs.append((counts / counts.sum()).float().to(self.device))

    def _sample(self, n, slot, num_samples):
        if num_samples == 0 or n == 0:
            return torch.zeros(n, num_samples, dtype=torch.long, device=self.device)
        return torch.multinomial(self._probs[slot], n * num_samples, replacement=True).view(n, num_samples)
