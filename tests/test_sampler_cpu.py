"""CPU: the device negative sampler's host-independent logic (kge/util/sampler.py) --
ranges, auto num_samples, shared sampling dropping each row's positive (sampler.py:199-255),
filtering of training positives (sampler.py:140-171), frequency sampling support."""
import torch

from kge import Config, Dataset
from kge.util.sampler import KgeSampler


def _ds(c, E=50, R=5):
    return Dataset.synthetic(c, "toy", seed=0, num_entities=E, num_relations=R, sizes=(1500, 10, 10))


def test_filtering_removes_training_positives():
    c = Config()
    c.set("negative_sampling.filtering.o", True)
    c.set("negative_sampling.filtering.s", True)
    c.set("negative_sampling.num_samples.s", 40)
    ds = _ds(c)
    smp = KgeSampler.create(c, "negative_sampling", ds, "cpu")
    assert smp.num_samples == [40, 0, 40]  # o copies s, p defaults to 0
    tr = ds.split("train")[:300].long()
    for slot in (0, 2):
        neg = smp.sample(tr, slot)
        assert neg.shape == (300, 40) and int(neg.min()) >= 0 and int(neg.max()) < 50
        assert not bool(smp._is_positive(neg, slot, tr).any())
        assert bool(smp._is_positive(tr[:, [slot]], slot, tr).all())


def test_shared_sampling_drops_own_positive():
    c = Config()
    c.set("negative_sampling.shared", True)
    c.set("negative_sampling.num_samples.s", 20)
    ds = _ds(c)
    smp = KgeSampler.create(c, "negative_sampling", ds, "cpu")
    tr = ds.split("train")[:300].long()
    for wr in (True, False):
        smp.with_replacement = wr
        for slot in (0, 2):
            neg = smp.sample(tr, slot)
            assert neg.shape == (300, 20)
            assert not bool((neg == tr[:, [slot]]).any())
            if not wr:  # WOR: distinct per row
                assert all(len(set(r.tolist())) == 20 for r in neg)


def test_frequency_sampler():
    c = Config()
    c.set("negative_sampling.sampling_type", "frequency")
    ds = _ds(c)
    smp = KgeSampler.create(c, "negative_sampling", ds, "cpu")
    tr = ds.split("train")[:100].long()
    neg = smp.sample(tr, 2, 1000)
    counts = torch.bincount(neg.view(-1), minlength=50).float()
    # Zipf-skewed synthetic data: the most frequent object id is drawn far more often
    freq = torch.bincount(ds.split("train")[:, 2].long(), minlength=50).float()
    assert counts[freq.argmax()] > 3 * counts[freq.argmin()]
