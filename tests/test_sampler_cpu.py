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


def test_filtering_of_relation_negatives():
    """filtering.p: sampled relations r with (s, r, o) in the training split are redrawn
    (sampler.py:140-171 with the so_to_p index); with 24 relations over 641 entity pairs (up to 15 positives each) many rows
    have a positive among their first draws."""
    c = Config()
    c.set("negative_sampling.filtering.p", True)
    c.set("negative_sampling.num_samples.p", 3)
    ds = _ds(c, E=30, R=24)
    smp = KgeSampler.create(c, "negative_sampling", ds, "cpu")
    assert smp.num_samples[1] == 3
    tr = ds.split("train")[:300].long()
    first = smp._sample(300, 1, 3)
    assert bool(smp._is_positive(first, 1, tr).any())  # unfiltered draws do hit positives
    neg = smp.sample(tr, 1)
    assert neg.shape == (300, 3) and int(neg.min()) >= 0 and int(neg.max()) < 24
    assert not bool(smp._is_positive(neg, 1, tr).any())
    assert bool(smp._is_positive(tr[:, [1]], 1, tr).all())
    train = {tuple(t) for t in ds.split("train").tolist()}
    for (s, p, o), row in zip(tr.tolist(), neg.tolist()):
        assert all((s, r, o) not in train for r in row)


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
