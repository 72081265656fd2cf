"""Filtered entity ranking at the full FB15K-237 entity count (E = 14,541, R = 237,
ComplEx-512, the BASELINE configs[1] model) against the CPU oracle's restatement of
EntityRankingJob (oracle/kge_oracle.py: entity_ranking, following entity_ranking.py:79-577).

Dyadic tables (k/8, |k| <= 16) make every score exact in fp32 and in the bf16x3 split, so
the size-independent property holds at full size: every rank (raw and filtered, both
directions, ties included) and every metric must be identical.  The first 4,096 triples of
the synthetic test split are evaluated (filtering uses all splits) to keep the float64
oracle within seconds."""
import numpy as np
import pytest
import torch

from oracle import kge_oracle as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["bf16x3", "fp32", "bf16x3_refined"])
def test_entity_ranking_fb15k237_size_dyadic(precision):
    from kge import Config, Dataset, KgeModel
    from kge.job import EntityRankingJob

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 512)
    c.set("engine.precision", precision.replace("_refined", ""))
    c.set("engine.eval_precision", precision)  # refined: every exact tie of the true score is rescored
    c.set("eval.split", "test")
    c.set("eval.batch_size", 1024)
    c.set("verbose", False)
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    ds._triples["test"] = ds._triples["test"][:4096].clone()
    E, R = ds.num_entities(), ds.num_relations()
    assert (E, R) == (14541, 237)
    g = torch.Generator().manual_seed(5)
    ent = torch.randint(-16, 17, (E, 512), generator=g).float() / 8
    rel = torch.randint(-16, 17, (R, 512), generator=g).float() / 8
    torch.manual_seed(0)
    model = KgeModel.create(c, ds)
    with torch.no_grad():
        model._entity_embedder._embeddings.weight.copy_(ent)
        model._relation_embedder._embeddings.weight.copy_(rel)
    model.eval()
    job = EntityRankingJob(c, ds, model=model)
    job.capture_ranks = True
    trace = job.run()

    splits = {k: ds.split(k).long().numpy() for k in ("train", "valid", "test")}
    ranks, metrics = K.entity_ranking("complex", ent.numpy(), rel.numpy(), splits, eval_split="test",
                                      filter_splits=("train", "valid"), batch_size=1024)
    assert set(job.ranks) == set(ranks)
    for k, v in ranks.items():
        np.testing.assert_array_equal(job.ranks[k], v, err_msg=k)
    for k, v in metrics.items():
        assert trace[k] == pytest.approx(v, rel=1e-6, abs=1e-9), k
    # a non-degenerate ranking: ties present, ranks spread
    assert trace["mean_reciprocal_rank_filtered"] > 0.0 and len(np.unique(ranks["o_filt"])) > 100


def test_engine_eval_batch_size_changes_the_grouping_not_the_result():
    """eval.batch_size 100 (the reference's default, config-default.yaml:324) with and without
    the engine's larger launch groups (engine.eval_batch_size): identical ranks and metrics, and
    the trace counts the batches of eval.batch_size either way."""
    from kge import Config, Dataset, KgeModel
    from kge.job import EntityRankingJob

    traces, ranks, groups = [], [], []
    for engine_bs in (0, 1024):
        c = Config()
        c.set("model", "complex")
        c._import("complex")
        c.set("job.device", "cuda")
        c.set("lookup_embedder.dim", 128)
        c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
        c.set("eval.split", "valid")
        c.set("eval.batch_size", 100)
        c.set("engine.eval_batch_size", engine_bs)
        c.set("verbose", False)
        ds = Dataset.synthetic(c, "toy", seed=0, num_entities=3000, num_relations=9, sizes=(20000, 2345, 500))
        torch.manual_seed(0)
        model = KgeModel.create(c, ds)
        model.eval()
        job = EntityRankingJob(c, ds, model=model)
        job.capture_ranks = True
        traces.append(job.run())
        ranks.append(job.ranks)
        groups.append(job._bs)
    assert groups == [100, 1024]
    assert traces[0]["batches"] == traces[1]["batches"] == 24 and traces[0]["size"] == 2345
    for k in ranks[0]:
        np.testing.assert_array_equal(ranks[0][k], ranks[1][k], err_msg=k)
    for k, v in traces[0].items():
        if k not in ("epoch_time",) and isinstance(v, float):
            assert traces[1][k] == v, k
