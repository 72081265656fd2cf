"""GPU parity at shapes that cross the production kernels' tiles, against reference-captured
fixtures (tests/golden/make_golden.py: RESCAL at d = 128, a 1vsAll trajectory over 1,600 entities,
the toy run's per-epoch tables and validation ranks) and, at BASELINE configs[1]'s full size,
against float64 autograd of the reference formulas."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, seeded_scorer_tables, table_checksum
from test_gpu_configs import base_config, dataset_from, set_tables, tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib

    _lib.lib()


def _seeded(meta, model, d_r):
    ent, rel = seeded_scorer_tables(meta["table_seed"], "normal", model, meta["E"], meta["R"], meta["dim"], d_r)
    assert table_checksum(ent) == meta["ent_checksum"] and table_checksum(rel) == meta["rel_checksum"], \
        "seeded tables differ from the ones the reference was run on (numpy stream changed?)"
    return ent, rel


@pytest.mark.parametrize("eval_precision", ["bf16x3_refined", "fp32"])
def test_rescal128_entity_ranking_vs_reference(eval_precision):
    """The reference's EntityRankingJob with RESCAL at d = 128 -- relation rows of 16,384 floats
    through prep_rescal -- rank for rank (rescal.py:15-53, entity_ranking.py:79-577)."""
    from kge import KgeModel
    from kge.job import EntityRankingJob

    f = np.load(os.path.join(GOLDEN, "eval_rescal128_normal.npz"))
    meta = json.loads(str(f["meta"]))
    ent, rel = _seeded(meta, "rescal", meta["dim"] ** 2)
    c = base_config("rescal", meta["dim"], meta["E"], meta["R"], {
        "eval.batch_size": meta["batch_size"], "eval.split": "valid", "engine.eval_precision": eval_precision})
    ds = dataset_from(c, f)
    model = KgeModel.create(c, ds)
    assert model._relation_embedder.dim == meta["dim"] ** 2
    set_tables(model, ent, rel)
    job = EntityRankingJob(c, ds, model=model)
    job.capture_ranks = True
    trace = job.run()
    ref = {k[5:]: f[k] for k in f.files if k.startswith("full_")}
    assert set(job.ranks) == set(ref)
    same = sum(int((job.ranks[k] == ref[k]).sum()) for k in ref)
    total = sum(len(v) for v in ref.values())
    assert same >= total - 2, (same, total)  # fp32 summation order may move a rank at a near-tie
    for k, v in json.loads(str(f["metrics"]))["full"].items():
        assert trace[k] == pytest.approx(v, rel=2e-3, abs=1e-9), k


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "recorded"])
@pytest.mark.parametrize("precision,gtol,atol,frac", [("fp32", 1e-5, 5e-5, 1e-3), ("bf16x3", 1e-4, 2e-4, 3e-3)])
def test_train_1vsall_large_vs_reference(precision, gtol, atol, frac, graph):
    """Three reference 1vsAll batches (ComplEx-128, Adagrad, kl) over 1,600 entities with 300
    triples each: seven entity panels and two (stacked: three) query tiles per contraction, the
    backward GEMMs' split-K over 1,600 rows.  The first batch's gradients (teacher-forced), the
    per-batch losses and the final tables; `recorded` replays the third batch from the job's HIP
    graph (two eager batches precede every recording).  Adagrad steps by g / sqrt(sum g^2), i.e.
    by about lr whatever the gradient's size: where a gradient nearly cancels, a rounding-level
    difference (1e-5 of the largest gradient with bf16x3) becomes a visible step, so a small
    fraction of the elements (measured 0.1 % with bf16x3) may lie beyond atol."""
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, "train1vsall_complex_large.npz"))
    meta = json.loads(str(f["meta"]))
    ent, rel = _seeded(meta, "complex", meta["dim"])
    c = base_config("complex", meta["dim"], meta["E"], meta["R"], {
        "train.type": "1vsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": meta["lr"]},
        "train.batch_size": meta["batch_size"], "engine.precision": precision, "engine.graph_step": graph})
    batches = torch.from_numpy(f["batches"].astype(np.int64))
    from kge import Dataset

    ds = Dataset(c, None)
    ds._triples = {"train": batches.reshape(-1, 3).int()}
    job = TrainingJob.create(c, ds)
    set_tables(job.model, ent, rel)
    job._prepare()
    # teacher-forced gradients of the first batch
    job.optimizer.zero_grad()
    job._process_batch(0, {"triples": batches[0]})
    ge = job.model._entity_embedder._embeddings.weight.grad.cpu().numpy()
    gr = job.model._relation_embedder._embeddings.weight.grad.cpu().numpy()
    assert np.abs(ge - f["g_ent_0"]).max() <= gtol * np.abs(f["g_ent_0"]).max()
    assert np.abs(gr - f["g_rel_0"]).max() <= gtol * np.abs(f["g_rel_0"]).max()
    job.optimizer.zero_grad()
    losses = []
    for b in range(len(batches)):
        res, _, _ = job.train_step(b, {"triples": batches[b]})
        losses.append(float(res.avg_loss))
    if graph:
        assert job._graph_step is not None and job._graph_step.graph is not None, job._graph_step.error
    np.testing.assert_allclose(losses, f["losses"], rtol=1e-5)
    e1, r1 = tables(job.model)
    for mine, ref in ((e1, f["ent1"]), (r1, f["rel1"])):
        diff = np.abs(mine - ref)
        assert int((diff > atol).sum()) <= max(8, frac * diff.size) and float(diff.mean()) < 1e-5


def test_c1_toy_validation_teacher_forced_vs_reference():
    """configs[0]: after every epoch of the reference's toy run, the reference's tables of that
    epoch go into this build's EntityRankingJob and its validation ranks must be the
    reference's -- the tables are the reference's own, so nothing but the scoring and ranking
    of that epoch is compared (the free-running trajectory test cannot pin the metrics tightly:
    Adagrad amplifies rounding)."""
    from kge import KgeModel
    from kge.job import EntityRankingJob

    f = np.load(os.path.join(GOLDEN, "train_toy_complex.npz"))
    g = np.load(os.path.join(GOLDEN, "train_toy_complex_epochs.npz"))
    meta = json.loads(str(f["meta"]))
    gmeta = json.loads(str(g["meta"]))
    ref_valids = json.loads(str(f["valids"]))
    c = base_config("complex", meta["dim"], meta["E"], meta["R"], {
        "eval.batch_size": meta["eval_batch_size"], "eval.split": "valid"})
    ds = dataset_from(c, f)
    model = KgeModel.create(c, ds)
    job = EntityRankingJob(c, ds, model=model)
    job.capture_ranks = True
    names = ("raw", "filt", "filt_test")[:gmeta["rankings"]]
    moved_total = 0
    for e in range(gmeta["epochs"]):
        set_tables(model, g[f"ent_{e}"], g[f"rel_{e}"])
        trace = job.run()
        moved = 0
        for d in "so":
            for r in names:
                mine, ref = job.ranks[f"{d}_{r}"], g[f"{d}_{r}_{e}"]
                assert mine.shape == ref.shape
                moved += int((mine != ref).sum())
                assert np.abs(mine - ref).max() <= 1  # a near-tie moves a rank by one place at most here
        moved_total += moved
        assert moved <= 2, (e, moved)
        for k, v in ref_valids[e].items():
            if k.startswith(("mean_rank", "mean_reciprocal_rank", "hits_at")):
                assert trace[k] == pytest.approx(v, rel=1e-3, abs=2e-3 if k.startswith("hits") else 1e-9), (e, k)
    print(f"\nC1 teacher-forced validation: {moved_total} ranks moved over {gmeta['epochs']} epochs")


def _c2_job(graph, precision="bf16x3"):
    from kge import Dataset
    from kge.job import TrainingJob

    c = base_config("complex", 512, 1, 1, {
        "train.type": "1vsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.2},
        "train.batch_size": 1024, "engine.precision": precision, "engine.graph_step": graph,
        "lookup_embedder.initialize_args": {"mean": 0.0, "std": 0.1}})
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    assert (ds.num_entities(), ds.num_relations()) == (14541, 237)
    torch.manual_seed(0)
    job = TrainingJob.create(c, ds)
    job._prepare()
    return job, ds


def test_c2_1vsall_job_step_fullsize_vs_float64():
    """One TrainingJob1vsAll step of configs[1] at full size -- ComplEx-512, E = 14,541, 1,024
    triples, both directions in one stacked engine pass -- through the job: the loss and the
    gradients of both tables against float64 autograd of the reference formulas (complex.py:19-44,
    train.py:1032-1062, loss.py:198-208), computed with torch in float64."""
    job, ds = _c2_job(graph=False)
    tr = ds.split("train")[torch.randperm(len(ds.split("train")), generator=torch.Generator().manual_seed(5))[:1024]]
    tr = tr.long()
    job.optimizer.zero_grad()
    res = job._process_batch(0, {"triples": tr})
    torch.cuda.synchronize()
    g_ent = job.model._entity_embedder._embeddings.weight.grad.double()
    g_rel = job.model._relation_embedder._embeddings.weight.grad.double()
    ent = job.model._entity_embedder._embeddings.weight.detach().double().requires_grad_()
    rel = job.model._relation_embedder._embeddings.weight.detach().double().requires_grad_()
    t = tr.cuda()
    s, p, o = t[:, 0], t[:, 1], t[:, 2]

    def cmul(a, b, conj_b=False):
        h = a.shape[1] // 2
        ar, ai, br, bi = a[:, :h], a[:, h:], b[:, :h], b[:, h:]
        if conj_b:
            bi = -bi
        return torch.cat([ar * br - ai * bi, ar * bi + ai * br], 1)

    ce = torch.nn.CrossEntropyLoss(reduction="sum")
    loss = (ce(cmul(ent[s], rel[p]) @ ent.t(), o) + ce(cmul(ent[o], rel[p], conj_b=True) @ ent.t(), s)) / 1024
    loss.backward()
    assert float(res.avg_loss) == pytest.approx(float(loss.detach()), rel=1e-5)
    for got, ref, name in ((g_ent, ent.grad, "entity"), (g_rel, rel.grad, "relation")):
        err = float((got - ref).abs().max() / ref.abs().max())
        assert err < 1e-4, (name, err)


def test_c2_1vsall_recorded_step_fullsize_equals_eager():
    """The recorded (HIP graph) configs[1] step at full size against the eager step on the same
    batches: the same kernels in the same order, so the losses and the tables after four steps
    (two eager, one recorded, one replayed) must agree to rounding -- up to the few elements
    (measured 0.01 %) whose nearly cancelling gradient lets Adagrad turn the order of the prep
    backward's atomic adds into a visible step."""
    out = []
    for graph in (False, True):
        job, ds = _c2_job(graph)
        train = ds.split("train")
        perm = torch.randperm(len(train), generator=torch.Generator().manual_seed(6))
        losses = []
        for b in range(4):
            res, _, _ = job.train_step(b, {"triples": train[perm[b * 1024:(b + 1) * 1024]].long()})
            losses.append(float(res.avg_loss))
        if graph:
            assert job._graph_step is not None and job._graph_step.graph is not None, job._graph_step.error
        out.append((losses, *tables(job.model)))
        del job
    (l0, e0, r0), (l1, e1, r1) = out
    np.testing.assert_allclose(l1, l0, rtol=1e-6)
    for a, b in ((e0, e1), (r0, r1)):
        diff = np.abs(a - b)
        assert int((diff > 1e-4).sum()) <= max(4, 1e-3 * diff.size) and float(diff.mean()) < 1e-6
