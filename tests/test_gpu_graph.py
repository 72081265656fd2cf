"""The 1vsAll training step replayed from a recorded HIP graph (engine.graph_step) vs the
eager step: same losses, weights and Adagrad state after warm-up, recording, replays and a
final partial batch; and the golden 3-step trajectory (fixture F4) through train_step,
whose third batch is the recorded one."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _job(graph, precision="fp32", E=700, R=9, dim=64, seed=0, reciprocal=False):
    from kge import Config, Dataset
    from kge.job import TrainingJob

    c = Config()
    if reciprocal:
        c.set("model", "reciprocal_relations_model")
        c._import("reciprocal_relations_model")
        c.set("reciprocal_relations_model.base_model.type", "complex")
    else:
        c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", dim)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", "1vsAll")
    c.set("train.batch_size", 64)
    c.set("engine.precision", precision)
    c.set("engine.graph_step", graph)
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.2})
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    c.set("verbose", False)
    ds = Dataset(c, None)
    g = torch.Generator().manual_seed(seed)
    tr = torch.stack([torch.randint(0, E, (600,), generator=g), torch.randint(0, R, (600,), generator=g),
                      torch.randint(0, E, (600,), generator=g)], 1).int()
    ds._triples = {"train": tr}
    torch.manual_seed(seed)
    job = TrainingJob.create(c, ds)
    job._prepare()
    return job, tr


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_graph_step_matches_eager(precision):
    runs = {}
    for graph in (False, True):
        job, tr = _job(graph, precision)
        losses = []
        for b, lo in enumerate(range(0, 64 * 7 + 30, 64)):  # 7 full batches + one of 30
            res, _, _ = job.train_step(b, {"triples": tr[lo:lo + 64].long()})
            losses.append(float(res.loss))
        if graph:
            assert job._graph_step is not None and job._graph_step.graph is not None, f"graph was not recorded: {job._graph_step.error}"
        else:
            assert job._graph_step is None
        st = job.optimizer.state
        ent = job.model._entity_embedder._embeddings.weight
        rel = job.model._relation_embedder._embeddings.weight
        runs[graph] = (np.array(losses), ent.detach().cpu().numpy(), rel.detach().cpu().numpy(),
                       st[ent]["sum"].cpu().numpy(), int(st[ent]["step"]), int(st[rel]["step"]))
    e, g = runs[False], runs[True]
    # The same kernels in the same order, but split-K and scatter atomics sum in run-dependent
    # order, and Adagrad turns a near-zero gradient's last-bit differences into steps of
    # ~lr (an eager run against an eager run shows the same): the losses -- which would
    # expose a stale or wrongly indexed replay at once -- are held tight, the weights to
    # a few differing elements.
    np.testing.assert_allclose(g[0], e[0], rtol=1e-5)
    for a, b in ((g[1], e[1]), (g[2], e[2])):
        off = np.abs(a - b) > 1e-5
        assert off.mean() < 0.05 and np.abs(a - b).max() < 2e-2, (off.mean(), np.abs(a - b).max())
    np.testing.assert_allclose(g[3], e[3], rtol=1e-2, atol=1e-3 * np.abs(e[3]).max())
    assert g[4] == e[4] == 8 and g[5] == e[5] == 8


def test_graph_step_golden_trajectory():
    """F4 (3 Adagrad steps captured from the reference) through job.train_step: batches 1-2
    eager, batch 3 recorded and replayed."""
    from kge import Config, Dataset
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, "train1vsall_complex.npz"))
    meta = json.loads(str(f["meta"]))
    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", meta["dim"])
    c.set("train.type", "1vsAll")
    c.set("engine.precision", "fp32")
    c.set("train.batch_size", int(f["batches"].shape[1]))
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": meta["lr"]})
    c.set("dataset.num_entities", meta["E"])
    c.set("dataset.num_relations", meta["R"])
    ds = Dataset(c, None)
    ds._triples = {"train": torch.from_numpy(f["batches"].reshape(-1, 3).astype(np.int32))}
    job = TrainingJob.create(c, ds)
    with torch.no_grad():
        job.model._entity_embedder._embeddings.weight.copy_(torch.from_numpy(f["ent0"]))
        job.model._relation_embedder._embeddings.weight.copy_(torch.from_numpy(f["rel0"]))
    job._prepare()
    losses = []
    for b in range(len(f["batches"])):
        res, _, _ = job.train_step(b, {"triples": torch.from_numpy(f["batches"][b]).long()})
        losses.append(float(res.loss))
    assert job._graph_step.graph is not None
    np.testing.assert_allclose(losses, f["losses"], rtol=1e-5)
    e1 = job.model._entity_embedder._embeddings.weight.detach().cpu().numpy()
    r1 = job.model._relation_embedder._embeddings.weight.detach().cpu().numpy()
    np.testing.assert_allclose(e1, f["ent1"], atol=1e-4)
    np.testing.assert_allclose(r1, f["rel1"], atol=1e-4)


def test_graph_step_not_used_when_unsafe():
    """lr_decay != 0 makes the effective learning rate step-dependent: eager steps only."""
    from kge import Config, Dataset
    from kge.job import TrainingJob

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 32)
    c.set("train.type", "1vsAll")
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.2, "lr_decay": 0.01})
    c.set("dataset.num_entities", 100)
    c.set("dataset.num_relations", 5)
    ds = Dataset(c, None)
    ds._triples = {"train": torch.zeros(8, 3, dtype=torch.int32)}
    job = TrainingJob.create(c, ds)
    job._prepare()
    assert job._graph_step is None


def test_graph_step_run_epoch_matches_eager():
    """Two epochs through run_epoch (the job's own loop: pinned one-batch-late loss reads,
    a partial last batch, the recorded step replayed from the third batch on) with and
    without engine.graph_step: same epoch losses."""
    traces = {}
    for graph in (False, True):
        job, _ = _job(graph, "fp32")
        job.generator.manual_seed(0)
        traces[graph] = [job.run_epoch()["avg_loss"] for _ in range(2)]
        if graph:
            assert job._graph_step.graph is not None
    np.testing.assert_allclose(traces[True], traces[False], rtol=1e-5)
    assert traces[True][1] < traces[True][0]


def _kvsall_job(graph, model, E=600, R=7, dim=64, seed=0, batch=64):
    from kge import Config, Dataset
    from kge.job import TrainingJob

    c = Config()
    c.set("model", model)
    c._import(model)
    if model == "reciprocal_relations_model":
        c.set("reciprocal_relations_model.base_model.type", "distmult")
        c._import("distmult")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", dim)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", "KvsAll")
    c.set("KvsAll.label_smoothing", 0.1)
    c.set("train.batch_size", batch)
    c.set("engine.graph_step", graph)
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.2})
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    c.set("verbose", False)
    ds = Dataset(c, None)
    g = torch.Generator().manual_seed(seed)
    # few distinct (s, p) / (p, o) keys: label lists of very different lengths
    tr = torch.stack([torch.randint(0, 40, (900,), generator=g), torch.randint(0, R, (900,), generator=g),
                      torch.randint(0, E, (900,), generator=g)], 1).int()
    ds._triples = {"train": tr}
    torch.manual_seed(seed)
    job = TrainingJob.create(c, ds)
    job._prepare()
    return job


@pytest.mark.parametrize("model", ["distmult", "complex", "reciprocal_relations_model"])
def test_kvsall_graph_step_matches_eager(model):
    """The KvsAll step recorded as a HIP graph -- stacked (s, p, ?) / (?, p, o) query rows whose
    split point and label CSR differ from batch to batch and are read from the recorded device
    block -- against the eager step on the same batches: losses per batch (the last query type's,
    as the reference reports), tables and Adagrad state; batches with only one query type, a
    partial batch and the batches after it included."""
    runs = {}
    for graph in (False, True):
        job = _kvsall_job(graph, model)
        n = job.num_examples
        perm = torch.randperm(n, generator=torch.Generator().manual_seed(3))
        n_first = job.query_last_example[0]
        batches = [perm[b:b + 64] for b in range(0, 64 * 6, 64)]
        batches.append(torch.arange(0, 64))                    # only the first query type
        batches.append(torch.arange(n - 64, n))                # only the second
        batches.append(perm[64 * 6:64 * 6 + 30])               # partial: eager
        batches.append(perm[64 * 7:64 * 8])                    # replayed again afterwards
        assert n_first > 64 and n - n_first > 64
        losses = []
        for b, ids in enumerate(batches):
            res, _, _ = job.train_step(b, job._collate(ids))
            losses.append(float(res.loss))
        if graph:
            assert job._graph_step is not None and job._graph_step.graph is not None, (
                f"graph was not recorded: {job._graph_step.error}")
        else:
            assert job._graph_step is None
        st = job.optimizer.state
        ent = job.model.get_s_embedder()._embeddings.weight
        rel = job.model.get_p_embedder()._embeddings.weight
        runs[graph] = (np.array(losses), ent.detach().cpu().numpy(), rel.detach().cpu().numpy(),
                       st[ent]["sum"].cpu().numpy(), int(st[ent]["step"]), int(st[rel]["step"]))
    e, g = runs[False], runs[True]
    np.testing.assert_allclose(g[0], e[0], rtol=2e-5, atol=1e-7)
    for a, b in ((g[1], e[1]), (g[2], e[2])):
        off = np.abs(a - b) > 1e-5
        assert off.mean() < 0.05 and np.abs(a - b).max() < 2e-2, (off.mean(), np.abs(a - b).max())
    np.testing.assert_allclose(g[3], e[3], rtol=1e-2, atol=1e-3 * np.abs(e[3]).max())
    assert g[4] == e[4] == len(batches) and g[5] == e[5] == len(batches)


@pytest.mark.parametrize("model", ["distmult", "complex"])
def test_kvsall_graph_step_with_dropout_one_recording_per_split_matches_eager(model):
    """KvsAll with dropout in the embedders: the query types are scored one after the other, each
    against its own dropped copy of the entity table, so the step is recorded once PER SPLIT POINT
    of the batch (train.py's _KvsAllSplitGraphStep; all recordings share one buffer and one memory
    pool).  Against the eager job from the same seed: torch's dropout draws the same masks in both
    (same calls, same shapes), so losses, tables and optimizer state must agree step after step --
    over 40 steps that record a dozen splits and replay each several times, in any order."""
    runs = {}
    for graph in (False, True):
        job = _kvsall_job(graph, model, batch=32)
        for e in (job.model.get_s_embedder(), job.model.get_p_embedder()):
            e.dropout.p = 0.3
        job._prepare()  # decides on the graph step with the dropout in place
        n = job.num_examples
        torch.manual_seed(11)
        g = torch.Generator().manual_seed(3)
        batches = [torch.randperm(n, generator=g)[:32] for _ in range(40)]
        batches.insert(7, torch.randperm(n, generator=g)[:20])  # a partial batch: eager
        losses, splits = [], []
        for b, ids in enumerate(batches):
            splits.append(int((ids < job.query_last_example[0]).sum()) if len(ids) == 32 else -1)
            res, _, _ = job.train_step(b, job._collate(ids))
            losses.append(float(res.loss))
        if graph:
            gs = job._graph_step
            assert gs is not None and gs.graphs, f"not recorded: {None if gs is None else gs.error}"
            recorded = set(splits[2:]) - {-1}  # (two eager warm-up steps)
            assert set(gs.graphs) == recorded and len(recorded) < len(splits) - 12  # splits were replayed
        else:
            assert job._graph_step is None
        st = job.optimizer.state
        ent = job.model.get_s_embedder()._embeddings.weight
        rel = job.model.get_p_embedder()._embeddings.weight
        runs[graph] = (np.array(losses), ent.detach().cpu().numpy(), rel.detach().cpu().numpy(),
                       st[ent]["sum"].cpu().numpy(), int(st[ent]["step"]))
    e, g = runs[False], runs[True]
    np.testing.assert_allclose(g[0], e[0], rtol=1e-4, atol=1e-7)
    for a, b in ((g[1], e[1]), (g[2], e[2])):  # (a different mask anywhere would move rows by O(0.1))
        assert np.abs(a - b).max() <= 1e-3 * np.abs(b).max() and np.abs(a - b).mean() <= 1e-5 * np.abs(b).max()
    np.testing.assert_allclose(g[3], e[3], rtol=1e-2, atol=1e-4 * np.abs(e[3]).max())
    assert g[4] == e[4] == len(batches)


def test_kvsall_graph_step_falls_back_when_labels_exceed_capacity():
    """A batch whose positives do not fit the recorded label buffer runs eagerly (same result)."""
    job = _kvsall_job(True, "distmult")
    job._graph_step.cap = 16  # far below any batch's label count
    for b in range(4):
        job.train_step(b, job._collate(torch.arange(b * 64, b * 64 + 64)))
    assert job._graph_step.graph is None and not job._graph_step.disabled


@pytest.mark.parametrize("train_type", ["1vsAll", "KvsAll"])
def test_job_loop_memorises_its_training_triples(train_type):
    """End to end through TrainingJob.run() with the default engine options (recorded graph
    step, fused loss and optimizer, refined bf16x3 evaluation, validation every few epochs):
    validation triples that are training triples must reach a filtered MRR near 1 -- the
    evaluation reads the tables the replayed steps update."""
    from kge import Config, Dataset
    from kge.job import TrainingJob

    E, R = 400, 6
    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 64)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", train_type)
    c.set("train.batch_size", 128)
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.5})
    c.set("train.max_epochs", 40)
    c.set("valid.every", 20)
    c.set("eval.batch_size", 100)
    c.set("engine.eval_batch_size", 0)  # the batches of eval.batch_size as they are
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    c.set("verbose", False)
    g = torch.Generator().manual_seed(11)
    tr = torch.stack([torch.randint(0, E, (1500,), generator=g), torch.randint(0, R, (1500,), generator=g),
                      torch.randint(0, E, (1500,), generator=g)], 1).int()
    ds = Dataset(c, None)
    ds._triples = {"train": tr, "valid": tr[:250].clone(), "test": tr[250:300].clone()}
    torch.manual_seed(0)
    job = TrainingJob.create(c, ds)
    traces = job.run()
    assert job._graph_step is not None and job._graph_step.graph is not None, job._graph_step.error
    assert traces[-1]["avg_loss"] < 0.5 * traces[0]["avg_loss"]
    assert len(job.valid_trace) == 2
    assert job.valid_trace[-1]["mean_reciprocal_rank_filtered"] > 0.9, job.valid_trace[-1]
    assert job.valid_trace[-1]["hits_at_1_filtered"] > 0.85


def test_kvsall_graph_step_not_used_when_the_plane_path_does_not_apply():
    """dim 50 rows cannot feed the plane-fed kernels: no graph step is set up and every batch runs
    eagerly, with the same losses as a job with engine.graph_step off."""
    losses = {}
    for graph in (True, False):
        job = _kvsall_job(graph, "distmult", dim=50)
        out = []
        for b in range(5):
            res, _, _ = job.train_step(b, job._collate(torch.arange(b * 64, b * 64 + 64)))
            out.append(float(res.loss))
        losses[graph] = out
        assert job._graph_step is None
    np.testing.assert_allclose(losses[True], losses[False], rtol=2e-5)


@pytest.mark.parametrize("graph", [True, False], ids=["graph_step", "eager"])
@pytest.mark.parametrize("tag", ["1vsall_w", "1vsall_u", "kvsall_w"])
def test_penalty_trajectories_vs_reference(tag, graph):
    """Three batch steps WITH embedding penalties (weighted L3 on entities, weighted L2 on
    relations; unweighted for 1vsall_u) captured from the reference's batch loop
    (train.py:309-429, lookup_embedder.py:112-158): losses, the penalty sum of every batch and
    the tables after the steps.  With engine.graph_step the third 1vsAll batch is the recorded
    one (weighted terms in their per-occurrence form); KvsAll with weighted terms steps eagerly
    (its triples vary in number) and builds them per batch like the reference collate."""
    from kge import Config, Dataset
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, "train_penalties.npz"))
    meta = json.loads(str(f["meta"]))
    case = meta["cases"][tag]
    c = Config()
    c.set("model", case["model"])
    c._import(case["model"])
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", meta["dim"])
    c.set("train.type", case["train_type"])
    c.set("engine.precision", "fp32")
    c.set("engine.graph_step", graph)
    c.set("train.batch_size", case["batch_size"])
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": meta["lr"]})
    c.set("dataset.num_entities", meta["E"])
    c.set("dataset.num_relations", meta["R"])
    c.set("verbose", False)
    for k, v in case["extra"].items():
        c.set(k, v)
    ds = Dataset(c, None)
    ds._triples = {"train": torch.from_numpy(f["tri_train"].astype(np.int32))}
    job = TrainingJob.create(c, ds)
    with torch.no_grad():
        job.model._entity_embedder._embeddings.weight.copy_(torch.from_numpy(f[tag + "_ent0"]))
        job.model._relation_embedder._embeddings.weight.copy_(torch.from_numpy(f[tag + "_rel0"]))
    job._prepare()
    losses, pens = [], []
    for b in range(meta["num_batches"]):
        if case["train_type"] == "1vsAll":
            batch = {"triples": torch.from_numpy(f[tag + "_batches"][b]).long()}
        else:
            batch = job._collate(torch.from_numpy(f[tag + "_examples"][b]))
        res, pen, _ = job.train_step(b, batch)
        losses.append(float(res.loss))
        pens.append(float(pen))
    recorded = job._graph_step is not None and job._graph_step.graph is not None
    assert recorded == (graph and case["train_type"] == "1vsAll"), getattr(job._graph_step, "error", None)
    np.testing.assert_allclose(losses, f[tag + "_losses"], rtol=1e-5)
    np.testing.assert_allclose(pens, f[tag + "_penalties"].sum(1), rtol=1e-5)
    e1 = job.model._entity_embedder._embeddings.weight.detach().cpu().numpy()
    r1 = job.model._relation_embedder._embeddings.weight.detach().cpu().numpy()
    # Adagrad's first steps are lr * g / |g|-like: where a gradient element is at rounding level its
    # last bits decide a visible step, so a handful of elements may differ (the allowance of the
    # eager-vs-graph comparison above); everything else is held to 1e-4
    for got, ref in ((e1, f[tag + "_ent1"]), (r1, f[tag + "_rel1"])):
        off = np.abs(got - ref) > 1e-4
        assert off.mean() < 1e-3 and np.abs(got - ref).max() < 2e-3, (off.sum(), np.abs(got - ref).max())


def test_graph_step_recorded_anew_when_the_learning_rate_changes():
    """The learning rate is an argument of the recorded optimizer kernel: after a scheduler
    changes it the next batch is recorded anew, and the run follows the eager one."""
    runs = {}
    for graph in (False, True):
        job, tr = _job(graph, "fp32")
        losses, recordings = [], []
        for b in range(9):
            if b == 5:
                for group in job.optimizer.param_groups:
                    group["lr"] = 0.02
            res, _, _ = job.train_step(b, {"triples": tr[b * 64:(b + 1) * 64].long()})
            losses.append(float(res.loss))
            if graph:
                recordings.append(job._graph_step.graph)
        if graph:
            assert recordings[1] is None and recordings[2] is not None
            assert recordings[4] is recordings[2] and recordings[5] is not recordings[4]
            assert recordings[8] is recordings[5]
            assert job._graph_step.hyper[0][0] == 0.02
        ent = job.model._entity_embedder._embeddings.weight
        runs[graph] = (np.array(losses), ent.detach().cpu().numpy())
    np.testing.assert_allclose(runs[True][0], runs[False][0], rtol=1e-5)
    off = np.abs(runs[True][1] - runs[False][1]) > 1e-5
    assert off.mean() < 0.05 and np.abs(runs[True][1] - runs[False][1]).max() < 2e-2


def test_graph_step_with_adam_matches_eager():
    """train.optimizer Adam: the step counters live on the device (capturable), so the step is
    recorded and replayed like the Adagrad one and follows the eager run."""
    from kge.util.optimizer import CapturableAdam

    runs = {}
    for graph in (False, True):
        from kge import Config, Dataset
        from kge.job import TrainingJob

        c = Config()
        c.set("model", "complex")
        c._import("complex")
        c.set("job.device", "cuda")
        c.set("lookup_embedder.dim", 64)
        c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
        c.set("train.type", "1vsAll")
        c.set("train.batch_size", 64)
        c.set("engine.precision", "fp32")
        c.set("engine.graph_step", graph)
        c.set("train.optimizer", "Adam")
        c.set("train.optimizer_args", {"lr": 0.01})
        c.set("dataset.num_entities", 700)
        c.set("dataset.num_relations", 9)
        c.set("verbose", False)
        ds = Dataset(c, None)
        g = torch.Generator().manual_seed(0)
        tr = torch.stack([torch.randint(0, 700, (600,), generator=g), torch.randint(0, 9, (600,), generator=g),
                          torch.randint(0, 700, (600,), generator=g)], 1).int()
        ds._triples = {"train": tr}
        torch.manual_seed(0)
        job = TrainingJob.create(c, ds)
        job._prepare()
        assert isinstance(job.optimizer, CapturableAdam) == graph
        losses = []
        for b in range(8):
            res, _, _ = job.train_step(b, {"triples": tr[b * 64:(b + 1) * 64].long()})
            losses.append(float(res.loss))
        if graph:
            assert job._graph_step is not None and job._graph_step.graph is not None, job._graph_step.error
            ent = job.model._entity_embedder._embeddings.weight
            assert int(job.optimizer.state[ent]["step"]) == 8
        else:
            assert job._graph_step is None
        runs[graph] = (np.array(losses), job.model._entity_embedder._embeddings.weight.detach().cpu().numpy())
    np.testing.assert_allclose(runs[True][0], runs[False][0], rtol=1e-5)
    # Adam's step is ~lr * sign(g) while the second moment is young: rounding-level gradient
    # elements may step the other way (as with Adagrad above)
    off = np.abs(runs[True][1] - runs[False][1]) > 1e-5
    assert off.mean() < 0.05 and np.abs(runs[True][1] - runs[False][1]).max() < 0.2


@pytest.mark.parametrize("reciprocal", [False, True])
@pytest.mark.parametrize("precision", ["bf16x3", "fp32"])
@pytest.mark.parametrize("direction", ["sp_", "_po"])
def test_fused_loss_with_embedder_dropout_matches_unfused(direction, precision, reciprocal):
    """lookup_embedder.dropout > 0 in training mode: score_sp_xent / score_po_xent score dropped
    query rows against a dropped copy of the table in one engine pass.  Under the same seed the
    unfused path (score_sp / score_po, torch cross entropy) draws the same masks: same loss, same
    gradients.  The reciprocal-relations model draws its (?, p, o) rows in its own order
    (reciprocal_relations_model.py:67-74)."""
    job, tr = _job(False, precision, reciprocal=reciprocal)
    m = job.model
    for e in (m._entity_embedder, m._relation_embedder):
        e.dropout.p = 0.3
    m.train()
    assert m._lookup_tables() is None and m._lookup_embedders_with_dropout()
    t = tr[:64].long().cuda()
    s, p, o = t[:, 0], t[:, 1], t[:, 2]
    ent, rel = m._entity_embedder._embeddings.weight, m._relation_embedder._embeddings.weight
    out = {}
    for fused in (True, False):
        ent.grad = rel.grad = None
        torch.manual_seed(5)
        if fused:
            loss = m.score_sp_xent(s, p, o, 1.0 / 64) if direction == "sp_" else m.score_po_xent(p, o, s, 1.0 / 64)
        else:
            scores = m.score_sp(s, p) if direction == "sp_" else m.score_po(p, o)
            loss = torch.nn.functional.cross_entropy(scores, o if direction == "sp_" else s, reduction="sum") / 64
        loss.backward()
        out[fused] = (float(loss.detach()), ent.grad.detach().clone(), rel.grad.detach().clone())
    tol = 2e-5 if precision == "fp32" else 2e-4
    assert out[True][0] == pytest.approx(out[False][0], rel=1e-5)
    for a, b in zip(out[True][1:], out[False][1:]):
        assert (a - b).abs().max().item() <= tol * b.abs().max().item()
    # the masks are redrawn per call
    torch.manual_seed(5)
    first = float(m.score_sp_xent(s, p, o, 1.0 / 64).detach())
    assert float(m.score_sp_xent(s, p, o, 1.0 / 64).detach()) != first


@pytest.mark.parametrize("reciprocal", [False, True])
def test_graph_step_with_embedder_dropout_records_and_redraws_masks(reciprocal):
    """Dropout in the lookup embedders keeps the step on the recorded path: torch's dropout is
    part of the recording and every replay draws new masks (replaying one batch twice gives two
    different losses); the loss falls over the run like the eager job's."""
    runs = {}
    for graph in (True, False):
        job, tr = _job(graph, "bf16x3", reciprocal=reciprocal)
        for e in (job.model._entity_embedder, job.model._relation_embedder):
            e.dropout.p = 0.2
        job._prepare()  # decides on the graph step with the dropout in place
        torch.manual_seed(1)
        losses = []
        for rep in range(5):
            for b in range(8):
                res, _, _ = job.train_step(b, {"triples": tr[b * 64:(b + 1) * 64].long()})
                losses.append(float(res.loss))
        recorded = job._graph_step is not None and job._graph_step.graph is not None
        assert recorded == graph, getattr(job._graph_step, "error", None)
        runs[graph] = np.array(losses)
        if graph:
            a = float(job.train_step(0, {"triples": tr[:64].long()})[0].loss)
            b = float(job.train_step(0, {"triples": tr[:64].long()})[0].loss)
            assert a != b
    for losses in runs.values():
        assert np.isfinite(losses).all() and losses[-8:].mean() < 0.8 * losses[:8].mean()
    assert runs[True][-8:].mean() == pytest.approx(runs[False][-8:].mean(), rel=0.25)


def test_graph_step_penalties_follow_eager_over_many_steps():
    """Frequency-weighted Lp penalties inside the recorded step (engine kernels over the
    occurrences of the batch's indexes, added into the held gradient) against the eager step's
    unique-index form: the same penalty and loss at every one of 12 steps, i.e. also on the
    replays after the recording, and after an lr change records the step anew."""
    runs = {}
    for graph in (True, False):
        job, tr = _job(graph, "fp32")
        for e, w, p in ((job.model._entity_embedder, 1e-2, 3), (job.model._relation_embedder, 5e-3, 2)):
            e.config.set(e.configuration_key + ".regularize_weight", w)
            e.config.set("lookup_embedder.regularize_args.weighted", True)
            e.config.set(e.configuration_key + ".regularize_args.p", p)
        job._prepare()
        assert job.model._entity_embedder.penalty_weighted()
        pens, losses = [], []
        for b in range(12):
            if b == 8:
                for group in job.optimizer.param_groups:
                    group["lr"] = 0.05
            res, pen, _ = job.train_step(b % 9, {"triples": tr[(b % 9) * 64:(b % 9 + 1) * 64].long()})
            pens.append(float(pen))
            losses.append(float(res.loss))
        recorded = job._graph_step is not None and job._graph_step.graph is not None
        assert recorded == graph, getattr(job._graph_step, "error", None)
        runs[graph] = (np.array(pens), np.array(losses))
    assert (runs[False][0] > 0).all()
    np.testing.assert_allclose(runs[True][0], runs[False][0], rtol=2e-5)
    np.testing.assert_allclose(runs[True][1], runs[False][1], rtol=2e-5)


def test_kvsall_graph_step_with_unweighted_penalty_matches_eager():
    """KvsAll records its step with UNWEIGHTED Lp penalties (whole-table norms: nothing
    batch-dependent) and follows the eager step; with frequency-weighted terms it steps eagerly
    (their triples vary in number) and its batches carry those triples."""
    runs = {}
    for graph in (True, False):
        job = _kvsall_job(graph, "distmult")
        for e, w in ((job.model._entity_embedder, 1e-3), (job.model._relation_embedder, 5e-4)):
            e.config.set(e.configuration_key + ".regularize_weight", w)
        job._prepare()
        assert (job._graph_step is not None) == graph
        perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(3))
        pens, losses = [], []
        for b in range(8):
            res, pen, _ = job.train_step(b, job._collate(perm[b * 64:(b + 1) * 64]))
            pens.append(float(pen))
            losses.append(float(res.loss))
        if graph:
            assert job._graph_step.graph is not None, job._graph_step.error
        runs[graph] = (np.array(pens), np.array(losses))
    assert (runs[False][0] > 0).all()
    np.testing.assert_allclose(runs[True][0], runs[False][0], rtol=2e-5)
    np.testing.assert_allclose(runs[True][1], runs[False][1], rtol=2e-5)
    job = _kvsall_job(True, "distmult")
    job.config.set("lookup_embedder.regularize_args.weighted", True)
    job.config.set("distmult.entity_embedder.regularize_weight", 1e-3)
    job._prepare()
    assert job._graph_step is None and job._weighted_penalty()
    batch = job._collate(torch.arange(64))
    assert batch["triples"].shape[1] == 3
    res, pen, _ = job.train_step(0, batch)
    assert float(pen) > 0


@pytest.mark.parametrize("model_name,per,extra", [
    ("complex", True, {}), ("distmult", False, {}), ("transe", False, {}),
    # entity chunks (counts accumulated over three chunks, histograms in a launch of their own)
    ("complex", False, {"entity_ranking.chunk_size": 600}),
    # a reciprocal-relations model: both directions' true scores, (?, p, o) as (o, p + R, ?)
    ("reciprocal", False, {"entity_ranking.filter_with_test": False}),
    ("complex", False, {"engine.eval_precision": "fp32", "engine.eval_streams": 1}),
])
def test_recorded_evaluation_pass_equals_eager_on_every_replay(model_name, per, extra):
    """engine.graph_eval: the job's first run is eager, its second records the device work of the
    run (all batches, both streams) and replays it, later runs only replay.  Every run must give
    the ranks and metrics of an eager job on the same weights -- also after the tables were
    updated in place between runs (a replay reads the weights as they are then), with eager
    device work and synchronisations between the replays."""
    from kge import Config, Dataset, KgeModel
    from kge.job import EntityRankingJob

    def config(graph):
        c = Config()
        if model_name == "reciprocal":
            c.set("model", "reciprocal_relations_model")
            c._import("reciprocal_relations_model")
            c.set("reciprocal_relations_model.base_model.type", "complex")
            c._import("complex")
        else:
            c.set("model", model_name)
            c._import(model_name)
        c.set("job.device", "cuda")
        c.set("lookup_embedder.dim", 128)
        c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
        c.set("eval.split", "valid")
        c.set("eval.batch_size", 256)
        c.set("engine.eval_batch_size", 0)  # five batches, the last one partial
        c.set("engine.graph_eval", graph)
        for k, v in extra.items():
            c.set(k, v)
        c.set("entity_ranking.metrics_per.head_and_tail", per)
        c.set("entity_ranking.metrics_per.relation_type", per)
        c.set("verbose", False)
        return c

    c = config(True)
    ds = Dataset.synthetic(c, "toy", seed=0, num_entities=1500, num_relations=7, sizes=(12000, 1100, 300))
    torch.manual_seed(0)
    model = KgeModel.create(c, ds)
    model.eval()
    job = EntityRankingJob(c, ds, model=model)
    job.capture_ranks = True
    eager = EntityRankingJob(config(False), ds, model=model)
    eager.capture_ranks = True
    g = torch.Generator(device="cuda").manual_seed(3)
    ent, rel = (t for t in model._lookup_tables())
    states = []
    for run in range(5):
        if run in (2, 4):  # the tables change in place, as an optimizer step changes them
            with torch.no_grad():
                ent.add_(torch.randn(ent.shape, device="cuda", generator=g) * 0.05)
                rel.add_(torch.randn(rel.shape, device="cuda", generator=g) * 0.05)
        got = job.run()
        got_ranks = {k: v.copy() for k, v in job.ranks.items()}
        states.append("graph" in job._graph_state)
        torch.cuda.synchronize()
        want = eager.run()  # eager device work between the replays
        assert "graph" not in eager._graph_state
        for k, v in eager.ranks.items():
            np.testing.assert_array_equal(got_ranks[k], v, err_msg=f"run {run} {k}")
        for k, v in want.items():
            if k != "epoch_time" and isinstance(v, float):
                assert got[k] == v, (run, k)
    assert states == [False, True, True, True, True], job._graph_state.get("error")
    # a job that now has to capture other ranks starts over: eager, then recorded again
    job.capture_ranks = False
    job.run()
    assert "graph" not in job._graph_state
    job.run()
    assert "graph" in job._graph_state


def test_evaluation_that_cannot_be_recorded_runs_eagerly():
    """A device pass that raises while it is being recorded (here: a hook that refuses to run under
    stream capture) switches engine.graph_eval off for the job: the same run and every later one
    evaluate eagerly, with the eager job's metrics."""
    from kge import Config, Dataset, KgeModel
    from kge.job import EntityRankingJob

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 64)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("eval.split", "valid")
    c.set("eval.batch_size", 128)
    c.set("verbose", False)
    ds = Dataset.synthetic(c, "toy", seed=1, num_entities=700, num_relations=5, sizes=(6000, 500, 100))
    torch.manual_seed(0)
    model = KgeModel.create(c, ds)
    model.eval()
    job = EntityRankingJob(c, ds, model=model)
    first = job.run()
    inner = job._rank_batches

    def refuses_capture(*a, **k):
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("not under capture")
        return inner(*a, **k)

    job._rank_batches = refuses_capture
    for _ in range(3):
        again = job.run()
        assert job._graph_state.get("disabled") and "not under capture" in job._graph_state["error"]
        for k, v in first.items():
            if k != "epoch_time" and isinstance(v, float):
                assert again[k] == v, k
