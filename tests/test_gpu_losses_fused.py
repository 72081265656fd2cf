"""GPU parity of the losses other than kl that the engine fuses: bce on the all-entities score
block (kge_bce_planes: KvsAll with label smoothing, 1vsAll index labels) and margin_ranking / bce
on negative-sampling blocks (kge_ns_loss) -- the kernels against torch's float64 losses, the jobs
against reference-captured trajectories (tests/golden/make_golden.py: kvsall_bce, onevsall_bce,
ns_complex_margin, ns_rotate_bce)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from test_gpu_configs import _example_ids, base_config, dataset_from, set_tables, tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib
    _lib.lib()
    return _lib


@pytest.mark.parametrize("n,m,smoothing,offset,csr", [
    (37, 1001, 0.1, 0.5, True), (16, 14541, 0.0, 0.0, True), (64, 40943, 0.1, -2.0, True), (50, 700, 0.0, 1.5, False)])
def test_bce_planes_vs_torch_float64(L, n, m, smoothing, offset, csr):
    """loss_i = sum_j BCEWithLogits(s_ij + offset, y_ij) and G = scale (sigmoid - y) as bf16 hi / lo
    planes (hi + lo = G to 2^-16), y the smoothed label rows of train.py:715-721 or one-hot rows."""
    rng = np.random.default_rng(n + m)
    sc = (rng.standard_normal((n, m)) * 6).astype(np.float32)
    sc[0, :5] = [90.0, -90.0, 0.0, 30.0, -30.0]  # softplus / sigmoid at the extremes
    if csr:
        lens = rng.integers(0, 6, size=n)
        lens[1] = 0
        ptr = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=ptr[1:])
        col = np.concatenate([rng.choice(m, size=k, replace=False) for k in lens] + [np.zeros(0, np.int64)]).astype(np.int64)
    else:
        ptr, col = None, rng.integers(0, m, size=n).astype(np.int64)
    y = np.zeros((n, m))
    for i in range(n):
        y[i, (col[ptr[i]:ptr[i + 1]] if csr else col[i:i + 1])] = 1.0
    if smoothing > 0:
        y = (1.0 - smoothing) * y + 1.0 / m
    x = torch.from_numpy(sc).double() + offset
    yt = torch.from_numpy(y)
    ref_loss = torch.nn.functional.binary_cross_entropy_with_logits(x, yt, reduction="none").sum(1).numpy()
    scale = 1.0 / n
    ref_g = (scale * (torch.sigmoid(x) - yt)).numpy()
    n_pad, ld = L.planes_layout(n, m)
    buf = torch.zeros(n_pad, ld, device="cuda")
    buf[:n, :m] = torch.from_numpy(sc).cuda()
    lab = torch.from_numpy(col).cuda()
    loss, gp = L.softmax_planes(buf, n, m, lab, torch.from_numpy(ptr).cuda() if csr else None, smoothing, scale,
                                loss_kind="bce", offset=offset)
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss.cpu().numpy(), ref_loss, rtol=2e-6 * np.sqrt(m) / 10 + 2e-6)
    g = (gp.hi[:n, :m].float() + gp.lo[:n, :m].float()).cpu().numpy()
    assert np.abs(g - ref_g).max() <= 3e-5 * np.abs(ref_g).max()
    # K padding: columns past m and rows past n are zero in both planes
    for pad in (gp.hi[:, m:], gp.lo[:, m:], gp.hi[n:], gp.lo[n:]):
        assert pad.numel() == 0 or float(pad.float().abs().max()) == 0.0


@pytest.mark.parametrize("n,m,c0,offset,strided", [
    (37, 130, 0, 0.0, False), (64, 257, 1000, -2.0, True), (5, 31, 7, 1.5, False), (130, 5000, 20000, 0.5, True),
    (1, 4, 0, 0.0, False)])
def test_bce_grad_planes_of_a_row_shard_vs_torch_float64(L, n, m, c0, offset, strided):
    """kge_bce_grad_planes: one shard's columns [c0, c0 + m) of the 1vsAll bce loss.  Labels that
    fall outside the shard contribute no hot column there; the block's loss sum and G = scale
    (sigmoid(s + offset) - y) (hi + lo planes) equal torch's float64; scores stay untouched."""
    rng = np.random.default_rng(n * 7 + m)
    sc = (rng.standard_normal((n, m)) * 6).astype(np.float32)
    sc[0, :4] = [90.0, -90.0, 0.0, 30.0]
    labels = rng.integers(max(c0 - m, 0), c0 + 2 * m, size=n).astype(np.int64)  # about a third inside
    labels[0] = c0  # first column, at the extreme score
    if n > 2:
        labels[1], labels[2] = c0 + m - 1, c0 + m  # last column / first one past the shard
    y = np.zeros((n, m))
    inside = (labels >= c0) & (labels < c0 + m)
    y[np.nonzero(inside)[0], labels[inside] - c0] = 1.0
    x = torch.from_numpy(sc).double() + offset
    yt = torch.from_numpy(y)
    ref_loss = float(torch.nn.functional.binary_cross_entropy_with_logits(x, yt, reduction="sum"))
    scale = 1.0 / 4096
    ref_g = (scale * (torch.sigmoid(x) - yt)).numpy()
    if strided:  # a column window of a wider score buffer (row stride != m)
        wide = torch.full((n, m + 24), 7.0, device="cuda")
        wide[:, 8:8 + m] = torch.from_numpy(sc).cuda()
        s = wide[:, 8:8 + m]
    else:
        s = torch.from_numpy(sc).cuda()
    before = s.clone()
    loss, gp = L.bce_grad_planes(s, c0, torch.from_numpy(labels).cuda(), offset, scale)
    torch.cuda.synchronize()
    assert loss.dtype == torch.float64 and loss.dim() == 0
    assert abs(float(loss) - ref_loss) <= 3e-6 * abs(ref_loss)
    assert torch.equal(s, before)
    g = (gp.hi[:n, :m].float() + gp.lo[:n, :m].float()).cpu().numpy()
    assert np.abs(g - ref_g).max() <= 3e-5 * np.abs(ref_g).max()
    for pad in (gp.hi[:, m:], gp.lo[:, m:], gp.hi[n:], gp.lo[n:]):
        assert pad.numel() == 0 or float(pad.float().abs().max()) == 0.0


@pytest.mark.parametrize("kind,arg", [("margin_ranking", 1.0), ("margin_ranking", 0.25), ("bce", 0.0), ("bce", -3.0)])
@pytest.mark.parametrize("n,k", [(64, 9), (512, 1025), (3, 1)])
def test_ns_loss_vs_torch_float64(L, kind, arg, n, k):
    from kge import engine

    rng = np.random.default_rng(n * k)
    sc = (rng.standard_normal((n, k)) * 2).astype(np.float32)
    if k > 2 and kind == "margin_ranking":
        # a pair exactly at the margin, in dyadic values (exact in fp32 and float64 alike): torch's
        # clamp passes the gradient there
        sc[0, 0], sc[0, 1] = 1.5, 1.5 - arg
    s = torch.from_numpy(sc).cuda().requires_grad_()
    scale = 1.0 / n
    loss = engine.ns_loss_column0(s, kind, arg, scale)
    loss.backward()
    x = torch.from_numpy(sc).double().requires_grad_()
    if kind == "margin_ranking":
        pos = x[:, :1].expand(n, k - 1).reshape(-1)
        ref = torch.nn.functional.margin_ranking_loss(pos, x[:, 1:].reshape(-1), torch.ones(n * (k - 1), dtype=torch.float64),
                                                      margin=arg, reduction="sum") * scale
    else:
        y = torch.zeros(n, k, dtype=torch.float64)
        y[:, 0] = 1.0
        ref = torch.nn.functional.binary_cross_entropy_with_logits(x + arg, y, reduction="sum") * scale
    ref.backward()
    assert float(loss.detach()) == pytest.approx(float(ref.detach()), rel=2e-6, abs=1e-7)
    np.testing.assert_allclose(s.grad.cpu().numpy(), x.grad.numpy(), rtol=4e-6, atol=1e-9)


@pytest.mark.parametrize("fused", [True, False], ids=["fused_bce", "torch_bce"])
@pytest.mark.parametrize("precision,atol", [("fp32", 1e-4), ("bf16x3", 2e-4)])
def test_kvsall_bce_trajectory_vs_reference(precision, atol, fused):
    """Three reference KvsAll batches with train.loss bce (offset 0.5, label smoothing 0.1: smoothed,
    not normalised label rows; loss.py:137-158, train.py:715-751): per-batch loss and gradients
    teacher-forced from the reference's tables, then the free-running tables."""
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, "train_kvsall_bce_distmult.npz"))
    meta = json.loads(str(f["meta"]))
    c = base_config("distmult", meta["dim"], meta["E"], meta["R"], {
        "train.type": "KvsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": meta["lr"]},
        "train.loss": "bce", "train.loss_arg": meta["loss_arg"],
        "train.batch_size": meta["batch_size"], "KvsAll.label_smoothing": meta["label_smoothing"],
        "engine.precision": precision, "engine.fused_loss": fused})
    ds = dataset_from(c, f)
    job = TrainingJob.create(c, ds)
    set_tables(job.model, f["ent0"], f["rel0"])
    job._prepare()
    assert (job._fused_loss_kind() == ("bce", 0.5)) == fused
    ent_w = job.model._entity_embedder._embeddings.weight
    rel_w = job.model._relation_embedder._embeddings.weight
    gtol = 5e-6 if precision == "fp32" else 1e-4
    batches = []
    for b in range(meta["num_batches"]):
        ids = _example_ids(job, f[f"queries_{b}"], f[f"qtype_{b}"])
        batches.append(ids)
        set_tables(job.model, f[f"ent_before_{b}"], f[f"rel_before_{b}"])
        job.optimizer.zero_grad()
        res = job.process_batch(b, {"examples": ids})
        assert float(res.avg_loss) == pytest.approx(float(f["losses"][b]), rel=2e-5)
        for w, key in ((ent_w, f"g_ent_{b}"), (rel_w, f"g_rel_{b}")):
            err = np.abs(w.grad.cpu().numpy() - f[key]).max() / np.abs(f[key]).max()
            assert err < gtol, (b, key, err)
    set_tables(job.model, f["ent0"], f["rel0"])
    job.optimizer = type(job.optimizer)(job.optimizer.param_groups[0]["params"], lr=meta["lr"])
    losses = []
    for b, ids in enumerate(batches):
        job.optimizer.zero_grad()
        res = job.process_batch(b, {"examples": ids})
        job.optimizer.step()
        losses.append(res.avg_loss)
    np.testing.assert_allclose(losses, f["losses"], rtol=2e-5)
    for got, want in zip(tables(job.model), (f["ent1"], f["rel1"])):
        diff = np.abs(got - want)
        assert int((diff > atol).sum()) <= max(4, 1e-3 * diff.size) and float(diff.mean()) < 1e-5


@pytest.mark.parametrize("mode", ["eager", "recorded", "torch_bce"])
@pytest.mark.parametrize("precision,gtol,atol", [("fp32", 1e-5, 1e-4), ("bf16x3", 1e-4, 2e-4)])
def test_1vsall_bce_trajectory_vs_reference(precision, gtol, atol, mode, monkeypatch):
    """Three reference 1vsAll batches with train.loss bce (index labels -> one-hot rows,
    loss.py:109-117): first batch's gradients, per-batch losses, final tables -- through the
    fused plane pass (eager, and replayed from the recorded step) and through torch's loss."""
    from kge import Dataset
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, "train1vsall_bce_complex.npz"))
    meta = json.loads(str(f["meta"]))
    c = base_config("complex", meta["dim"], meta["E"], meta["R"], {
        "train.type": "1vsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": meta["lr"]},
        "train.loss": "bce", "train.batch_size": meta["batch_size"], "engine.precision": precision,
        "engine.fused_loss": mode != "torch_bce", "engine.graph_step": mode == "recorded"})
    batches = torch.from_numpy(f["batches"].astype(np.int64))
    ds = Dataset(c, None)
    ds._triples = {"train": batches.reshape(-1, 3).int()}
    job = TrainingJob.create(c, ds)
    set_tables(job.model, f["ent0"], f["rel0"])
    job._prepare()
    job.optimizer.zero_grad()
    # the bf16x3 fused path must run kge_bce_planes (not fall through to torch's loss)
    from kge import _lib
    calls = []
    orig = _lib.softmax_planes
    monkeypatch.setattr(_lib, "softmax_planes", lambda *a, **k: (calls.append(a[7] if len(a) > 7 else k.get("loss_kind", "kl")), orig(*a, **k))[1])
    job.process_batch(0, {"triples": batches[0]})
    monkeypatch.setattr(_lib, "softmax_planes", orig)
    assert calls == (["bce"] if (precision == "bf16x3" and mode != "torch_bce") else []), calls
    ge = job.model._entity_embedder._embeddings.weight.grad.cpu().numpy()
    gr = job.model._relation_embedder._embeddings.weight.grad.cpu().numpy()
    assert np.abs(ge - f["g_ent_0"]).max() <= gtol * np.abs(f["g_ent_0"]).max()
    assert np.abs(gr - f["g_rel_0"]).max() <= gtol * np.abs(f["g_rel_0"]).max()
    job.optimizer.zero_grad()
    losses = []
    for b in range(len(batches)):
        res, _, _ = job.train_step(b, {"triples": batches[b]})
        losses.append(float(res.avg_loss))
    if mode == "recorded":
        assert job._graph_step is not None and job._graph_step.graph is not None, job._graph_step.error
    np.testing.assert_allclose(losses, f["losses"], rtol=2e-5)
    for got, want in zip(tables(job.model), (f["ent1"], f["rel1"])):
        diff = np.abs(got - want)
        assert int((diff > atol).sum()) <= max(8, 3e-3 * diff.size) and float(diff.mean()) < 1e-5


@pytest.mark.parametrize("fused", [True, False], ids=["fused", "torch_loss"])
@pytest.mark.parametrize("impl", ["triple", "all", "batch"])
@pytest.mark.parametrize("name,model", [("train_ns_complex_margin_ranking.npz", "complex"),
                                        ("train_ns_rotate_bce.npz", "rotate")])
def test_negative_sampling_margin_and_bce_steps_vs_reference(name, model, impl, fused):
    """Two reference negative-sampling batches with train.loss margin_ranking (margin 2, ComplEx) and
    bce (offset -3, RotatE), the reference sampler's negatives injected: per-batch loss and
    gradients from the reference's tables, then the free-running tables."""
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, name))
    meta = json.loads(str(f["meta"]))
    extra = {"train.type": "negative_sampling", "train.optimizer": "Adagrad",
             "train.optimizer_args": {"lr": meta["lr"]}, "train.batch_size": meta["batch_size"],
             "train.loss": meta["loss"], "train.loss_arg": meta["loss_arg"],
             "negative_sampling.num_samples.s": meta["num_negatives"], "negative_sampling.num_samples.o": -1,
             "negative_sampling.num_samples.p": 0, "negative_sampling.implementation": impl,
             "engine.precision": "fp32", "engine.fused_loss": fused}
    if meta["l_norm"] is not None:
        extra[f"{model}.l_norm"] = float(meta["l_norm"])
    c = base_config(model, meta["dim"], meta["E"], meta["R"], extra)
    ds = dataset_from(c, f)
    job = TrainingJob.create(c, ds)
    set_tables(job.model, f["ent0"], f["rel0"])
    job._prepare()
    assert (job._fused_loss is not None) == fused
    ent_w = job.model._entity_embedder._embeddings.weight
    rel_w = job.model._relation_embedder._embeddings.weight
    batches = []
    for b in range(meta["num_batches"]):
        neg_s, neg_o = torch.from_numpy(f[f"neg_s_{b}"]), torch.from_numpy(f[f"neg_o_{b}"])
        batch = {"triples": torch.from_numpy(f[f"triples_{b}"]),
                 "negative_samples": [neg_s, torch.zeros(len(neg_s), 0, dtype=torch.int64), neg_o]}
        batches.append(batch)
        set_tables(job.model, f[f"ent_before_{b}"], f[f"rel_before_{b}"])
        job.optimizer.zero_grad()
        res = job.process_batch(b, batch)
        assert float(res.avg_loss) == pytest.approx(float(f["losses"][b]), rel=2e-5)
        for w, key in ((ent_w, f"g_ent_{b}"), (rel_w, f"g_rel_{b}")):
            err = np.abs(w.grad.cpu().numpy() - f[key]).max() / np.abs(f[key]).max()
            assert err < 1e-5, (b, key, err)
    set_tables(job.model, f["ent0"], f["rel0"])
    job.optimizer = type(job.optimizer)(job.optimizer.param_groups[0]["params"], lr=meta["lr"])
    losses = []
    for b, batch in enumerate(batches):
        job.optimizer.zero_grad()
        res = job.process_batch(b, batch)
        job.optimizer.step()
        losses.append(res.avg_loss)
    np.testing.assert_allclose(losses, f["losses"], rtol=2e-5)
    for got, want in zip(tables(job.model), (f["ent1"], f["rel1"])):
        diff = np.abs(got - want)
        assert int((diff > 2e-4).sum()) <= max(4, 1e-3 * diff.size) and float(diff.mean()) < 1e-5


@pytest.mark.parametrize("impl", ["triple", "batch"])
@pytest.mark.parametrize("name,model", [("train_ns_transe_bce_self_adversarial.npz", "transe"),
                                        ("train_ns_distmult_bce_mean.npz", "distmult"),
                                        ("train_ns_complex_soft_margin.npz", "complex"),
                                        ("train_ns_simple_se.npz", "simple")])
def test_negative_sampling_other_losses_vs_reference(name, model, impl):
    """The losses the engine does not fuse -- bce_self_adversarial (temperature 0.5 from the user
    section, offset 6; loss.py:169-187), bce_mean, soft_margin, se -- on reference negative-sampling
    batches: torch's loss chain on the engine's score block, loss and gradients per batch."""
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, name))
    meta = json.loads(str(f["meta"]))
    extra = {"train.type": "negative_sampling", "train.optimizer": "Adagrad",
             "train.optimizer_args": {"lr": meta["lr"]}, "train.batch_size": meta["batch_size"],
             "train.loss": meta["loss"],
             "negative_sampling.num_samples.s": meta["num_negatives"], "negative_sampling.num_samples.o": -1,
             "negative_sampling.num_samples.p": 0, "negative_sampling.implementation": impl,
             "engine.precision": "fp32"}
    if meta["loss_arg"] is not None:
        extra["train.loss_arg"] = meta["loss_arg"]
    extra.update(meta["extra"])
    if meta["l_norm"] is not None:
        extra[f"{model}.l_norm"] = float(meta["l_norm"])
    c = base_config(model, meta["dim"], meta["E"], meta["R"], extra)
    ds = dataset_from(c, f)
    job = TrainingJob.create(c, ds)
    set_tables(job.model, f["ent0"], f["rel0"])
    job._prepare()
    assert job._fused_loss is None
    ent_w = job.model._entity_embedder._embeddings.weight
    rel_w = job.model._relation_embedder._embeddings.weight
    for b in range(meta["num_batches"]):
        neg_s, neg_o = torch.from_numpy(f[f"neg_s_{b}"]), torch.from_numpy(f[f"neg_o_{b}"])
        batch = {"triples": torch.from_numpy(f[f"triples_{b}"]),
                 "negative_samples": [neg_s, torch.zeros(len(neg_s), 0, dtype=torch.int64), neg_o]}
        set_tables(job.model, f[f"ent_before_{b}"], f[f"rel_before_{b}"])
        job.optimizer.zero_grad()
        res = job.process_batch(b, batch)
        assert float(res.avg_loss) == pytest.approx(float(f["losses"][b]), rel=2e-5)
        for w, key in ((ent_w, f"g_ent_{b}"), (rel_w, f"g_rel_{b}")):
            err = np.abs(w.grad.cpu().numpy() - f[key]).max() / np.abs(f[key]).max()
            assert err < 2e-5, (b, key, err)


@pytest.mark.parametrize("impl", ["triple", "all", "batch"])
def test_sparse_embeddings_negative_sampling_vs_reference(impl):
    """lookup_embedder.sparse: True (lookup_embedder.py:30-45: the reference's nn.Embedding then hands the
    optimizer row-sparse gradients): two reference negative-sampling batches captured with the
    option on -- losses, densified gradients, and the tables after two Adagrad steps."""
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, "train_ns_complex_sparse.npz"))
    meta = json.loads(str(f["meta"]))
    extra = {"train.type": "negative_sampling", "train.optimizer": "Adagrad",
             "train.optimizer_args": {"lr": meta["lr"]}, "train.batch_size": meta["batch_size"],
             "negative_sampling.num_samples.s": meta["num_negatives"], "negative_sampling.num_samples.o": -1,
             "negative_sampling.num_samples.p": 0, "negative_sampling.implementation": impl,
             "engine.precision": "fp32"}
    extra.update(meta["extra"])
    assert extra["lookup_embedder.sparse"] is True
    c = base_config("complex", meta["dim"], meta["E"], meta["R"], extra)
    ds = dataset_from(c, f)
    job = TrainingJob.create(c, ds)
    assert job.model._entity_embedder.sparse and job.model._entity_embedder._embeddings.sparse
    set_tables(job.model, f["ent0"], f["rel0"])
    job._prepare()
    ent_w = job.model._entity_embedder._embeddings.weight
    rel_w = job.model._relation_embedder._embeddings.weight
    batches = []
    for b in range(meta["num_batches"]):
        neg_s, neg_o = torch.from_numpy(f[f"neg_s_{b}"]), torch.from_numpy(f[f"neg_o_{b}"])
        batch = {"triples": torch.from_numpy(f[f"triples_{b}"]),
                 "negative_samples": [neg_s, torch.zeros(len(neg_s), 0, dtype=torch.int64), neg_o]}
        batches.append(batch)
        set_tables(job.model, f[f"ent_before_{b}"], f[f"rel_before_{b}"])
        job.optimizer.zero_grad()
        res = job.process_batch(b, batch)
        assert float(res.avg_loss) == pytest.approx(float(f["losses"][b]), rel=2e-5)
        for w, key in ((ent_w, f"g_ent_{b}"), (rel_w, f"g_rel_{b}")):
            g = w.grad.to_dense() if w.grad.is_sparse else w.grad
            err = np.abs(g.cpu().numpy() - f[key]).max() / np.abs(f[key]).max()
            assert err < 1e-5, (b, key, err)
    set_tables(job.model, f["ent0"], f["rel0"])
    job.optimizer = type(job.optimizer)(job.optimizer.param_groups[0]["params"], lr=meta["lr"])
    for b, batch in enumerate(batches):
        job.optimizer.zero_grad()
        job.process_batch(b, batch)
        job.optimizer.step()
    for got, want in zip(tables(job.model), (f["ent1"], f["rel1"])):
        diff = np.abs(got - want)
        assert int((diff > 2e-4).sum()) <= max(4, 1e-3 * diff.size) and float(diff.mean()) < 1e-5
