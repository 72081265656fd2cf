"""GPU parity of the drop-in plugin API (kge.model.KgeModel / RelationalScorer /
LookupEmbedder, kge.job.EntityRankingJob / TrainingJob1vsAll) against the reference's
golden vectors.  Everything here runs on libkgescore; a missing library raises."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_scorer_fixture
from oracle import kge_oracle as K

pytestmark = pytest.mark.gpu
SCORER_FILES = sorted(glob.glob(os.path.join(GOLDEN, "scorer_*.npz")))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib
    _lib.lib()


def make_model(model, dim, E, R, ent, rel, extra=None, precision="bf16x3"):
    from kge import Config, Dataset, KgeModel

    c = Config()
    c.set("model", model)
    c._import(model)
    c.set("job.device", "cuda")
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    c.set("lookup_embedder.dim", dim)
    c.set("engine.precision", precision)
    for k, v in (extra or {}).items():
        c.set(k, v)
    m = KgeModel.create(c, Dataset(c, None))
    with torch.no_grad():
        m._entity_embedder._embeddings.weight.copy_(torch.from_numpy(ent))
        m._relation_embedder._embeddings.weight.copy_(torch.from_numpy(rel))
    return m


def model_from_fixture(f, precision):
    meta = json.loads(str(f["meta"]))
    extra = {}
    if meta["model"] in ("transe", "rotate"):
        extra[f"{meta['model']}.l_norm"] = float(meta["l_norm"])
    m = make_model(meta["model"], f["ent"].shape[1], f["ent"].shape[0], f["rel"].shape[0], f["ent"], f["rel"], extra,
                   precision)
    return m, meta


def rel_err(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.abs(ref).max(axis=-1, keepdims=True) if ref.ndim == 2 else np.abs(ref).max()
    return float((np.abs(x - ref) / np.maximum(scale, 1e-30)).max())


def check(meta, name, got, ref, prec):
    model = meta["model"]
    exact = meta["regime"] == "dyadic" and (model in K.BILINEAR or (model == "transe" and meta["l_norm"] == 1
                                                                      and name != "spo"))
    if exact:
        np.testing.assert_array_equal(got, ref, err_msg=name)
    else:
        tol = 1e-5 if (model in K.DISTANCE or name == "spo") else (2e-5 if prec == "bf16x3" else 2e-6)
        assert rel_err(got, ref) < tol, (name, rel_err(got, ref))


@pytest.mark.parametrize("path", ["lookup", "emb"])
@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
@pytest.mark.parametrize("fn", SCORER_FILES, ids=lambda f: os.path.basename(f)[7:-4])
def test_model_scores_and_grads(fn, prec, path):
    f = load_scorer_fixture(fn)
    m, meta = model_from_fixture(f, prec)
    dev = "cuda"
    s, p, o, sub = (torch.from_numpy(f[k]).to(dev) for k in ("s", "p", "o", "subset"))
    m.train()
    if path == "lookup":
        spo = m.score_spo(s, p, o)
        sp_all = m.score_sp(s, p)
        po_all = m.score_po(p, o)
    else:  # generic plugin path: embeddings into RelationalScorer.score_emb
        es, ep, eo = m.get_s_embedder().embed(s), m.get_p_embedder().embed(p), m.get_o_embedder().embed(o)
        allE = m.get_o_embedder().embed_all()
        spo = m.get_scorer().score_emb(es, ep, eo, "spo").view(-1)
        sp_all = m.get_scorer().score_emb(es, ep, allE, "sp_")
        po_all = m.get_scorer().score_emb(allE, ep, eo, "_po")
    w_sp, w_po, w_spo = (torch.from_numpy(f[k]).to(dev) for k in ("w_sp", "w_po", "w_spo"))
    loss = (w_sp * sp_all).sum() + (w_po * po_all).sum() + (w_spo * spo).sum()
    m.zero_grad()
    loss.backward()
    with torch.no_grad():
        outs = dict(spo=spo, sp_all=sp_all, po_all=po_all, sp_sub=m.score_sp(s, p, sub), po_sub=m.score_po(p, o, sub),
                    sppo_sub=m.score_sp_po(s, p, o, sub), sppo_all=m.score_sp_po(s, p, o))
    for k, v in outs.items():
        if k in f:  # the larger fixtures leave the [n, 2 E] score_sp_po block out
            check(meta, k, v.detach().cpu().numpy(), f[k], prec)
    ge = m._entity_embedder._embeddings.weight.grad.cpu().numpy()
    gr = m._relation_embedder._embeddings.weight.grad.cpu().numpy()
    tol = 1e-4 if (prec == "bf16x3" and meta["model"] in K.BILINEAR) else 1e-5
    assert np.abs(ge - f["g_ent"]).max() <= tol * np.abs(f["g_ent"]).max()
    assert np.abs(gr - f["g_rel"]).max() <= tol * np.abs(f["g_rel"]).max()


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
@pytest.mark.parametrize("fn", SCORER_FILES, ids=lambda f: os.path.basename(f)[7:-4])
def test_fused_xent_matches_unfused(fn, prec):
    """KgeModel.score_sp_xent / score_po_xent (scores -> CE -> gradient in the engine) give
    the loss and gradients of score_sp / score_po + torch CrossEntropyLoss(sum) / B."""
    f = load_scorer_fixture(fn)
    if json.loads(str(f["meta"]))["regime"] != "normal":
        pytest.skip("one regime is enough")
    s, p, o = (torch.from_numpy(f[k]).cuda() for k in ("s", "p", "o"))
    B = len(s)
    res = []
    for fused in (True, False):
        m, meta = model_from_fixture(f, prec)
        m.train()
        m.zero_grad()
        if fused:
            loss = m.score_sp_xent(s, p, o, 1.0 / B) + m.score_po_xent(p, o, s, 1.0 / B)
        else:
            ce = torch.nn.CrossEntropyLoss(reduction="sum")
            loss = ce(m.score_sp(s, p), o) / B + ce(m.score_po(p, o), s) / B
        loss.backward()
        res.append((loss.item(), m._entity_embedder._embeddings.weight.grad.cpu().numpy(),
                    m._relation_embedder._embeddings.weight.grad.cpu().numpy()))
    (l1, ge1, gr1), (l0, ge0, gr0) = res
    assert abs(l1 - l0) <= 1e-5 * abs(l0)
    tol = 1e-4 if (prec == "bf16x3" and meta["model"] in K.BILINEAR) else 1e-5
    assert np.abs(ge1 - ge0).max() <= tol * np.abs(ge0).max()
    assert np.abs(gr1 - gr0).max() <= tol * np.abs(gr0).max()


def eval_job(f, tag, precision, extra=None):
    from kge import Config, Dataset
    from kge.job import EntityRankingJob

    meta = json.loads(str(f["meta"]))
    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", meta["dim"])
    c.set("engine.precision", precision.replace("_refined", ""))
    c.set("engine.eval_precision", precision)
    c.set("eval.batch_size", meta["batch_size"])
    c.set("engine.eval_batch_size", 0)  # the batches of eval.batch_size as they are
    c.set("eval.split", "valid")
    c.set("entity_ranking.chunk_size", -1 if tag == "full" else meta["chunk8"])
    c.set("dataset.num_entities", meta["E"])
    c.set("dataset.num_relations", meta["R"])
    for k, v in (extra or {}).items():
        c.set(k, v)
    ds = Dataset(c, None)
    ds._triples = {k: torch.from_numpy(f["tri_" + k].astype(np.int32)) for k in ("train", "valid", "test")}
    m = make_model("complex", meta["dim"], meta["E"], meta["R"], f["ent"], f["rel"],
                   precision=precision.replace("_refined", ""))
    m.config = c
    m.get_scorer().config = c
    job = EntityRankingJob(c, ds, model=m)
    job.capture_ranks = True
    trace = job.run()
    return job, trace


@pytest.mark.parametrize("regime,precision", [("dyadic", "bf16x3"), ("dyadic", "fp32"), ("normal", "fp32"),
                                              ("dyadic", "bf16x3_refined"), ("normal", "bf16x3_refined")])
@pytest.mark.parametrize("tag", ["full", "chunk8"])
def test_entity_ranking_vs_golden(regime, precision, tag):
    f = np.load(os.path.join(GOLDEN, f"eval_{regime}.npz"))
    ref_metrics = json.loads(str(f["metrics"]))[tag]
    job, trace = eval_job(f, tag, precision)
    for k, v in job.ranks.items():
        np.testing.assert_array_equal(v, f[f"{tag}_{k}"], err_msg=k)
    for k, v in ref_metrics.items():
        assert trace[k] == pytest.approx(v, rel=1e-6, abs=1e-9), k


@pytest.mark.parametrize("tag", ["full", "chunk8"])
def test_entity_ranking_metrics_per_group_vs_golden(tag):
    """entity_ranking.metrics_per.{head_and_tail, relation_type, argument_frequency}: the
    dataset's relation classes and frequency quartiles and every metric of the reference's
    epoch trace (729 of them), in the reference's order, unchunked and in 8 entity chunks."""
    f = np.load(os.path.join(GOLDEN, "eval_metrics_per.npz"))
    f = dict(f)
    meta = json.loads(str(f["meta"]))
    meta["chunk8"] = -(-meta["E"] // 8)
    f["meta"] = np.array(json.dumps(meta))
    job, trace = eval_job(f, tag, "bf16x3_refined",
                          {"entity_ranking.metrics_per." + k: True
                           for k in ("head_and_tail", "relation_type", "argument_frequency")})
    assert job.dataset.index("relation_types") == json.loads(str(f["relation_types"]))
    percs = job.dataset.index("frequency_percentiles")
    assert {a: {q: sorted(v) for q, v in d.items()} for a, d in percs.items()} == json.loads(
        str(f["frequency_percentiles"]))
    ref_metrics = json.loads(str(f["metrics"]))
    order = json.loads(str(f["metric_order"]))
    assert [k for k in trace if k in ref_metrics] == order
    for k, v in ref_metrics.items():
        assert trace[k] == pytest.approx(v, rel=1e-6, abs=1e-9), k


@pytest.mark.parametrize("streams", [1, 2, 3])
def test_entity_ranking_same_ranks_on_any_number_of_streams(streams):
    """engine.eval_streams: the evaluation batches take turns on that many HIP streams; the
    ranks and every metric are the reference's whatever the number, twice in a row (the second
    run reuses the job's streams and their cached buffers)."""
    f = np.load(os.path.join(GOLDEN, "eval_normal.npz"))
    ref_metrics = json.loads(str(f["metrics"]))["full"]
    meta = json.loads(str(f["meta"]))
    assert len(f["tri_valid"]) > 2 * meta["batch_size"]  # three batches
    job, trace = eval_job(f, "full", "bf16x3_refined", {"engine.eval_streams": streams})
    assert len(job._streams.streams) == (streams if streams > 1 else 0)
    for run in range(2):
        for k, v in job.ranks.items():
            np.testing.assert_array_equal(v, f[f"full_{k}"], err_msg=f"{k} run {run}")
        for k, v in ref_metrics.items():
            assert trace[k] == pytest.approx(v, rel=1e-6, abs=1e-9), k
        trace = job.run()


def test_batch_streams_score_sp_identical_to_one_stream():
    """kge.engine.BatchStreams: score_sp batches launched on alternating streams give the
    scores of the same batches on the caller's stream, bit for bit, and leaving the block
    orders the caller's stream behind every batch."""
    from kge import engine

    f = np.load(os.path.join(GOLDEN, "eval_normal.npz"))
    meta = json.loads(str(f["meta"]))
    m = make_model("complex", meta["dim"], meta["E"], meta["R"], f["ent"], f["rel"])
    g = torch.Generator().manual_seed(3)
    s = torch.randint(0, meta["E"], (12, 257), generator=g).cuda()
    p = torch.randint(0, meta["R"], (12, 257), generator=g).cuda()
    with torch.no_grad():
        ref = [m.score_sp(s[i], p[i]) for i in range(12)]
        for count in (2, 3):
            outs = []
            with engine.BatchStreams("cuda", count) as lanes:
                assert len(lanes.streams) == count
                for i in range(12):
                    with lanes.batch(i):
                        outs.append(m.score_sp(s[i], p[i]))
            total = torch.stack(outs).sum()  # on the caller's stream, after the block
            assert torch.equal(torch.stack(outs), torch.stack(ref))
            assert torch.isfinite(total)
    with engine.BatchStreams("cuda", 1) as lanes:  # one stream: the caller's own
        assert lanes.streams == []
        with lanes.batch(0):
            assert torch.cuda.current_stream() == torch.cuda.default_stream()


def test_entity_ranking_bf16x3_normal_near_ties_only():
    """bf16x3 scoring on real-valued data: a rank may differ from the reference's only where
    unfiltered competitors lie within the score tolerance of the true score -- asserted per
    moved rank against exact (float64) score rows, with |rank change| bounded by the number
    of such competitors (test_gpu_configs.assert_rank_moves_are_near_ties)."""
    from test_gpu_configs import assert_rank_moves_are_near_ties

    f = np.load(os.path.join(GOLDEN, "eval_normal.npz"))
    ref_metrics = json.loads(str(f["metrics"]))["full"]
    job, trace = eval_job(f, "full", "bf16x3")
    ref = {k: f["full_" + k] for k in job.ranks}
    splits = {k: f["tri_" + k].astype(np.int64) for k in ("train", "valid", "test")}
    moved, worst = assert_rank_moves_are_near_ties(job.ranks, ref, f["ent"], f["rel"], splits["valid"], splits,
                                                   3e-5, "bf16x3")
    n_q = 2 * len(splits["valid"])
    for k, v in ref_metrics.items():
        if k.startswith("hits_at"):
            assert abs(trace[k] - v) <= moved / n_q + 1e-7, k
    assert trace["mean_reciprocal_rank_filtered"] == pytest.approx(ref_metrics["mean_reciprocal_rank_filtered"],
                                                                   rel=1e-3 if moved else 1e-6)


@pytest.mark.parametrize("fused", [True, False], ids=["fused_xent", "torch_ce"])
@pytest.mark.parametrize("precision,atol", [("fp32", 1e-4), ("bf16x3", 2e-4)])
def test_train_1vsall_vs_golden(precision, atol, fused):
    """Three Adagrad 1vsAll steps vs the golden trajectory.  Adagrad divides by the root of
    the accumulated squared gradient, so an element whose gradient is tiny moves by ~lr
    whatever its size; the bf16x3 backward (~1e-5 of the row scale per product, split-K
    atomics in nondeterministic order) therefore gets a slightly wider bound on the weights
    than the exact fp32 path.  Losses are held to rtol 1e-5 in both."""
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
    c.set("engine.precision", precision)
    c.set("engine.fused_loss", fused)
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
        job.optimizer.zero_grad()
        res = job._process_batch(b, {"triples": torch.from_numpy(f["batches"][b])})
        job.optimizer.step()
        losses.append(res.avg_loss)
    np.testing.assert_allclose(losses, f["losses"], rtol=1e-5)
    e1 = job.model._entity_embedder._embeddings.weight.detach().cpu().numpy()
    r1 = job.model._relation_embedder._embeddings.weight.detach().cpu().numpy()
    np.testing.assert_allclose(e1, f["ent1"], atol=atol)
    np.testing.assert_allclose(r1, f["rel1"], atol=atol)


def test_reciprocal_relations_model():
    """(?, p, o) answered as (o, p + R, ?) with the sp_ kernel (reciprocal_relations_model.py:67-74)."""
    from kge import Config, Dataset, KgeModel

    torch.manual_seed(0)
    c = Config()
    c.set("model", "reciprocal_relations_model")
    c._import("reciprocal_relations_model")
    c.set("reciprocal_relations_model.base_model.type", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 32)
    c.set("dataset.num_entities", 50)
    c.set("dataset.num_relations", 5)
    m = KgeModel.create(c, Dataset(c, None))
    ent = m._entity_embedder._embeddings.weight.detach().double().cpu().numpy()
    rel = m._relation_embedder._embeddings.weight.detach().double().cpu().numpy()
    p = torch.tensor([0, 1, 4], device="cuda")
    o = torch.tensor([3, 7, 49], device="cuda")
    got = m.score_po(p, o).detach().cpu().numpy()
    ref = K.prep_sp("complex", ent[o.cpu().numpy()], rel[p.cpu().numpy() + 5]) @ ent.T
    assert rel_err(got, ref) < 2e-5
    with pytest.raises(Exception):
        m.score_spo(p, p, o)


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
@pytest.mark.parametrize("fn", SCORER_FILES, ids=lambda f: os.path.basename(f)[7:-4])
def test_fused_xent2_matches_separate(fn, prec):
    """KgeModel.score_sp_po_xent (both directions stacked into one contraction, one loss
    launch, one backward that writes dE) == score_sp_xent + score_po_xent."""
    f = load_scorer_fixture(fn)
    if json.loads(str(f["meta"]))["regime"] != "normal":
        pytest.skip("one regime is enough")
    s, p, o = (torch.from_numpy(f[k]).cuda() for k in ("s", "p", "o"))
    B = len(s)
    res = []
    for combined in (True, False):
        m, meta = model_from_fixture(f, prec)
        m.train()
        m.zero_grad()
        if combined:
            both = m.score_sp_po_xent(s, p, o, 1.0 / B)
            if both is None:
                assert meta["model"] in K.DISTANCE or meta["model"] == "cp"
                pytest.skip("not fusable across directions")
            total, (l_sp, l_po) = both
            assert not l_sp.requires_grad and abs(total.item() - (l_sp + l_po).item()) <= 1e-6 * abs(total.item())
            (0.75 * total).backward()  # an upstream gradient other than 1
        else:
            l_sp, l_po = m.score_sp_xent(s, p, o, 1.0 / B), m.score_po_xent(p, o, s, 1.0 / B)
            (0.75 * (l_sp + l_po)).backward()
        res.append((l_sp.item(), l_po.item(), m._entity_embedder._embeddings.weight.grad.cpu().numpy(),
                    m._relation_embedder._embeddings.weight.grad.cpu().numpy()))
    (a1, b1, ge1, gr1), (a0, b0, ge0, gr0) = res
    assert abs(a1 - a0) <= 1e-5 * abs(a0) and abs(b1 - b0) <= 1e-5 * abs(b0)
    assert np.abs(ge1 - ge0).max() <= 2e-5 * np.abs(ge0).max()
    assert np.abs(gr1 - gr0).max() <= 2e-5 * np.abs(gr0).max()


def test_reciprocal_fused_xent():
    """ReciprocalRelationsModel.score_po_xent == CE over score_po (base sp_ kernel, p + R)."""
    from kge import Config, Dataset, KgeModel

    torch.manual_seed(0)
    c = Config()
    c.set("model", "reciprocal_relations_model")
    c._import("reciprocal_relations_model")
    c.set("reciprocal_relations_model.base_model.type", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 32)
    c.set("dataset.num_entities", 50)
    c.set("dataset.num_relations", 5)
    m = KgeModel.create(c, Dataset(c, None))
    p = torch.tensor([0, 1, 4], device="cuda")
    o = torch.tensor([3, 7, 49], device="cuda")
    s = torch.tensor([9, 0, 17], device="cuda")
    fused = m.score_po_xent(p, o, s, 0.5)
    ref = torch.nn.CrossEntropyLoss(reduction="sum")(m.score_po(p, o), s) * 0.5
    assert abs(fused.item() - ref.item()) <= 1e-5 * abs(ref.item())
    total, both = m.score_sp_po_xent(s, p, o, 0.5)  # both halves as "sp_" queries in one pass
    ref_sp = torch.nn.CrossEntropyLoss(reduction="sum")(m.score_sp(s, p), o) * 0.5
    assert abs(both[0].item() - ref_sp.item()) <= 1e-5 * abs(ref_sp.item())
    assert abs(both[1].item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert abs(total.item() - (ref_sp + ref).item()) <= 1e-5 * abs(total.item())
