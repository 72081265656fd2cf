"""Every BASELINE configuration on the GPU, pinned to fixtures captured from the reference
(tests/golden/make_golden.py) where a fixture can be captured, and to float64 arithmetic
(torch CPU double, independent of the engine) at the full configuration sizes.

  C1  toy-complex options (1vsAll, dim 128, Adagrad 0.2, ReduceLROnPlateau, lp penalty
      0.8e-7, N(0, 0.1)): the reference's TrainingJob._run trajectory, epoch by epoch.
  C2  ComplEx-512 entity ranking at E = 14,541 on real-valued tables, default
      configuration: ranks against the reference's, any difference checked to be a near-tie.
  C3  DistMult KvsAll: reference-captured three-batch trajectory (label smoothing, sp_ + _po)
      and one step at E = 40,943, B = 512, d = 512 against float64.
  C4  negative sampling: reference-captured steps with the negatives injected (RotatE,
      ComplEx) and the candidate kernel at d = 1024, k = 1025 against float64.
  C5  score_sp over one rank's Wikidata5M shard (574,311 rows) through RowShardedScorer.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib
    _lib.lib()


def base_config(model, dim, E, R, extra=None):
    from kge import Config

    c = Config()
    c.set("model", model)
    c._import(model)
    c.set("job.device", "cuda")
    c.set("verbose", False)
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    c.set("lookup_embedder.dim", dim)
    c.set("engine.eval_batch_size", 0)  # evaluation in the batches of eval.batch_size, as the fixtures were captured
    for k, v in (extra or {}).items():
        c.set(k, v)
    return c


def dataset_from(c, f):
    from kge import Dataset

    ds = Dataset(c, None)
    ds._triples = {k[4:]: torch.from_numpy(f[k].astype(np.int32)) for k in f.files if k.startswith("tri_")}
    return ds


def set_tables(model, ent, rel):
    with torch.no_grad():
        model._entity_embedder._embeddings.weight.copy_(torch.as_tensor(ent))
        model._relation_embedder._embeddings.weight.copy_(torch.as_tensor(rel))


def tables(model):
    return (model._entity_embedder._embeddings.weight.detach().cpu().numpy(),
            model._relation_embedder._embeddings.weight.detach().cpu().numpy())


# ------------------------------------------------------------------------------ C2 eval

#: engine.eval_precision of config-default.yaml
DEFAULT_EVAL_PRECISION = "bf16x3_refined"


def seeded_tables(seed, E, R, d_e, d_r, std=0.1):
    """The generator of tests/golden/make_golden.py (numpy PCG64 stream)."""
    rng = np.random.default_rng(seed)
    ent = (rng.standard_normal((E, d_e), dtype=np.float32) * np.float32(std)).astype(np.float32)
    rel = (rng.standard_normal((R, d_r), dtype=np.float32) * np.float32(std)).astype(np.float32)
    return ent, rel


def table_checksum(x):
    return [float(x.astype(np.float64).sum()), float(np.abs(x.astype(np.float64)).sum()),
            float(x[0, 0]), float(x[-1, -1])]


def complex_rows_f64(ent, rel, e_idx, p_idx, direction):
    """Exact (float64) ComplEx score rows of queries against every entity
    (complex.py:19-44 restated: sp_ = cmul(s, r) . E^T, _po = cmul(conj(r), o) . E^T)."""
    e = ent[e_idx].astype(np.float64)
    r = rel[p_idx].astype(np.float64)
    h = ent.shape[1] // 2
    er, ei, rr, ri = e[:, :h], e[:, h:], r[:, :h], r[:, h:]
    if direction == "sp":
        q = np.concatenate([er * rr - ei * ri, er * ri + ei * rr], 1)
    else:
        q = np.concatenate([rr * er + ri * ei, rr * ei - ri * er], 1)
    return q @ ent.astype(np.float64).T


def complex_spo_f64(ent, rel, s, p, o):
    e_s, r, e_o = ent[s].astype(np.float64), rel[p].astype(np.float64), ent[o].astype(np.float64)
    h = ent.shape[1] // 2
    qr = e_s[:, :h] * r[:, :h] - e_s[:, h:] * r[:, h:]
    qi = e_s[:, :h] * r[:, h:] + e_s[:, h:] * r[:, :h]
    return (qr * e_o[:, :h]).sum(1) + (qi * e_o[:, h:]).sum(1)


def assert_rank_moves_are_near_ties(got, ref, ent, rel, tri, splits, tol, what):
    """Every rank that differs from the reference's must be explained by near-ties: the
    number of unfiltered competitors whose exact score lies within tol * rowmax of the exact
    true score bounds |rank - reference rank| (a competitor that far from the true score
    cannot change sides under a score error below tol * rowmax, entity_ranking.py:469-529).
    Returns (#moved, largest |competitor - true| / rowmax needed to explain a move)."""
    moved, worst = 0, 0.0
    known = {}
    for key in got:
        d, ranking = key[0], key[2:]
        bad = np.flatnonzero(got[key] != ref[key])
        if len(bad) == 0:
            continue
        moved += len(bad)
        s, p, o = tri[bad, 0], tri[bad, 1], tri[bad, 2]
        if d == "o":
            rows = complex_rows_f64(ent, rel, s, p, "sp")
            target, qa, qb, va, vb, vt = o, s, p, 0, 1, 2
        else:
            rows = complex_rows_f64(ent, rel, o, p, "po")
            target, qa, qb, va, vb, vt = s, p, o, 1, 2, 0
        true = complex_spo_f64(ent, rel, s, p, o)
        for j, i in enumerate(bad):
            names = {"raw": [], "filt": ["train", "valid"], "filt_test": ["train", "valid", "test"]}[ranking]
            mask = np.zeros(ent.shape[0], bool)
            for nme in names:
                t = splits[nme]
                mask[t[(t[:, va] == qa[j]) & (t[:, vb] == qb[j]), vt]] = True
            mask[target[j]] = True  # the true entry takes the true score: never a competitor
            row = rows[j]
            scale = np.abs(row).max()
            dist = np.abs(row - true[j]) / scale
            dist[mask] = np.inf
            delta = abs(int(got[key][i]) - int(ref[key][i]))
            near = np.sort(dist)[:delta]
            assert near[-1] <= tol, (f"{what}: {key}[{i}] moved by {delta} but the {delta} nearest competitors are "
                                     f"{near} of the row maximum away from the true score (tolerance {tol})")
            worst = max(worst, float(near[-1]))
    return moved, worst


@pytest.mark.parametrize("chunk", [-1, 5000], ids=["one_chunk", "chunk5000"])
@pytest.mark.parametrize("eval_precision", [None, "fp32", "bf16x3", "bf16x3_refined"])
def test_c2_entity_ranking_fullsize_real_valued_vs_reference(eval_precision, chunk):
    """The reference's EntityRankingJob at E = 14,541 (ComplEx-512, N(0, 0.1) tables, 512
    validation triples, filtered + filtered-with-test) against this build's job in its DEFAULT
    configuration and with every engine.eval_precision: fp32 contraction, plain bf16x3, and
    bf16x3 with near-ties of the true score rescored exactly (bf16x3_refined).

    Two fp32 implementations of a K = 512 contraction differ by ~1e-6 of the row maximum
    (summation order), so on real-valued tables a competitor closer than that to the true
    score can legitimately change sides.  The bar: every rank equals the reference's, except
    where near-ties explain the move (contract tolerance 1e-4 of the row maximum; asserted
    much tighter: 1e-5 for fp32 and bf16x3_refined, 3e-5 for bf16x3), and the metrics agree
    accordingly."""
    from kge.job import EntityRankingJob
    from kge import KgeModel

    f = np.load(os.path.join(GOLDEN, "eval_fullsize_normal.npz"))
    meta = json.loads(str(f["meta"]))
    E, R, dim = meta["E"], meta["R"], meta["dim"]
    ent, rel = seeded_tables(meta["table_seed"], E, R, dim, dim, meta["std"])
    assert table_checksum(ent) == meta["ent_checksum"] and table_checksum(rel) == meta["rel_checksum"], \
        "seeded tables differ from the ones the reference was run on (numpy stream changed?)"
    if chunk > 0 and eval_precision in (None, "bf16x3"):
        pytest.skip("chunked scoring is covered with fp32 and bf16x3_refined")
    c = base_config("complex", dim, E, R, {"eval.batch_size": meta["batch_size"], "eval.split": "valid",
                                           "entity_ranking.chunk_size": chunk})
    assert c.get("engine.eval_precision") == DEFAULT_EVAL_PRECISION and c.get("engine.precision") == "bf16x3"
    if eval_precision is not None:
        c.set("engine.eval_precision", eval_precision)
    exactish = (eval_precision or DEFAULT_EVAL_PRECISION) != "bf16x3"
    ds = dataset_from(c, f)
    model = KgeModel.create(c, ds)
    set_tables(model, ent, rel)
    job = EntityRankingJob(c, ds, model=model)
    job.capture_ranks = True
    trace = job.run()
    ref = {k[5:]: f[k] for k in f.files if k.startswith("full_")}
    assert set(job.ranks) == set(ref)
    splits = {k: ds.split(k).long().numpy() for k in ("train", "valid", "test")}
    tol = 1e-5 if exactish else 3e-5
    moved, worst = assert_rank_moves_are_near_ties(job.ranks, ref, ent, rel, splits["valid"], splits, tol,
                                                   f"eval_precision={eval_precision or 'default'}")
    total = sum(len(v) for v in ref.values())
    print(f"\nC2 full-size eval ({eval_precision or 'default ' + DEFAULT_EVAL_PRECISION}, chunk {chunk}): {moved} of "
          f"{total} ranks differ from the reference, all near-ties (largest gap {worst:.2e} of the row maximum)")
    assert moved <= (0.005 if exactish else 0.02) * total
    # metrics: the job's own numbers follow from its ranks by the reference's formulas
    # (entity_ranking.py:553-577), and differ from the reference's by no more than the moved
    # ranks account for
    ref_metrics = json.loads(str(f["metrics"]))["full"]
    for ranking, suffix in (("raw", ""), ("filt", "_filtered"), ("filt_test", "_filtered_with_test")):
        mine = np.concatenate([job.ranks[f"s_{ranking}"], job.ranks[f"o_{ranking}"]]).astype(np.float64)
        theirs = np.concatenate([ref[f"s_{ranking}"], ref[f"o_{ranking}"]]).astype(np.float64)
        n_q = len(mine)
        assert trace["mean_rank" + suffix] == pytest.approx((mine + 1).mean(), rel=1e-6)
        assert trace["mean_reciprocal_rank" + suffix] == pytest.approx((1 / (mine + 1)).mean(), rel=1e-5)
        assert abs(trace["mean_rank" + suffix] - ref_metrics["mean_rank" + suffix]) <= \
            np.abs(mine - theirs).sum() / n_q + 1e-6 * ref_metrics["mean_rank" + suffix]
        assert abs(trace["mean_reciprocal_rank" + suffix] - ref_metrics["mean_reciprocal_rank" + suffix]) <= \
            np.abs(1 / (mine + 1) - 1 / (theirs + 1)).sum() / n_q + 1e-5 * ref_metrics["mean_reciprocal_rank" + suffix]
        for k in (1, 3, 10, 50, 100, 200, 300, 400, 500, 1000):
            crossed = ((mine < k) != (theirs < k)).sum()
            assert abs(trace[f"hits_at_{k}{suffix}"] - ref_metrics[f"hits_at_{k}{suffix}"]) <= crossed / n_q + 1e-7


def test_eval_precision_is_applied_and_restored():
    """engine.eval_precision governs the scorer during the run only (it used to be a dead key)."""
    from kge import KgeModel
    from kge.job import EntityRankingJob
    from kge import _lib

    f = np.load(os.path.join(GOLDEN, "eval_normal.npz"))
    meta = json.loads(str(f["meta"]))
    seen = []
    for ep in ("fp32", "bf16x3", "bf16x3_refined"):
        c = base_config("complex", meta["dim"], meta["E"], meta["R"], {"engine.eval_precision": ep})
        ds = dataset_from(c, f)
        model = KgeModel.create(c, ds)
        scorer = model.get_scorer()
        orig = scorer.precision

        def spy(orig=orig):
            seen.append(orig())
            return seen[-1]

        scorer.precision = spy
        EntityRankingJob(c, ds, model=model).run()
        # the refined mode contracts in bf16x3 and rescores near-ties in the ranking launch
        assert set(seen) == {_lib.PRECISIONS[ep.replace("_refined", "")]}, (ep, set(seen))
        seen.clear()
        scorer.precision = orig
        assert scorer.precision_override is None and scorer.precision() == _lib.PREC_BF16X3
    c = base_config("complex", 32, 10, 3, {"engine.eval_precision": "fp16"})
    ds = dataset_from(c, f)
    with pytest.raises(ValueError):
        EntityRankingJob(c, ds, model=KgeModel.create(c, ds)).run()


def test_metrics_per_head_and_tail_and_group_keys():
    """entity_ranking.metrics_per.head_and_tail: the head (subject) and tail (object)
    histograms of eval.py:125-146 -- checked against the metrics recomputed from the
    reference-captured per-direction ranks; each of the other metrics_per keys adds its
    groups' metrics, whose query counts add up to the ungrouped ones (the reference-pinned
    values are checked in test_gpu_api.test_entity_ranking_metrics_per_group_vs_golden)."""
    from kge import KgeModel
    from kge.job import EntityRankingJob

    f = np.load(os.path.join(GOLDEN, "eval_dyadic.npz"))
    meta = json.loads(str(f["meta"]))
    c = base_config("complex", meta["dim"], meta["E"], meta["R"],
                    {"eval.batch_size": meta["batch_size"], "entity_ranking.metrics_per.head_and_tail": True})
    ds = dataset_from(c, f)
    model = KgeModel.create(c, ds)
    set_tables(model, f["ent"], f["rel"])
    trace = EntityRankingJob(c, ds, model=model).run()
    E = meta["E"]
    for slot, d in (("head", "s"), ("tail", "o")):
        for ranking, suffix in (("raw", ""), ("filt", "_filtered"), ("filt_test", "_filtered_with_test")):
            r = f[f"full_{d}_{ranking}"].astype(np.float64)
            assert trace[f"mean_rank{suffix}_{slot}"] == pytest.approx((r + 1).mean(), rel=1e-6)
            assert trace[f"mean_reciprocal_rank{suffix}_{slot}"] == pytest.approx((1 / (r + 1)).mean(), rel=1e-5)
            assert trace[f"hits_at_10{suffix}_{slot}"] == pytest.approx((r < 10).mean(), abs=1e-7)
    assert E > 10
    n_q = 2 * len(f["tri_valid"])
    for key, groups in (("relation_type", ds.index("relations_per_type")),
                        ("argument_frequency", ["relation_" + q for q in ("25%", "50%", "75%", "top")])):
        c2 = base_config("complex", meta["dim"], meta["E"], meta["R"],
                         {"eval.batch_size": meta["batch_size"], "entity_ranking.metrics_per." + key: True})
        t2 = EntityRankingJob(c2, ds, model=model).run()
        assert t2["mean_rank_filtered"] == trace["mean_rank_filtered"]
        # mean rank is a per-group average: weighting by the group sizes gives the overall mean back
        sizes = {}
        p = f["tri_valid"][:, 1]
        for g in groups:
            if key == "relation_type":
                sizes[g] = 2 * int(np.isin(p, list(ds.index("relations_per_type")[g])).sum())
            else:
                sizes[g] = 2 * int(np.isin(p, list(ds.index("frequency_percentiles")["relation"][g[9:]])).sum())
        assert sum(sizes.values()) == n_q
        total = sum(t2[f"mean_rank_filtered_{g}"] * k for g, k in sizes.items())
        assert total / n_q == pytest.approx(trace["mean_rank_filtered"], rel=1e-5)


# ------------------------------------------------------------------------------ C1 toy


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_c1_toy_complex_options_trajectory_vs_reference(precision):
    """examples/toy-complex-train.yaml's options through TrainingJob._run: six epochs of
    1vsAll with the lp penalty, validation after every epoch and ReduceLROnPlateau on the
    validation metric, batches in the recorded order.  Compared with the reference's run:
    learning rate schedule exactly (it depends on the order of the validation metrics),
    per-epoch loss / penalty, every validation metric, the final tables."""
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, "train_toy_complex.npz"))
    meta = json.loads(str(f["meta"]))
    c = base_config("complex", meta["dim"], meta["E"], meta["R"], {
        "train.type": "1vsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": meta["lr"]},
        "train.lr_scheduler": meta["lr_scheduler"], "train.lr_scheduler_args": meta["lr_scheduler_args"],
        "lookup_embedder.regularize_weight": meta["regularize_weight"],
        "train.batch_size": meta["batch_size"], "train.max_epochs": meta["max_epochs"],
        "valid.every": meta["valid_every"], "valid.early_stopping.patience": 0,
        "eval.batch_size": meta["eval_batch_size"], "engine.precision": precision,
    })
    assert c.get("valid.metric") == meta["valid_metric"]
    ds = dataset_from(c, f)
    job = TrainingJob.create(c, ds)
    set_tables(job.model, f["ent0"], f["rel0"])
    perms = torch.from_numpy(f["perms"].astype(np.int64))
    bs = meta["batch_size"]

    def batches():  # the recorded order instead of the job's own shuffle
        perm = perms[job.epoch - 1]
        for b in range(0, len(perm), bs):
            yield perm[b:b + bs]

    job._batches = batches
    traces = job.run()
    ref_epochs = json.loads(str(f["epochs"]))
    ref_valids = json.loads(str(f["valids"]))
    assert len(traces) == len(ref_epochs) and len(job.valid_trace) == len(ref_valids)
    # the penalty is part of the recorded step, and the step is recorded anew after each lr change
    assert job._graph_step is not None and job._graph_step.graph is not None, job._graph_step.error
    assert job._graph_step.hyper[0][0] == ref_epochs[-1]["lr"][0] < meta["lr"]  # the last epoch's rate
    for t, r in zip(traces, ref_epochs):
        assert t["epoch"] == r["epoch"] and t["batches"] == r["batches"] and t["size"] == r["size"]
        assert t["lr"] == pytest.approx(r["lr"], rel=1e-12), f"lr schedule at epoch {r['epoch']}"
        assert t["avg_loss"] == pytest.approx(r["avg_loss"], rel=2e-4), r["epoch"]
        assert t["avg_penalty"] == pytest.approx(r["avg_penalty"], rel=2e-4), r["epoch"]
        assert t["avg_cost"] == pytest.approx(r["avg_cost"], rel=2e-4), r["epoch"]
    for t, r in zip(job.valid_trace, ref_valids):
        assert t["epoch"] == r["epoch"]
        for k, v in r.items():
            if k.startswith("mean_rank"):
                assert t[k] == pytest.approx(v, rel=0.02), (r["epoch"], k)
            elif k.startswith("mean_reciprocal_rank"):
                assert t[k] == pytest.approx(v, rel=0.05, abs=1e-3), (r["epoch"], k)
    assert [g["lr"] for g in job.optimizer.param_groups] == pytest.approx(list(f["final_lr"]), rel=1e-12)
    e1, r1 = tables(job.model)
    # 120 Adagrad steps: early steps move every element by ~lr whatever the gradient's size,
    # so the tables are compared by their overall distance from the reference's
    assert np.abs(e1 - f["ent1"]).mean() < 2e-3 * np.abs(f["ent1"]).mean()
    assert np.abs(r1 - f["rel1"]).mean() < 2e-3 * np.abs(f["rel1"]).mean()


# ------------------------------------------------------------------------------ C3 KvsAll


def _example_ids(job, queries, qtype):
    """This build's example ids (positions in its own (sp_, _po) index order) of the
    reference batch's queries."""
    ids = []
    for (a, b), qt in zip(queries.tolist(), qtype.tolist()):
        ix = job.query_indexes[qt]
        start = 0 if qt == 0 else job.query_last_example[qt - 1]
        ids.append(start + ix._dict()[(a, b)])
    return torch.tensor(ids, dtype=torch.int64)


@pytest.mark.parametrize("query_types", [["sp_", "_po"], ["sp_", "s_o", "_po"]], ids=["sp_po", "sp_so_po"])
@pytest.mark.parametrize("fused", [True, False], ids=["fused_kl", "torch_kl"])
@pytest.mark.parametrize("precision,atol", [("fp32", 1e-4), ("bf16x3", 2e-4)])
def test_c3_kvsall_trajectory_vs_reference(precision, atol, fused, query_types):
    """Three reference KvsAll batches (DistMult, sp_ + _po queries, label smoothing 0.1, KL,
    Adagrad): the same queries with the same label sets, the loss the reference reports per
    batch (its last query type's, train.py:747) and the tables after the three steps.  With
    (s, ?, o) queries as well: relation targets through score_so, not smoothed (train.py:715-751)."""
    from kge.job import TrainingJob

    name = "train_kvsall_so_distmult.npz" if "s_o" in query_types else "train_kvsall_distmult.npz"
    f = np.load(os.path.join(GOLDEN, name))
    meta = json.loads(str(f["meta"]))
    assert meta["query_types"] == query_types
    c = base_config("distmult", meta["dim"], meta["E"], meta["R"], {
        "train.type": "KvsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": meta["lr"]},
        "train.batch_size": meta["batch_size"], "KvsAll.label_smoothing": meta["label_smoothing"],
        "KvsAll.query_types.s_o": "s_o" in query_types,
        "engine.precision": precision, "engine.fused_loss": fused})
    ds = dataset_from(c, f)
    job = TrainingJob.create(c, ds)
    set_tables(job.model, f["ent0"], f["rel0"])
    job._prepare()
    assert job.query_types == meta["query_types"]
    ent_w = job.model._entity_embedder._embeddings.weight
    rel_w = job.model._relation_embedder._embeddings.weight
    gtol = 5e-6 if precision == "fp32" else 1e-4
    batches = []
    for b in range(meta["num_batches"]):
        queries, qtype, coords = f[f"queries_{b}"], f[f"qtype_{b}"], f[f"label_coords_{b}"]
        ids = _example_ids(job, queries, qtype)
        # the label sets this build's index holds for these queries are the reference's
        for row, (ex, qt) in enumerate(zip(ids.tolist(), qtype.tolist())):
            ix = job.query_indexes[qt]
            e = ex - (0 if qt == 0 else job.query_last_example[qt - 1])
            mine = ix.values[ix.offsets[e]:ix.offsets[e + 1]]
            assert sorted(mine.tolist()) == sorted(coords[coords[:, 0] == row, 1].tolist())
        batches.append(ids)
        # the batch's true triples, one per (query, label) in batch order (train.py:625-674)
        assert np.array_equal(job._batch_triples(ids.numpy()).numpy(), f[f"triples_{b}"])
        # (1) from the reference's tables before this batch: its loss and its gradients
        set_tables(job.model, f[f"ent_before_{b}"], f[f"rel_before_{b}"])
        job.optimizer.zero_grad()
        res = job._process_batch(b, {"examples": ids})
        assert float(res.avg_loss) == pytest.approx(float(f["losses"][b]), rel=2e-5)
        for w, key in ((ent_w, f"g_ent_{b}"), (rel_w, f"g_rel_{b}")):
            err = np.abs(w.grad.cpu().numpy() - f[key]).max() / np.abs(f[key]).max()
            assert err < gtol, (b, key, err)
    # (2) free-running from the initial tables: three Adagrad steps.  Adagrad's first steps
    # move an element by ~lr whatever the size of its gradient, so an element whose gradient
    # nearly cancels is ill-conditioned; all but a handful of elements must agree to atol
    set_tables(job.model, f["ent0"], f["rel0"])
    job.optimizer = type(job.optimizer)(job.optimizer.param_groups[0]["params"], lr=meta["lr"])
    losses = []
    for b, ids in enumerate(batches):
        job.optimizer.zero_grad()
        res = job._process_batch(b, {"examples": ids})
        job.optimizer.step()
        losses.append(res.avg_loss)
    np.testing.assert_allclose(losses, f["losses"], rtol=2e-5)
    e1, r1 = tables(job.model)
    for got, want in ((e1, f["ent1"]), (r1, f["rel1"])):
        diff = np.abs(got - want)
        n_off, mean_off = int((diff > atol).sum()), float(diff.mean())
        assert n_off <= max(4, 1e-3 * diff.size) and mean_off < 1e-5, (n_off, mean_off)


def test_c3_kvsall_step_at_wn18rr_size_vs_float64():
    """One KvsAll step of configs[2] at full size -- DistMult-512, E = 40,943, 512 examples
    (sp_ and _po queries mixed, label smoothing) -- through the job's fused path: the loss
    and the gradients of both tables against torch CPU float64 autograd of the reference
    formulas (distmult.py:14-26; train.py:698-751; loss.py:209-213)."""
    from kge import Dataset
    from kge.job import TrainingJob

    c = base_config("distmult", 512, 1, 1, {
        "train.type": "KvsAll", "train.batch_size": 512, "KvsAll.label_smoothing": 0.1,
        "lookup_embedder.initialize_args": {"mean": 0.0, "std": 0.1}})
    ds = Dataset.synthetic(c, "wn18rr", seed=0)
    E, R = ds.num_entities(), ds.num_relations()
    assert (E, R) == (40943, 11)
    torch.manual_seed(0)
    job = TrainingJob.create(c, ds)
    job._prepare()
    ex = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(3))[:512]
    job.optimizer.zero_grad()
    res = job._process_batch(0, {"examples": ex})
    torch.cuda.synchronize()
    g_ent = job.model._entity_embedder._embeddings.weight.grad.cpu().double()
    g_rel = job.model._relation_embedder._embeddings.weight.grad.cpu().double()

    ent = job.model._entity_embedder._embeddings.weight.detach().cpu().double().requires_grad_()
    rel = job.model._relation_embedder._embeddings.weight.detach().cpu().double().requires_grad_()
    exn = ex.numpy()
    last = None
    start = 0
    for qi, qt in enumerate(job.query_types):
        end = job.query_last_example[qi]
        sel = exn[(exn >= start) & (exn < end)] - start
        start = end
        ix = job.query_indexes[qi]
        q = torch.from_numpy(ix.keys[sel].astype(np.int64))
        labels = torch.zeros(len(sel), E, dtype=torch.float64)
        for row, e in enumerate(sel):
            labels[row, torch.from_numpy(ix.values[ix.offsets[e]:ix.offsets[e + 1]].astype(np.int64))] = 1.0
        labels = (1.0 - 0.1) * labels + 1.0 / E
        if qt == "sp_":
            scores = (ent[q[:, 0]] * rel[q[:, 1]]) @ ent.t()
        else:
            scores = (ent[q[:, 1]] * rel[q[:, 0]]) @ ent.t()
        loss = torch.nn.functional.kl_div(torch.log_softmax(scores, 1),
                                          torch.nn.functional.normalize(labels, p=1, dim=1), reduction="sum") / 512
        loss.backward()
        last = float(loss.detach())
    assert float(res.avg_loss) == pytest.approx(last, rel=1e-5)
    for got, ref, name in ((g_ent, ent.grad, "entity"), (g_rel, rel.grad, "relation")):
        err = float((got - ref).abs().max() / ref.abs().max())
        assert err < 1e-4, (name, err)


# ------------------------------------------------------------------------------ C4 negative sampling


@pytest.mark.parametrize("impl", ["triple", "all", "batch"])
@pytest.mark.parametrize("fixture", ["rotate", "complex", "rotate_n128", "complex_n128", "transe_n128"])
def test_c4_negative_sampling_steps_vs_reference(fixture, impl):
    """Two reference negative-sampling batches (KL with the positive in column 0, eight
    negatives per corrupted slot, Adagrad) with the reference sampler's negatives injected:
    per-batch loss and the tables after both steps, for every scoring implementation.  The
    _n128 fixtures carry 128 negatives per slot: lists the "triple" implementation scores in
    ascending candidate order (kge_score_cand_ordered), results in the reference's columns."""
    from kge import engine
    from kge.job import TrainingJob

    f = np.load(os.path.join(GOLDEN, f"train_ns_{fixture}.npz"))
    meta = json.loads(str(f["meta"]))
    model = meta["model"]
    ordered = engine._cand_order(torch.zeros(meta["batch_size"], 1 + meta["num_negatives"], dtype=torch.int64,
                                             device="cuda"), meta["E"]) is not None
    assert ordered == fixture.endswith("_n128")
    if model == "transe" and impl != "triple":
        # the fixture is the reference's "triple" run: score_spo = -pairwise_distance (eps 1e-6
        # inside the norm, transe.py:17), while "all" / "batch" score with -cdist (no eps,
        # transe.py:19-23) -- the L1 gradients sign(x + eps) and sign(x) differ wherever
        # |x| < 1e-6, a handful of the 5e5 components of such a step, in the reference too
        pytest.skip("TransE-L1: the reference's own implementations differ at |x| < eps")
    extra = {"train.type": "negative_sampling", "train.optimizer": "Adagrad",
             "train.optimizer_args": {"lr": meta["lr"]}, "train.batch_size": meta["batch_size"],
             "negative_sampling.num_samples.s": meta["num_negatives"], "negative_sampling.num_samples.o": -1,
             "negative_sampling.num_samples.p": 0, "negative_sampling.implementation": impl,
             "engine.precision": "fp32"}
    if meta["l_norm"] is not None:
        extra[f"{model}.l_norm"] = float(meta["l_norm"])
    c = base_config(model, meta["dim"], meta["E"], meta["R"], extra)
    ds = dataset_from(c, f)
    job = TrainingJob.create(c, ds)
    assert tuple(job.model._entity_embedder._embeddings.weight.shape) == f["ent0"].shape
    assert tuple(job.model._relation_embedder._embeddings.weight.shape) == f["rel0"].shape
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
        # from the reference's tables before this batch: its loss and its gradients
        set_tables(job.model, f[f"ent_before_{b}"], f[f"rel_before_{b}"])
        job.optimizer.zero_grad()
        res = job._process_batch(b, batch)
        assert float(res.avg_loss) == pytest.approx(float(f["losses"][b]), rel=2e-5)
        for w, key in ((ent_w, f"g_ent_{b}"), (rel_w, f"g_rel_{b}")):
            err = np.abs(w.grad.cpu().numpy() - f[key]).max() / np.abs(f[key]).max()
            assert err < 1e-5, (b, key, err)
    # free-running from the initial tables
    set_tables(job.model, f["ent0"], f["rel0"])
    job.optimizer = type(job.optimizer)(job.optimizer.param_groups[0]["params"], lr=meta["lr"])
    losses = []
    for b, batch in enumerate(batches):
        job.optimizer.zero_grad()
        res = job._process_batch(b, batch)
        job.optimizer.step()
        losses.append(res.avg_loss)
    np.testing.assert_allclose(losses, f["losses"], rtol=2e-5)
    e1, r1 = tables(job.model)
    for got, want in ((e1, f["ent1"]), (r1, f["rel1"])):
        diff = np.abs(got - want)
        n_off, mean_off = int((diff > 2e-4).sum()), float(diff.mean())
        assert n_off <= max(4, 1e-3 * diff.size) and mean_off < 1e-5, (n_off, mean_off)


def _rotate_cand_f64(ent, rel, eidx, ridx, cand, direction):
    """RotatE scores of each query against its own candidates, exact arithmetic
    (rotate.py:18-63: +sum_k |s o rot(p) - o|_C; the _po form through conj(rot))."""
    h = ent.shape[1] // 2
    e = ent[eidx]
    er, ei = e[:, :h], e[:, h:]
    cr, sr = torch.cos(rel[ridx]), torch.sin(rel[ridx])
    if direction == 0:  # s o rot(p)
        qr, qi = er * cr - ei * sr, er * sr + ei * cr
    else:  # o o conj(rot(p))
        qr, qi = er * cr + ei * sr, ei * cr - er * sr
    c = ent[cand]  # [n, k, d]
    dr, di = qr[:, None, :] - c[:, :, :h], qi[:, None, :] - c[:, :, h:]
    return torch.sqrt(dr * dr + di * di).sum(-1)


@pytest.mark.parametrize("direction", [0, 1], ids=["o_slot", "s_slot"])
def test_c4_candidate_kernel_at_rotate1024_1025_candidates_vs_float64(direction):
    """kge_score_cand and its backward at the configs[3] shape -- RotatE, entity dim 1024,
    1 positive + 1024 negatives per query, the FB15K-237 entity count -- through the model
    API (KgeModel.score_sp_cand / score_po_cand), against float64 autograd of the scorer's
    formula: scores, and the gradients that reach the entity and the relation table."""
    from kge import Dataset, KgeModel

    E, R, d, n, k = 14541, 237, 1024, 48, 1025
    c = base_config("rotate", d, E, R)
    torch.manual_seed(4)
    model = KgeModel.create(c, Dataset(c, None))
    model.train()
    ent_w = model._entity_embedder._embeddings.weight
    rel_w = model._relation_embedder._embeddings.weight
    assert tuple(rel_w.shape) == (R, d // 2)
    g = torch.Generator().manual_seed(8)
    eidx = torch.randint(0, E, (n,), generator=g)
    ridx = torch.randint(0, R, (n,), generator=g)
    cand = torch.randint(0, E, (n, k), generator=g)
    cand[:, 1] = cand[:, 0]  # repeated candidates inside a row
    cand[1] = cand[0]        # and across rows (the entity gradient sums them)
    w = torch.randn(n, k, generator=g)
    fn = model.score_sp_cand if direction == 0 else model.score_po_cand
    args = (eidx.cuda(), ridx.cuda()) if direction == 0 else (ridx.cuda(), eidx.cuda())
    got = fn(*args, cand.cuda())
    (got * w.cuda()).sum().backward()
    torch.cuda.synchronize()

    ent = ent_w.detach().cpu().double().requires_grad_()
    rel = rel_w.detach().cpu().double().requires_grad_()
    ref = _rotate_cand_f64(ent, rel, eidx, ridx, cand, direction)
    (ref * w.double()).sum().backward()
    err = float((got.detach().cpu().double() - ref.detach()).abs().max() / ref.detach().abs().max())
    assert err < 1e-5, err
    for gg, rr, name in ((ent_w.grad, ent.grad, "entity"), (rel_w.grad, rel.grad, "relation")):
        e = float((gg.cpu().double() - rr).abs().max() / rr.abs().max())
        assert e < 1e-4, (name, e)


# ------------------------------------------------------------------------------ C5 shard


def test_c5_wikidata5m_shard_score_sp_through_row_sharded_scorer():
    """configs[4] per GPU: one rank's shard of ceil(4,594,485 / 8) = 574,311 entity rows
    scored by 1,024 ComplEx-512 queries through RowShardedScorer (RCCL, world 1): sampled
    query rows against float64, and a dyadic copy of the tables bit-exact (every partial sum
    is exactly representable, in fp32 and in the bf16x3 split)."""
    import torch.distributed as dist
    from kge import _lib
    from kge.sharded import EngineOps, RowShardedScorer, shard_bounds

    E_full, R, d, B = 4594485, 822, 512, 1024
    lo, hi = shard_bounds(E_full, 8, 3)
    assert hi - lo == 574311
    created = not dist.is_initialized()
    if created:
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        g = torch.Generator(device="cuda").manual_seed(2)
        for regime in ("normal", "dyadic"):
            if regime == "normal":
                ent = torch.randn(hi - lo, d, device="cuda", generator=g) * 0.1
                rel = torch.randn(R, d, device="cuda", generator=g) * 0.1
            else:
                ent = torch.randint(-16, 17, (hi - lo, d), device="cuda", generator=g).float() / 8
                rel = torch.randint(-16, 17, (R, d), device="cuda", generator=g).float() / 8
            sc = RowShardedScorer(ent, lo, hi, E_full, rel, EngineOps(_lib.COMPLEX, _lib.PREC_BF16X3))
            s = torch.randint(lo, hi, (B,), device="cuda", generator=g)  # subjects this rank owns
            p = torch.randint(0, R, (B,), device="cuda", generator=g)
            scores = sc.score_sp(s, p)
            assert tuple(scores.shape) == (B, hi - lo)
            rows = torch.tensor([0, 1, 255, 256, 511, 777, 1023], device="cuda")
            e64, r64 = ent[s[rows] - lo].double(), rel[p[rows]].double()
            h = d // 2
            q = torch.cat([e64[:, :h] * r64[:, :h] - e64[:, h:] * r64[:, h:],
                           e64[:, :h] * r64[:, h:] + e64[:, h:] * r64[:, :h]], 1)
            ref = q @ ent.double().t()
            got = scores[rows].double()
            if regime == "dyadic":
                assert torch.equal(got, ref)
            else:
                err = float(((got - ref).abs().max(1).values / ref.abs().max(1).values).max())
                assert err < 2e-5, err
            # the shard's last columns (the ragged last tile) against the same reference
            assert torch.isfinite(scores[:, -300:]).all()
            del scores, sc, ent, ref, got
            torch.cuda.empty_cache()
    finally:
        if created:
            dist.destroy_process_group()


# ------------------------------------------------------------------------------ A5: the s_o combine


def test_score_so_and_generic_s_o_combine_vs_reference():
    """KgeModel.score_so (kge_model.py:684-704) -- all relations and a subset -- runs through
    RelationalScorer.score_emb's generic "s_o" expansion (kge_model.py:166-174), whose row-wise
    scores come from the engine's spo kernel.  Against reference-captured outputs."""
    from kge import Dataset, KgeModel

    f = np.load(os.path.join(GOLDEN, "score_so.npz"))
    for case in json.loads(str(f["meta"]))["cases"]:
        nm = case["name"]
        ent, rel = f[f"{nm}_ent"], f[f"{nm}_rel"]
        extra = {}
        if case["l_norm"] is not None:
            extra[f"{case['model']}.l_norm"] = float(case["l_norm"])
        c = base_config(case["model"], ent.shape[1], ent.shape[0], rel.shape[0], extra)
        m = KgeModel.create(c, Dataset(c, None))
        set_tables(m, ent, rel)
        s, o, psub = (torch.from_numpy(f[f"{nm}_{k}"]).cuda() for k in ("s", "o", "psub"))
        with torch.no_grad():
            so_all = m.score_so(s, o).cpu().numpy()
            so_sub = m.score_so(s, o, psub).cpu().numpy()
        for got, ref in ((so_all, f[f"{nm}_so_all"]), (so_sub, f[f"{nm}_so_sub"])):
            assert got.shape == ref.shape
            scale = np.abs(ref).max(axis=1, keepdims=True)
            assert float((np.abs(got - ref) / scale).max()) < 1e-5, nm
        with pytest.raises(ValueError):
            m.get_scorer().score_emb(torch.zeros(2, ent.shape[1]).cuda(), torch.zeros(2, rel.shape[1]).cuda(),
                                     torch.zeros(2, ent.shape[1]).cuda(), "sp*")


# ------------------------------------------------------------------------------ the reference's examples


@pytest.mark.parametrize("name,opts", [
    ("toy-complex-train", {
        "model": "complex", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.2},
        "train.lr_scheduler": "ReduceLROnPlateau", "train.lr_scheduler_args": {"mode": "max", "patience": 4},
        "lookup_embedder.dim": 100, "lookup_embedder.regularize_weight": 0.8e-7,
        "lookup_embedder.initialize": "normal_",
        "lookup_embedder.initialize_args": {"normal_": {"mean": 0.0, "std": 0.1}}}),
    ("toy-complex-train-sampling", {
        "model": "complex", "train.type": "negative_sampling", "train.optimizer": "Adagrad",
        "train.optimizer_args": {"lr": 0.6, "weight_decay": 0.4e-7}, "train.loss": "margin_ranking",
        "train.loss_arg": 2.0, "train.batch_size": 512, "lookup_embedder.dim": 100,
        "negative_sampling.num_samples.s": 30, "negative_sampling.num_samples.p": 30,
        "negative_sampling.num_samples.o": -1, "negative_sampling.filtering.s": True,
        "negative_sampling.filtering.o": True, "negative_sampling.filtering.p": True}),
    ("toy-transe-train", {
        "model": "transe", "train.batch_size": 256, "train.loss": "margin_ranking", "train.loss_arg": 4.0,
        "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.1}, "train.type": "negative_sampling"}),
], ids=lambda x: x if isinstance(x, str) else "")
def test_reference_training_examples_run(name, opts):
    """The options of the reference's runnable training examples (examples/toy-complex-train.yaml,
    toy-complex-train-sampling.yaml, toy-transe-train.yaml)
    through TrainingJob.run with validation every epoch, on the small dataset the reference's own
    tests ship: every key is accepted, the jobs train and evaluate, costs and metrics are finite."""
    from kge import Config, Dataset
    from kge.job import TrainingJob

    c = Config()
    c.set("model", opts["model"])
    c._import(opts["model"])
    c.set("job.device", "cuda")
    c.set("verbose", False)
    c.set("train.max_epochs", 3)
    c.set("valid.every", 1)
    for k, v in opts.items():
        if k != "model":
            c.set(k, v)
    ds = Dataset.create(c, folder=os.path.join(GOLDEN, "dataset_test"))
    torch.manual_seed(0)
    job = TrainingJob.create(c, ds)
    traces = job.run()
    assert len(traces) == 3 and len(job.valid_trace) == 3
    for t in traces:
        assert np.isfinite(t["avg_cost"]) and np.isfinite(t["avg_loss"]) and t["batches"] >= 1
    for v in job.valid_trace:
        assert 0.0 < v["mean_reciprocal_rank_filtered"] <= 1.0 and v["mean_rank"] >= 1.0
