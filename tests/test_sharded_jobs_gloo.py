"""World-size-2 gloo test (CPU) of the JOBS over a row-sharded entity table:
TrainingJob1vsAll (engine.row_sharded: vocab-parallel 1vsAll through
RowShardedScorer.train_1vsall_global, Adagrad state on each rank's rows, validation after
every epoch) and EntityRankingJob (per-shard rank counts, one all_reduce).

The jobs, the exchange logic and the optimizer wiring are the product code; only the per-shard
compute is injected (torch / numpy CPU ops restating the engine kernels), as this container
has no GPU.  Compared with the UNSHARDED objective computed independently here: torch
autograd of  sum_dir CE(Q E^T, target) / B  with torch.optim.Adagrad over the same batches
(train.py:1032-1062), and the CPU oracle's entity ranking (entity_ranking.py:79-577)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import kge_oracle as K
from test_sharded_gloo import OracleOps
from test_sharded_train_gloo import TorchOps, _prep

E, R, D, BS, EPOCHS, SEED = 41, 4, 8, 16, 2, 5


class JobOps(TorchOps):
    """TorchOps (training) + float64 eval ops."""

    def score(self, q, tab, out=None):
        s = (q.double() @ tab.double().T).float()
        if out is not None:
            out.copy_(s)
            return out
        return s

    spo = OracleOps.spo
    rank_counts = OracleOps.rank_counts

    def rank_rows(self, s, n_a, c0, part_a, part_b, f_col, t_col, greater, ties, refine=None):
        """kge_rank_rows on the CPU: the stacked block's counts, laid out [ranking][row]."""
        n = s.shape[0]
        for first, rows, (true_idx, true_score, f_ptr, t_ptr) in ((0, s[:n_a], part_a), (n_a, s[n_a:], part_b)):
            nb = rows.shape[0]
            g = torch.zeros(3 * nb, dtype=torch.int64)
            t = torch.zeros(3 * nb, dtype=torch.int64)
            OracleOps.rank_counts(self, rows, c0, true_idx, true_score, f_ptr, f_col, t_ptr, t_col, g, t)
            for r in range(1 + (f_ptr is not None) + (t_ptr is not None)):
                greater[r * n + first:r * n + first + nb] += g[r * nb:(r + 1) * nb]
                ties[r * n + first:r * n + first + nb] += t[r * nb:(r + 1) * nb]

    def rank_hist_multi(self, greater, ties, rows_per_hist, tie_handling, ranks, hists):
        assert tie_handling == "rounded_mean_rank"
        r = greater + ties // 2
        ranks.copy_(r)
        for h in range(hists.shape[0]):
            part = r[h * rows_per_hist:(h + 1) * rows_per_hist]
            hists[h] += torch.bincount(part, minlength=hists.shape[1]).float()


def _splits():
    rng = np.random.default_rng(1)
    seen, out = set(), []
    while len(out) < 120:
        t = (int(rng.integers(E)), int(rng.integers(R)), int(rng.integers(E)))
        if t not in seen:
            seen.add(t)
            out.append(t)
    t = np.array(out, dtype=np.int64)
    return {"train": t[:80], "valid": t[80:100], "test": t[100:]}


def _tables():
    g = torch.Generator().manual_seed(3)
    return torch.randn(E, D, generator=g) * 0.5, torch.randn(R, D, generator=g) * 0.5


def _config():
    from kge import Config

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cpu")
    c.set("verbose", False)
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    c.set("lookup_embedder.dim", D)
    c.set("train.type", "1vsAll")
    c.set("train.batch_size", BS)
    c.set("train.max_epochs", EPOCHS)
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.1})
    c.set("valid.every", 1)
    c.set("valid.early_stopping.patience", 0)
    c.set("eval.batch_size", 7)
    c.set("engine.eval_batch_size", 0)  # the batches of eval.batch_size as they are
    c.set("engine.eval_exchange_group", 3)  # several exchange groups per evaluation, the last one ragged
    c.set("random_seed.torch", SEED)
    return c


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


#: penalty cases: (weight, p, weighted) of the entity and of the relation embedder
PENALTIES = {"ent_weighted_l3": ((2e-2, 3, True), (1e-2, 2, False)),
             "ent_unweighted_l2": ((5e-3, 2, False), (2e-2, 3, True))}


def _set_penalties(job, case):
    m = job.model
    for e, (w, p, weighted) in zip((m._entity_embedder, m._relation_embedder), PENALTIES[case]):
        e.config.set(e.configuration_key + ".regularize_weight", w)
        e.config.set(e.configuration_key + ".regularize_args.p", p)
        e.config.set(e.configuration_key + ".regularize_args.weighted", weighted)
        assert e.penalty_active() and e.penalty_weighted() == weighted


def _lp(table, idx, w, p, weighted):
    """lookup_embedder.py:112-158 on the whole table."""
    if not weighted:
        return w / p * table.norm(p=p) ** p
    u, cnt = torch.unique(idx, return_counts=True)
    rows = table[u].abs() if p % 2 == 1 else table[u]
    return (w / p * (rows ** p * cnt.float().view(-1, 1))).sum() / len(idx)


def _worker(rank, world, port, out_q, penalties=None, bce_offset=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge import Dataset
        from kge.job import EntityRankingJob, TrainingJob

        c = _config()
        if bce_offset is not None:
            c.set("train.loss", "bce")
            c.set("train.loss_arg", bce_offset)
            c.set("valid.every", 0)
        ds = Dataset(c, None)
        ds._triples = {k: torch.from_numpy(v.astype(np.int32)) for k, v in _splits().items()}
        job = TrainingJob.create(c, ds)
        if penalties:
            _set_penalties(job, penalties)
        ent0, rel0 = _tables()
        with torch.no_grad():
            job.model._entity_embedder._embeddings.weight.copy_(ent0)
            job.model._relation_embedder._embeddings.weight.copy_(rel0)
        job.sharded_ops = JobOps()
        traces = job.run()
        assert job._sharded is not None and job._sharded.world == world
        lo, hi = job._sharded.lo, job._sharded.hi
        if bce_offset is not None:
            assert job._sharded.loss == ("bce", bce_offset) and job._sharded.scorer.collectives_last_step == 4
            job._sharded.sync_model()
            out_q.put((rank, [t["avg_loss"] for t in traces],
                       job.model._entity_embedder._embeddings.weight.detach().numpy().copy(),
                       job.model._relation_embedder._embeddings.weight.detach().numpy().copy()))
            return
        if penalties:
            job._sharded.sync_model()
            out_q.put((rank, [t["avg_loss"] for t in traces], [t["avg_penalty"] for t in traces],
                       job.model._entity_embedder._embeddings.weight.detach().numpy().copy(),
                       job.model._relation_embedder._embeddings.weight.detach().numpy().copy()))
            return
        state_rows = [tuple(st["sum"].shape) for st in job.optimizer.state.values()]
        job._sharded.sync_model()
        for k in ("head_and_tail", "relation_type", "argument_frequency"):
            c.set("entity_ranking.metrics_per." + k, True)
        ev = EntityRankingJob(c, ds, model=job.model)
        ev.sharded_ops = JobOps()
        ev.capture_ranks = True
        etrace = ev.run()
        out_q.put((rank, lo, hi, [t["avg_loss"] for t in traces],
                   [v["mean_reciprocal_rank_filtered_with_test"] for v in job.valid_trace], state_rows,
                   job.model._entity_embedder._embeddings.weight.detach().numpy().copy(),
                   job.model._relation_embedder._embeddings.weight.detach().numpy().copy(),
                   {k: v.copy() for k, v in ev.ranks.items()},
                   {k: v for k, v in etrace.items() if isinstance(v, float)}))
    finally:
        dist.destroy_process_group()


def _unsharded_reference(penalties=None, bce_offset=None):
    """The same training run without any sharding, by torch autograd."""
    splits = _splits()
    ent0, rel0 = _tables()
    ent = ent0.clone().requires_grad_(True)
    rel = rel0.clone().requires_grad_(True)
    opt = torch.optim.Adagrad([ent, rel], lr=0.1)
    gen = torch.Generator().manual_seed(SEED)
    train = torch.from_numpy(splits["train"])
    losses, valid_mrr, pens = [], [], []
    for _ in range(EPOCHS):
        perm = torch.randperm(len(train), generator=gen)
        tot = 0.0
        pen_tot, n_batches = 0.0, 0
        for b in range(0, len(train), BS):
            tr = train[perm[b:b + BS]]
            opt.zero_grad()
            loss = 0.0
            for direction, e_col, lab_col in ((0, 0, 2), (1, 2, 0)):
                q = _prep(direction, ent, tr[:, e_col], rel, tr[:, 1])
                if bce_offset is None:
                    loss = loss + torch.nn.functional.cross_entropy(q @ ent.T, tr[:, lab_col], reduction="sum") / len(tr)
                else:  # loss.py:137-158: BCEWithLogits(sum) on scores + offset against the one-hot rows
                    y = torch.zeros(len(tr), E)
                    y[torch.arange(len(tr)), tr[:, lab_col]] = 1.0
                    loss = loss + torch.nn.functional.binary_cross_entropy_with_logits(
                        q @ ent.T + bce_offset, y, reduction="sum") / len(tr)
            if penalties:  # kge_model.py:588-605: subjects, relations, objects
                (we, pe, ee), (wr, pr, er) = PENALTIES[penalties]
                pen = (_lp(ent, tr[:, 0], we, pe, ee) + _lp(rel, tr[:, 1], wr, pr, er)
                       + _lp(ent, tr[:, 2], we, pe, ee))
                pen_tot += float(pen.detach())
                loss = loss + pen
            n_batches += 1
            loss.backward()
            opt.step()
            tot += float(loss.detach()) * len(tr) - (float(pen.detach()) * len(tr) if penalties else 0.0)
        losses.append(tot / len(train))
        pens.append(pen_tot / n_batches)
        if penalties or bce_offset is not None:
            continue
        _, m = K.entity_ranking("complex", ent.detach().double().numpy(), rel.detach().double().numpy(), splits,
                                eval_split="valid", filter_splits=("train", "valid"), batch_size=7)
        valid_mrr.append(m["mean_reciprocal_rank_filtered_with_test"])
    if penalties:
        return losses, pens, ent.detach().numpy(), rel.detach().numpy()
    return losses, valid_mrr, ent.detach().numpy(), rel.detach().numpy()


def test_sharded_training_and_eval_jobs_world2_match_unsharded():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    ref_losses, ref_mrr, ref_ent, ref_rel = _unsharded_reference()
    splits = _splits()
    per = -(-E // world)
    for rank, lo, hi, losses, mrr, state_rows, ent, rel, ranks, metrics in res:
        assert (lo, hi) == (rank * per, min(E, (rank + 1) * per))
        # the optimizer state covers this rank's rows only (and the replicated relation table)
        assert sorted(state_rows) == sorted([(hi - lo, D), (R, D)])
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
        np.testing.assert_allclose(mrr, ref_mrr, rtol=1e-5)
        # after sync_model every rank holds the whole trained table
        np.testing.assert_allclose(ent, ref_ent, atol=2e-5)
        np.testing.assert_allclose(rel, ref_rel, atol=2e-5)
    # the sharded evaluation job on the trained model vs the oracle on the same tables
    oranks, ometrics = K.entity_ranking("complex", res[0][6].astype(np.float64), res[0][7].astype(np.float64),
                                        splits, eval_split="valid", filter_splits=("train", "valid"), batch_size=7,
                                        head_and_tail=True, relation_type=True, argument_frequency=True)
    assert any(k.endswith("_object_top") for k in ometrics) and any(k.endswith("_tail") for k in ometrics)
    for rank, *_, ranks, metrics in res:
        assert set(ranks) == set(oranks)
        for k, v in oranks.items():
            np.testing.assert_array_equal(ranks[k], v, err_msg=k)
        for k, v in ometrics.items():
            assert metrics[k] == pytest.approx(v, rel=1e-5, abs=1e-9), k


def test_sharded_training_job_with_bce_world2_matches_unsharded():
    """train.loss bce (with an offset) through the row-sharded TrainingJob1vsAll: every shard forms
    its slice of the loss and of the gradient by itself (4 collectives per step, no statistics
    exchange); loss trajectory and trained tables equal the unsharded autograd run."""
    world, offset = 2, -2.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, None, offset)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    ref_losses, _, ref_ent, ref_rel = _unsharded_reference(bce_offset=offset)
    for rank, losses, ent, rel in res:
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
        np.testing.assert_allclose(ent, ref_ent, atol=2e-5)
        np.testing.assert_allclose(rel, ref_rel, atol=2e-5)


@pytest.mark.parametrize("case", sorted(PENALTIES))
def test_sharded_training_with_embedding_penalties_world2_matches_unsharded(case):
    """Lp penalties on a row-sharded table: every rank differentiates the entity terms over its
    own rows (frequency-weighted over the global batch's indexes that fall into them, or its
    share of the whole-table norm), the relation term is replicated; loss, reported penalty and
    trained tables equal the unsharded run's."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    ref_losses, ref_pens, ref_ent, ref_rel = _unsharded_reference(case)
    assert min(ref_pens) > 0
    for rank, losses, pens, ent, rel in res:
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
        np.testing.assert_allclose(pens, ref_pens, rtol=1e-5)
        np.testing.assert_allclose(ent, ref_ent, atol=2e-5)
        np.testing.assert_allclose(rel, ref_rel, atol=2e-5)


def _worker_reciprocal(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge.sharded import RowShardedScorer, shard_bounds

        g = torch.Generator().manual_seed(0)
        ent = torch.randn(E, D, generator=g)
        rel = torch.randn(2 * R, D, generator=g)  # reciprocal model: relations r and r + R
        lo, hi = shard_bounds(E, world, rank)
        sc = RowShardedScorer(ent[lo:hi].clone(), lo, hi, E, rel, OracleOps())
        ge = torch.Generator().manual_seed(7)
        B = 9
        es, ep, eo = (torch.randint(0, n, (B,), generator=ge) for n in (E, R, E))
        f_ptr = torch.arange(0, 2 * B + 1, 2)
        f_col = torch.randint(0, E, (2 * B,), generator=ge)
        counts = sc.rank_counts(es, ep, eo, (f_ptr, f_col), (f_ptr, f_col), p_inverse=ep + R)
        out_q.put((rank, counts.numpy(), [x.numpy() for x in (es, ep, eo, f_ptr, f_col)]))
    finally:
        dist.destroy_process_group()


def test_sharded_rank_counts_reciprocal_relations_world2():
    """The (?, p, o) side of a reciprocal-relations model is the sp_ score of (o, p + R, ?),
    queries and true score alike (reciprocal_relations_model.py:57-74): sharded counts vs
    the unsharded computation."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_reciprocal, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    g = torch.Generator().manual_seed(0)
    ent = torch.randn(E, D, generator=g)
    rel = torch.randn(2 * R, D, generator=g)
    es, ep, eo, f_ptr, f_col = (torch.from_numpy(x) for x in res[0][2])
    B = len(es)
    ops = OracleOps()
    ref = np.zeros((2, 2, 3 * B), np.int64)
    sides = ((es, ep, eo, ops.spo(ent[es], rel, ep, ent[eo])), (eo, ep + R, es, ops.spo(ent[eo], rel, ep + R, ent[es])))
    for di, (e_idx, rel_ids, tgt, true) in enumerate(sides):
        scores = ops.score(ops.prep(0, ent, e_idx, rel, rel_ids), ent)
        gr = torch.zeros(3 * B, dtype=torch.int64)
        ti = torch.zeros(3 * B, dtype=torch.int64)
        ops.rank_counts(scores, 0, tgt, true, f_ptr, f_col, None, None, gr, ti)
        ref[di, 0], ref[di, 1] = gr.numpy(), ti.numpy()
    for _, counts, _ in res:
        np.testing.assert_array_equal(counts[:, :, :2 * B], ref[:, :, :2 * B])
    # and the two sides really differ (an undirected true score would be wrong here)
    assert not np.array_equal(ref[0], ref[1])


@pytest.mark.parametrize("train_type", ["KvsAll", "negative_sampling"])
def test_row_sharded_on_is_refused_by_the_training_types_that_do_not_shard(train_type):
    """engine.row_sharded: on with a training type that has no row-sharded step fails loudly
    instead of silently training replicas."""
    from kge import Dataset
    from kge.job import TrainingJob

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        c = _config()
        c.set("train.type", train_type)
        c.set("engine.row_sharded", "on")
        ds = Dataset(c, None)
        ds._triples = {k: torch.from_numpy(v.astype(np.int32)) for k, v in _splits().items()}
        job = TrainingJob.create(c, ds)
        with pytest.raises(NotImplementedError, match="does not shard"):
            job._prepare()
        c.set("engine.row_sharded", "auto")  # a world of one process: nothing to say, nothing sharded
        job._replicas_only()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("train_loss", ["bce_mean", "soft_margin"])
def test_row_sharded_1vsall_refuses_losses_it_cannot_split_by_rows(train_loss):
    """Row-sharded 1vsAll training serves kl and bce; any other train.loss fails loudly when the
    sharded step is set up instead of training on a wrong objective."""
    from kge import Dataset
    from kge.job import TrainingJob

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        c = _config()
        c.set("train.loss", train_loss)
        c.set("engine.row_sharded", "on")
        ds = Dataset(c, None)
        ds._triples = {k: torch.from_numpy(v.astype(np.int32)) for k, v in _splits().items()}
        job = TrainingJob.create(c, ds)
        job.sharded_ops = JobOps()
        with pytest.raises(NotImplementedError, match="kl and bce"):
            job._prepare()
    finally:
        dist.destroy_process_group()


def _worker_shard_only(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge import Dataset
        from kge.job import TrainingJob

        c = _config()
        ds = Dataset(c, None)
        ds._triples = {k: torch.from_numpy(v.astype(np.int32)) for k, v in _splits().items()}
        job = TrainingJob.create(c, ds)
        ent0, rel0 = _tables()
        with torch.no_grad():
            job.model._entity_embedder._embeddings.weight.copy_(ent0)
            job.model._relation_embedder._embeddings.weight.copy_(rel0)
        job.sharded_ops = JobOps()
        seen = []

        def after_epoch(j, trace):  # what the model holds while the job trains
            emb = j.model._entity_embedder
            seen.append((tuple(emb._embeddings.weight.shape), emb.shard, j._sharded.scorer.collectives_last_step,
                         emb._embeddings.weight.detach().numpy().copy()))

        job.post_epoch_hooks.append(after_epoch)
        job.run()
        emb = job.model._entity_embedder
        after_run = (tuple(emb._embeddings.weight.shape), emb.shard)
        # the unsharded scoring path takes the model again once sync_model has run (job.run ends
        # with it): here it gets as far as the engine, which refuses CPU tensors ...
        from kge._lib import EngineError

        try:
            job.model.score_sp(torch.tensor([1, 2]), torch.tensor([0, 1]))
            full_ok = False
        except EngineError:
            full_ok = True
        best = job.best_state_full()
        key = "_entity_embedder._embeddings.weight"
        best_shard_shape = tuple(job.best_state[key].shape)
        best_epoch = max(range(len(job.valid_trace)), key=lambda i: job.valid_trace[i][c.get("valid.metric")])
        # ... and a further batch cuts the model down to this rank's rows again
        job._sharded.process_batch({"triples": ds.split("train")[:BS].long()})
        refused = False
        try:
            job.model.score_sp(torch.tensor([1]), torch.tensor([0]))
        except RuntimeError as e:
            refused = "row-sharded" in str(e)
        out_q.put((rank, job._sharded.lo, job._sharded.hi, seen, after_run, full_ok,
                   best[key].numpy().copy(), best_shard_shape, best_epoch, emb.shard, refused))
    finally:
        dist.destroy_process_group()


def test_sharded_job_holds_only_its_rows_and_best_state_reassembles():
    """While a row-sharded job trains, the model's entity parameter is [hi - lo, d] (the whole
    table exists only after sync_model); a step takes 4 collectives; best_state keeps every
    rank's rows of the best epoch and best_state_full() assembles that epoch's whole table."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_shard_only, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert res[0][8] == res[1][8]  # both ranks picked the same best epoch
    best_epoch = res[0][8]
    for rank, lo, hi, seen, after_run, full_ok, best_full, best_shard_shape, _, shard_again, refused in res:
        assert len(seen) == EPOCHS
        for shape, shard, collectives, _rows in seen:
            assert shape == (hi - lo, D) and shard == (lo, hi) and collectives == 4
        assert after_run == ((E, D), None) and full_ok
        assert best_shard_shape == (hi - lo, D) and best_full.shape == (E, D)
        assert shard_again == (lo, hi) and refused
        # the assembled best table is every rank's rows as they were after the best epoch
        for r2 in res:
            np.testing.assert_array_equal(best_full[r2[1]:r2[2]], r2[3][best_epoch][3])
    np.testing.assert_array_equal(res[0][6], res[1][6])


def test_exchange_plan_slots():
    """ExchangePlan: owner-major slots with equal blocks of cap rows per rank."""
    from kge.sharded import ExchangePlan

    e = np.array([5, 0, 9, 3, 7, 1, 8, 4])  # per = 4: owners 1 0 2 0 1 0 2 1
    plans = [ExchangePlan(e, 4, 3, r, "cpu") for r in range(3)]
    assert [p.cap for p in plans] == [3, 3, 3] and [p.count for p in plans] == [3, 3, 2]
    assert plans[0].mine.tolist() == [1, 3, 5] and plans[1].mine.tolist() == [0, 4, 7] and plans[2].mine.tolist() == [2, 6]
    assert plans[0].slot.tolist() == [3, 0, 6, 1, 4, 2, 7, 5]
    # gathering rank-major blocks of cap rows and reading them through slot gives the batch order back
    blocks = np.full(9, -1)
    for r, p in enumerate(plans):
        blocks[r * 3:r * 3 + p.count] = e[p.mine.numpy()]
    np.testing.assert_array_equal(blocks[plans[0].slot.numpy()], e)
    empty = ExchangePlan(np.zeros(0, np.int64), 4, 2, 0, "cpu")
    assert empty.cap == 1 and empty.count == 0 and empty.slot.numel() == 0
