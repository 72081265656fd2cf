"""GPU parity of the negative-sampling path (RotatE-1024 with 1,024 negatives at FB15K-237 size included):

* kge_score_cand (+ backward) against the oracle's score_spo semantics on the expanded
  B x (1 + N) triples, for all five scorers, both corrupted slots, duplicate candidates;
* the job's implementations agree: fused triple == expanded-triple score_spo == all == batch;
* the device sampler honours its constraints (range, shared drop of the positive,
  filtering of training positives);
* an NS training run (RotatE, FB15K-237 shape subset) lowers its loss.
"""
import glob
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_scorer_fixture
from oracle import kge_oracle as K

pytestmark = pytest.mark.gpu

MODEL_IDS = {"complex": 0, "distmult": 1, "rescal": 2, "transe": 3, "rotate": 4, "cp": 5, "simple": 6}
FILES = sorted(glob.glob(os.path.join(GOLDEN, "scorer_*_normal.npz")))


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib
    _lib.lib()
    return _lib


@pytest.mark.parametrize("slot", ["o", "s"])
@pytest.mark.parametrize("fn", FILES, ids=lambda f: os.path.basename(f)[7:-11])
def test_score_cand_vs_oracle(L, fn, slot):
    from kge import engine

    f = load_scorer_fixture(fn)
    meta = json.loads(str(f["meta"]))
    model, ln = meta["model"], meta["l_norm"] or 1.0
    ent64, rel64 = f["ent"].astype(np.float64), f["rel"].astype(np.float64)
    E, R = ent64.shape[0], rel64.shape[0]
    rng = np.random.default_rng(7)
    n, k = 9, 17
    s, p, o = rng.integers(0, E, n), rng.integers(0, R, n), rng.integers(0, E, n)
    cand = rng.integers(0, E, (n, k))
    cand[:, 3] = cand[:, 5]  # duplicates within a row (atomic accumulation in backward)
    # expanded triples exactly as the reference's "triple" implementation builds them
    S_, P_, O_ = np.repeat(s, k), np.repeat(p, k), np.repeat(o, k)
    if slot == "o":
        O_ = cand.reshape(-1)
    else:
        S_ = cand.reshape(-1)
    ref = K.score_emb(model, ent64[S_], rel64[P_], ent64[O_], "spo", ln).reshape(n, k)
    w = rng.standard_normal((n, k))
    zeros = np.zeros((n * k, E))
    g_ent_ref, g_rel_ref = K.model_grads(model, ent64, rel64, S_, P_, O_, zeros, zeros, w.reshape(-1), ln)

    ent = torch.tensor(f["ent"], device="cuda", requires_grad=True)
    rel = torch.tensor(f["rel"], device="cuda", requires_grad=True)
    d = L.DIR_SP if slot == "o" else L.DIR_PO
    eidx = torch.from_numpy(s if slot == "o" else o).cuda()
    out = engine.score_cand(MODEL_IDS[model], d, ln, ent, eidx, rel, torch.from_numpy(p).cuda(),
                            torch.from_numpy(cand).cuda())
    (out * torch.from_numpy(w).float().cuda()).sum().backward()
    got = out.detach().cpu().numpy()
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() <= 2e-6 * scale, np.abs(got - ref).max() / scale
    ge, gr = ent.grad.cpu().numpy(), rel.grad.cpu().numpy()
    assert np.abs(ge - g_ent_ref).max() <= 1e-5 * np.abs(g_ent_ref).max()
    assert np.abs(gr - g_rel_ref).max() <= 1e-5 * np.abs(g_rel_ref).max()


def _ns_job(model, impl, num_neg=31, dim=64, shared=False, filtering=False, E=500, R=11):
    from kge import Config, Dataset
    from kge.job import TrainingJob

    c = Config()
    c.set("model", model)
    c._import(model)
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", dim)
    c.set("train.type", "negative_sampling")
    c.set("train.loss", "kl")
    c.set("negative_sampling.num_samples.s", num_neg)
    c.set("negative_sampling.implementation", impl)
    c.set("negative_sampling.shared", shared)
    c.set("negative_sampling.filtering.s", filtering)
    c.set("negative_sampling.filtering.o", filtering)
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.1})
    c.set("train.batch_size", 128)
    c.set("verbose", False)
    torch.manual_seed(0)
    ds = Dataset.synthetic(c, "toy", seed=0, num_entities=E, num_relations=R, sizes=(3000, 100, 100))
    job = TrainingJob.create(c, ds)
    job._prepare()
    return job


@pytest.mark.parametrize("model,ln", [("distmult", 1.0), ("transe", 1.0), ("transe", 2.0), ("rotate", 1.0),
                                      ("rotate", 2.0)])
@pytest.mark.parametrize("d", [128, 1024, 30])  # 30: rows float4 loads cannot read (scalar kernels)
def test_score_cand_ordered_lists_vs_plain(L, model, ln, d):
    """The engine orders long candidate lists (ascending per query, kge_score_cand_ordered /
    kge_score_cand_bwd_q_ordered) when the rows repeat across queries: the scores must be the
    SAME BITS as kge_score_cand's in the caller's column order (a pair's arithmetic does not
    depend on its position), the gradients equal up to the summation order."""
    from kge import engine

    torch.manual_seed(5)
    E, R, n, k = 900, 7, 70, 300
    kind = MODEL_IDS[model]
    d_r = d // 2 if model == "rotate" else d
    ent = (torch.randn(E, d, device="cuda") * 0.3).requires_grad_()
    rel = (torch.randn(R, d_r, device="cuda") * 0.3).requires_grad_()
    eidx = torch.randint(0, E, (n,), device="cuda")
    ridx = torch.randint(0, R, (n,), device="cuda")
    cand = torch.randint(0, E, (n, k), device="cuda")
    cand[:, 7] = cand[:, 11]  # duplicates within a row
    w = torch.randn(n, k, device="cuda")
    w[3, 5] = 0.0  # pairs without gradient are skipped
    assert engine._cand_order(cand, E) is not None
    for direction in (L.DIR_SP, L.DIR_PO):
        out = engine.score_cand(kind, direction, ln, ent, eidx, rel, ridx, cand)
        (out * w).sum().backward()
        ge, gr = ent.grad.clone(), rel.grad.clone()
        ent.grad = rel.grad = None
        # the plain kernels on the same inputs
        with torch.no_grad():
            q = L.prep_query(kind, direction, ent, eidx, rel, ridx, n, d, d_r)
            s = L.score_cand(kind, ln, direction, q, ent, cand)
            assert torch.equal(out, s)
            dq = torch.empty_like(q)
            d_ent, d_rel = torch.zeros_like(ent), torch.zeros_like(rel)
            grouped = L.score_cand_bwd_ent(kind, ln, direction, q, ent, cand, s, w, d_ent)
            assert grouped == (d % 8 == 0)
            L.score_cand_bwd(kind, ln, direction, q, ent, cand, s, w, dq, None if grouped else d_ent)
            L.prep_query_bwd(kind, direction, ent, eidx, rel, ridx, n, d, d_r, dq, d_ent, d_rel)
        assert (ge - d_ent).abs().max() <= 2e-5 * d_ent.abs().max()
        assert (gr - d_rel).abs().max() <= 2e-5 * d_rel.abs().max()


@pytest.mark.parametrize("n,k,ld", [(5, 1, 1), (3, 2, 7), (64, 1025, 1025), (9, 300, 301), (2, 8192, 8192), (1, 777, 777),
                                    (4, 3, 3), (4, 5, 5), (7, 64, 64), (7, 255, 256), (7, 256, 256), (7, 257, 300),
                                    (3, 512, 512), (3, 1024, 1024), (3, 2048, 2048), (3, 2049, 2049)])
def test_sort_rows_is_torch_stable_sort(L, n, k, ld):
    """kge_sort_rows (bitonic network in LDS) against torch.sort(stable=True): ids and positions,
    with many repeated ids per row."""
    torch.manual_seed(n + k)
    buf = torch.randint(0, max(2, k // 3), (n, ld), device="cuda")
    buf[0, :k] = 2 ** 40 + 5  # large ids; a row of equal ids keeps its order
    x = buf[:, :k]
    srt, col = L.sort_rows(x)
    exp = torch.sort(x, dim=1, stable=True)
    assert torch.equal(srt, exp.values) and torch.equal(col, exp.indices)
    # with a bound on the ids (32-bit keys below 2^21 and up to 2,048 columns)
    buf[0, :k] = 7
    exp = torch.sort(x, dim=1, stable=True)
    for bound in (max(8, k // 3 + 1), 1 << 21, (1 << 21) + 1):
        srt, col = L.sort_rows(x, bound)
        assert torch.equal(srt, exp.values) and torch.equal(col, exp.indices), bound


@pytest.mark.parametrize("n,k,E", [(512, 1025, 14541), (70, 300, 900), (3, 40, 5000), (600, 33, 100), (1, 1, 1),
                                   (16, 64, 300000)])
def test_group_sorted_rows_is_the_counting_sort(L, n, k, E):
    """kge_group_sorted_rows (grouping from sorted candidate lists, LDS counters per entity range)
    against the bincount / cumsum grouping of the flattened candidate matrix: the same segment
    pointers, and every entity's segment holds exactly its pairs (in the caller's columns)."""
    torch.manual_seed(n * k)
    cand = torch.randint(0, E, (n, k), device="cuda")
    if k > 8:
        cand[:, 3] = cand[:, 5]  # duplicates within a row
        cand[0, :] = E - 1       # a row of one (the last) entity
    srt, col = L.sort_rows(cand)
    order, seg_ptr = L.group_sorted_rows(srt, col, E)
    flat = cand.reshape(-1)
    exp_ptr = torch.zeros(E + 1, dtype=torch.int64, device="cuda")
    exp_ptr[1:] = torch.cumsum(torch.bincount(flat, minlength=E), 0)
    assert torch.equal(seg_ptr, exp_ptr)
    # a permutation of all pairs, each in the segment of its entity
    assert torch.equal(torch.sort(order).values, torch.arange(n * k, device="cuda"))
    ent_of_slot = torch.repeat_interleave(torch.arange(E, device="cuda"), seg_ptr[1:] - seg_ptr[:-1])
    assert torch.equal(flat[order], ent_of_slot)


@pytest.mark.parametrize("ordered", [False, True])
def test_score_cand_rotate_dim_3072_vs_float64(L, ordered):
    """RotatE with 3,072-float entity rows (the backward takes up to 3,584): scores and both
    gradients against float64 autograd of rotate.py:18-50's arithmetic.  The vector form of the
    query-gradient pass would need more LDS than a kernel gets without asking: it runs its
    scalar form at this width."""
    from kge import engine

    torch.manual_seed(3)
    E, R, d = 600, 5, 3072
    n, k = (24, 420) if ordered else (5, 40)
    ent = (torch.randn(E, d, device="cuda") * 0.3).requires_grad_()
    rel = ((torch.rand(R, d // 2, device="cuda") * 2 - 1) * 3.14159).requires_grad_()
    eidx = torch.randint(0, E, (n,), device="cuda")
    ridx = torch.randint(0, R, (n,), device="cuda")
    cand = torch.randint(0, E, (n, k), device="cuda")
    w = torch.randn(n, k, device="cuda")
    assert (engine._cand_order(cand, E) is not None) == ordered
    out = engine.score_cand(MODEL_IDS["rotate"], L.DIR_SP, 1.0, ent, eidx, rel, ridx, cand)
    (out * w).sum().backward()
    e64, r64 = ent.detach().double().requires_grad_(), rel.detach().double().requires_grad_()
    h = d // 2
    s = e64[eidx]
    c, sn = torch.cos(r64[ridx]), torch.sin(r64[ridx])
    qr, qi = s[:, :h] * c - s[:, h:] * sn, s[:, :h] * sn + s[:, h:] * c
    o = e64[cand]  # [n, k, d]
    ref = torch.sqrt((qr[:, None] - o[..., :h]) ** 2 + (qi[:, None] - o[..., h:]) ** 2).sum(-1)
    (ref * w.double()).sum().backward()
    assert (out.double() - ref).abs().max() <= 2e-6 * ref.abs().max()
    assert (ent.grad.double() - e64.grad).abs().max() <= 2e-5 * e64.grad.abs().max()
    assert (rel.grad.double() - r64.grad).abs().max() <= 2e-5 * r64.grad.abs().max()


@pytest.mark.parametrize("num_neg", [31, 255])
@pytest.mark.parametrize("model", ["rotate", "complex", "transe", "cp", "simple"])
def test_ns_implementations_agree(model, num_neg):
    """Column 0 = the positive; same negatives through every scoring implementation (255
    negatives: the candidate lists are long enough for the engine to order them)."""
    job = _ns_job(model, "triple", num_neg=num_neg)
    tr = job.dataset.split("train")[:64].long().cuda()
    torch.manual_seed(1)
    for slot in (0, 2):
        neg = job._sampler.sample(tr, slot)
        fused = job._scores(tr, slot, neg)
        ref = {}
        for impl in ("all", "batch"):
            job._implementation = impl
            ref[impl] = job._scores(tr, slot, neg)
        job._implementation = "triple"
        t = tr.repeat(1, neg.shape[1] + 1).view(-1, 3)
        t[:, slot] = torch.cat((tr[:, [slot]], neg), 1).reshape(-1)
        ref["spo"] = job.model.score_spo(t[:, 0], t[:, 1], t[:, 2], direction="o" if slot == 2 else "s").view(64, -1)
        for name, r in ref.items():
            err = (fused - r).abs().max().item() / r.abs().max().item()
            assert err < 2e-5, (slot, name, err)


def test_sampler_constraints():
    job = _ns_job("distmult", "triple", num_neg=50, filtering=True, E=60)
    tr = job.dataset.split("train")[:200].long().cuda()
    for slot in (0, 2):
        neg = job._sampler.sample(tr, slot)
        assert neg.shape == (200, 50) and int(neg.min()) >= 0 and int(neg.max()) < 60
        assert not bool(job._sampler._is_positive(neg, slot, tr).any())
        # the positives themselves are recognised
        assert bool(job._sampler._is_positive(tr[:, [slot]], slot, tr).all())
    shared = _ns_job("distmult", "triple", num_neg=20, shared=True, E=60)
    for slot in (0, 2):
        neg = shared._sampler.sample(tr, slot)
        assert neg.shape == (200, 20)
        assert not bool((neg == tr[:, [slot]]).any())  # each row's own positive dropped


def test_ns_training_lowers_loss():
    job = _ns_job("rotate", "triple", num_neg=63, dim=128)
    first = last = None
    for epoch in range(4):
        tr = job.run_epoch()
        first = tr["avg_loss"] if first is None else first
        last = tr["avg_loss"]
    assert np.isfinite(last) and last < first


@pytest.mark.parametrize("model,num_neg", [("complex", 7), ("rotate", 200), ("transe", 40)])
def test_recorded_ns_step_replays_like_the_eager_step(model, num_neg):
    """engine.graph_step for negative sampling: the step recorded once and replayed (negatives
    drawn inside the recording, torch's generator advancing per replay) against the same job
    stepping eagerly from the same seed -- the same negatives, hence the same losses and tables,
    replay after replay, with eager work and synchronisations of the test in between."""
    def run(graph):
        job = _ns_job(model, "triple", num_neg=num_neg)
        job.config.set("engine.graph_step", graph)
        job._prepare()
        torch.manual_seed(123)
        perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))
        losses, tables = [], []
        for i in range(9):
            res, _, _ = job.train_step(i, job._collate(perm[i * 128:(i + 1) * 128]))
            losses.append(float(res.avg_loss))
            torch.cuda.synchronize()
            tables.append(job.model._entity_embedder._embeddings.weight.detach().clone())
            _ = (tables[-1] * 2).sum().item()  # unrelated eager work between the replays
        return job, losses, tables

    job_g, loss_g, tab_g = run(True)
    job_e, loss_e, tab_e = run(False)
    assert job_g._graph_step is not None and job_g._graph_step.graph is not None, job_g._graph_step.error
    assert job_e._graph_step is None
    np.testing.assert_allclose(loss_g, loss_e, rtol=1e-4)
    for i, (a, b) in enumerate(zip(tab_g, tab_e)):
        # the entity-grouped sums add their pairs in no fixed order: differences of an ulp, which an
        # L1 distance turns into a flipped sign(x) for the odd component with |x| ~ 1e-7 -- a
        # handful of elements may move by a step's worth, the tables as a whole not at all
        diff = (a - b).abs()
        off = int((diff > 2e-5 * b.abs().max()).sum())
        assert off <= 64 and float(diff.mean()) <= 1e-6 * float(b.abs().max()), (i, off, float(diff.mean()))
    assert len(set(loss_g)) == len(loss_g)  # every replay drew new negatives (and saw a new batch)


def test_in_place_row_gradients_reach_the_backward_on_the_device(monkeypatch):
    """in_place_row_gradients() must be seen by backward functions that autograd runs on its
    DEVICE thread (every CUDA backward): the second corrupted slot of a negative-sampling step adds
    its candidate and query rows into the gradient the first slot left (no zero fill of a
    table-sized buffer, no sum of two of them), with the same gradients as the plain path."""
    from kge import Config, Dataset
    from kge.job import TrainingJob
    from kge.model.embedder import lookup_embedder as le

    def job():
        c = Config()
        c.set("model", "complex")
        c._import("complex")
        c.set("job.device", "cuda")
        c.set("lookup_embedder.dim", 64)
        c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
        c.set("train.type", "negative_sampling")
        c.set("train.loss", "kl")
        c.set("negative_sampling.num_samples.s", 40)
        c.set("negative_sampling.implementation", "triple")
        c.set("train.optimizer", "Adagrad")
        c.set("train.batch_size", 64)
        c.set("engine.graph_step", False)
        c.set("verbose", False)
        ds = Dataset.synthetic(c, "toy", seed=0, num_entities=500, num_relations=5, sizes=(2000, 100, 100))
        torch.manual_seed(0)
        j = TrainingJob.create(c, ds)
        j._prepare()
        return j

    seen = []
    real = le._in_place_ok

    def spy(held, weight, dtype):
        ok = real(held, weight, dtype)
        seen.append(ok)
        return ok

    monkeypatch.setattr(le, "_in_place_ok", spy)
    a, b = job(), job()
    batch = a._collate(torch.arange(64))
    g = torch.Generator(device="cuda").manual_seed(5)
    negs = [torch.randint(0, 500, (64, 40), device="cuda", generator=g) for _ in range(3)]
    batch["negative_samples"] = negs
    a.optimizer.zero_grad()
    with le.in_place_row_gradients():
        a.process_batch(0, batch)
    assert any(seen), "no backward saw the in-place flag"
    seen.clear()
    b.optimizer.zero_grad()
    b.process_batch(0, batch)  # outside the context: autograd sums the slots' gradients
    assert not any(seen)
    for pa, pb in zip(a.model.parameters(), b.model.parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-5, atol=1e-7)
