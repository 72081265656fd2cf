"""GPU: the vocab-parallel pieces on the engine -- kge_softmax_row_stats / kge_softmax_grad
against torch on column slices, and RowShardedScorer.train_1vsall_grads with EngineOps at
world size 1 (RCCL, in-process) against the fused single-GPU 1vsAll gradients."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib
    _lib.lib()
    return _lib


@pytest.mark.parametrize("m,ld", [(1001, 1004), (777, 777), (4096, 4096)])
def test_row_stats_and_grad_on_slice(L, m, ld):
    rng = np.random.default_rng(m)
    n, c0 = 19, 300
    buf = torch.zeros(n, ld, device="cuda")
    s = buf[:, :m]
    s.copy_(torch.from_numpy((rng.standard_normal((n, m)) * 4).astype(np.float32)))
    labels = torch.from_numpy(rng.integers(0, c0 + m + 200, size=n)).cuda()  # some outside the slice
    mx, sm, tg = L.softmax_row_stats(s, c0, labels)
    ref_mx = s.max(1).values
    assert torch.equal(mx, ref_mx)
    torch.testing.assert_close(sm, torch.exp(s - ref_mx[:, None]).sum(1), rtol=2e-6, atol=0)
    c = labels - c0
    inside = (c >= 0) & (c < m)
    ref_tg = torch.where(inside, s[torch.arange(n), c.clamp(0, m - 1)], torch.zeros_like(mx))
    assert torch.equal(tg, ref_tg)
    lse = ref_mx + torch.log(torch.exp(s - ref_mx[:, None]).sum(1)) + 0.25  # any global lse
    g = torch.empty_like(s)
    L.softmax_grad(s, c0, labels, lse, 0.5, g)
    ref = 0.5 * torch.exp(s - lse[:, None])
    rows = torch.nonzero(inside).view(-1)
    ref[rows, c[rows]] -= 0.5
    torch.testing.assert_close(g, ref, rtol=0, atol=2e-6 * 0.5)


def _free_port():
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


@pytest.mark.parametrize("prec,planes", [("bf16x3", False), ("bf16x3", True), ("fp32", False)])
def test_train_1vsall_grads_world1_matches_fused(L, prec, planes):
    """planes: the shard's gradient slice leaves the loss kernel as bf16 hi / lo planes
    (kge_softmax_grad_planes) for the plane-fed backward GEMMs -- what large shards use; forced
    here on a small one whose 300 rows need K padding."""
    from kge import Config, Dataset, KgeModel
    from kge.sharded import EngineOps, RowShardedScorer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        c = Config()
        c.set("model", "complex")
        c._import("complex")
        c.set("job.device", "cuda")
        c.set("lookup_embedder.dim", 128)
        c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
        c.set("engine.precision", prec)
        c.set("dataset.num_entities", 3001)
        c.set("dataset.num_relations", 17)
        m = KgeModel.create(c, Dataset(c, None))
        ent = m._entity_embedder._embeddings.weight
        rel = m._relation_embedder._embeddings.weight
        g = torch.Generator().manual_seed(3)
        B = 300
        s, p, o = (torch.randint(0, n, (B,), generator=g).cuda() for n in (3001, 17, 3001))
        loss = m.score_sp_xent(s, p, o, 1.0 / B) + m.score_po_xent(p, o, s, 1.0 / B)
        loss.backward()
        sc = RowShardedScorer(ent.detach(), 0, 3001, 3001, rel.detach(), EngineOps(0, L.PRECISIONS[prec]))
        used = []
        if planes:
            sc.PLANES_MIN_ELEMS = 0
            inner = sc.ops.softmax_grad_planes
            sc.ops.softmax_grad_planes = lambda *a: (used.append(1), inner(*a))[1]
        l2, d_ent, d_rel = sc.train_1vsall_grads(s, p, o)
        assert len(used) == (1 if planes else 0)  # both directions in one stacked pass
        assert abs(l2 - loss.item()) <= 1e-5 * abs(loss.item())
        tol = 1e-4 if prec == "bf16x3" else 1e-5
        assert (d_ent - ent.grad).abs().max() <= tol * ent.grad.abs().max()
        assert (d_rel - rel.grad).abs().max() <= tol * rel.grad.abs().max()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("train_loss", ["kl", "bce"])
def test_sharded_jobs_world1_rccl_match_unsharded_jobs(L, train_loss):
    """TrainingJob1vsAll (train.loss kl, and bce with an offset) and EntityRankingJob with
    engine.row_sharded on, over an RCCL world of one process (the degenerate single shard,
    EngineOps = the HIP kernels): the same loss trajectory, tables and ranks as the unsharded
    jobs from the same start."""
    from kge import Config, Dataset
    from kge.job import EntityRankingJob, TrainingJob

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        runs = {}
        for mode in ("off", "on"):
            c = Config()
            c.set("model", "complex")
            c._import("complex")
            c.set("job.device", "cuda")
            c.set("verbose", False)
            c.set("lookup_embedder.dim", 64)
            c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
            c.set("train.type", "1vsAll")
            c.set("train.batch_size", 256)
            c.set("train.max_epochs", 2)
            c.set("train.optimizer_args", {"lr": 0.1})
            if train_loss == "bce":
                c.set("train.loss", "bce")
                c.set("train.loss_arg", -3.0)
            c.set("valid.every", 0)
            c.set("eval.batch_size", 100)
            c.set("engine.eval_batch_size", 0)  # the batches of eval.batch_size as they are
            c.set("random_seed.torch", 3)
            c.set("engine.precision", "fp32")
            c.set("engine.graph_step", False)
            c.set("engine.row_sharded", mode)
            ds = Dataset.synthetic(c, "toy", seed=1, num_entities=700, num_relations=9, sizes=(2000, 150, 150))
            torch.manual_seed(11)
            job = TrainingJob.create(c, ds)
            traces = job.run()
            assert (job._sharded is not None) == (mode == "on")
            ev = EntityRankingJob(c, ds, model=job.model)
            ev.capture_ranks = True
            et = ev.run()
            runs[mode] = ([t["avg_loss"] for t in traces],
                          job.model._entity_embedder._embeddings.weight.detach().cpu().numpy(),
                          job.model._relation_embedder._embeddings.weight.detach().cpu().numpy(), ev.ranks,
                          et["mean_reciprocal_rank_filtered_with_test"])
        np.testing.assert_allclose(runs["on"][0], runs["off"][0], rtol=1e-5)
        for i in (1, 2):  # tables after 16 Adagrad steps: all but a handful of ill-conditioned elements
            diff = np.abs(runs["on"][i] - runs["off"][i])
            # Adagrad divides every gradient by its own running magnitude, so where the gradient is
            # nearly zero a rounding-level difference becomes a visible step: here that is one
            # complex component (columns 31 / 63), whose common-mode gradient sum_i q_i nearly
            # cancels -- measured 44-64 of 44,800 elements beyond 1e-4, all in those two columns,
            # whichever order the shards sum in
            assert int((diff > 1e-4).sum()) <= max(4, 2e-3 * diff.size) and float(diff.mean()) < 1e-5
        same = sum(int((runs["on"][3][k] == runs["off"][3][k]).sum()) for k in runs["on"][3])
        total = sum(len(v) for v in runs["on"][3].values())
        assert same >= 0.99 * total  # two fp32 trajectories: a rare near-tie may sit on another side
        assert runs["on"][4] == pytest.approx(runs["off"][4], rel=1e-2)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,prec,d", [("complex", "bf16x3", 64), ("distmult", "bf16x3", 40), ("complex", "fp32", 64),
                                          ("transe", "bf16x3", 64)])
def test_pipelined_exchange_world1_matches_direct_scoring(L, kind, prec, d):
    """submit_queries_local / score_submitted (the N > 1 bench's step: query rows exchanged as
    packed bf16 planes where the split contraction applies, as fp32 rows otherwise) at world
    size 1 over RCCL against score_sp_local and against the engine's own score_all -- identical."""
    from kge import engine
    from kge.sharded import EngineOps, RowShardedScorer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        E, R, B = 333, 5, 48
        k = {"complex": L.COMPLEX, "distmult": L.DISTMULT, "transe": L.TRANSE}[kind]
        g = torch.Generator().manual_seed(d)
        ent = (torch.randn(E, d, generator=g) * 0.3).cuda()
        rel = (torch.randn(R, d, generator=g) * 0.3).cuda()
        ops = EngineOps(k, L.PRECISIONS[prec])
        lo = 56  # this rank's rows start here: the queries carry GLOBAL entity ids
        shard = ent[lo:]
        sh = RowShardedScorer(shard, lo, E, E, rel, ops)
        s = torch.randint(lo, E, (3, B), generator=g).cuda()
        p = torch.randint(0, R, (3, B), generator=g).cuda()
        assert ops.planes_ok(shard, L.DIR_SP) == (prec == "bf16x3" and kind != "transe")
        tickets = [sh.submit_queries_local(s[0], p[0])]
        outs = []
        for i in range(3):  # batch i + 1 in flight while batch i is scored
            if i + 1 < 3:
                tickets.append(sh.submit_queries_local(s[i + 1], p[i + 1]))
            outs.append(sh.score_submitted(tickets.pop(0)))
        torch.cuda.synchronize()
        for i in range(3):
            direct = sh.score_sp_local(s[i], p[i])
            assert torch.equal(outs[i], direct)
            ref = engine.score_all(k, L.DIR_SP, L.PRECISIONS[prec], 1.0, ent, s[i], rel, p[i], shard, None)
            assert torch.equal(outs[i], ref)
        # three batches in ONE exchange, scored block by block: the same scores
        group = sh.submit_queries_local(s.reshape(-1), p.reshape(-1))
        for i in range(3):
            assert torch.equal(sh.score_submitted(group, (i, 3)), outs[i])
        assert group.work is None  # waited for once
        with pytest.raises(ValueError):
            sh.score_submitted(group, (0, 5))  # 144 rows do not split into 5 blocks
        with pytest.raises(ValueError):
            sh.score_submitted(group, (3, 3))
    finally:
        dist.destroy_process_group()


def complex_q(e, r, direction):
    """float64 query rows of ComplEx: (s o r) for sp_, (o o conj r) for _po (complex.py:19-44)."""
    h = e.shape[1] // 2
    er, ei, rr, ri = e[:, :h], e[:, h:], r[:, :h], r[:, h:]
    if direction == 0:
        return torch.cat((er * rr - ei * ri, er * ri + ei * rr), 1)
    return torch.cat((rr * er + ri * ei, rr * ei - ri * er), 1)


def test_c5_rank_shapes_at_n8_past_2_32_elements(L):
    """What ONE rank sees at N = 8 on the Wikidata5M configuration: 8,192 global queries against a
    574,311-row shard -- a [8192, 574311] score block of 4.7e9 elements, past 2^32 -- through the
    row-sharded scoring and training paths (gradient planes) at world size 1 over RCCL, with the
    loss and sampled scores / dE rows checked in float64."""
    from kge.sharded import EngineOps, RowShardedScorer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        _c5_rank_shapes(L, EngineOps, RowShardedScorer)
    finally:
        dist.destroy_process_group()
        torch.cuda.empty_cache()


def _c5_rank_shapes(L, EngineOps, RowShardedScorer):
    E, R, B, d = 574311, 237, 8192, 512
    torch.manual_seed(0)
    ent = torch.randn(E, d, device="cuda") * 0.1
    rel = torch.randn(R, d, device="cuda") * 0.1
    sh = RowShardedScorer(ent, 0, E, E, rel, EngineOps(L.COMPLEX, L.PREC_BF16X3))
    g = torch.Generator().manual_seed(1)
    s = torch.randint(0, E, (B,), generator=g).cuda()
    p = torch.randint(0, R, (B,), generator=g).cuda()
    o = torch.randint(0, E, (B,), generator=g).cuda()
    rows = torch.tensor([0, 1, 4095, 4096, 7000, 8191]).cuda()      # rows on both sides of 2^32 / E
    cols = torch.tensor([0, 5, 300000, 523775, 574310]).cuda()

    # ---- scoring (what bench.py's row_sharded_c5 runs per rank at N = 8)
    scores = sh.score_submitted(sh.submit_queries_local(s, p))
    q64 = complex_q(ent[s[rows]].double(), rel[p[rows]].double(), 0)
    ref = q64 @ ent[cols].double().T
    got = scores[rows][:, cols].double()
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-5
    del scores
    torch.cuda.empty_cache()

    # ---- training gradients (vocab-parallel 1vsAll; gradient planes at this size)
    tr = torch.stack([s, p, o], 1)
    loss, d_ent, d_rel = sh.train_1vsall_global(tr)
    # the loss in float64, every row, in column chunks
    total = 0.0
    for direction, e_idx, lab in ((0, s, o), (1, o, s)):
        for b0 in range(0, B, 512):
            sl = slice(b0, b0 + 512)
            q64 = complex_q(ent[e_idx[sl]].double(), rel[p[sl]].double(), direction)
            acc_max = torch.full((512,), -float("inf"), device="cuda", dtype=torch.float64)
            acc_sum = torch.zeros(512, device="cuda", dtype=torch.float64)
            for c0 in range(0, E, 65536):
                lg = q64 @ ent[c0:c0 + 65536].double().T
                m = torch.maximum(acc_max, lg.max(1).values)
                acc_sum = acc_sum * torch.exp(acc_max - m) + torch.exp(lg - m[:, None]).sum(1)
                acc_max = m
            tgt = (q64 * ent[lab[sl]].double()).sum(1)
            total += float((acc_max + torch.log(acc_sum) - tgt).sum())
    ref_loss = total / B
    assert abs(float(loss) - ref_loss) < 1e-5 * abs(ref_loss)
    # dE rows: sum over both directions of G^T Q restricted to sampled entity rows
    ref_de = torch.zeros(len(cols), d, device="cuda", dtype=torch.float64)
    for direction, e_idx, lab in ((0, s, o), (1, o, s)):
        for b0 in range(0, B, 512):
            sl = slice(b0, b0 + 512)
            q64 = complex_q(ent[e_idx[sl]].double(), rel[p[sl]].double(), direction)
            acc_max = torch.full((512,), -float("inf"), device="cuda", dtype=torch.float64)
            acc_sum = torch.zeros(512, device="cuda", dtype=torch.float64)
            for c0 in range(0, E, 65536):
                lg = q64 @ ent[c0:c0 + 65536].double().T
                m = torch.maximum(acc_max, lg.max(1).values)
                acc_sum = acc_sum * torch.exp(acc_max - m) + torch.exp(lg - m[:, None]).sum(1)
                acc_max = m
            lse = acc_max + torch.log(acc_sum)
            gcols = torch.exp(q64 @ ent[cols].double().T - lse[:, None])          # [512, 5]
            gcols -= (lab[sl][:, None] == cols[None, :]).double()
            ref_de += (gcols / B).T @ q64
    # the query rows' own contribution (prep backward) lands on rows s / o, not on the sampled cols
    # unless they coincide: mask those out of the comparison
    touched = torch.isin(cols, torch.cat((s, o)))
    got = d_ent[cols].double()
    err = ((got - ref_de)[~touched]).abs().max().item() / ref_de.abs().max().item()
    assert err < 1e-4


@pytest.mark.parametrize("planes", [True, False])
def test_row_sharded_bce_step_world1_vs_float64_autograd(L, planes):
    """train_1vsall_global with loss ("bce", offset) on the engine (gradient planes, or the fp32
    gradient block) at world size 1 over RCCL: loss and both tables' gradients against autograd of
    BCEWithLogits(sum) / B on float64 ComplEx scores (train.py:1041-1057 with loss.py:137-158)."""
    from kge.sharded import EngineOps, RowShardedScorer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        E, R, B, d, offset = 1517, 11, 96, 64, -1.0
        torch.manual_seed(3)
        ent = torch.randn(E, d, device="cuda") * 0.4
        rel = torch.randn(R, d, device="cuda") * 0.4
        g = torch.Generator().manual_seed(4)
        tr = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                          torch.randint(0, E, (B,), generator=g)], 1).cuda()
        e64, r64 = ent.double().requires_grad_(), rel.double().requires_grad_()
        ref = 0.0
        for direction, q_col, lab_col in ((0, 0, 2), (1, 2, 0)):
            q = complex_q(e64[tr[:, q_col]], r64[tr[:, 1]], direction)
            y = torch.zeros(B, E, device="cuda", dtype=torch.float64)
            y[torch.arange(B), tr[:, lab_col]] = 1.0
            ref = ref + torch.nn.functional.binary_cross_entropy_with_logits(q @ e64.T + offset, y, reduction="sum") / B
        ref.backward()
        ref = float(ref.detach())
        sh = RowShardedScorer(ent, 0, E, E, rel, EngineOps(L.COMPLEX, L.PREC_BF16X3))
        sh.PLANES_MIN_ELEMS = sh.BCE_PLANES_MIN_ELEMS = 0 if planes else 1 << 62
        loss, d_ent, d_rel = sh.train_1vsall_global(tr, loss=("bce", offset))
        torch.cuda.synchronize()
        assert sh.collectives_last_step == 4
        assert abs(float(loss) - ref) <= 2e-5 * abs(ref)
        assert float((d_ent.double() - e64.grad).abs().max()) <= 2e-4 * float(e64.grad.abs().max())
        assert float((d_rel.double() - r64.grad).abs().max()) <= 2e-4 * float(r64.grad.abs().max())
    finally:
        dist.destroy_process_group()


def _world2_batch():
    """Tables and one global batch for the two-rank test; some targets sit right past the end of
    shard 0 (rows 502 .. 511 of 1,003: inside the K padding of shard 0's gradient planes) and
    right before shard 1."""
    from kge.sharded import shard_bounds

    E, R, d, B = 1003, 11, 64, 96
    g = torch.Generator().manual_seed(5)
    ent = torch.randn(E, d, generator=g) * 0.2
    rel = torch.randn(R, d, generator=g) * 0.2
    tr = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                      torch.randint(0, E, (B,), generator=g)], 1)
    hi0 = shard_bounds(E, 2, 0)[1]
    tr[0, 2], tr[1, 2], tr[2, 0], tr[3, 0], tr[4, 2] = hi0, hi0 + 3, hi0, hi0 - 1, hi0 - 1
    return E, R, d, B, ent, rel, tr


def _world2_worker(rank, world, port, planes, out_q, loss=("kl", 0.0)):
    """One of two ranks sharing the GPU; collectives over gloo (device tensors staged through host
    memory by kge.sharded), compute on the engine."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge import _lib
        from kge.sharded import EngineOps, RowShardedScorer, shard_bounds

        E, R, d, B, ent, rel, tr = _world2_batch()
        lo, hi = shard_bounds(E, world, rank)
        sc = RowShardedScorer(ent[lo:hi].cuda().contiguous(), lo, hi, E, rel.cuda(),
                              EngineOps(_lib.COMPLEX, _lib.PREC_BF16X3))
        sc.PLANES_MIN_ELEMS = sc.BCE_PLANES_MIN_ELEMS = 0 if planes else 1 << 62
        value, d_ent, d_rel = sc.train_1vsall_global(tr.cuda(), loss=loss)
        assert sc.collectives_last_step == 4
        out_q.put((rank, lo, hi, float(value), d_ent.cpu().numpy(), d_rel.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("planes", [True, False], ids=["planes", "fp32_block"])
def test_train_1vsall_world2_on_the_engine_matches_fused(L, planes):
    """Vocab-parallel 1vsAll gradients with TWO ranks on the engine's kernels (both on this GPU,
    collectives over gloo through host memory): every rank's shard of dE, the relation gradient
    and the loss equal the single-GPU fused step's -- with targets that live in the other shard,
    including the columns right past a shard's end (the K padding of its gradient planes)."""
    import torch.multiprocessing as mp

    from kge import Config, Dataset, KgeModel

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world2_worker, args=(r, world, port, planes, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    E, R, d, B, ent, rel, tr = _world2_batch()
    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", d)
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    m = KgeModel.create(c, Dataset(c, None))
    we, wr = m._entity_embedder._embeddings.weight, m._relation_embedder._embeddings.weight
    with torch.no_grad():
        we.copy_(ent)
        wr.copy_(rel)
    t = tr.cuda()
    loss = m.score_sp_xent(t[:, 0], t[:, 1], t[:, 2], 1.0 / B) + m.score_po_xent(t[:, 1], t[:, 2], t[:, 0], 1.0 / B)
    loss.backward()
    ref_e, ref_r = we.grad.cpu().numpy(), wr.grad.cpu().numpy()
    for rank, lo, hi, l2, d_ent, d_rel in res:
        assert l2 == pytest.approx(loss.item(), rel=1e-5)
        assert np.abs(d_ent - ref_e[lo:hi]).max() <= 1e-4 * np.abs(ref_e).max(), rank
        assert np.abs(d_rel - ref_r).max() <= 1e-4 * np.abs(ref_r).max(), rank


@pytest.mark.parametrize("planes", [True, False], ids=["planes", "fp32_block"])
def test_train_1vsall_bce_world2_on_the_engine_vs_float64_autograd(L, planes):
    """train.loss bce (offset -1.5) over TWO ranks on the engine's kernels (both on this GPU,
    collectives over gloo through host memory): each rank's share of the loss summed by the final
    all_reduce, its shard of dE and the relation gradient against float64 autograd of
    BCEWithLogits(sum) / B on the whole table -- with hot columns that belong to the other shard,
    also right past a shard's end (the K padding of its gradient planes)."""
    import torch.multiprocessing as mp

    world, offset = 2, -1.5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world2_worker, args=(r, world, port, planes, q, ("bce", offset))) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    E, R, d, B, ent, rel, tr = _world2_batch()
    e64, r64 = ent.double().requires_grad_(), rel.double().requires_grad_()
    ref = 0.0
    for direction, q_col, lab_col in ((0, 0, 2), (1, 2, 0)):
        qq = complex_q(e64[tr[:, q_col]], r64[tr[:, 1]], direction)
        y = torch.zeros(B, E, dtype=torch.float64)
        y[torch.arange(B), tr[:, lab_col]] = 1.0
        ref = ref + torch.nn.functional.binary_cross_entropy_with_logits(qq @ e64.T + offset, y, reduction="sum") / B
    ref.backward()
    ref_e, ref_r = e64.grad.numpy(), r64.grad.numpy()
    for rank, lo, hi, value, d_ent, d_rel in res:
        assert value == pytest.approx(float(ref.detach()), rel=1e-5)
        assert np.abs(d_ent - ref_e[lo:hi]).max() <= 1e-4 * np.abs(ref_e).max(), rank
        assert np.abs(d_rel - ref_r).max() <= 1e-4 * np.abs(ref_r).max(), rank


def _world2_score_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge import _lib
        from kge.sharded import EngineOps, RowShardedScorer, shard_bounds

        E, R, d, B, ent, rel, tr = _world2_batch()
        lo, hi = shard_bounds(E, world, rank)
        sc = RowShardedScorer(ent[lo:hi].cuda().contiguous(), lo, hi, E, rel.cuda(),
                              EngineOps(_lib.COMPLEX, _lib.PREC_BF16X3))
        g = torch.Generator().manual_seed(40 + rank)
        k = 2
        s = torch.randint(lo, hi, (k, 48), generator=g).cuda()   # shard-affine queries: own subjects
        p = torch.randint(0, R, (k, 48), generator=g).cuda()
        single = [sc.score_submitted(sc.submit_queries_local(s[i], p[i])).cpu().numpy() for i in range(k)]
        group = sc.submit_queries_local(s.reshape(-1), p.reshape(-1))
        blocks = [sc.score_submitted(group, (x, k)).cpu().numpy() for x in range(k)]
        # the generic path: any subjects, owner-computed query rows + all_reduce
        s_any = torch.randint(0, E, (48,), generator=g).cuda()
        generic = sc.score_sp(s_any, p[0])
        tv, ti = sc.topk(generic, 5)
        # evaluation counts of a batch every rank holds
        t = tr[:32].cuda()
        f_ptr = torch.arange(0, 65, 2).cuda()
        f_col = torch.randint(0, E, (64,), generator=torch.Generator().manual_seed(9)).cuda()
        counts = sc.rank_counts(t[:, 0], t[:, 1], t[:, 2], (f_ptr, f_col), (f_ptr, f_col))
        out_q.put((rank, lo, hi, s.cpu().numpy(), p.cpu().numpy(), single, blocks, s_any.cpu().numpy(),
                   generic.cpu().numpy(), tv.cpu().numpy(), ti.cpu().numpy(), counts.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_scoring_and_ranking_world2_on_the_engine(L):
    """Two ranks on the engine's kernels: shard-affine scoring through the packed-plane exchange
    (single batches and one grouped exchange of two batches), the generic owner-computes path,
    the top-k merge and the evaluation counts -- against the unsharded engine on the whole table."""
    import torch.multiprocessing as mp

    from kge import engine

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world2_score_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    E, R, d, B, ent, rel, tr = _world2_batch()
    ent, rel = ent.cuda(), rel.cuda()

    def full(s, p):
        return engine.score_all(L.COMPLEX, L.DIR_SP, L.PREC_BF16X3, 1.0, ent, torch.as_tensor(s).cuda(), rel,
                                torch.as_tensor(p).cuda(), ent, None).cpu().numpy()

    k = 2
    s_ranks, p_ranks = [r[3] for r in res], [r[4] for r in res]
    for rank, lo, hi, _, _, single, blocks, s_any, generic, tv, ti, counts in res:
        for i in range(k):  # step i: rank 0's batch i, then rank 1's
            ref = full(np.concatenate([s_ranks[0][i], s_ranks[1][i]]), np.concatenate([p_ranks[0][i], p_ranks[1][i]]))
            np.testing.assert_allclose(single[i], ref[:, lo:hi], rtol=0, atol=2e-5 * np.abs(ref).max())
        # grouped: rank-major rows (rank 0's two batches, then rank 1's), scored in two blocks
        s_g = np.concatenate([s_ranks[0].reshape(-1), s_ranks[1].reshape(-1)])
        p_g = np.concatenate([p_ranks[0].reshape(-1), p_ranks[1].reshape(-1)])
        ref = full(s_g, p_g)
        np.testing.assert_allclose(np.concatenate(blocks), ref[:, lo:hi], rtol=0, atol=2e-5 * np.abs(ref).max())
    # generic path: the global batch is rank 0's queries then rank 1's
    s_all = np.concatenate([r[7] for r in res])
    p_all = np.concatenate([p_ranks[0][0], p_ranks[1][0]])
    ref = full(s_all, p_all)
    for rank, lo, hi, *_rest in res:
        generic, tv, ti = _rest[5], _rest[6], _rest[7]
        np.testing.assert_allclose(generic, ref[:, lo:hi], rtol=0, atol=2e-5 * np.abs(ref).max())
        np.testing.assert_allclose(tv, np.sort(ref, 1)[:, ::-1][:, :5], rtol=0, atol=2e-5 * np.abs(ref).max())
        np.testing.assert_allclose(np.take_along_axis(ref, ti, 1), tv, rtol=0, atol=2e-5 * np.abs(ref).max())
    np.testing.assert_array_equal(res[0][11], res[1][11])  # the reduced counts are global
    # the same counts from one rank holding the whole table
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from kge.sharded import EngineOps, RowShardedScorer

        one = RowShardedScorer(ent, 0, E, E, rel, EngineOps(L.COMPLEX, L.PREC_BF16X3))
        t = tr[:32].cuda()
        f_ptr = torch.arange(0, 65, 2).cuda()
        f_col = torch.randint(0, E, (64,), generator=torch.Generator().manual_seed(9)).cuda()
        ref_counts = one.rank_counts(t[:, 0], t[:, 1], t[:, 2], (f_ptr, f_col), (f_ptr, f_col)).cpu().numpy()
    finally:
        dist.destroy_process_group()
    # bf16x3 scores of a shard and of the whole table agree to rounding: counts may differ only
    # where a competitor ties the true score within that rounding -- none on these random tables
    np.testing.assert_array_equal(res[0][11], ref_counts)


def _jobs_config(mode, precision="fp32"):
    from kge import Config

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda")
    c.set("verbose", False)
    c.set("lookup_embedder.dim", 64)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", "1vsAll")
    c.set("train.batch_size", 256)
    c.set("train.max_epochs", 2)
    c.set("train.optimizer_args", {"lr": 0.1})
    c.set("valid.every", 0)
    c.set("eval.batch_size", 100)
    c.set("engine.eval_batch_size", 0)  # the batches of eval.batch_size as they are
    c.set("random_seed.torch", 3)
    c.set("engine.precision", precision)
    c.set("engine.graph_step", False)
    c.set("engine.row_sharded", mode)
    return c


def _run_jobs(c, penalties=False):
    from kge import Dataset
    from kge.job import EntityRankingJob, TrainingJob

    ds = Dataset.synthetic(c, "toy", seed=1, num_entities=700, num_relations=9, sizes=(2000, 150, 150))
    torch.manual_seed(11)
    job = TrainingJob.create(c, ds)
    if penalties:  # frequency-weighted L3 on the (sharded) entity table, plain L2 on the relations
        for e, w, p, weighted in ((job.model._entity_embedder, 1e-2, 3, True),
                                  (job.model._relation_embedder, 5e-3, 2, False)):
            e.config.set(e.configuration_key + ".regularize_weight", w)
            e.config.set(e.configuration_key + ".regularize_args.p", p)
            e.config.set(e.configuration_key + ".regularize_args.weighted", weighted)
    traces = job.run()
    if penalties:
        assert min(t["avg_penalty"] for t in traces) > 0
    ev = EntityRankingJob(c, ds, model=job.model)
    ev.capture_ranks = True
    et = ev.run()
    return ([t["avg_loss"] + t["avg_penalty"] for t in traces], job.model._entity_embedder._embeddings.weight.detach().cpu().numpy(),
            job.model._relation_embedder._embeddings.weight.detach().cpu().numpy(), ev.ranks,
            et["mean_reciprocal_rank_filtered_with_test"], job._sharded is not None)


def _world2_jobs_worker(rank, world, port, out_q, penalties):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out_q.put((rank,) + _run_jobs(_jobs_config("on"), penalties))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("penalties", [False, True], ids=["plain", "lp_penalties"])
def test_sharded_jobs_world2_on_the_engine_match_unsharded_jobs(L, penalties):
    """TrainingJob1vsAll and EntityRankingJob row-sharded over TWO ranks with the engine's kernels
    (both on this GPU, gloo through host memory): after sync_model both ranks hold the tables the
    unsharded job trains, the loss (plus penalty) trajectory and the evaluation ranks are the same;
    also with Lp penalties, whose entity terms every rank differentiates over its own rows."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world2_jobs_worker, args=(r, world, port, q, penalties)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    off = _run_jobs(_jobs_config("off"), penalties)
    assert not off[5]
    for r in res:
        on = r[1:]
        assert on[5]
        np.testing.assert_allclose(on[0], off[0], rtol=1e-5)
        for i in (1, 2):
            diff = np.abs(on[i] - off[i])
            # Adagrad divides every gradient by its own running magnitude, so where the gradient is
            # nearly zero a rounding-level difference becomes a visible step: here that is one
            # complex component (columns 31 / 63), whose common-mode gradient sum_i q_i nearly
            # cancels -- measured 44-64 of 44,800 elements beyond 1e-4, all in those two columns,
            # whichever order the shards sum in
            assert int((diff > 1e-4).sum()) <= max(4, 2e-3 * diff.size) and float(diff.mean()) < 1e-5
        same = sum(int((on[3][k] == off[3][k]).sum()) for k in on[3])
        total = sum(len(v) for v in on[3].values())
        assert same >= 0.99 * total
        assert on[4] == pytest.approx(off[4], rel=1e-2)


def _world2_fullsize_eval_worker(rank, world, port, eval_precision, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import json

        from conftest import GOLDEN
        from kge import KgeModel
        from kge.job import EntityRankingJob
        from test_gpu_configs import base_config, dataset_from, seeded_tables, set_tables

        f = np.load(os.path.join(GOLDEN, "eval_fullsize_normal.npz"))
        meta = json.loads(str(f["meta"]))
        E, R, dim = meta["E"], meta["R"], meta["dim"]
        ent, rel = seeded_tables(meta["table_seed"], E, R, dim, dim, meta["std"])
        c = base_config("complex", dim, E, R, {"eval.batch_size": meta["batch_size"], "eval.split": "valid",
                                               "engine.row_sharded": "on", "engine.eval_precision": eval_precision})
        ds = dataset_from(c, f)
        model = KgeModel.create(c, ds)
        set_tables(model, ent, rel)
        job = EntityRankingJob(c, ds, model=model)
        job.capture_ranks = True
        trace = job.run()
        out_q.put((rank, {k: v.copy() for k, v in job.ranks.items()},
                   {k: v for k, v in trace.items() if isinstance(v, float)}, job._shard_refinement is not None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("eval_precision", ["bf16x3_refined", "fp32"])
def test_sharded_eval_world2_fullsize_vs_reference(L, eval_precision):
    """The row-sharded EntityRankingJob over TWO ranks (both on this GPU, gloo through host
    memory) against the reference's full-size capture (E = 14,541, ComplEx-512, 512 validation
    triples, filtered + filtered-with-test): with the default eval precision every shard
    contracts in bf16x3 and rescores the near-ties of the true score among its own columns, so
    the summed counts are those of exactly computed scores -- every rank that differs from the
    reference's must be explained by near-ties within 1e-5 of the row maximum, as for the
    unsharded job."""
    import json

    import torch.multiprocessing as mp

    from conftest import GOLDEN
    from test_gpu_configs import assert_rank_moves_are_near_ties, seeded_tables

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world2_fullsize_eval_worker, args=(r, world, port, eval_precision, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    f = np.load(os.path.join(GOLDEN, "eval_fullsize_normal.npz"))
    meta = json.loads(str(f["meta"]))
    ent, rel = seeded_tables(meta["table_seed"], meta["E"], meta["R"], meta["dim"], meta["dim"], meta["std"])
    ref = {k[5:]: f[k] for k in f.files if k.startswith("full_")}
    splits = {k: f["tri_" + k].astype(np.int64) for k in ("train", "valid", "test")}
    total = sum(len(v) for v in ref.values())
    for rank, ranks, metrics, refined in res:
        assert refined == (eval_precision == "bf16x3_refined")
        assert set(ranks) == set(ref)
        moved, worst = assert_rank_moves_are_near_ties(ranks, ref, ent, rel, splits["valid"], splits, 1e-5,
                                                       f"sharded x2 rank {rank} {eval_precision}")
        print(f"\nsharded x2 rank {rank} ({eval_precision}): {moved} of {total} ranks differ, largest gap {worst:.2e}")
        assert moved <= 0.005 * total
    for k in res[0][1]:  # every rank holds the same global ranks
        np.testing.assert_array_equal(res[0][1][k], res[1][1][k])
