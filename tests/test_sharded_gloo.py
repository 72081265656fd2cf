"""World-size-2 gloo test (CPU) of the entity-row-sharded exchange logic (kge/sharded.py).

The collectives, shard bounds, owner-computed query rows, count reduction and top-k
merge are the product code; only the per-shard compute is injected (numpy oracle ops)
because this container has no GPU.  On a GPU the same class runs with EngineOps."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import kge_oracle as K


class OracleOps:
    def prep(self, direction, ent, eidx, rel, ridx):
        e = ent[eidx].double().numpy()
        r = rel[ridx].double().numpy()
        q = K.prep_sp("complex", e, r) if direction == 0 else K.prep_po("complex", r, e)
        return torch.from_numpy(q).float()

    def score(self, q, tab):
        return (q.double() @ tab.double().T).float()

    def spo(self, ent_s, rel, p, ent_o):
        q = K.prep_sp("complex", ent_s.double().numpy(), rel[p].double().numpy())
        return torch.from_numpy((q * ent_o.double().numpy()).sum(1)).float()

    def rank_counts(self, s, c0, true_idx, true_score, fp, fc, tp, tc, greater, ties):
        S = s.double().numpy().copy()
        n, m = S.shape
        t = true_score.double().numpy()
        ti = true_idx.numpy() - c0
        for i in range(n):
            if 0 <= ti[i] < m:
                S[i, ti[i]] = t[i]
        g0, e0 = K.rank_and_ties(S, t)
        greater[:n] += torch.from_numpy(g0)
        ties[:n] += torch.from_numpy(e0)
        for r, (ptr, col) in enumerate(((fp, fc), (tp, tc))):
            if ptr is None:
                continue
            for i in range(n):
                for j in col[ptr[i]:ptr[i + 1]].tolist():
                    if 0 <= j - c0 < m and j - c0 != ti[i]:
                        S[i, j - c0] = -np.inf
            g, e = K.rank_and_ties(S, t)
            greater[(1 + r) * n:(2 + r) * n] += torch.from_numpy(g)
            ties[(1 + r) * n:(2 + r) * n] += torch.from_numpy(e)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge.sharded import RowShardedScorer, shard_bounds

        g = torch.Generator().manual_seed(0)
        E, R, d, B = 53, 5, 8, 6
        ent = torch.randn(E, d, generator=g)
        rel = torch.randn(R, d, generator=g)
        lo, hi = shard_bounds(E, world, rank)
        sc = RowShardedScorer(ent[lo:hi].clone(), lo, hi, E, rel, OracleOps())
        # each rank contributes its own queries
        gq = torch.Generator().manual_seed(100 + rank)
        s = torch.randint(0, E, (B,), generator=gq)
        p = torch.randint(0, R, (B,), generator=gq)
        local = sc.score_sp(s, p)
        tv, ti = sc.topk(local, 5)
        # identical eval batch on every rank
        ge = torch.Generator().manual_seed(7)
        es, ep, eo = (torch.randint(0, n, (B,), generator=ge) for n in (E, R, E))
        f_ptr = torch.arange(0, 2 * B + 1, 2)
        f_col = torch.randint(0, E, (2 * B,), generator=ge)
        counts = sc.rank_counts(es, ep, eo, (f_ptr, f_col), (f_ptr, f_col))
        out_q.put((rank, lo, hi, local.numpy(), tv.numpy(), ti.numpy(), counts.numpy(),
                   [x.numpy() for x in (s, p, es, ep, eo, f_ptr, f_col)]))
    finally:
        dist.destroy_process_group()


def test_row_sharded_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    g = torch.Generator().manual_seed(0)
    E, R, d, B = 53, 5, 8, 6
    ent = torch.randn(E, d, generator=g).double().numpy()
    rel = torch.randn(R, d, generator=g).double().numpy()
    # global queries in rank order
    s_all = np.concatenate([r[7][0] for r in res])
    p_all = np.concatenate([r[7][1] for r in res])
    full = K.prep_sp("complex", ent[s_all], rel[p_all]) @ ent.T
    for rank, lo, hi, local, tv, ti, counts, _ in res:
        np.testing.assert_allclose(local, full[:, lo:hi], rtol=1e-5, atol=1e-5)
        ref_top = np.sort(full, 1)[:, ::-1][:, :5]
        np.testing.assert_allclose(tv, ref_top, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(np.take_along_axis(full, ti, 1), tv, rtol=1e-5, atol=1e-5)
    # eval counts: every rank holds the same reduced counts == unsharded computation
    es, ep, eo, f_ptr, f_col = res[0][7][2:]
    ops = OracleOps()
    entt, relt = torch.from_numpy(ent).float(), torch.from_numpy(rel).float()
    true = ops.spo(entt[torch.from_numpy(es)], relt, torch.from_numpy(ep), entt[torch.from_numpy(eo)])
    ref = np.zeros((2, 2, 3 * B), np.int64)
    for di, (e_idx, direction, tgt) in enumerate(((es, 0, eo), (eo, 1, es))):
        qv = ops.prep(direction, entt, torch.from_numpy(e_idx), relt, torch.from_numpy(ep))
        scores = ops.score(qv, entt)
        gr = torch.zeros(3 * B, dtype=torch.int64)
        ti = torch.zeros(3 * B, dtype=torch.int64)
        ops.rank_counts(scores, 0, torch.from_numpy(tgt), true, torch.from_numpy(f_ptr), torch.from_numpy(f_col),
                        None, None, gr, ti)
        ref[di, 0], ref[di, 1] = gr.numpy(), ti.numpy()
    for r in res:
        np.testing.assert_array_equal(r[6][:, :, :2 * B], ref[:, :, :2 * B])


def _worker_local(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge.sharded import RowShardedScorer, shard_bounds

        g = torch.Generator().manual_seed(0)
        E, R, d, B = 41, 4, 8, 5
        ent = torch.randn(E, d, generator=g)
        rel = torch.randn(R, d, generator=g)
        lo, hi = shard_bounds(E, world, rank)
        sc = RowShardedScorer(ent[lo:hi].clone(), lo, hi, E, rel, OracleOps())
        gq = torch.Generator().manual_seed(200 + rank)
        s = torch.randint(lo, hi, (B,), generator=gq)
        p = torch.randint(0, R, (B,), generator=gq)
        out_q.put((rank, lo, hi, sc.score_sp_local(s, p).numpy(), s.numpy(), p.numpy()))
        try:
            sc.score_sp_local(torch.tensor([hi % E] * B), p)  # not owned -> error on one rank at least
            bad = False
        except ValueError:
            bad = True
        out_q.put((rank, "err", bad))
    finally:
        dist.destroy_process_group()


def test_row_sharded_local_queries_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_local, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    items = [q.get(timeout=120) for _ in range(2 * world)]
    for pr in procs:
        pr.join(timeout=60)
    res = sorted([x for x in items if x[1] != "err"], key=lambda x: x[0])
    errs = [x[2] for x in items if x[1] == "err"]
    g = torch.Generator().manual_seed(0)
    E, R, d, B = 41, 4, 8, 5
    ent = torch.randn(E, d, generator=g).double().numpy()
    rel = torch.randn(R, d, generator=g).double().numpy()
    s_all = np.concatenate([r[4] for r in res])
    p_all = np.concatenate([r[5] for r in res])
    full = K.prep_sp("complex", ent[s_all], rel[p_all]) @ ent.T
    for rank, lo, hi, local, _, _ in res:
        np.testing.assert_allclose(local, full[:, lo:hi], rtol=1e-5, atol=1e-5)
    assert all(errs)


def _worker_grouped(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge.sharded import RowShardedScorer, shard_bounds

        g = torch.Generator().manual_seed(0)
        E, R, d, B, k = 41, 4, 8, 5, 3
        ent = torch.randn(E, d, generator=g)
        rel = torch.randn(R, d, generator=g)
        lo, hi = shard_bounds(E, world, rank)
        sc = RowShardedScorer(ent[lo:hi].clone(), lo, hi, E, rel, OracleOps())
        gq = torch.Generator().manual_seed(300 + rank)
        s = torch.randint(lo, hi, (k, B), generator=gq)
        p = torch.randint(0, R, (k, B), generator=gq)
        # k single-batch exchanges, the next one in flight while a batch is scored
        tickets = [sc.submit_queries_local(s[0], p[0])]
        single = []
        for i in range(k):
            if i + 1 < k:
                tickets.append(sc.submit_queries_local(s[i + 1], p[i + 1]))
            single.append(sc.score_submitted(tickets.pop(0)).numpy())
        # the same k batches in ONE exchange, scored in k blocks
        group = sc.submit_queries_local(s.reshape(-1), p.reshape(-1))
        blocks = [sc.score_submitted(group, (x, k)).numpy() for x in range(k)]
        out_q.put((rank, lo, hi, single, blocks, s.numpy(), p.numpy()))
    finally:
        dist.destroy_process_group()


def test_row_sharded_grouped_exchange_world2():
    """One all_gather for k batches per rank (submit_queries_local on k B queries) and
    score_submitted(ticket, (x, k)): block x holds the gathered rows [x W B, (x + 1) W B) in
    rank-major order, every query is scored exactly once, and the scores are those of the k
    single-batch exchanges."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_grouped, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    g = torch.Generator().manual_seed(0)
    E, R, d, B, k = 41, 4, 8, 5, 3
    ent = torch.randn(E, d, generator=g).double().numpy()
    rel = torch.randn(R, d, generator=g).double().numpy()
    # gathered order: rank 0's k B queries, then rank 1's
    s_g = np.concatenate([r[5].reshape(-1) for r in res])
    p_g = np.concatenate([r[6].reshape(-1) for r in res])
    full = K.prep_sp("complex", ent[s_g], rel[p_g]) @ ent.T  # [W k B, E]
    for rank, lo, hi, single, blocks, _, _ in res:
        got = np.concatenate(blocks)
        assert got.shape == (world * k * B, hi - lo)
        np.testing.assert_allclose(got, full[:, lo:hi], rtol=1e-5, atol=1e-5)
        # the same rows as the single-batch steps: step i holds (rank w, batch i) at rows w B ..
        for i in range(k):
            for w in range(world):
                np.testing.assert_array_equal(single[i][w * B:(w + 1) * B],
                                              got[(w * k + i) * B:(w * k + i + 1) * B])
