"""World-size-2 (and 3) gloo test (CPU) of vocab-parallel 1vsAll training over the
row-sharded entity table (kge/sharded.py RowShardedScorer.train_1vsall_grads).

The collectives -- triple all_gather, owner-computed query rows, MAX / SUM reductions of
the row statistics, the dQ all_reduce, the relation-gradient all_reduce -- are the product
code; only the per-shard compute is injected (torch CPU ops restating the engine kernels:
ComplEx prep, contraction, softmax row stats / gradient, backward GEMMs).  The result must
equal the unsharded objective  sum_dir CE(Q E^T, target) / (W B)  by torch autograd."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _prep(direction, ent, eidx, rel, ridx):
    e, r = ent[eidx], rel[ridx]
    h = e.shape[1] // 2
    er, ei, rr, ri = e[:, :h], e[:, h:], r[:, :h], r[:, h:]
    if direction == 0:  # s * r
        return torch.cat([er * rr - ei * ri, er * ri + ei * rr], 1)
    return torch.cat([rr * er + ri * ei, rr * ei - ri * er], 1)  # conj(r) * o


class TorchOps:
    def prep(self, direction, ent, eidx, rel, ridx):
        return _prep(direction, ent, eidx, rel, ridx)

    def score(self, q, tab, out=None):
        s = q @ tab.T
        if out is not None:
            out.copy_(s)
            return out
        return s

    def row_stats(self, s, c0, labels):
        mx = s.max(1).values
        sm = torch.exp(s - mx[:, None]).sum(1)
        c = labels - c0
        inside = (c >= 0) & (c < s.shape[1])
        tg = torch.where(inside, s[torch.arange(len(s)), c.clamp(0, s.shape[1] - 1)], torch.zeros_like(mx))
        return mx, sm, tg

    def softmax_grad(self, s, c0, labels, lse, scale, g):
        out = scale * torch.exp(s - lse[:, None])
        c = labels - c0
        rows = torch.nonzero((c >= 0) & (c < s.shape[1])).view(-1)
        out[rows, c[rows]] -= scale
        g.copy_(out)
        return g

    def bce_grad(self, s, c0, labels, offset, scale, g):
        from kge.sharded import bce_grad_block

        return bce_grad_block(s, c0, labels, offset, scale, g)

    def score_bwd(self, g, q, tab, dq, d_tab):
        dq.copy_(g @ tab)
        d_tab += g.T @ q

    def prep_bwd(self, direction, ent, eidx, rel, ridx, dq, d_ent, d_rel):
        e = ent.detach().clone().requires_grad_(True)
        r = rel.detach().clone().requires_grad_(True)
        q = _prep(direction, e, eidx, r, ridx)
        ge, gr = torch.autograd.grad(q, (e, r), dq)
        d_ent += ge
        d_rel += gr


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


E, R, D, B = 37, 5, 8, 6


def _data():
    g = torch.Generator().manual_seed(0)
    return torch.randn(E, D, generator=g, dtype=torch.float64).float(), \
        torch.randn(R, D, generator=g, dtype=torch.float64).float()


def _worker(rank, world, port, out_q, loss=("kl", 0.0)):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kge.sharded import RowShardedScorer, shard_bounds

        ent, rel = _data()
        lo, hi = shard_bounds(E, world, rank)
        sc = RowShardedScorer(ent[lo:hi].clone(), lo, hi, E, rel.clone(), TorchOps())
        gq = torch.Generator().manual_seed(50 + rank)
        s, p, o = (torch.randint(0, n, (B,), generator=gq) for n in (E, R, E))
        if loss[0] == "kl":
            value, d_ent, d_rel = sc.train_1vsall_grads(s, p, o)
        else:  # every rank passes the whole batch (as the job does)
            tr = torch.stack([s, p, o], 1)
            value, d_ent, d_rel = sc.train_1vsall_global(sc._all_gather_1d(tr.reshape(-1)).view(-1, 3), loss=loss)
            value = float(value)
            assert sc.collectives_last_step == 4
        out_q.put((rank, lo, hi, value, d_ent.numpy(), d_rel.numpy(), torch.stack([s, p, o], 1).numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_vocab_parallel_1vsall_grads(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # unsharded reference on the gathered batch (rank order), torch autograd
    ent, rel = _data()
    ent = ent.double().requires_grad_(True)
    rel = rel.double().requires_grad_(True)
    tr = torch.from_numpy(np.concatenate([r[6] for r in res]))
    n = len(tr)
    ce = torch.nn.CrossEntropyLoss(reduction="sum")
    loss = (ce(_prep(0, ent, tr[:, 0], rel, tr[:, 1]) @ ent.T, tr[:, 2]) +
            ce(_prep(1, ent, tr[:, 2], rel, tr[:, 1]) @ ent.T, tr[:, 0])) / n
    loss.backward()
    g_ent, g_rel = ent.grad.numpy(), rel.grad.numpy()
    for rank, lo, hi, l, d_ent, d_rel, _ in res:
        assert abs(l - loss.item()) < 1e-5 * abs(loss.item())
        np.testing.assert_allclose(d_ent, g_ent[lo:hi], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(d_rel, g_rel, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("world,offset", [(2, 0.0), (3, -1.5)])
def test_row_sharded_1vsall_bce_grads(world, offset):
    """train.loss bce over the row shards (no softmax statistics: each shard's slice of the loss
    and of G by itself, one scalar all_reduce) against the unsharded objective
    sum_dir BCEWithLogits(Q E^T + offset, one-hot target, reduction sum) / (W B) by autograd
    (loss.py:137-158, train.py:1041-1057)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, ("bce", offset))) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    ent, rel = _data()
    ent = ent.double().requires_grad_(True)
    rel = rel.double().requires_grad_(True)
    tr = torch.from_numpy(np.concatenate([r[6] for r in res]))
    n = len(tr)
    bce = torch.nn.BCEWithLogitsLoss(reduction="sum")

    def term(scores, target):
        y = torch.zeros_like(scores)
        y[torch.arange(n), target] = 1.0
        return bce(scores + offset, y)

    loss = (term(_prep(0, ent, tr[:, 0], rel, tr[:, 1]) @ ent.T, tr[:, 2]) +
            term(_prep(1, ent, tr[:, 2], rel, tr[:, 1]) @ ent.T, tr[:, 0])) / n
    loss.backward()
    g_ent, g_rel = ent.grad.numpy(), rel.grad.numpy()
    for rank, lo, hi, l, d_ent, d_rel, _ in res:
        assert abs(l - loss.item()) < 1e-5 * abs(loss.item())
        np.testing.assert_allclose(d_ent, g_ent[lo:hi], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(d_rel, g_rel, rtol=1e-4, atol=1e-6)
