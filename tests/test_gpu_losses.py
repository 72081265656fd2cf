"""GPU parity of the fused training losses: kge_softmax_kl (KvsAll) against the oracle, and
the fused KvsAll / 1vsAll jobs against their unfused (torch loss) form."""
import numpy as np
import pytest
import torch

from oracle import kge_oracle as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib
    _lib.lib()
    return _lib


def _csr(lists):
    ptr = np.zeros(len(lists) + 1, np.int64)
    ptr[1:] = np.cumsum([len(x) for x in lists])
    col = np.concatenate([np.asarray(x, np.int64) for x in lists]) if ptr[-1] else np.zeros(0, np.int64)
    return ptr, col


@pytest.mark.parametrize("m", [5, 1001, 40943])
@pytest.mark.parametrize("eps", [0.0, 0.1])
@pytest.mark.parametrize("layout", ["padded_inplace", "tight_out"])
def test_softmax_kl_vs_oracle(L, m, eps, layout):
    rng = np.random.default_rng(m + int(eps * 10))
    n = 23
    S = (rng.standard_normal((n, m)) * 4).astype(np.float32)
    lists = [rng.choice(m, size=min(m, k), replace=False) for k in rng.integers(0, 9, size=n)]
    lists[0] = np.zeros(0, np.int64)          # empty row
    lists[1] = np.arange(min(m, 300))         # many positives (more than one wave)
    scale = 1.0 / n
    ref_loss, ref_g = K.softmax_kl(S.astype(np.float64), lists, eps, scale)
    ptr, col = _csr(lists)
    ld = (m + 3) // 4 * 4 if layout == "padded_inplace" else m
    buf = torch.zeros((n, ld), device="cuda")
    s = buf[:, :m]
    s.copy_(torch.from_numpy(S).cuda())
    g = s if layout == "padded_inplace" else torch.zeros((n, m), device="cuda")
    loss = L.softmax_kl(s, torch.from_numpy(ptr).cuda(), torch.from_numpy(col).cuda(), eps, scale, g=g)
    torch.cuda.synchronize()
    lo = loss.cpu().numpy()
    # the loss combines terms of size ~|S| (lse, row sums): absolute bound on that scale
    bound = 2e-6 * (np.abs(S).max() + np.log(m)) * (1 + eps * m * np.abs(S).mean())
    assert np.abs(lo - ref_loss).max() <= bound, (np.abs(lo - ref_loss).max(), bound)
    assert np.abs(g.cpu().numpy() - ref_g).max() <= 2e-6 * scale


def test_softmax_xent_is_kl_with_one_positive(L):
    rng = np.random.default_rng(1)
    n, m = 16, 777
    S = torch.from_numpy((rng.standard_normal((n, m)) * 3).astype(np.float32)).cuda()
    lab = torch.from_numpy(rng.integers(0, m, size=n)).cuda()
    g1, g2 = torch.zeros_like(S), torch.zeros_like(S)
    l1 = L.softmax_xent(S, lab, 0.5, g=g1)
    l2 = L.softmax_kl(S, torch.arange(n + 1, device="cuda"), lab, 0.0, 0.5, g=g2)
    torch.cuda.synchronize()
    assert torch.allclose(l1, l2, rtol=1e-6, atol=1e-5)
    assert torch.allclose(g1, g2, atol=1e-7)


def _kvsall_job(model, fused, smoothing):
    from kge import Config, Dataset
    from kge.job import TrainingJob

    c = Config()
    c.set("model", model)
    c._import(model)
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 64)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", "KvsAll")
    c.set("train.loss", "kl")
    c.set("KvsAll.label_smoothing", smoothing)
    c.set("engine.fused_loss", fused)
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.1})
    c.set("train.batch_size", 64)
    c.set("verbose", False)
    torch.manual_seed(0)
    ds = Dataset.synthetic(c, "toy", seed=0, num_entities=300, num_relations=7, sizes=(2000, 100, 100))
    job = TrainingJob.create(c, ds)
    job._prepare()
    return job


@pytest.mark.parametrize("model,smoothing", [("distmult", 0.0), ("distmult", 0.1), ("complex", 0.05)])
def test_kvsall_fused_matches_unfused(model, smoothing):
    """KvsAll batches of sp_ and of _po queries: the fused KL gives the loss and the table
    gradients of the dense-label torch KL path.  Gradients, not optimizer steps, are
    compared: Adagrad's first step is lr * sign(g) for any g != 0, which turns 1e-9-sized
    differences of near-zero gradient entries into lr-sized weight differences."""
    res = []
    for fused in (True, False):
        job = _kvsall_job(model, fused, smoothing)
        out = []
        mixed = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(5))[:64]  # sp_ and _po
        for b, ex in enumerate((torch.arange(0, 64), torch.arange(job.num_examples - 64, job.num_examples), mixed)):
            job.optimizer.zero_grad()
            loss = job._process_batch(b, job._collate(ex)).avg_loss
            out.append((loss, job.model._entity_embedder._embeddings.weight.grad.cpu().numpy().copy(),
                        job.model._relation_embedder._embeddings.weight.grad.cpu().numpy().copy()))
        res.append(out)
    for (l1, ge1, gr1), (l0, ge0, gr0) in zip(*res):
        assert abs(l1 - l0) <= 2e-5 * abs(l0)
        tol = 1e-4  # bf16x3 backward GEMMs on both paths; G from the fused kernel vs torch
        assert np.abs(ge1 - ge0).max() <= tol * np.abs(ge0).max()
        assert np.abs(gr1 - gr0).max() <= tol * np.abs(gr0).max()


@pytest.mark.parametrize("kw", [{}, {"lr_decay": 0.01, "weight_decay": 0.1}, {"maximize": True, "eps": 1e-6},
                                {"initial_accumulator_value": 0.5}])
def test_fused_adagrad_matches_torch(kw):
    """util.optimizer.FusedAdagrad (kge_adagrad_step) == torch.optim.Adagrad, step by step,
    including a parameter that falls back to torch (odd size: scalar kernel path; CPU)."""
    from kge.util.optimizer import FusedAdagrad

    torch.manual_seed(0)
    # more tensors than one launch takes (8), vector and scalar layouts mixed, an empty one
    shapes = [(300, 64), (7, 33), (5,), (64, 4), (0, 8), (1000, 128), (3,), (16, 16), (2, 2), (33, 7), (128,)]
    ref = [torch.randn(s, device="cuda") for s in shapes] + [torch.randn(4, 4)]
    mine = [t.clone() for t in ref]
    for t in ref + mine:
        t.requires_grad_(True)
    o_ref = torch.optim.Adagrad(ref, lr=0.1, **kw)
    o_mine = FusedAdagrad(mine, lr=0.1, **kw)
    for _ in range(4):
        grads = [torch.randn_like(t) for t in ref]
        for a, b, g in zip(ref, mine, grads):
            a.grad, b.grad = g.clone(), g.clone()
        o_ref.step()
        o_mine.step()
    for a, b in zip(ref, mine):
        if a.numel() == 0:
            continue
        assert torch.allclose(a, b, rtol=0, atol=1e-6 * a.abs().max().item()), (a - b).abs().max()
    sd = o_mine.state_dict()  # torch's layout: loads into a stock Adagrad
    o2 = torch.optim.Adagrad(ref, lr=0.1, **kw)
    o2.load_state_dict(sd)


@pytest.mark.parametrize("p", [1, 2, 3, 4])
def test_lp_rows_kernels_vs_torch(p):
    """kge_lp_rows / kge_lp_rows_bwd (the frequency-weighted Lp penalty over the occurrences of a
    batch's indexes, lookup_embedder.py:138-158) against torch: row sums of |x|^p, the gradient
    scattered into an existing buffer with repeated rows adding up, values on a grid so that
    exact zeros occur (p = 1: sign(0) = 0), an odd row width, a leading dimension wider than the
    rows."""
    from kge import _lib as L

    g = torch.Generator().manual_seed(p)
    wide = (torch.randint(-6, 7, (300, 70), generator=g) / 8.0).cuda()
    w = wide[:, :67]  # ld 70, d 67
    idx = torch.randint(0, 300, (513,), generator=g).cuda()
    idx[:7] = 11  # one row many times
    sums = L.lp_rows(w, idx, p)
    ref = w[idx].double().abs().pow(p).sum(1)
    assert torch.allclose(sums.double(), ref, rtol=1e-6, atol=1e-7)
    gs = torch.tensor([0.75], device="cuda")
    dw = torch.full((300, 67), 0.5, device="cuda")
    L.lp_rows_bwd(w, idx, p, gs, 0.3, dw)
    wr = w.double().clone().requires_grad_(True)
    (0.3 * 0.75 * wr[idx].abs().pow(p).sum()).backward()
    assert torch.allclose((dw - 0.5).double(), wr.grad, rtol=1e-5, atol=1e-6)
    # no scale pointer: factor 1; nothing to do for an empty index vector
    dw2 = torch.zeros(300, 67, device="cuda")
    L.lp_rows_bwd(w, idx, p, None, 0.3, dw2)
    assert torch.allclose(dw2.double() * 0.75, wr.grad, rtol=1e-5, atol=1e-6)
    assert L.lp_rows(w, idx[:0], p).numel() == 0


@pytest.mark.parametrize("n,m", [(37, 130), (64, 257), (5, 31)])
def test_softmax_grad_planes_slice_vs_float64(n, m):
    """kge_softmax_grad_planes on a column slice [c0, c0 + m) of rows whose labels are GLOBAL ids:
    hi + lo reproduces scale * (exp(s - lse) - onehot) to the split's 2^-16; labels that belong to
    another shard -- below c0, past the slice, and in particular inside the slice's K padding
    [m, ld) -- leave no trace; padding columns and rows are zero."""
    from kge import _lib as L

    g = torch.Generator().manual_seed(n * 1000 + m)
    c0 = 11
    s = torch.randn(n, m, generator=g).cuda()
    lse = (torch.logsumexp(s.double(), 1) + 0.3).float()
    labels = torch.randint(0, c0 + m + 40, (n,), generator=g)
    labels[0] = c0 + m          # first padding column
    labels[1 % n] = c0 - 1      # just below the slice
    labels[2 % n] = c0 + m - 1  # last column of the slice
    labels = labels.cuda()
    gp = L.softmax_grad_planes(s, c0, labels, lse, 0.5)
    ref = 0.5 * torch.exp(s.double() - lse.double()[:, None])
    lab = labels - c0
    own = (lab >= 0) & (lab < m)
    ref[torch.arange(n, device="cuda")[own], lab[own]] -= 0.5
    got = gp.hi[:n, :m].double() + gp.lo[:n, :m].double()
    assert (got - ref).abs().max().item() <= 3e-5 * ref.abs().max().item()
    for plane in (gp.hi, gp.lo):
        assert float(plane[:, m:].float().abs().sum()) == 0.0
        assert float(plane[n:].float().abs().sum()) == 0.0
