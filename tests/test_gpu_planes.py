"""GPU parity of the plane-fed backward path through the C ABI: the fused losses that leave
their gradient as bf16 hi / lo planes in place of the scores (kge_softmax_xent_planes /
kge_softmax_kl_planes) against the CPU oracle's loss + gradient, and the two backward GEMMs
that read the planes (kge_score_dot_bwd_q_planes / kge_score_dot_bwd_t_planes) against float64
products of the very planes they were given (1e-4 of the max |entry|: the bf16x3 contract)."""
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


def _scores(L, n, m, seed, scale=3.0):
    n_pad, ld = L.planes_layout(n, m)
    g = torch.Generator(device="cuda").manual_seed(seed)
    buf = torch.full((n_pad, ld), 7.5, device="cuda")  # stale contents everywhere
    buf[:n, :m] = torch.randn(n, m, device="cuda", generator=g) * scale
    return buf


@pytest.mark.parametrize("n,m", [(5, 37), (33, 1000), (64, 14541), (40, 8193), (8, 40943), (6, 20001), (3, 60000),
                                 (2, 65536)])
def test_xent_planes_vs_oracle(L, n, m):
    buf = _scores(L, n, m, n * 1000 + m)
    s = buf[:n, :m].double().cpu().numpy()
    labels = torch.randint(0, m, (n,), generator=torch.Generator().manual_seed(m)).cuda()
    scale = 1.0 / n
    loss, gp = L.softmax_planes(buf, n, m, labels, None, 0.0, scale)
    torch.cuda.synchronize()
    ref_loss, ref_g = K.softmax_xent(s, labels.cpu().numpy(), scale)
    np.testing.assert_allclose(loss.cpu().numpy(), ref_loss, rtol=2e-5, atol=2e-5)
    g = (gp.hi.float() + gp.lo.float()).double().cpu().numpy()
    gmax = np.abs(ref_g).max()
    assert np.abs(g[:n, :m] - ref_g).max() <= 3e-5 * gmax
    # hi is the bf16 rounding of the value, lo the rest: |G - hi - lo| <= 2^-16 |G|
    assert np.all(np.abs(g[:n, :m] - ref_g) <= 2.0 ** -15 * np.abs(ref_g) + 1e-7 * gmax)
    # K padding: columns [m, ld) and rows [n, n_pad) of both planes are zero
    if gp.hi.shape[1] > m:
        assert float(gp.hi[:, m:].float().abs().max()) == 0.0 and float(gp.lo[:, m:].float().abs().max()) == 0.0
    if gp.n_pad > n:
        assert float(gp.hi[n:].float().abs().max()) == 0.0 and float(gp.lo[n:].float().abs().max()) == 0.0


@pytest.mark.parametrize("n,m,eps", [(7, 300, 0.0), (20, 5000, 0.1), (16, 40943, 0.1), (5, 30011, 0.05), (4, 65533, 0.1)])
def test_kl_planes_vs_oracle(L, n, m, eps):
    buf = _scores(L, n, m, 17 * n + m)
    s = buf[:n, :m].double().cpu().numpy()
    rng = np.random.default_rng(m)
    lens = rng.integers(0, 9, size=n)
    lens[0] = 0  # a query without positives
    lens[-1] = min(m, 300)
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=ptr[1:])
    col = np.concatenate([rng.choice(m, size=k, replace=False) for k in lens]).astype(np.int64)
    scale = 1.0 / n
    loss, gp = L.softmax_planes(buf, n, m, torch.from_numpy(col).cuda(), torch.from_numpy(ptr).cuda(), eps, scale)
    torch.cuda.synchronize()
    ref_loss, ref_g = K.softmax_kl(s, [col[ptr[i]:ptr[i + 1]] for i in range(n)], eps, scale)
    np.testing.assert_allclose(loss.cpu().numpy(), ref_loss, rtol=3e-5, atol=3e-5)
    g = (gp.hi.float() + gp.lo.float()).double().cpu().numpy()
    assert np.abs(g[:n, :m] - ref_g).max() <= 3e-5 * np.abs(ref_g).max()
    assert float(gp.hi[:, m:].float().abs().max()) == 0.0


def _planes(L, n, m, seed):
    """Random gradient planes as the loss kernel leaves them (through the loss kernel itself)."""
    buf = _scores(L, n, m, seed)
    labels = torch.randint(0, m, (n,), generator=torch.Generator().manual_seed(seed)).cuda()
    _, gp = L.softmax_planes(buf, n, m, labels, None, 0.0, 1.0)
    g64 = (gp.hi.float().double() + gp.lo.float().double())[:n, :m]
    return gp, g64


@pytest.mark.parametrize("n,m,d", [(100, 501, 64), (300, 3001, 128), (2048, 14541, 512), (512, 40943, 512),
                                   (1, 40, 8), (64, 700, 1024), (50, 333, 104)])
def test_bwd_q_planes_vs_float64(L, n, m, d):
    gp, g64 = _planes(L, n, m, n + m + d)
    gen = torch.Generator(device="cuda").manual_seed(d)
    t = torch.randn(m, d, device="cuda", generator=gen) * 0.1
    ref = g64 @ t.double()
    dq = L.score_dot_bwd_q_planes(gp, t)
    torch.cuda.synchronize()
    assert float((dq.double() - ref).abs().max() / ref.abs().max()) < 1e-4
    # deterministic (fixed-order slab sum), scaled and accumulated forms
    assert torch.equal(dq, L.score_dot_bwd_q_planes(gp, t))
    alpha = torch.tensor([0.375], device="cuda")
    seed = torch.randn(n, d, device="cuda", generator=gen)
    acc = seed.clone()
    L.score_dot_bwd_q_planes(gp, t, gscale=alpha, dq=acc, accumulate=True)
    want = seed.double() + 0.375 * ref
    assert float((acc.double() - want).abs().max() / want.abs().max()) < 1e-4


@pytest.mark.parametrize("n,m,d", [(100, 501, 64), (300, 3001, 128), (2048, 14541, 512), (512, 40943, 512),
                                   (1, 40, 8), (64, 700, 1024), (50, 333, 104)])
def test_bwd_t_planes_vs_float64(L, n, m, d):
    gp, g64 = _planes(L, n, m, 3 * n + m + d)
    gen = torch.Generator(device="cuda").manual_seed(d + 1)
    q = torch.randn(n, d, device="cuda", generator=gen) * 0.1
    ldp = (d + 31) // 32 * 32
    qh = torch.zeros(gp.n_pad, ldp, device="cuda", dtype=torch.bfloat16)
    ql = torch.zeros_like(qh)
    h, l = L.split_rows(q)
    qh[:n], ql[:n] = h, l
    q64 = (qh.float().double() + ql.float().double())[:n, :d]
    ref = g64.T @ q64
    dt = torch.full((m, d), float("nan"), device="cuda")
    L.score_dot_bwd_t_planes(gp, qh, ql, dt)
    torch.cuda.synchronize()
    assert float((dt.double() - ref).abs().max() / ref.abs().max()) < 1e-4
    # reproducible bit for bit, and a column permutation of the query planes permutes dT's columns
    dt2 = torch.full((m, d), float("nan"), device="cuda")
    L.score_dot_bwd_t_planes(gp, qh, ql, dt2)
    assert torch.equal(dt, dt2)
    if d % 8 == 0:
        cperm = torch.randperm(d, generator=torch.Generator().manual_seed(d)).cuda()
        qhp, qlp = torch.zeros_like(qh), torch.zeros_like(ql)
        qhp[:, :d], qlp[:, :d] = qh[:, :d][:, cperm], ql[:, :d][:, cperm]
        L.score_dot_bwd_t_planes(gp, qhp, qlp, dt2)
        assert torch.equal(dt2, dt[:, cperm])
    alpha = torch.tensor([-2.0], device="cuda")
    seed = torch.randn(m, d, device="cuda", generator=gen)
    acc = seed.clone()
    L.score_dot_bwd_t_planes(gp, qh, ql, acc, gscale=alpha, accumulate=True)
    want = seed.double() - 2.0 * ref
    assert float((acc.double() - want).abs().max() / want.abs().max()) < 1e-4


def test_planes_entry_points_reject_bad_layouts(L):
    buf = torch.zeros(32, 100, device="cuda")  # leading dimension not a multiple of 32
    with pytest.raises(L.EngineError):
        L.softmax_planes(buf, 4, 90, torch.zeros(4, dtype=torch.int64, device="cuda"), None, 0.0, 1.0)
    assert not L.planes_ok(70000) and L.planes_ok(40943)


@pytest.mark.parametrize("model", ["complex", "distmult", "rescal", "transe", "rotate", "cp", "simple"])
@pytest.mark.parametrize("aligned", [True, False], ids=["vector", "scalar"])
def test_two_part_prep_equals_the_per_direction_launches(L, model, aligned):
    """kge_prep_query_split2 / kge_prep_query_bwd2 (rows [0, n_a) in one direction, the rest in
    the other, split point on the host or in device memory) against the per-direction entry
    points on the same rows: forward bit-identical (fp32 rows and both planes), backward equal up
    to the order of the float atomics."""
    kind = {"complex": L.COMPLEX, "distmult": L.DISTMULT, "rescal": L.RESCAL, "transe": L.TRANSE,
            "rotate": L.ROTATE, "cp": L.CP, "simple": L.SIMPLE}[model]
    d_e = (16 if model == "rescal" else 64) + (0 if aligned else 2)
    d_r = K.relation_dim(model, d_e) if model != "cp" else d_e // 2
    E, R, n, n_a = 50, 7, 37, 13
    g = torch.Generator().manual_seed(d_e + kind)
    ent = torch.randn(E, d_e, generator=g).cuda()
    rel = torch.randn(R, d_r, generator=g).cuda()
    eidx = torch.randint(0, E, (n,), generator=g).cuda()
    ridx = torch.randint(0, R, (n,), generator=g).cuda()
    qw = L.query_width(kind, d_e)
    ldp = (qw + 31) // 32 * 32

    def bufs():
        return (torch.full((n, qw), 7.0, device="cuda"), torch.full((n, ldp), 3.0, device="cuda", dtype=torch.bfloat16),
                torch.full((n, ldp), 3.0, device="cuda", dtype=torch.bfloat16))

    q0, h0, l0 = bufs()
    L.prep_query_split(kind, L.DIR_PO, ent, eidx[:n_a], rel, ridx[:n_a], n_a, d_e, d_r, out=(q0[:n_a], h0[:n_a], l0[:n_a]))
    L.prep_query_split(kind, L.DIR_SP, ent, eidx[n_a:], rel, ridx[n_a:], n - n_a, d_e, d_r,
                       out=(q0[n_a:], h0[n_a:], l0[n_a:]))
    n_a_dev = torch.tensor([n_a], dtype=torch.int64, device="cuda")
    for host_n_a, dev in ((n_a, None), (0, n_a_dev)):
        q1, h1, l1 = bufs()
        L.prep_query_split2(kind, L.DIR_PO, L.DIR_SP, host_n_a, dev, ent, eidx, rel, ridx, d_e, d_r, out=(q1, h1, l1))
        torch.cuda.synchronize()
        assert torch.equal(q0, q1) and torch.equal(h0, h1) and torch.equal(l0, l1)
    dq = torch.randn(n, qw, generator=g).cuda()
    de0, dr0 = torch.zeros_like(ent), torch.zeros_like(rel)
    L.prep_query_bwd(kind, L.DIR_PO, ent, eidx[:n_a], rel, ridx[:n_a], n_a, d_e, d_r, dq[:n_a], de0, dr0)
    L.prep_query_bwd(kind, L.DIR_SP, ent, eidx[n_a:], rel, ridx[n_a:], n - n_a, d_e, d_r, dq[n_a:], de0, dr0)
    for host_n_a, dev in ((n_a, None), (0, n_a_dev)):
        de1, dr1 = torch.zeros_like(ent), torch.zeros_like(rel)
        L.prep_query_bwd2(kind, L.DIR_PO, L.DIR_SP, host_n_a, dev, ent, eidx, rel, ridx, d_e, d_r, dq, de1, dr1)
        torch.cuda.synchronize()
        assert float((de0 - de1).abs().max()) <= 1e-5 * float(de0.abs().max())
        assert float((dr0 - dr1).abs().max()) <= 1e-5 * float(dr0.abs().max())
    # the reductions of a two-part loss with the split point in device memory
    loss = torch.randn(n, generator=g).cuda()
    t0, p0 = L.loss_sums(loss, n_a, 0.5)
    t1, p1 = L.loss_sums(loss, 0, 0.5, n_a_dev)
    assert torch.equal(t0, t1) and torch.equal(p0, p1)
    assert float(p0[0]) == pytest.approx(0.5 * float(loss[:n_a].double().sum()), rel=1e-5, abs=1e-6)
