"""GPU parity of the C-ABI kernels (libkgescore.so) against the reference's golden
vectors and the CPU oracle.  Every call goes through the C ABI via kge._lib.

Tolerances (north star: 1e-4 relative to the row max, fp32):
  * dyadic fixtures: bit-exact for the bilinear models in both precisions (all partial
    sums are exact), bit-exact for TransE L1 sp_/_po;
  * N(0, 0.1) fixtures: <= 2e-5 of the row max for bf16x3, <= 2e-6 for fp32, <= 1e-5
    for the VALU distance kernels; gradients <= 1e-4 of the max |grad| (bf16x3) /
    2e-6 (fp32).
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


def win(model, direction, t):
    """Entity-row columns a query contracts with (CP: second half for sp_, first for _po)."""
    if model != "cp":
        return t
    h = t.shape[1] // 2
    return t[:, h:] if direction == 0 else t[:, :h]
SCORER_FILES = sorted(glob.glob(os.path.join(GOLDEN, "scorer_*.npz")))


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib
    _lib.lib()
    return _lib


def dev(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def rel_err(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.abs(ref).max(axis=-1, keepdims=True) if ref.ndim == 2 else np.abs(ref).max()
    return float((np.abs(x - ref) / np.maximum(scale, 1e-30)).max())


def dist_kind(model, l_norm):
    if model == "transe":
        return (0 if l_norm == 1 else 1), -1.0
    return (2 if l_norm == 1 else 3), 1.0


def forward_all(L, meta, f, prec):
    model = meta["model"]
    mk = MODEL_IDS[model]
    ln = meta["l_norm"] or 1.0
    ent, rel = dev(f["ent"]), dev(f["rel"])
    s, p, o, sub = (dev(f[k], torch.int64) for k in ("s", "p", "o", "subset"))
    d_e, d_r = ent.shape[1], rel.shape[1]
    n = s.numel()
    out = {}
    q_sp = L.prep_query(mk, L.DIR_SP, ent, s, rel, p, n, d_e, d_r)
    q_po = L.prep_query(mk, L.DIR_PO, ent, o, rel, p, n, d_e, d_r)
    if model in K.BILINEAR:
        e_sp, e_po = win(model, 0, ent), win(model, 1, ent)
        out["sp_all"] = L.score_dot(q_sp, e_sp, None, prec)
        out["po_all"] = L.score_dot(q_po, e_po, None, prec)
        out["sp_sub"] = L.score_dot(q_sp, e_sp, sub, prec)
        out["po_sub"] = L.score_dot(q_po, e_po, sub, prec)
    else:
        kind, sign = dist_kind(model, ln)
        out["sp_all"] = L.score_dist(kind, sign, q_sp, ent, None)
        out["po_all"] = L.score_dist(kind, sign, q_po, ent, None)
        out["sp_sub"] = L.score_dist(kind, sign, q_sp, ent, sub)
        out["po_sub"] = L.score_dist(kind, sign, q_po, ent, sub)
    out["spo"] = L.score_spo(mk, ln, ent, s, rel, p, o, d_e, d_r)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
@pytest.mark.parametrize("fn", SCORER_FILES, ids=lambda f: os.path.basename(f)[7:-4])
def test_forward_vs_golden(L, fn, prec):
    f = load_scorer_fixture(fn)
    meta = json.loads(str(f["meta"]))
    out = forward_all(L, meta, f, L.PRECISIONS[prec])
    model = meta["model"]
    for k, v in out.items():
        ref = f[k]
        if meta["regime"] == "dyadic" and (model in K.BILINEAR or (model == "transe" and meta["l_norm"] == 1 and k != "spo")):
            np.testing.assert_array_equal(v, ref, err_msg=f"{k} not bit-exact")
        else:
            tol = 1e-5 if model in K.DISTANCE else (2e-5 if prec == "bf16x3" else 2e-6)
            if k == "spo":
                tol = 2e-6
            assert rel_err(v, ref) < tol, (k, rel_err(v, ref))


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
@pytest.mark.parametrize("fn", SCORER_FILES, ids=lambda f: os.path.basename(f)[7:-4])
def test_gradients_vs_golden(L, fn, prec):
    f = load_scorer_fixture(fn)
    meta = json.loads(str(f["meta"]))
    model = meta["model"]
    mk = MODEL_IDS[model]
    ln = meta["l_norm"] or 1.0
    P = L.PRECISIONS[prec]
    ent, rel = dev(f["ent"]), dev(f["rel"])
    s, p, o = (dev(f[k], torch.int64) for k in ("s", "p", "o"))
    w_sp, w_po, w_spo = dev(f["w_sp"]), dev(f["w_po"]), dev(f["w_spo"])
    d_e, d_r = ent.shape[1], rel.shape[1]
    n = s.numel()
    g_ent = torch.zeros_like(ent)
    g_rel = torch.zeros_like(rel)
    for direction, e_idx, w in ((L.DIR_SP, s, w_sp), (L.DIR_PO, o, w_po)):
        q = L.prep_query(mk, direction, ent, e_idx, rel, p, n, d_e, d_r)
        dq = torch.zeros_like(q)
        if model in K.BILINEAR:
            L.score_dot_bwd_q(w, win(model, direction, ent), None, P, dq=dq, accumulate=False)
            L.score_dot_bwd_t(w, q, None, win(model, direction, g_ent), P)
        else:
            kind, sign = dist_kind(model, ln)
            L.score_dist_bwd(kind, sign, w, q, ent, None, dq, g_ent)
        L.prep_query_bwd(mk, direction, ent, e_idx, rel, p, n, d_e, d_r, dq, g_ent, g_rel)
    L.score_spo_bwd(mk, ln, ent, s, rel, p, o, d_e, d_r, w_spo, g_ent, g_rel)
    torch.cuda.synchronize()
    tol = 1e-4 if (prec == "bf16x3" and model in K.BILINEAR) else 1e-5
    ge, gr = g_ent.cpu().numpy(), g_rel.cpu().numpy()
    assert np.abs(ge - f["g_ent"]).max() <= tol * np.abs(f["g_ent"]).max()
    assert np.abs(gr - f["g_rel"]).max() <= tol * np.abs(f["g_rel"]).max()


def test_rank_counts_vs_oracle(L):
    rng = np.random.default_rng(3)
    n, m, c0 = 37, 1000, 500
    # quantised scores -> many ties; some NaN / inf
    S = (rng.integers(-20, 20, size=(n, m)) / 4).astype(np.float32)
    S[rng.random((n, m)) < 0.01] = np.nan
    S[rng.random((n, m)) < 0.005] = np.inf
    true_idx = rng.integers(c0 - 50, c0 + m + 50, size=n)
    true_score = (rng.integers(-20, 20, size=n) / 4).astype(np.float32)
    true_score[0] = np.nan
    true_score[1] = -np.inf
    fl = [np.unique(rng.integers(c0 - 100, c0 + m + 100, size=rng.integers(0, 40))) for _ in range(n)]
    tl = [np.setdiff1d(np.unique(rng.integers(c0, c0 + m, size=rng.integers(0, 10))), f) for f in fl]
    fl[2] = np.append(fl[2], true_idx[2]) if true_idx[2] not in fl[2] else fl[2]

    def csr(lists):
        ptr = np.zeros(n + 1, np.int64)
        ptr[1:] = np.cumsum([len(x) for x in lists])
        col = np.concatenate(lists).astype(np.int64) if ptr[-1] else np.zeros(1, np.int64)
        return ptr, col

    fp, fc = csr(fl)
    tp, tc = csr(tl)
    greater = torch.zeros(3 * n, dtype=torch.int64, device="cuda")
    ties = torch.zeros(3 * n, dtype=torch.int64, device="cuda")
    L.rank_counts(dev(S), c0, dev(true_idx), dev(true_score), dev(fp), dev(fc), dev(tp), dev(tc), greater, ties)
    g = greater.view(3, n).cpu().numpy()
    t = ties.view(3, n).cpu().numpy()
    # oracle: overwrite the true entry, then -inf the filtered ones (never the true one)
    Sx = S.astype(np.float64).copy()
    for i in range(n):
        if c0 <= true_idx[i] < c0 + m:
            Sx[i, true_idx[i] - c0] = true_score[i]
    raw = K.rank_and_ties(Sx, true_score.astype(np.float64))
    for r, lists in ((1, fl), (2, None)):
        for i in range(n):
            cols = fl[i] if r == 1 else tl[i]
            for j in cols:
                if c0 <= j < c0 + m and j != true_idx[i]:
                    Sx[i, j - c0] = -np.inf
        gr, tr = K.rank_and_ties(Sx, true_score.astype(np.float64))
        np.testing.assert_array_equal(g[r], gr)
        np.testing.assert_array_equal(t[r], tr)
    np.testing.assert_array_equal(g[0], raw[0])
    np.testing.assert_array_equal(t[0], raw[1])


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
def test_score_sp_c2_shape(L, prec):
    """ComplEx-512 at the C2 shape (B=1024, E=14,541): check 64 random rows against the
    float64 oracle, plus a dyadic copy bit-exact (size-independent exactness)."""
    torch.manual_seed(0)
    E, R, B, d = 14541, 237, 1024, 512
    ent = (torch.randn(E, d) * 0.1).cuda()
    rel = (torch.randn(R, d) * 0.1).cuda()
    s = torch.randint(0, E, (B,)).cuda()
    p = torch.randint(0, R, (B,)).cuda()
    q = L.prep_query(0, L.DIR_SP, ent, s, rel, p, B, d, d)
    S = L.score_dot(q, ent, None, L.PRECISIONS[prec])
    rows = torch.randint(0, B, (64,))
    ref = K.prep_sp("complex", ent[s[rows]].double().cpu().numpy(), rel[p[rows]].double().cpu().numpy()) @ \
        ent.double().cpu().numpy().T
    err = rel_err(S[rows.cuda()].cpu().numpy(), ref)
    assert err < (2e-5 if prec == "bf16x3" else 2e-6), err
    # dyadic: exact
    entd = (torch.randint(-16, 17, (E, d)) / 8).float().cuda()
    reld = (torch.randint(-16, 17, (R, d)) / 8).float().cuda()
    qd = L.prep_query(0, L.DIR_SP, entd, s, reld, p, B, d, d)
    Sd = L.score_dot(qd, entd, None, L.PRECISIONS[prec])
    ref = qd.double() @ entd.double().T
    assert torch.equal(Sd.double(), ref)


@pytest.mark.parametrize("n,m,d", [(1, 1, 4), (100, 300, 100), (129, 255, 64), (1024, 14541, 512),
                                   (256, 1000, 36), (300, 2049, 128)])
def test_score_dot_split_shapes(L, n, m, d):
    """Production bf16x3 path (kge_split_rows + kge_score_dot_split): ragged tile edges,
    K tails (d not a multiple of 32), subsets with duplicates; dyadic inputs bit-exact."""
    g = torch.Generator().manual_seed(n * 7 + m + d)
    E = m + 17
    t = (torch.randn(E, d, generator=g) * 0.1).cuda()
    q = (torch.randn(n, d, generator=g) * 0.1).cuda()
    tidx = torch.randint(0, E, (m,), generator=g).cuda()
    hi, lo = L.split_rows(q)
    for ti in (None, tidx):
        s = L.score_dot_split(hi, lo, t, ti, d)
        tt = t if ti is None else t[ti]
        ref = (q.double() @ tt.double().T).cpu().numpy()
        assert rel_err(s.cpu().numpy(), ref) < 2e-5
    qd = (torch.randint(-16, 17, (n, d), generator=g) / 8).float().cuda()
    td = (torch.randint(-16, 17, (E, d), generator=g) / 8).float().cuda()
    hi, lo = L.split_rows(qd)
    s = L.score_dot_split(hi, lo, td, tidx, d)
    assert torch.equal(s.double(), qd.double() @ td[tidx].double().T)


@pytest.mark.parametrize("n,m,d", [(1024, 14541, 512), (512, 40943, 512), (300, 100003, 128)])
def test_score_dot_split_fullsize_properties(L, n, m, d):
    """Size-independent properties of the production contraction at the BASELINE shapes, on
    real-valued N(0, 0.1) operands, all BITWISE (the K order of every element's accumulation does
    not depend on where the element sits in a tile or in the launch):
      * scoring a row-permuted entity table gives the column-permuted score matrix, and the same
        through a candidate index vector (with duplicates);
      * scoring a permutation / a slice of the query rows gives those rows;
      * an entity chunk [c0, c1) scores to the corresponding column slice (the chunked / sharded
        evaluation's decomposition);
      * a second launch reproduces the first."""
    g = torch.Generator().manual_seed(n + m + d)
    t = (torch.randn(m, d, generator=g) * 0.1).cuda()
    q = (torch.randn(n, d, generator=g) * 0.1).cuda()
    hi, lo = L.split_rows(q)
    s = L.score_dot_split(hi, lo, t, None, d)
    assert torch.equal(s, L.score_dot_split(hi, lo, t, None, d))
    perm = torch.randperm(m, generator=g).cuda()
    assert torch.equal(L.score_dot_split(hi, lo, t[perm].contiguous(), None, d), s[:, perm])
    tidx = torch.cat([perm[:m // 2], perm[:m // 3]])  # a subset with duplicates
    assert torch.equal(L.score_dot_split(hi, lo, t, tidx, d), s[:, tidx])
    qperm = torch.randperm(n, generator=g).cuda()
    hp, lp = L.split_rows(q[qperm].contiguous())
    assert torch.equal(L.score_dot_split(hp, lp, t, None, d), s[qperm])
    k = max(1, n // 3)
    hs, ls = L.split_rows(q[:k].contiguous())
    assert torch.equal(L.score_dot_split(hs, ls, t, None, d), s[:k])
    c0, c1 = m // 5 + 3, m // 5 + 3 + (m // 8 + 1)
    assert torch.equal(L.score_dot_split(hi, lo, t[c0:c1], None, d), s[:, c0:c1])
    # and the values themselves, on sampled rows, against float64
    rows = torch.arange(0, n, max(1, n // 32), device="cuda")
    ref = (q[rows].double() @ t.double().T).cpu().numpy()
    assert rel_err(s[rows].cpu().numpy(), ref) < 2e-5


def test_score_dot_split_multitile(L):
    """Persistent schedule with many tiles per workgroup (m = 200,003: 782 column tiles x 4
    row tiles over <= 256 workgroups), launched repeatedly: the schedule under which an
    in-flight register load once had its registers reused (a rare memory fault).  Rows are
    checked against float64 after the last launch; a dyadic copy must be bit-exact."""
    g = torch.Generator().manual_seed(11)
    n, m, d = 1024, 200003, 512
    t = (torch.randint(-16, 17, (m, d), generator=g) / 8).float().cuda()
    q = (torch.randint(-16, 17, (n, d), generator=g) / 8).float().cuda()
    hi, lo = L.split_rows(q)
    s = torch.empty(n, m, device="cuda")
    for _ in range(20):
        L.score_dot_split(hi, lo, t, None, d, out=s)
    torch.cuda.synchronize()
    rows = torch.arange(0, n, 61, device="cuda")
    assert torch.equal(s[rows].double(), q[rows].double() @ t.double().T)
    tr = (torch.randn(m, d, generator=g) * 0.1).cuda()
    L.score_dot_split(hi, lo, tr, None, d, out=s)
    ref = (q[rows].double() @ tr.double().T).cpu().numpy()
    assert rel_err(s[rows].cpu().numpy(), ref) < 2e-5


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("d", [64, 512, 30])
def test_score_dist_tiled_and_generic_kernels(L, kind, d):
    """Both all-entities distance kernels against float64 and against each other: the
    register-tiled kernel (score_dist2.hip) takes 16-B-aligned rows with a component count
    that is a multiple of 4; any other layout -- here rows with an odd leading dimension, and
    d = 30 (RotatE: 15 complex components) -- takes the generic kernel (score_dist.hip)."""
    g = torch.Generator().manual_seed(kind * 100 + d)
    n, m = 100, 501
    q = (torch.randn(n, d, generator=g) * 0.1).cuda()
    t = (torch.randn(m + 7, d, generator=g) * 0.1).cuda()
    sub = torch.randint(0, m + 7, (m,), generator=g).cuda()
    # the same values in rows that are only 4-B aligned (leading dimension d + 1)
    q_odd = torch.zeros(n, d + 1, device="cuda")[:, :d]
    q_odd.copy_(q)
    t_odd = torch.zeros(m + 7, d + 1, device="cuda")[:, :d]
    t_odd.copy_(t)
    outs = {2: (L.score_dist(kind, -1.0, q, t, None), L.score_dist(kind, -1.0, q, t, sub)),
            1: (L.score_dist(kind, -1.0, q_odd, t_odd, None), L.score_dist(kind, -1.0, q_odd, t_odd, sub))}
    qq, tt = q.double().cpu(), t.double().cpu()
    if kind < 2:
        diff = qq[:, None, :] - tt[None, :, :]
        ref = -(diff.abs().sum(-1) if kind == 0 else diff.pow(2).sum(-1).sqrt())
    else:
        h = d // 2
        dr = qq[:, None, :h] - tt[None, :, :h]
        di = qq[:, None, h:] - tt[None, :, h:]
        mod = (dr * dr + di * di).sqrt()
        ref = -(mod.sum(-1) if kind == 2 else mod.pow(2).sum(-1).sqrt())
    for impl in (1, 2):
        a, b = outs[impl]
        assert rel_err(a.cpu().numpy(), ref.numpy()) < 1e-5, (impl, "all")
        assert rel_err(b.cpu().numpy(), ref[:, sub.cpu()].numpy()) < 1e-5, (impl, "subset")
    assert rel_err(outs[2][0].cpu().numpy(), outs[1][0].cpu().double().numpy()) < 1e-5


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("d", [72, 512, 30])
def test_score_dist_bwd_owner_and_generic_kernels(L, kind, d):
    """Backward of the all-entities distance scores against float64 autograd, for dL/dS = G:
    the owner-computes kernels (score_dist_bwd2.hip: L1 kinds directly, L2 kinds through pair
    weights G / dist) on float4-readable rows -- d = 72 leaves a partial block of components,
    the candidate subset repeats rows (their gradients add up), n and m are ragged -- and the
    generic kernel on rows with an odd leading dimension and on d = 30; both accumulate into
    dq / dt."""
    g = torch.Generator().manual_seed(kind * 100 + d)
    n, m, extra = 131, 300, 9
    # values on a grid so that exact zeros of q - t occur (sign(0) = 0, |0| has gradient 0)
    q = (torch.randint(-8, 9, (n, d), generator=g) / 16.0).cuda()
    t = (torch.randint(-8, 9, (m + extra, d), generator=g) / 16.0).cuda()
    sub = torch.randint(0, m + extra, (m,), generator=g).cuda()
    sign = -1.0 if kind < 2 else 1.0

    def reference(rows, G):
        qq = q.double().cpu().requires_grad_(True)
        tt = t.double().cpu().requires_grad_(True)
        tr = tt if rows is None else tt[rows.cpu()]
        if kind < 2:
            diff = qq[:, None, :] - tr[None, :, :]
            dist = diff.abs().sum(-1) if kind == 0 else diff.pow(2).sum(-1).sqrt()
        else:
            h = d // 2
            dr = qq[:, None, :h] - tr[None, :, :h]
            di = qq[:, None, h:] - tr[None, :, h:]
            sq = dr * dr + di * di
            mod = torch.where(sq > 0, sq.clamp_min(1e-300).sqrt(), torch.zeros_like(sq))
            dist = mod.sum(-1) if kind == 2 else sq.sum(-1).sqrt()
        (sign * dist * G.double().cpu()).sum().backward()
        return qq.grad.numpy(), tt.grad.numpy()

    for rows in (None, sub):
        cols = m + extra if rows is None else m
        G = torch.randn(n, cols, generator=g).cuda()
        ref_q, ref_t = reference(rows, G)
        tol = 2e-5 * max(1.0, float(np.abs(ref_q).max()), float(np.abs(ref_t).max()))
        for odd in (False, True):
            if odd:  # rows that are only 4-B aligned: the generic kernel
                q_in = torch.zeros(n, d + 1, device="cuda")[:, :d]
                q_in.copy_(q)
                t_in = torch.zeros(m + extra, d + 1, device="cuda")[:, :d]
                t_in.copy_(t)
            else:
                q_in, t_in = q, t
            dq = torch.full((n, d), 0.5, device="cuda")
            dt = torch.full((m + extra, d), -0.25, device="cuda")
            L.score_dist_bwd(kind, sign, G, q_in, t_in, rows, dq, dt)
            got_q, got_t = (dq - 0.5).cpu().numpy(), (dt + 0.25).cpu().numpy()
            assert np.abs(got_q - ref_q).max() < tol, (kind, d, rows is None, odd, "dq")
            assert np.abs(got_t - ref_t).max() < tol, (kind, d, rows is None, odd, "dt")


def test_contract_dispatch_and_errors(L):
    q = torch.randn(8, 6).cuda()
    t = torch.randn(20, 6).cuda()
    s = L.contract(q, t, None, L.PREC_BF16X3)  # d % 4 != 0 -> generic kernel
    assert rel_err(s.cpu().numpy(), (q.double() @ t.double().T).cpu().numpy()) < 2e-5
    with pytest.raises(ValueError):
        L.score_dot(q, torch.randn(20, 5).cuda(), None, L.PREC_BF16X3)


@pytest.mark.parametrize("m", [1, 7, 1001, 14541])
@pytest.mark.parametrize("layout", ["padded_inplace", "padded_out", "tight_inplace"])
def test_softmax_xent_vs_oracle(L, m, layout):
    """kge_softmax_xent: per-row CE + G = scale * (softmax - onehot), vectorised (rows
    padded to 16 B) and scalar (tight, odd leading dimension) paths, in place and not."""
    rng = np.random.default_rng(m)
    n = 37
    S = (rng.standard_normal((n, m)) * 5).astype(np.float32)
    if m > 8:
        S[3, :] = -np.inf          # -inf entries add 0 ...
        S[3, : m // 2] = rng.standard_normal(m // 2)
        S[5, 1::3] = -np.inf
    labels = rng.integers(0, m, size=n)
    scale = 1.0 / n
    ref_loss, ref_g = K.softmax_xent(S.astype(np.float64), labels, scale)
    ld = (m + 3) // 4 * 4 if layout.startswith("padded") else m
    buf = torch.full((n, ld), 123.0, device="cuda")
    s = buf[:, :m]
    s.copy_(dev(S))
    g = s if layout.endswith("inplace") else torch.zeros((n, ld), device="cuda")[:, :m]
    loss = L.softmax_xent(s, dev(labels, torch.int64), scale, g=g)
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss.cpu().numpy(), ref_loss, rtol=2e-6, atol=2e-6 * np.abs(ref_loss).max())
    gg = g.cpu().numpy()
    assert np.abs(gg - ref_g).max() <= 2e-6 * scale, np.abs(gg - ref_g).max() / scale
    if ld > m:  # padding columns untouched
        assert torch.all(buf[:, m:] == 123.0) if layout == "padded_inplace" else True


def test_softmax_xent_edge_cases(L):
    n, m = 4, 50
    S = np.zeros((n, m), np.float32)
    S[1, 7] = np.nan
    S[2, :] = -np.inf
    labels = np.array([0, 1, 2, m + 5])  # last label out of range
    s = dev(S)
    lab = dev(labels, torch.int64)
    out = torch.empty(n, device="cuda")
    # raw C ABI: the Python wrapper's index check (KGE_CHECK_INDEX) would reject the label
    assert L.lib().kge_softmax_xent(L.ptr(s), m, n, m, L.ptr(lab), 1.0, L.ptr(out), None, 0, L.stream()) == 0
    loss = out.cpu().numpy()
    assert abs(loss[0] - np.log(m)) < 1e-6   # uniform row
    assert np.isnan(loss[1])                 # NaN score -> NaN loss (torch CE likewise)
    assert np.isnan(loss[2])                 # all -inf row -> NaN (torch: nan)
    assert np.isnan(loss[3])                 # label out of range
    assert L.lib().kge_softmax_xent(L.ptr(s), m - 1, n, m, L.ptr(lab), 1.0, L.ptr(out), None, 0,
                                    L.stream()) == 1001  # KGE_ERR_ARG: lds < m


@pytest.mark.parametrize("n,m,d", [(300, 1001, 64), (1024, 2053, 512), (5, 17, 8)])
@pytest.mark.parametrize("g_layout", ["padded", "tight"])
@pytest.mark.parametrize("gather", [False, True])
def test_backward_gemms_layouts(L, n, m, d, g_layout, gather):
    """dQ = G.T[tidx] and dT[tidx] += G^T.Q in bf16x3: the vectorised kernel (G rows padded
    to 16 B, as kge_softmax_xent writes them; transposed LDS reads) and the scalar one
    (tight odd leading dimension, as autograd hands G over), with and without a candidate
    gather (duplicates included), against float64."""
    rng = np.random.default_rng(n + m + d)
    G = rng.standard_normal((n, m)).astype(np.float32)
    Q = rng.standard_normal((n, d)).astype(np.float32)
    E = m + 7 if gather else m
    T = rng.standard_normal((E, d)).astype(np.float32)
    tidx = rng.integers(0, E, size=m) if gather else None
    ld = (m + 3) // 4 * 4 + 4 if g_layout == "padded" else m
    gb = torch.zeros((n, ld), device="cuda")
    gb[:, :m] = dev(G)
    g = gb[:, :m]
    Tr = T[tidx] if gather else T
    dq = L.score_dot_bwd_q(g, dev(T), dev(tidx, torch.int64) if gather else None, L.PREC_BF16X3)
    dt = torch.zeros(E, d, device="cuda")
    L.score_dot_bwd_t(g, dev(Q), dev(tidx, torch.int64) if gather else None, dt, L.PREC_BF16X3)
    torch.cuda.synchronize()
    ref_q = G.astype(np.float64) @ Tr.astype(np.float64)
    ref_t = np.zeros((E, d))
    np.add.at(ref_t, tidx if gather else np.arange(m), G.T.astype(np.float64) @ Q.astype(np.float64))
    assert rel_err(dq.cpu().numpy(), ref_q) < 2e-5
    assert rel_err(dt.cpu().numpy(), ref_t) < 2e-5
