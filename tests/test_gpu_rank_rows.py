"""GPU parity of the stacked ranking launch (kge_rank_rows) through the C ABI:
* its counts, ranks and histograms against the CPU oracle's rank_and_ties / get_ranks
  (entity_ranking.py:469-551 restated) and against the per-direction kge_rank_counts +
  kge_rank_hist_multi pair it replaces -- bit-exact (integer work);
* its refinement of reduced-precision scores: counts must EQUAL those of exactly computed
  scores (float64 dot products rounded to fp32) on inputs built to be full of near-ties that
  the bf16x3 contraction mis-orders."""
import math

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


def _csr(rng, n, m, max_len):
    lens = rng.integers(0, max_len + 1, size=n)
    lens[0] = 0
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=ptr[1:])
    col = np.concatenate([rng.choice(m, size=k, replace=False) for k in lens] + [np.zeros(0, np.int64)])
    return ptr, col.astype(np.int64)


def _minus(ptr_a, col_a, ptr_b, col_b):
    """Per-row A \\ B."""
    out_ptr, out = [0], []
    for i in range(len(ptr_a) - 1):
        b = set(col_b[ptr_b[i]:ptr_b[i + 1]].tolist())
        keep = [c for c in col_a[ptr_a[i]:ptr_a[i + 1]].tolist() if c not in b]
        out += keep
        out_ptr.append(len(out))
    return np.asarray(out_ptr, np.int64), np.asarray(out, np.int64)


def _oracle_counts(scores, c0, true_idx, true_score, lists):
    """[1 + len(lists)] x (greater, ties) of one batch: the true entry takes the true score,
    list entries (global ids, cumulative over the lists) go to -inf."""
    sc = scores.copy()
    n, m = sc.shape
    for i in range(n):
        j = true_idx[i] - c0
        if 0 <= j < m:
            sc[i, j] = true_score[i]
    out = [K.rank_and_ties(sc, true_score)]
    for ptr, col in lists:
        for i in range(n):
            for j in col[ptr[i]:ptr[i + 1]]:
                if c0 <= j < c0 + m and j != true_idx[i]:
                    sc[i, j - c0] = -np.inf
        out.append(K.rank_and_ties(sc, true_score))
    return out


def _dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


@pytest.mark.parametrize("n_a,n_b,m,c0,ld,with_test", [
    (37, 37, 1001, 0, 1004, True),      # padded rows: vector loads
    (16, 9, 517, 100, 517, True),       # odd leading dimension: scalar loads; a chunk at c0 = 100
    (5, 0, 64, 0, 64, False),           # one batch only, raw + filtered
    (64, 64, 14541, 0, 14544, True),    # FB15K-237 width
])
def test_rank_rows_counts_ranks_hists_vs_oracle_and_rank_counts(L, n_a, n_b, m, c0, ld, with_test):
    rng = np.random.default_rng(n_a * 7 + m)
    n = n_a + n_b
    E = c0 + m + 50  # entity ids beyond the chunk exist
    # coarse scores: plenty of exact ties; NaN and infinities sprinkled in
    sc = np.round(rng.standard_normal((n, m)).astype(np.float32) * 4) / 4
    sc[rng.random((n, m)) < 0.002] = np.nan
    sc[rng.random((n, m)) < 0.001] = np.inf
    sc[rng.random((n, m)) < 0.001] = -np.inf
    true_idx = rng.integers(0, E, size=n).astype(np.int64)
    true_score = (np.round(rng.standard_normal(n).astype(np.float32) * 4) / 4).astype(np.float32)
    true_score[0] = np.nan
    if n > 3:
        true_score[3] = -np.inf
    f_ptr_a, f_col_a = _csr(rng, n_a, E, 40)
    f_ptr_b, f_col_b = _csr(rng, n_b, E, 40) if n_b else (np.zeros(1, np.int64), np.zeros(0, np.int64))
    t_a = _minus(*_csr(rng, n_a, E, 25), f_ptr_a, f_col_a)
    t_b = _minus(*_csr(rng, n_b, E, 25), f_ptr_b, f_col_b) if n_b else (np.zeros(1, np.int64), np.zeros(0, np.int64))
    nrank = 3 if with_test else 2

    exp = []  # per batch: [(greater, ties)] * nrank
    for r0, r1, (fp, fc), (tp, tc) in ((0, n_a, (f_ptr_a, f_col_a), t_a), (n_a, n, (f_ptr_b, f_col_b), t_b)):
        lists = [(fp, fc)] + ([(tp, tc)] if with_test else [])
        exp.append(_oracle_counts(sc[r0:r1], c0, true_idx[r0:r1], true_score[r0:r1], lists))
    exp_g = np.stack([np.concatenate([exp[0][r][0], exp[1][r][0]]) for r in range(nrank)])
    exp_t = np.stack([np.concatenate([exp[0][r][1], exp[1][r][1]]) for r in range(nrank)])

    buf = torch.full((n, ld), 3.25, device="cuda")
    buf[:, :m] = _dev(sc)
    s = buf[:, :m]
    ti, ts = _dev(true_idx), _dev(true_score)
    f_col = _dev(np.concatenate([f_col_a, f_col_b, np.zeros(1, np.int64)]))
    t_col = _dev(np.concatenate([t_a[1], t_b[1], np.zeros(1, np.int64)]))
    fpa, fpb = _dev(f_ptr_a), _dev(f_ptr_b + len(f_col_a))
    tpa, tpb = (_dev(t_a[0]), _dev(t_b[0] + len(t_a[1]))) if with_test else (None, None)
    part_a = (ti[:n_a], ts[:n_a], fpa, tpa)
    part_b = (ti[n_a:], ts[n_a:], fpb, tpb) if n_b else None

    for tie in ("rounded_mean_rank", "best_rank", "worst_rank"):
        g = torch.full((nrank * n,), -7, dtype=torch.int64, device="cuda")  # overwritten, not added to
        t = torch.full((nrank * n,), -7, dtype=torch.int64, device="cuda")
        rk = torch.empty(nrank * n, dtype=torch.int64, device="cuda")
        rows_per_hist = n_a if n_b == n_a else n
        hists = torch.zeros(nrank * n // rows_per_hist, E, device="cuda")
        L.rank_rows(s, n_a, c0, part_a, part_b, f_col, t_col if with_test else None, g, t, accumulate=False,
                    tie_handling=tie, ranks=rk, hists=hists, rows_per_hist=rows_per_hist)
        torch.cuda.synchronize()
        assert np.array_equal(g.view(nrank, n).cpu().numpy(), exp_g)
        assert np.array_equal(t.view(nrank, n).cpu().numpy(), exp_t)
        exp_rk = K.get_ranks(exp_g, exp_t, tie)
        assert np.array_equal(rk.view(nrank, n).cpu().numpy(), exp_rk)
        flat = exp_rk.reshape(-1)
        exp_h = np.zeros((nrank * n // rows_per_hist, E), np.float32)
        for x, r in enumerate(flat):
            if 0 <= r < E:
                exp_h[x // rows_per_hist, r] += 1
        assert np.array_equal(hists.cpu().numpy(), exp_h)

    # accumulate mode adds to what the buffers hold; the per-direction kernel it replaces agrees
    g = torch.full((nrank * n,), 5, dtype=torch.int64, device="cuda")
    t = torch.full((nrank * n,), 2, dtype=torch.int64, device="cuda")
    L.rank_rows(s, n_a, c0, part_a, part_b, f_col, t_col if with_test else None, g, t, accumulate=True)
    assert np.array_equal(g.view(nrank, n).cpu().numpy(), exp_g + 5)
    assert np.array_equal(t.view(nrank, n).cpu().numpy(), exp_t + 2)
    for r0, r1, fp, fc, tp, tc in ((0, n_a, f_ptr_a, f_col_a, *t_a), (n_a, n, f_ptr_b, f_col_b, *t_b)):
        if r1 == r0:
            continue
        k = r1 - r0
        g1 = torch.zeros(3 * k, dtype=torch.int64, device="cuda")
        t1 = torch.zeros(3 * k, dtype=torch.int64, device="cuda")
        L.rank_counts(s[r0:r1], c0, ti[r0:r1], ts[r0:r1], _dev(fp), _dev(np.concatenate([fc, [0]])),
                      _dev(tp) if with_test else None, _dev(np.concatenate([tc, [0]])) if with_test else None, g1, t1)
        assert np.array_equal(g1.view(3, k)[:nrank].cpu().numpy(), exp_g[:, r0:r1])
        assert np.array_equal(t1.view(3, k)[:nrank].cpu().numpy(), exp_t[:, r0:r1])


@pytest.mark.parametrize("d,m", [(512, 3000), (128, 1500)])
def test_rank_rows_refinement_equals_exact_scoring(L, d, m):
    """Candidate rows built as tiny perturbations of each query's true row give scores within
    1e-7 .. 1e-5 of the true score: the bf16x3 contraction (error up to ~1e-5 of the row
    maximum) puts many of them on the wrong side; the refined counts must equal the counts of
    float64 dot products rounded to fp32 -- for the raw and the filtered ranking."""
    rng = np.random.default_rng(d + m)
    n = 48
    q = (rng.standard_normal((n, d)) * 0.3).astype(np.float32)
    t = (rng.standard_normal((m, d)) * 0.3).astype(np.float32)
    true_idx = rng.choice(m, size=n, replace=False).astype(np.int64)
    # 20 near-copies of every query's true row, at relative distances 1e-7 .. 1e-5
    for i in range(n):
        for c in range(20):
            j = (true_idx[i] + 1 + c * 53 + i) % m
            if j in true_idx:
                continue
            eps = 10.0 ** rng.uniform(-7, -5) * rng.choice([-1.0, 1.0])
            t[j] = (t[true_idx[i]].astype(np.float64) * (1.0 + eps)
                    + rng.standard_normal(d) * 1e-7).astype(np.float32)
    exact = (q.astype(np.float64) @ t.astype(np.float64).T).astype(np.float32)
    true_score = exact[np.arange(n), true_idx].copy()
    f_ptr, f_col = _csr(rng, n, m, 30)
    # filter lists that hit near-ties too: add each row's first near-copy
    cols = [np.unique(np.append(f_col[f_ptr[i]:f_ptr[i + 1]], (true_idx[i] + 1 + i) % m)) for i in range(n)]
    f_ptr = np.zeros(n + 1, np.int64)
    np.cumsum([len(c) for c in cols], out=f_ptr[1:])
    f_col = np.concatenate(cols).astype(np.int64)
    exp = _oracle_counts(exact, 0, true_idx, true_score, [(f_ptr, f_col)])

    qd, td = _dev(q), _dev(t)
    hi, lo = L.split_rows(qd)
    buf = torch.empty(n, (m + 3) // 4 * 4, device="cuda")
    s = L.score_dot_split(hi, lo, td, None, d, out=buf[:, :m])
    part = (_dev(true_idx), _dev(true_score), _dev(f_ptr), None)
    f_col_d = _dev(np.concatenate([f_col, [0]]))

    def counts(refine):
        g = torch.empty(2 * n, dtype=torch.int64, device="cuda")
        tt = torch.empty(2 * n, dtype=torch.int64, device="cuda")
        L.rank_rows(s, n, 0, part, None, f_col_d, None, g, tt, accumulate=False, refine=refine)
        return g.view(2, n).cpu().numpy(), tt.view(2, n).cpu().numpy()

    tmax = L.row_norm_max(td)
    assert float(tmax) == pytest.approx(np.linalg.norm(t.astype(np.float64), axis=1).max(), rel=1e-5)
    g0, t0 = counts(None)
    wrong = int((g0[0] != exp[0][0]).sum())
    g1, t1 = counts((qd, td, 1e-4, tmax))
    for r in range(2):
        assert np.array_equal(g1[r], exp[r][0]), f"ranking {r}: refined 'greater' counts differ from exact scoring"
        assert np.array_equal(t1[r], exp[r][1]), f"ranking {r}: refined tie counts differ from exact scoring"
    # the inputs do exercise the refinement: plain bf16x3 scores mis-count some rows
    assert wrong > 0, "test inputs too easy: bf16x3 ranked every near-tie correctly"
    # the contraction's error is far inside the band the refinement assumes
    err = np.abs(s.cpu().numpy().astype(np.float64) - q.astype(np.float64) @ t.astype(np.float64).T)
    bound = np.linalg.norm(q.astype(np.float64), axis=1)[:, None] * float(tmax)
    assert (err / bound).max() < 0.25e-4


@pytest.mark.parametrize("m,near", [(6000, 5000), (6000, 2048), (6000, 2049), (9001, 9000)])
def test_rank_rows_refinement_rows_with_thousands_of_near_ties(L, m, near):
    """More entries inside the band than the kernel's near-tie ring holds (2,048): such a row is
    scanned a second time, rescoring after every step.  `near` candidate rows are copies of the
    true row up to a 1e-6 relative perturbation; refined counts must equal exact scoring, raw and
    filtered, on rows of both kinds in the same launch."""
    rng = np.random.default_rng(m + near)
    n, d = 6, 128
    q = (rng.standard_normal((n, d)) * 0.3).astype(np.float32)
    t = (rng.standard_normal((m, d)) * 0.3).astype(np.float32)
    true_idx = np.arange(n, dtype=np.int64) * 7
    crowded = [3]  # this query's true row is copied `near` times
    pool = np.setdiff1d(np.arange(m), true_idx)
    for i in crowded:
        js = rng.choice(pool, size=min(near, len(pool)), replace=False)
        eps = rng.uniform(-1e-6, 1e-6, size=(len(js), 1))
        t[js] = (t[true_idx[i]].astype(np.float64)[None] * (1.0 + eps)).astype(np.float32)
        # make them near-ties of query i only by giving query i a large component along its true row
        q[i] = (t[true_idx[i]] * 2.0 + q[i] * 0.01).astype(np.float32)
    exact = (q.astype(np.float64) @ t.astype(np.float64).T).astype(np.float32)
    true_score = exact[np.arange(n), true_idx].copy()
    f_ptr, f_col = _csr(rng, n, m, 40)
    exp = _oracle_counts(exact, 0, true_idx, true_score, [(f_ptr, f_col)])
    qd, td = _dev(q), _dev(t)
    hi, lo = L.split_rows(qd)
    buf = torch.empty(n, (m + 3) // 4 * 4, device="cuda")
    s = L.score_dot_split(hi, lo, td, None, d, out=buf[:, :m])
    part = (_dev(true_idx), _dev(true_score), _dev(f_ptr), None)
    g = torch.empty(2 * n, dtype=torch.int64, device="cuda")
    tt = torch.empty(2 * n, dtype=torch.int64, device="cuda")
    tmax = L.row_norm_max(td)
    band = 1e-4
    L.rank_rows(s, n, 0, part, None, _dev(np.concatenate([f_col, [0]])), None, g, tt, accumulate=False,
                refine=(qd, td, band, tmax))
    in_band = (np.abs(s.cpu().numpy() - true_score[:, None])
               <= band * np.linalg.norm(q, axis=1)[:, None] * float(tmax)).sum(1)
    assert (in_band[crowded] >= min(near, len(pool))).all() and in_band[1] < 2048
    g, tt = g.view(2, n).cpu().numpy(), tt.view(2, n).cpu().numpy()
    for r in range(2):
        assert np.array_equal(g[r], exp[r][0]), (r, g[r], exp[r][0])
        assert np.array_equal(tt[r], exp[r][1]), (r, tt[r], exp[r][1])


@pytest.mark.parametrize("model,dim", [("distmult", 64), ("rescal", 16), ("simple", 64), ("complex", 64), ("cp", 64),
                                       ("transe", 64), ("rotate", 64), ("complex", 50), ("distmult", 37)])
@pytest.mark.parametrize("chunk", [-1, 700])
def test_refined_eval_job_every_model_vs_exact_scoring(model, dim, chunk):
    """EntityRankingJob with engine.eval_precision bf16x3_refined (the default) for every
    scorer against the oracle's job on float64 scores rounded to fp32 (entity_ranking.py:79-577
    restated): DistMult / RESCAL / SimplE / ComplEx take the refined bf16x3 path, CP, the
    distance models and row widths the rescoring cannot read as float4 (dim 50, 37) fall back to
    fp32 scoring.  The engine prepares its query rows in fp32, so
    a rank may differ from exact scoring only at a near-tie at the level of fp32 rounding:
    every moved rank is checked against the float64 score row (1e-6 of the row maximum)."""
    from test_gpu_configs import base_config, set_tables
    from kge import Dataset, KgeModel
    from kge.job import EntityRankingJob

    E, R, n_eval = 2000, 11, 300
    rng = np.random.default_rng(sum(map(ord, model)) + dim)
    ent = (rng.standard_normal((E, dim)) * 0.3).astype(np.float32)

    def triples(k):
        return np.stack([rng.integers(0, E, k), rng.integers(0, R, k), rng.integers(0, E, k)], 1).astype(np.int64)

    splits = {"train": triples(4000), "valid": triples(n_eval), "test": triples(500)}
    # near-ties on purpose: entity rows that nearly repeat other rows
    for j in range(0, 200, 2):
        ent[1000 + j] = ent[j] * np.float32(1 + 3e-7 * (j % 5 - 2))
    c = base_config(model, dim, E, R, {"eval.batch_size": 128, "eval.split": "valid",
                                       "entity_ranking.chunk_size": chunk})
    assert c.get("engine.eval_precision") == "bf16x3_refined"
    ds = Dataset(c, None)
    ds._triples = {k: torch.from_numpy(v.astype(np.int32)) for k, v in splits.items()}
    m = KgeModel.create(c, ds)
    d_r = m._relation_embedder._embeddings.weight.shape[1]  # config-derived (rotate d/2, rescal d^2, cp d/2)
    rel = (rng.standard_normal((R, d_r)) * 0.3).astype(np.float32)
    if model == "rotate":
        rel = (rng.uniform(-np.pi, np.pi, (R, d_r))).astype(np.float32)
    set_tables(m, ent, rel)
    job = EntityRankingJob(c, ds, model=m)
    job.capture_ranks = True
    job.run()
    l_norm = float(c.get(model + ".l_norm")) if model in K.DISTANCE else 1.0
    ranks, _ = K.entity_ranking(model, ent, rel, splits, eval_split="valid", filter_splits=("train", "valid"),
                                batch_size=128, l_norm=l_norm)
    assert set(job.ranks) == set(ranks)
    tri = splits["valid"]
    moved = 0
    for key, exp in ranks.items():
        bad = np.flatnonzero(job.ranks[key] != exp)
        moved += len(bad)
        for i in bad:
            s, p, o = tri[i:i + 1, 0], tri[i:i + 1, 1], tri[i:i + 1, 2]
            sc = K.model_scores(model, ent, rel, s, p, o, np.arange(1), l_norm)
            row = sc["sp_all"][0] if key[0] == "o" else sc["po_all"][0]
            dist = np.abs(row - sc["spo"][0]) / np.abs(row).max()
            dist[o[0] if key[0] == "o" else s[0]] = np.inf
            delta = abs(int(job.ranks[key][i]) - int(exp[i]))
            assert np.sort(dist)[delta - 1] <= 1e-6, (key, i, delta, np.sort(dist)[:delta])
    assert moved <= 0.02 * sum(len(v) for v in ranks.values())


def _near_tie_tables(rng, n, m, d, copies):
    """Query rows, candidate rows and true columns with `copies` near-copies of every query's
    true row at relative distances 1e-7 .. 1e-5 (scores the bf16x3 contraction mis-orders)."""
    q = (rng.standard_normal((n, d)) * 0.3).astype(np.float32)
    t = (rng.standard_normal((m, d)) * 0.3).astype(np.float32)
    true_idx = rng.choice(m, size=n, replace=False).astype(np.int64)
    for i in range(n):
        for c in range(copies):
            j = (true_idx[i] + 1 + c * 53 + i) % m
            if j in true_idx:
                continue
            eps = 10.0 ** rng.uniform(-7, -5) * rng.choice([-1.0, 1.0])
            t[j] = (t[true_idx[i]].astype(np.float64) * (1.0 + eps) + rng.standard_normal(d) * 1e-7).astype(np.float32)
    return q, t, true_idx


def _random_rank_cases(count, seed=20):
    """Seeded random shapes for the fused-ranking test: ragged batches (the second one empty now and
    then), entity counts around and between the 256-column panels, row widths that are multiples of 4
    but not of the 32-column K stage, chunk offsets, padded code rows."""
    rng = np.random.default_rng(seed)
    cases = []
    for _ in range(count):
        n_a = int(rng.integers(5, 420))
        n_b = 0 if rng.random() < 0.2 else (n_a if rng.random() < 0.3 else int(rng.integers(1, 420)))
        m = int(rng.choice([rng.integers(n_a + n_b, n_a + n_b + 300), rng.integers(1000, 6000),
                            256 * rng.integers(4, 12) + rng.integers(-1, 2)]))
        m = max(m, n_a + n_b)
        c0 = int(rng.choice([0, 0, rng.integers(1, 900)]))
        max_filt = min(int(rng.choice([3, 30, 300])), (c0 + m + 40) // 2)  # lists drawn without replacement
        cases.append((n_a, n_b, m, c0, int(rng.choice([8, 20, 36, 64, 100, 132, 256, 516])), bool(rng.random() < 0.5),
                      bool(rng.random() < 0.7), max_filt, int(rng.choice([0, 0, 1, 2, 3]))))
    return cases


@pytest.mark.parametrize("n_a,n_b,m,c0,d,with_test,refined,max_filt,ld_pad", _random_rank_cases(12) + [
    (300, 300, 3001, 0, 512, True, True, 30, 0),     # two 256-row tiles per batch, a ragged last entity panel
    (100, 100, 1000, 700, 128, True, True, 30, 0),   # 128-row tiles; a chunk starting at column 700
    (64, 0, 257, 0, 64, False, True, 30, 0),         # one batch; one column past a panel
    (300, 211, 2050, 0, 256, True, False, 30, 0),    # no refinement: the bf16x3 scores compared as they are
    (40, 40, 40000, 0, 64, True, True, 700, 0),      # rows of more than 256 word quads, filter lists of more
                                                     # than 256 columns: the ranking kernel's later rounds
    (40, 40, 40000, 300, 64, True, False, 700, 0),
    (100, 100, 1000, 700, 128, True, True, 400, 3),  # code rows off 16-byte boundaries: read word by word
])
def test_fused_rank_codes_give_the_score_block_counts(L, n_a, n_b, m, c0, d, with_test, refined, max_filt, ld_pad):
    """kge_score_dot_split_rank + kge_rank_rows_codes (the scores never written: compared with
    the true score in the contraction's epilogue, 2-bit codes out) against kge_score_dot_split +
    kge_rank_rows on the score block: the same contraction, the same band, the same exact
    rescoring -- every count, rank and histogram must be IDENTICAL, with filter lists, a true
    column outside the chunk, NaN / -inf true scores and near-ties in the table."""
    rng = np.random.default_rng(n_a + 3 * m)
    n = n_a + n_b
    E = c0 + m + 40
    q, t, true_local = _near_tie_tables(rng, n, m, d, 12)
    true_idx = true_local + c0
    true_idx[1] = c0 + m + 5  # the true entity lies outside this chunk
    exact = (q.astype(np.float64) @ t.astype(np.float64).T).astype(np.float32)
    true_score = exact[np.arange(n), true_local].copy()
    true_score[2] = np.nan
    true_score[4] = -np.inf
    f_ptr_a, f_col_a = _csr(rng, n_a, E, max_filt)
    f_ptr_b, f_col_b = _csr(rng, n_b, E, max_filt) if n_b else (np.zeros(1, np.int64), np.zeros(0, np.int64))
    n_test = max_filt * 2 // 3
    t_a = _minus(*_csr(rng, n_a, E, n_test), f_ptr_a, f_col_a)
    t_b = _minus(*_csr(rng, n_b, E, n_test), f_ptr_b, f_col_b) if n_b else (np.zeros(1, np.int64), np.zeros(0, np.int64))
    nrank = 3 if with_test else 2
    qd, td = _dev(q), _dev(t)
    hi, lo = L.split_rows(qd)
    ti, ts = _dev(true_idx), _dev(true_score)
    f_col = _dev(np.concatenate([f_col_a, f_col_b, np.zeros(1, np.int64)]))
    t_col = _dev(np.concatenate([t_a[1], t_b[1], np.zeros(1, np.int64)])) if with_test else None
    fpa, fpb = _dev(f_ptr_a), _dev(f_ptr_b + len(f_col_a))
    tpa, tpb = (_dev(t_a[0]), _dev(t_b[0] + len(t_a[1]))) if with_test else (None, None)
    part_a = (ti[:n_a], ts[:n_a], fpa, tpa)
    part_b = (ti[n_a:], ts[n_a:], fpb, tpb) if n_b else None
    tmax = L.row_norm_max(td)
    band_rel = 1e-4
    refine = (qd, td, band_rel, tmax) if refined else None
    rows_per_hist = n_a if n_b == n_a else n

    def run(codes_path):
        g = torch.full((nrank * n,), -7, dtype=torch.int64, device="cuda")
        tt = torch.full((nrank * n,), -7, dtype=torch.int64, device="cuda")
        rk = torch.empty(nrank * n, dtype=torch.int64, device="cuda")
        hists = torch.zeros(nrank * n // rows_per_hist, E, device="cuda")
        kw = dict(accumulate=False, tie_handling="rounded_mean_rank", ranks=rk, hists=hists,
                  rows_per_hist=rows_per_hist, refine=refine)
        if codes_path:
            band = L.rank_band(qd, band_rel, tmax) if refined else torch.full((n,), -1.0, device="cuda")
            ldc = L.rank_codes_ld(m)
            codes = torch.empty(n, ldc + ld_pad, dtype=torch.int32, device="cuda")[:, :ldc] if ld_pad else None
            codes = L.score_dot_split_rank(hi, lo, td, d, n_a, (ti[:n_a], ts[:n_a]),
                                           (ti[n_a:], ts[n_a:]) if n_b else None, band, c0, codes=codes)
            assert codes.shape == (n, ldc) and L.lib().kge_rank_codes_ld(m) == ldc
            L.rank_rows(None, n_a, c0, part_a, part_b, f_col, t_col, g, tt, codes=codes, m=m, **kw)
        else:
            buf = torch.empty(n, (m + 3) // 4 * 4, device="cuda")
            s = L.score_dot_split(hi, lo, td, None, d, out=buf[:, :m])
            L.rank_rows(s, n_a, c0, part_a, part_b, f_col, t_col, g, tt, **kw)
        torch.cuda.synchronize()
        return g.cpu().numpy(), tt.cpu().numpy(), rk.cpu().numpy(), hists.cpu().numpy()

    ref, got = run(False), run(True)
    for a, b, name in zip(ref, got, ("greater", "ties", "ranks", "histograms")):
        assert np.array_equal(a, b), name
    if refined:  # and both equal exact scoring (the near-ties are there: plain bf16x3 differs)
        exp = _oracle_counts(exact[:n_a], c0, true_idx[:n_a], np.where(np.isnan(true_score[:n_a]), -np.inf,
                                                                         true_score[:n_a]), [])
        assert np.array_equal(got[0][:n_a], exp[0][0])
        assert np.array_equal(got[1][:n_a], exp[0][1])


def test_fused_rank_codes_rows_with_thousands_of_near_ties(L):
    """More code-3 entries in a row than the ranking kernel's near-tie ring holds: the row is
    scanned a second time with a drain per step -- same counts as exact scoring."""
    rng = np.random.default_rng(77)
    n, m, d, near = 6, 6000, 128, 5000
    q = (rng.standard_normal((n, d)) * 0.3).astype(np.float32)
    t = (rng.standard_normal((m, d)) * 0.3).astype(np.float32)
    true_idx = np.array([3, 100, 2000, 4000, 5999, 17], np.int64)
    for j in range(near):  # row 0's true row copied (almost) into most of the table
        if j not in true_idx:
            t[j] = (t[true_idx[0]].astype(np.float64) * (1.0 + rng.uniform(-1e-6, 1e-6))).astype(np.float32)
    exact = (q.astype(np.float64) @ t.astype(np.float64).T).astype(np.float32)
    true_score = exact[np.arange(n), true_idx].copy()
    exp = _oracle_counts(exact, 0, true_idx, true_score, [])
    qd, td = _dev(q), _dev(t)
    hi, lo = L.split_rows(qd)
    tmax = L.row_norm_max(td)
    ti, ts = _dev(true_idx), _dev(true_score)
    codes = L.score_dot_split_rank(hi, lo, td, d, n, (ti, ts), None, L.rank_band(qd, 1e-4, tmax), 0)
    g = torch.empty(n, dtype=torch.int64, device="cuda")
    tt = torch.empty(n, dtype=torch.int64, device="cuda")
    L.rank_rows(None, n, 0, (ti, ts, None, None), None, None, None, g, tt, accumulate=False, codes=codes, m=m,
                refine=(qd, td, 1e-4, tmax))
    torch.cuda.synchronize()
    assert np.array_equal(g.cpu().numpy(), exp[0][0]) and np.array_equal(tt.cpu().numpy(), exp[0][1])


@pytest.mark.parametrize("k,e,kmax", [(3, 14541, 10), (1, 5, 10), (40, 700, 3)])
def test_rank_metrics_vs_torch_formula(k, e, kmax):
    """kge_rank_metrics against the stacked torch arithmetic of entity_ranking.py:553-577 (fp32
    operands, fp64 sums): counts and hits are exact, the weighted sums agree to 1e-12."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib

    g = torch.Generator().manual_seed(k * e)
    h = torch.randint(0, 50, (k, e), generator=g).float()
    h[0] = 0 if k > 1 else h[0]  # an empty histogram: every metric 0 on the host side
    hd = h.cuda()
    got = _lib.rank_metrics(hd, kmax).cpu()
    ranks = torch.arange(1, e + 1).float()
    n = h.sum(1, keepdim=True)
    want_s1 = (h.double() * ranks.double()).sum(1)
    want_s2 = (h.double() * (1.0 / ranks).double()).sum(1)
    assert torch.equal(got[:, 0], n.double().view(-1))
    torch.testing.assert_close(got[:, 1], want_s1, rtol=1e-12, atol=0)
    torch.testing.assert_close(got[:, 2], want_s2, rtol=1e-12, atol=0)
    cum = torch.cumsum(torch.nn.functional.pad(h, (0, max(0, kmax - e)))[:, :kmax], 1)
    hits = torch.where(n > 0, cum / n, torch.zeros(()))
    assert torch.equal(got[:, 3:], hits.double())
    # a view with a leading dimension of its own
    wide = torch.zeros(k, e + 7, device="cuda")
    wide[:, :e] = hd
    assert torch.equal(_lib.rank_metrics(wide[:, :e], kmax).cpu(), got)


@pytest.mark.parametrize("model,d", [("complex", 512), ("distmult", 64), ("simple", 128), ("rescal", 16)])
def test_prep_split2_band_matches_separate_launches(L, model, d):
    """kge_prep_query_split2_band = kge_prep_query_split2 + kge_rank_band: identical query rows and
    planes, bands equal to the separate launch's up to summation order (RESCAL takes the separate
    launches inside the entry point)."""
    kind = {"complex": L.COMPLEX, "distmult": L.DISTMULT, "simple": L.SIMPLE, "rescal": L.RESCAL}[model]
    g = torch.Generator(device="cuda").manual_seed(d)
    E, R, n, n_a = 300, 7, 37, 20
    d_r = d * d if model == "rescal" else d
    ent = torch.randn(E, d, device="cuda", generator=g) * 0.1
    rel = torch.randn(R, d_r, device="cuda", generator=g) * 0.1
    eidx = torch.randint(0, E, (n,), device="cuda", generator=g)
    ridx = torch.randint(0, R, (n,), device="cuda", generator=g)
    qw = L.query_width(kind, d)
    ldp = (qw + 31) // 32 * 32

    def bufs():
        return (torch.empty(n, qw, device="cuda"), torch.empty(n, ldp, device="cuda", dtype=torch.bfloat16),
                torch.empty(n, ldp, device="cuda", dtype=torch.bfloat16))

    tmax = L.row_norm_max(ent)
    q0, h0, l0 = L.prep_query_split2(kind, L.DIR_SP, L.DIR_PO, n_a, None, ent, eidx, rel, ridx, d, d_r, out=bufs())
    b0 = L.rank_band(q0, 7e-5, tmax)
    q1, h1, l1, b1 = L.prep_query_split2_band(kind, L.DIR_SP, L.DIR_PO, n_a, ent, eidx, rel, ridx, d, d_r, bufs(), 7e-5,
                                              tmax)
    torch.cuda.synchronize()
    assert torch.equal(q0, q1) and torch.equal(h0.view(torch.int16), h1.view(torch.int16))
    assert torch.equal(l0.view(torch.int16), l1.view(torch.int16))
    torch.testing.assert_close(b1, b0, rtol=2e-6, atol=0)
    # and against float64: the band is never narrower than band_rel |q| tmax
    exact = 7e-5 * q0.double().norm(dim=1) * float(tmax)
    assert bool((b1.double() >= exact * (1 - 1e-7)).all())


@pytest.mark.parametrize("m,d,ld", [(1, 4, 4), (7, 512, 512), (1001, 516, 516), (333, 260, 264), (65, 1000, 1000),
                                    (50, 30, 31), (14541, 512, 512)])
def test_row_norm_max_is_a_tight_upper_bound_of_the_largest_row_norm(L, m, d, ld):
    """kge_row_norm_max (the table factor of the refinement band): never below the largest
    Euclidean row norm in float64, at most a few 1e-6 above it -- on the float4 path (rows of a
    multiple of 4 floats, 16-B aligned; odd row counts, a d / 4 that is not a multiple of 64 or
    128) and on the scalar path (d = 30, ld = 31); a NaN row poisons it."""
    g = torch.Generator().manual_seed(m * 1000 + d)
    buf = torch.randn(m, ld, generator=g).cuda()
    t = buf[:, :d]
    want = float(t.double().norm(dim=1).max())
    got = float(L.row_norm_max(t))
    assert want <= got <= want * (1 + 1e-5), (want, got)
    if m > 1:
        buf[m - 1, d - 1] = float("nan")
        assert math.isnan(float(L.row_norm_max(t)))
