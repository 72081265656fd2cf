"""CPU oracle for the LibKGE scoring hot path.  TEST INFRASTRUCTURE ONLY.

Restatement of the reference's algorithm in numpy (float64), used only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg -- as the checker,
never as the thing measured or shipped.  The product path (``kge-1_amd/kge``) never
imports this module and fails loudly when its HIP library is missing.

Pinning: every function here is checked against the golden vectors in
``tests/golden/*.npz`` (``tests/test_oracle_golden.py``), which were produced by running
the reference itself (``tests/golden/make_golden.py``).  The reference's own unit tests
(tests/test_dataset.py) pin nothing on this path, so the captured
fixtures are the pin.

All citations are ``file:line`` into the reference checkout (kge/...).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

BILINEAR = ("complex", "distmult", "rescal", "cp", "simple")
DISTANCE = ("transe", "rotate")
PAIRWISE_EPS = 1e-6  # torch.nn.functional.pairwise_distance default eps


# --------------------------------------------------------------------------- helpers


def _halves(x):
    h = x.shape[-1] // 2
    return x[..., :h], x[..., h:]


def _cat(re, im):
    return np.concatenate([re, im], axis=-1)


def _lp(x, p, axis=-1):
    """torch.norm(x, p) along ``axis`` for p in {1, 2}."""
    if p == 1:
        return np.abs(x).sum(axis=axis)
    if p == 2:
        return np.sqrt((x * x).sum(axis=axis))
    return (np.abs(x) ** p).sum(axis=axis) ** (1.0 / p)


# --------------------------------------------------------------- query preparation
# Every bilinear scorer is "prep + one contraction with the entity table".


def window(model: str, direction: str, e: np.ndarray) -> np.ndarray:
    """The columns of a candidate entity row that the query contracts with: CP scores
    subjects with the first half and objects with the second (cp.py:17-19), so sp_
    contracts with e[d/2:] and _po with e[:d/2]; every other model uses the whole row."""
    if model == "cp":
        h = e.shape[-1] // 2
        return e[..., h:] if direction == "sp_" else e[..., :h]
    return e


def prep_sp(model: str, s: np.ndarray, r: np.ndarray) -> np.ndarray:
    """Query vector q such that score(s, r, e) = q . window(e) for every entity e.

    complex  -- complex.py:31-38: (s_all * r_all) @ o_all^T with
               s_all=[s_re,s_im,s_re,s_im], r_all=[r_re,r_re,r_im,-r_im],
               o_all=[o_re,o_im,o_im,o_re]  ==  cmul(s, r) . [e_re | e_im].
    distmult -- distmult.py:20: (s * p) @ o^T.
    rescal   -- rescal.py:37-43: s^T M_r, M_r = p.view(d, d) (row-major).
    cp       -- cp.py:23: (s_h * p) @ o_t^T.
    simple   -- simple.py:24-26,34: ((s_h * p_f) @ o_t^T + (s_t * p_b) @ o_h^T) / 2
               == 0.5 [s_t * p_b | s_h * p_f] . [e_h | e_t].
    """
    if model == "cp":
        return _halves(s)[0] * r
    if model == "simple":
        s_h, s_t = _halves(s)
        r_f, r_b = _halves(r)
        return 0.5 * _cat(s_t * r_b, s_h * r_f)
    if model == "complex":
        s_re, s_im = _halves(s)
        r_re, r_im = _halves(r)
        return _cat(s_re * r_re - s_im * r_im, s_re * r_im + s_im * r_re)
    if model == "distmult":
        return s * r
    if model == "rescal":
        d = s.shape[-1]
        M = r.reshape(-1, d, d)
        return np.einsum("ni,nij->nj", s, M)
    raise ValueError(model)


def prep_po(model: str, r: np.ndarray, o: np.ndarray) -> np.ndarray:
    """Query vector q such that score(e, r, o) = q . e for every entity e.

    complex  -- complex.py:40: (r_all * o_all) @ s_all^T == conj(r) * o.
    distmult -- distmult.py:22: (o * p) @ s^T.
    rescal   -- rescal.py:44-49: M_r o.
    cp       -- cp.py:25: (o_t * p) @ s_h^T.
    simple   -- simple.py:28-30,34: ((o_t * p_f) @ s_h^T + (o_h * p_b) @ s_t^T) / 2
               == 0.5 [o_t * p_f | o_h * p_b] . [e_h | e_t].
    """
    if model == "cp":
        return _halves(o)[1] * r
    if model == "simple":
        o_h, o_t = _halves(o)
        r_f, r_b = _halves(r)
        return 0.5 * _cat(o_t * r_f, o_h * r_b)
    if model == "complex":
        r_re, r_im = _halves(r)
        o_re, o_im = _halves(o)
        return _cat(r_re * o_re + r_im * o_im, r_re * o_im - r_im * o_re)
    if model == "distmult":
        return o * r
    if model == "rescal":
        d = o.shape[-1]
        M = r.reshape(-1, d, d)
        return np.einsum("nij,nj->ni", M, o)
    raise ValueError(model)


def _rot(r):
    return np.cos(r), np.sin(r)  # rotate.py:26


def rotate_q_sp(s, r):
    """s * rot(r) -- rotate.py:43-45 (hadamard_complex, rotate.py:118-122)."""
    s_re, s_im = _halves(s)
    c, si = _rot(r)
    return _cat(s_re * c - s_im * si, s_re * si + s_im * c)


# ----------------------------------------------------------------------- scorers


def score_emb(model: str, s, p, o, combine: str, l_norm: float = 1.0) -> np.ndarray:
    """RelationalScorer.score_emb (kge_model.py:120-182) for the five in-scope scorers.

    combine: "spo" -> [n]; "sp_" -> [n, |o|]; "_po" -> [n, |s|].
    """
    n = p.shape[0]
    if model in BILINEAR:
        if combine == "spo":
            return (prep_sp(model, s, p) * window(model, "sp_", o)).sum(-1)
        if combine == "sp_":
            return prep_sp(model, s, p) @ window(model, "sp_", o).T
        if combine == "_po":
            return prep_po(model, p, o) @ window(model, "_po", s).T
    elif model == "transe":
        # transe.py:16-21: spo uses F.pairwise_distance (adds eps to the difference),
        # sp_/_po use torch.cdist (no eps).  Scores are NEGATED distances.
        if combine == "spo":
            return -_lp((s + p) - o + PAIRWISE_EPS, l_norm)
        if combine == "sp_":
            return -_lp((s + p)[:, None, :] - o[None, :, :], l_norm)
        if combine == "_po":
            return -_lp((o - p)[:, None, :] - s[None, :, :], l_norm)
    elif model == "rotate":
        # rotate.py:28-60.  Scores are POSITIVE distances.
        if combine == "spo":
            q = rotate_q_sp(s, p)
            d_re, d_im = _halves(q - o)
            return _lp(np.sqrt(d_re ** 2 + d_im ** 2), l_norm)
        if combine == "sp_":
            q = rotate_q_sp(s, p)
            q_re, q_im = _halves(q)
            o_re, o_im = _halves(o)
            d_re = q_re[:, None, :] - o_re[None]
            d_im = q_im[:, None, :] - o_im[None]
            return _lp(np.sqrt(d_re ** 2 + d_im ** 2), l_norm)
        if combine == "_po":
            # pairwise_hadamard_complex(s, rot(p)) - o, norm, transpose (rotate.py:51-60)
            s_re, s_im = _halves(s)
            c, si = _rot(p)
            o_re, o_im = _halves(o)
            x_re = s_re[:, None, :] * c[None] - s_im[:, None, :] * si[None]
            x_im = s_re[:, None, :] * si[None] + s_im[:, None, :] * c[None]
            d_re = x_re - o_re[None]
            d_im = x_im - o_im[None]
            return _lp(np.sqrt(d_re ** 2 + d_im ** 2), l_norm).T
    raise ValueError('cannot handle combine="{}".format(combine)')


def model_scores(model, ent, rel, s, p, o, subset, l_norm=1.0) -> Dict[str, np.ndarray]:
    """KgeModel.score_spo / score_sp / score_po / score_sp_po (kge_model.py:620-746)
    with LookupEmbedder gathers (lookup_embedder.py:91-107, dropout 0)."""
    ent = ent.astype(np.float64)
    rel = rel.astype(np.float64)
    S, P, O = ent[s], rel[p], ent[o]
    E_sub = ent[subset]
    sp_sub = score_emb(model, S, P, E_sub, "sp_", l_norm)
    po_sub = score_emb(model, E_sub, P, O, "_po", l_norm)
    sp_all = score_emb(model, S, P, ent, "sp_", l_norm)
    po_all = score_emb(model, ent, P, O, "_po", l_norm)
    return dict(
        spo=score_emb(model, S, P, O, "spo", l_norm),
        sp_all=sp_all,
        po_all=po_all,
        sp_sub=sp_sub,
        po_sub=po_sub,
        sppo_sub=np.concatenate([sp_sub, po_sub], 1),
        sppo_all=np.concatenate([sp_all, po_all], 1),
    )


# --------------------------------------------------------------------- gradients
# Autograd parity (F2): gradient of
#   L = sum(W_sp * score_sp(s,p)) + sum(W_po * score_po(p,o)) + sum(w_spo * score_spo)
# w.r.t. both tables, restated as explicit vector-Jacobian products.


def _vjp_prep_sp(model, s, r, dq):
    if model == "cp":
        s_h = _halves(s)[0]
        return _cat(dq * r, np.zeros_like(s_h)), dq * s_h
    if model == "simple":
        s_h, s_t = _halves(s)
        r_f, r_b = _halves(r)
        g1, g2 = _halves(dq)
        return 0.5 * _cat(g2 * r_f, g1 * r_b), 0.5 * _cat(g2 * s_h, g1 * s_t)
    if model == "complex":
        s_re, s_im = _halves(s)
        r_re, r_im = _halves(r)
        g_re, g_im = _halves(dq)
        ds = _cat(g_re * r_re + g_im * r_im, -g_re * r_im + g_im * r_re)
        dr = _cat(g_re * s_re + g_im * s_im, -g_re * s_im + g_im * s_re)
        return ds, dr
    if model == "distmult":
        return dq * r, dq * s
    if model == "rescal":
        d = s.shape[-1]
        M = r.reshape(-1, d, d)
        ds = np.einsum("nij,nj->ni", M, dq)
        dM = np.einsum("ni,nj->nij", s, dq)
        return ds, dM.reshape(r.shape)
    raise ValueError(model)


def _vjp_prep_po(model, r, o, dq):
    if model == "cp":
        o_t = _halves(o)[1]
        return dq * o_t, _cat(np.zeros_like(o_t), dq * r)
    if model == "simple":
        o_h, o_t = _halves(o)
        r_f, r_b = _halves(r)
        g1, g2 = _halves(dq)
        return 0.5 * _cat(g1 * o_t, g2 * o_h), 0.5 * _cat(g2 * r_b, g1 * r_f)
    if model == "complex":
        r_re, r_im = _halves(r)
        o_re, o_im = _halves(o)
        g_re, g_im = _halves(dq)
        dr = _cat(g_re * o_re + g_im * o_im, g_re * o_im - g_im * o_re)
        do = _cat(g_re * r_re - g_im * r_im, g_re * r_im + g_im * r_re)
        return dr, do
    if model == "distmult":
        return dq * o, dq * r
    if model == "rescal":
        d = o.shape[-1]
        M = r.reshape(-1, d, d)
        do = np.einsum("nij,ni->nj", M, dq)
        dM = np.einsum("ni,nj->nij", dq, o)
        return dM.reshape(r.shape), do
    raise ValueError(model)


def _dlp(diff, p, out_norm):
    """d||diff||_p / d diff, zero where undefined (torch convention)."""
    if p == 1:
        return np.sign(diff)
    with np.errstate(invalid="ignore", divide="ignore"):
        g = diff / out_norm[..., None]
    return np.where(out_norm[..., None] == 0, 0.0, g)


def _rotate_abs_grad(d_re, d_im, l_norm):
    """For f = ||(|d_k|)_k||_p, returns (df/dd_re, df/dd_im)."""
    a = np.sqrt(d_re ** 2 + d_im ** 2)
    f = _lp(a, l_norm)
    if l_norm == 1:
        ga = np.ones_like(a)
    else:
        with np.errstate(invalid="ignore", divide="ignore"):
            ga = np.where(f[..., None] == 0, 0.0, a / f[..., None])
    with np.errstate(invalid="ignore", divide="ignore"):
        gr = np.where(a == 0, 0.0, ga * d_re / a)
        gi = np.where(a == 0, 0.0, ga * d_im / a)
    return gr, gi


def model_grads(model, ent, rel, s, p, o, w_sp, w_po, w_spo, l_norm=1.0):
    ent = ent.astype(np.float64)
    rel = rel.astype(np.float64)
    g_ent = np.zeros_like(ent)
    g_rel = np.zeros_like(rel)
    S, P, O = ent[s], rel[p], ent[o]
    if model in BILINEAR:
        # sp_: scores = q_sp @ window_sp(E)^T
        q = prep_sp(model, S, P)
        window(model, "sp_", g_ent)[...] += w_sp.T @ q
        ds, dr = _vjp_prep_sp(model, S, P, w_sp @ window(model, "sp_", ent))
        np.add.at(g_ent, s, ds)
        np.add.at(g_rel, p, dr)
        # _po: scores = q_po @ window_po(E)^T
        q = prep_po(model, P, O)
        window(model, "_po", g_ent)[...] += w_po.T @ q
        dr, do = _vjp_prep_po(model, P, O, w_po @ window(model, "_po", ent))
        np.add.at(g_rel, p, dr)
        np.add.at(g_ent, o, do)
        # spo: sum(q_sp * window_sp(o))
        q = prep_sp(model, S, P)
        g_o = np.zeros_like(O)
        window(model, "sp_", g_o)[...] = w_spo[:, None] * q
        np.add.at(g_ent, o, g_o)
        ds, dr = _vjp_prep_sp(model, S, P, w_spo[:, None] * window(model, "sp_", O))
        np.add.at(g_ent, s, ds)
        np.add.at(g_rel, p, dr)
        return g_ent, g_rel
    if model == "transe":
        sgn = -1.0
        # sp_: -||(s+p) - e||
        x = S + P
        diff = x[:, None, :] - ent[None]
        gd = sgn * w_sp[..., None] * _dlp(diff, l_norm, _lp(diff, l_norm))
        gx = gd.sum(1)
        g_ent -= gd.sum(0)
        np.add.at(g_ent, s, gx)
        np.add.at(g_rel, p, gx)
        # _po: -||(o-p) - e||
        x = O - P
        diff = x[:, None, :] - ent[None]
        gd = sgn * w_po[..., None] * _dlp(diff, l_norm, _lp(diff, l_norm))
        gx = gd.sum(1)
        g_ent -= gd.sum(0)
        np.add.at(g_ent, o, gx)
        np.add.at(g_rel, p, -gx)
        # spo: -||s+p-o+eps||
        diff = (S + P) - O + PAIRWISE_EPS
        gd = sgn * w_spo[:, None] * _dlp(diff, l_norm, _lp(diff, l_norm))
        np.add.at(g_ent, s, gd)
        np.add.at(g_rel, p, gd)
        np.add.at(g_ent, o, -gd)
        return g_ent, g_rel
    if model == "rotate":
        c, si = _rot(P)
        # sp_: ||| s*rot(p) - e |||
        q = rotate_q_sp(S, P)
        q_re, q_im = _halves(q)
        e_re, e_im = _halves(ent)
        gr, gi = _rotate_abs_grad(q_re[:, None] - e_re[None], q_im[:, None] - e_im[None], l_norm)
        gr *= w_sp[..., None]
        gi *= w_sp[..., None]
        g_ent -= _cat(gr.sum(0), gi.sum(0))
        gq_re, gq_im = gr.sum(1), gi.sum(1)
        s_re, s_im = _halves(S)
        np.add.at(g_ent, s, _cat(gq_re * c + gq_im * si, -gq_re * si + gq_im * c))
        np.add.at(g_rel, p, gq_re * (-q_im) + gq_im * q_re)
        # _po: ||| e*rot(p) - o |||  (pairwise over entities e)
        o_re, o_im = _halves(O)
        x_re = e_re[None] * c[:, None] - e_im[None] * si[:, None]  # [n, E, h]
        x_im = e_re[None] * si[:, None] + e_im[None] * c[:, None]
        gr, gi = _rotate_abs_grad(x_re - o_re[:, None], x_im - o_im[:, None], l_norm)
        gr *= w_po[..., None]
        gi *= w_po[..., None]
        g_ent += _cat((gr * c[:, None] + gi * si[:, None]).sum(0),
                      (-gr * si[:, None] + gi * c[:, None]).sum(0))
        np.add.at(g_rel, p, (gr * (-x_im) + gi * x_re).sum(1))
        np.add.at(g_ent, o, -_cat(gr.sum(1), gi.sum(1)))
        # spo
        d_re, d_im = q_re - o_re, q_im - o_im
        gr, gi = _rotate_abs_grad(d_re, d_im, l_norm)
        gr *= w_spo[:, None]
        gi *= w_spo[:, None]
        np.add.at(g_ent, s, _cat(gr * c + gi * si, -gr * si + gi * c))
        np.add.at(g_rel, p, gr * (-q_im) + gi * q_re)
        np.add.at(g_ent, o, -_cat(gr, gi))
        return g_ent, g_rel
    raise ValueError(model)


# ------------------------------------------------------------- entity ranking (F3)


def rank_and_ties(scores: np.ndarray, true_scores: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """_get_ranks_and_num_ties (entity_ranking.py:505-529): NaN -> -inf, then count
    entries strictly greater than / equal to the true score per row (int64)."""
    sc = np.where(np.isnan(scores), -np.inf, scores)
    t = np.where(np.isnan(true_scores), -np.inf, true_scores)[:, None]
    return (sc > t).sum(1).astype(np.int64), (sc == t).sum(1).astype(np.int64)


def get_ranks(rank, ties, tie_handling="rounded_mean_rank"):
    """_get_ranks (entity_ranking.py:531-551)."""
    if tie_handling == "rounded_mean_rank":
        return rank + ties // 2
    if tie_handling == "best_rank":
        return rank
    if tie_handling == "worst_rank":
        return rank + ties - 1
    raise NotImplementedError


def compute_metrics(rank_hist: np.ndarray, hits_at_k_s: Sequence[int], suffix=""):
    """_compute_metrics (entity_ranking.py:553-577), fp32 like the reference."""
    hist = rank_hist.astype(np.float32)
    n = float(hist.sum(dtype=np.float64))
    ranks = np.arange(1, len(hist) + 1, dtype=np.float32)
    m = {}
    m["mean_rank" + suffix] = float((hist * ranks).sum(dtype=np.float64)) / n if n > 0 else 0.0
    rr = np.float32(1.0) / ranks
    m["mean_reciprocal_rank" + suffix] = (
        float((hist * rr).sum(dtype=np.float64)) / n if n > 0 else 0.0)
    kmax = max(hits_at_k_s)
    hits = (np.cumsum(hist[:kmax].astype(np.float64)) / n) if n > 0 else np.zeros(kmax)
    for k in hits_at_k_s:
        m["hits_at_{}{}".format(k, suffix)] = float(hits[k - 1])
    return m


def sp_po_index(triples: np.ndarray):
    """{(s,p): set(o)}, {(p,o): set(s)} -- the sp_to_o / po_to_s indexes
    (indexing.py:8-98, used by job/util.py:5-38)."""
    sp, po = {}, {}
    for s, p, o in triples.tolist():
        sp.setdefault((s, p), set()).add(o)
        po.setdefault((p, o), set()).add(s)
    return sp, po


def relation_types(train: np.ndarray, num_relations: int) -> List[str]:
    """index_relation_types (indexing.py:142-179): per relation, the mean number of subjects per
    distinct (p, o) and of objects per distinct (s, p) over the training triples (duplicates
    counted, as the index's value lists keep them, indexing.py:37-53), each compared with 1.5 in
    fp32; a relation without training triples gives nan > 1.5 = False, i.e. "1-1"."""
    stats = np.zeros((num_relations, 4), np.float32)  # num_s, distinct po, num_o, distinct sp
    seen_po, seen_sp = set(), set()
    for s, p, o in train.tolist():
        stats[p, 0] += 1
        stats[p, 2] += 1
        if (p, o) not in seen_po:
            seen_po.add((p, o))
            stats[p, 1] += 1
        if (s, p) not in seen_sp:
            seen_sp.add((s, p))
            stats[p, 3] += 1
    with np.errstate(invalid="ignore", divide="ignore"):
        is_m = stats[:, 0] / stats[:, 1] > 1.5
        is_n = stats[:, 2] / stats[:, 3] > 1.5
    return ["{}-{}".format("M" if m else "1", "N" if n else "1") for m, n in zip(is_m, is_n)]


def relations_per_type(types: Sequence[str]) -> Dict[str, set]:
    """index_relations_per_type (indexing.py:182-197): type -> set of relations, in order of
    each type's first relation."""
    out: Dict[str, set] = {}
    for i, k in enumerate(types):
        out.setdefault(k, set()).add(i)
    return out


PERCENTILES = (("25%", 0.0, 0.25), ("50%", 0.25, 0.5), ("75%", 0.5, 0.75), ("top", 0.75, 1.0))


def frequency_percentiles(train: np.ndarray, num_entities: int, num_relations: int) -> Dict[str, Dict[str, set]]:
    """index_frequency_percentiles (indexing.py:200-263): ids sorted by their training frequency
    in the slot (stable, so ties stay in id order), cut at int(fraction * num)."""
    out = {}
    for arg, col, num in (("subject", 0, num_entities), ("relation", 1, num_relations), ("object", 2, num_entities)):
        freq = [0] * num
        for x in train[:, col].tolist():
            freq[x] += 1
        order = [i for i, _ in sorted(enumerate(freq), key=lambda x: x[1])]
        out[arg] = {name: set(order[int(b * num):int(e * num)]) for name, b, e in PERCENTILES}
    return out


def grouped_histograms(ranks_s, ranks_o, triples, num_entities, head_and_tail=False, rel_types=None,
                       freq_percs=None) -> Dict[str, np.ndarray]:
    """The histogram hooks of the evaluation job for one ranking: hist_all, hist_per_relation_type
    and hist_per_frequency_percentile (eval.py:148-224).  Returns key -> rank histogram in the
    reference's key order; ranks_s rank the subject of (?, p, o), ranks_o the object of (s, p, ?)."""
    E = num_entities
    s, p, o = (triples[:, i] for i in range(3))

    def hist(ranks, mask=None):
        r = ranks if mask is None else ranks[mask]
        return np.bincount(r, minlength=E)[:E].astype(np.float32)

    h = {"all": hist(ranks_o) + hist(ranks_s)}
    if head_and_tail:
        h["head"], h["tail"] = hist(ranks_s), hist(ranks_o)
    if rel_types is not None:
        for t, rels in relations_per_type(rel_types).items():
            m = np.array([int(x) in rels for x in p], bool)
            h[t] = hist(ranks_o, m) + hist(ranks_s, m)
            if head_and_tail:
                h[t + "_head"], h[t + "_tail"] = hist(ranks_s, m), hist(ranks_o, m)
    if freq_percs is not None:
        def member(arg, perc, ids):
            return np.array([int(x) in freq_percs[arg][perc] for x in ids], bool)

        for arg in ("subject", "relation", "object"):
            for perc, _, _ in PERCENTILES:
                if arg == "subject":
                    h[f"{arg}_{perc}"] = hist(ranks_s, member(arg, perc, s))
                elif arg == "object":
                    h[f"{arg}_{perc}"] = hist(ranks_o, member(arg, perc, o))
                else:
                    m = member(arg, perc, p)
                    h[f"{arg}_{perc}"] = hist(ranks_s, m) + hist(ranks_o, m)
    return h


def entity_ranking(model, ent, rel, splits: Dict[str, np.ndarray], eval_split="valid",
                   filter_splits=("train", "valid"), filter_with_test=True,
                   batch_size=100, chunk_size=-1, tie_handling="rounded_mean_rank",
                   hits_at_k_s=(1, 3, 10, 50, 100, 200, 300, 400, 500, 1000),
                   l_norm=1.0, score_dtype=np.float32, head_and_tail=False, relation_type=False,
                   argument_frequency=False):
    """EntityRankingJob._run (entity_ranking.py:79-426), hist_all (eval.py:148-171).

    Scores are computed in float64 and rounded to ``score_dtype``; true scores come
    from score_spo (entity_ranking.py:139-140) and overwrite the matrix entries
    (172-177).  Filtering subtracts +inf labels with the own label zeroed (180-210,
    497-502); _filt_test builds on the _filt scores.  Returns (ranks dict, metrics).
    """
    ent64 = ent.astype(np.float64)
    rel64 = rel.astype(np.float64)
    E = ent.shape[0]
    triples = splits[eval_split]
    filter_splits = list(filter_splits)
    if eval_split not in filter_splits:
        filter_splits.append(eval_split)
    use_test = "test" not in filter_splits and filter_with_test
    rankings = ["_raw", "_filt", "_filt_test"] if use_test else ["_raw", "_filt"]
    filt_sp, filt_po = sp_po_index(np.concatenate([splits[k] for k in filter_splits]))
    test_sp, test_po = sp_po_index(splits["test"]) if use_test else ({}, {})
    kmax = min(E, max(hits_at_k_s))
    hits_at_k_s = [k for k in hits_at_k_s if k <= kmax]
    if chunk_size < 0:
        chunk_size = E
    out = {f"{d}{r}": [] for d in "so" for r in rankings}
    for b0 in range(0, len(triples), batch_size):
        batch = triples[b0:b0 + batch_size]
        s, p, o = batch[:, 0], batch[:, 1], batch[:, 2]
        Sv, Pv, Ov = ent64[s], rel64[p], ent64[o]
        o_true = score_emb(model, Sv, Pv, Ov, "spo", l_norm).astype(score_dtype)
        s_true = o_true.copy()  # score_spo(..., "o") == score_spo(..., "s") (no reciprocal)
        acc = {f"{d}{r}": [np.zeros(len(batch), np.int64), np.zeros(len(batch), np.int64)]
               for d in "so" for r in rankings}
        for c0 in range(0, E, chunk_size):
            c1 = min(c0 + chunk_size, E)
            sub = ent64[c0:c1]
            sc_sp = score_emb(model, Sv, Pv, sub, "sp_", l_norm).astype(score_dtype)
            sc_po = score_emb(model, sub, Pv, Ov, "_po", l_norm).astype(score_dtype)
            for i in range(len(batch)):
                if c0 <= o[i] < c1:
                    sc_sp[i, o[i] - c0] = o_true[i]
                if c0 <= s[i] < c1:
                    sc_po[i, s[i] - c0] = s_true[i]
            for r in rankings:
                if r != "_raw":
                    isp, ipo = (filt_sp, filt_po) if r == "_filt" else (test_sp, test_po)
                    for i in range(len(batch)):
                        for j in isp.get((int(s[i]), int(p[i])), ()):
                            if c0 <= j < c1 and j != o[i]:
                                sc_sp[i, j - c0] = -np.inf
                        for j in ipo.get((int(p[i]), int(o[i])), ()):
                            if c0 <= j < c1 and j != s[i]:
                                sc_po[i, j - c0] = -np.inf
                ro, to = rank_and_ties(sc_sp, o_true)
                rs, ts = rank_and_ties(sc_po, s_true)
                acc["o" + r][0] += ro
                acc["o" + r][1] += to
                acc["s" + r][0] += rs
                acc["s" + r][1] += ts
        for k, (rk, tk) in acc.items():
            out[k].append(get_ranks(rk, tk, tie_handling))
    ranks = {k: np.concatenate(v) for k, v in out.items()}
    metrics = {}
    names = {"_raw": "", "_filt": "_filtered", "_filt_test": "_filtered_with_test"}
    R = rel.shape[0]
    types = relation_types(splits["train"], R) if relation_type else None
    percs = frequency_percentiles(splits["train"], E, R) if argument_frequency else None
    grouped = {r: grouped_histograms(ranks["s" + r], ranks["o" + r], triples, E, head_and_tail, types, percs)
               for r in rankings}
    for key in grouped["_raw"]:  # entity_ranking.py:376-387: per key, every ranking
        for r in rankings:
            metrics.update(compute_metrics(grouped[r][key], hits_at_k_s,
                                           names[r] + ("_" + key if key != "all" else "")))
    return ranks, metrics


# ------------------------------------------------------------ 1vsAll training (F4)


def softmax_xent(logits: np.ndarray, labels: np.ndarray, scale: float = 1.0):
    """Per-row CrossEntropy(reduction="sum") of score rows against index labels and the
    gradient of scale * sum_i loss_i w.r.t. the scores -- KLDivWithSoftmaxKgeLoss with
    index labels (loss.py:192-208), divided by the batch size (train.py:1042,1052).
    Returns (loss [n], G [n, m]) with G = scale * (softmax - onehot)."""
    x = logits.astype(np.float64)
    n = x.shape[0]
    mx = x.max(1, keepdims=True)
    lse = np.log(np.exp(x - mx).sum(1, keepdims=True)) + mx
    loss = lse[:, 0] - x[np.arange(n), labels]
    G = np.exp(x - lse)
    G[np.arange(n), labels] -= 1.0
    return loss, G * scale


def softmax_kl(logits: np.ndarray, positives: Sequence[np.ndarray], smoothing: float = 0.0, scale: float = 1.0):
    """KvsAll loss per row: KLDivLoss(reduction="sum")(log_softmax(S), normalize(labels, p=1))
    (loss.py:209-213) with labels = 0/1 rows of the positive lists, label-smoothed as
    (1 - eps) * labels + 1 / m when eps > 0 (train.py:715-721).  Returns (loss [n], G) with
    G the gradient of scale * sum_i loss_i w.r.t. the scores."""
    x = logits.astype(np.float64)
    n, m = x.shape
    y = np.zeros((n, m))
    for i, cols in enumerate(positives):
        y[i, np.asarray(cols, np.int64)] = 1.0
    if smoothing > 0.0:
        y = (1.0 - smoothing) * y + 1.0 / m
    t = y / np.maximum(np.abs(y).sum(1, keepdims=True), 1e-12)
    mx = x.max(1, keepdims=True)
    lse = np.log(np.exp(x - mx).sum(1, keepdims=True)) + mx
    logsm = x - lse
    with np.errstate(divide="ignore", invalid="ignore"):
        tlogt = np.where(t > 0, t * np.log(np.where(t > 0, t, 1.0)), 0.0)
    loss = (tlogt - t * logsm).sum(1)
    G = np.exp(logsm) * t.sum(1, keepdims=True) - t
    return loss, G * scale


def train_1vsall(model, ent, rel, batches: Sequence[np.ndarray], lr=0.2, eps=1e-10):
    """TrainingJob1vsAll._process_batch (train.py:1032-1062) + Adagrad step.

    Per batch: loss_sp = CE(score_sp(s,p), o)/B (loss.py:198-208, reduction sum),
    backward; loss_po = CE(score_po(p,o), s)/B, backward; then torch.optim.Adagrad
    (state += g^2; w -= lr * g / (sqrt(state) + eps)).  Bilinear models only.
    """
    ent = ent.astype(np.float64).copy()
    rel = rel.astype(np.float64).copy()
    st_e = np.zeros_like(ent)
    st_r = np.zeros_like(rel)
    losses = []
    for batch in batches:
        s, p, o = batch[:, 0], batch[:, 1], batch[:, 2]
        B = len(batch)
        g_ent = np.zeros_like(ent)
        g_rel = np.zeros_like(rel)
        total = 0.0
        for direction in ("sp", "po"):
            S, P, O = ent[s], rel[p], ent[o]
            if direction == "sp":
                q = prep_sp(model, S, P)
                target = o
            else:
                q = prep_po(model, P, O)
                target = s
            loss_rows, G = softmax_xent(q @ ent.T, target, 1.0 / B)
            total += float(loss_rows.sum() / B)
            g_ent += G.T @ q
            dq = G @ ent
            if direction == "sp":
                ds, dr = _vjp_prep_sp(model, S, P, dq)
                np.add.at(g_ent, s, ds)
                np.add.at(g_rel, p, dr)
            else:
                dr, do = _vjp_prep_po(model, P, O, dq)
                np.add.at(g_rel, p, dr)
                np.add.at(g_ent, o, do)
        losses.append(total)
        st_e += g_ent ** 2
        st_r += g_rel ** 2
        ent -= lr * g_ent / (np.sqrt(st_e) + eps)
        rel -= lr * g_rel / (np.sqrt(st_r) + eps)
    return np.array(losses), ent, rel


def relation_dim(model: str, d_e: int, d_r: int = -1) -> int:
    """Config-derived relation dims: rotate.py:82-87 (d/2), rescal.py:79-96 (d^2)."""
    if d_r >= 0:
        return d_r
    if model == "rotate":
        return d_e // 2
    if model == "rescal":
        return d_e * d_e
    return d_e
