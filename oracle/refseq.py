"""Reference-op-sequence CPU replicas: ComplEx score_sp / score_po, the 1vsAll training step,
entity ranking, the DistMult KvsAll training step and the RotatE negative-sampling step.
TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's ``cpu_baseline`` leg and tests/).

Replays the exact ATen op sequence the reference issues on the CPU for
KgeModel.score_sp -> ComplExScorer.score_emb(..., "sp_") (kge_model.py:652-659,
lookup_embedder.py:91-107, complex.py:27-40): index_select gathers, the arange
embed_all() copy, the .contiguous() halves, the three torch.cat's and the K = 2d mm.
It is checked bit-for-bit against the golden vectors captured from the reference itself
(tests/test_oracle_golden.py::test_refseq_bitwise), so timing it on the GPU box's host
cores measures the reference's CPU path without shipping reference code.
"""
import torch


def _gather(table, idx):
    return torch.nn.functional.embedding(idx, table)


def complex_score_sp(ent: torch.Tensor, rel: torch.Tensor, s: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    s_emb = _gather(ent, s)
    p_emb = _gather(rel, p)
    o_emb = _gather(ent, torch.arange(ent.shape[0]))
    p_re, p_im = (t.contiguous() for t in p_emb.chunk(2, dim=1))
    o_re, o_im = (t.contiguous() for t in o_emb.chunk(2, dim=1))
    s_all = torch.cat((s_emb, s_emb), dim=1)
    r_all = torch.cat((p_re, p_emb, -p_im), dim=1)
    o_all = torch.cat((o_emb, o_im, o_re), dim=1)
    return (s_all * r_all).mm(o_all.transpose(0, 1))


def complex_score_po(ent: torch.Tensor, rel: torch.Tensor, p: torch.Tensor, o: torch.Tensor) -> torch.Tensor:
    s_emb = _gather(ent, torch.arange(ent.shape[0]))
    o_emb = _gather(ent, o)
    p_emb = _gather(rel, p)
    p_re, p_im = (t.contiguous() for t in p_emb.chunk(2, dim=1))
    o_re, o_im = (t.contiguous() for t in o_emb.chunk(2, dim=1))
    s_all = torch.cat((s_emb, s_emb), dim=1)
    r_all = torch.cat((p_re, p_emb, -p_im), dim=1)
    o_all = torch.cat((o_emb, o_im, o_re), dim=1)
    return (r_all * o_all).mm(s_all.transpose(0, 1))


def complex_score_spo(ent: torch.Tensor, rel: torch.Tensor, s: torch.Tensor, p: torch.Tensor,
                      o: torch.Tensor) -> torch.Tensor:
    """KgeModel.score_spo -> ComplExScorer.score_emb(..., "spo") (kge_model.py:620-637,
    complex.py:27-36)."""
    s_emb, p_emb, o_emb = _gather(ent, s), _gather(rel, p), _gather(ent, o)
    p_re, p_im = (t.contiguous() for t in p_emb.chunk(2, dim=1))
    o_re, o_im = (t.contiguous() for t in o_emb.chunk(2, dim=1))
    s_all = torch.cat((s_emb, s_emb), dim=1)
    r_all = torch.cat((p_re, p_emb, -p_im), dim=1)
    o_all = torch.cat((o_emb, o_im, o_re), dim=1)
    return (s_all * o_all * r_all).sum(dim=1)


def train_step_1vsall(ent: torch.nn.Parameter, rel: torch.nn.Parameter, optimizer, triples: torch.Tensor) -> float:
    """One TrainingJob1vsAll batch as the reference runs it on the CPU (train.py:314-375,
    1032-1062): zero_grad; score_sp -> CrossEntropyLoss(sum) / B -> .item() -> backward; the
    same for score_po with the subjects as targets; optimizer.step().  Returns the batch
    loss.  (No penalty term: lookup_embedder.regularize_weight is 0 by default.)"""
    ce = torch.nn.CrossEntropyLoss(reduction="sum")
    n = len(triples)
    optimizer.zero_grad()
    loss_sp = ce(complex_score_sp(ent, rel, triples[:, 0], triples[:, 1]), triples[:, 2]) / n
    loss = loss_sp.item()
    loss_sp.backward()
    loss_po = ce(complex_score_po(ent, rel, triples[:, 1], triples[:, 2]), triples[:, 0]) / n
    loss += loss_po.item()
    loss_po.backward()
    optimizer.step()
    return loss


def distmult_score_sp(ent, rel, s, p):
    """KgeModel.score_sp -> DistMultScorer.score_emb(..., "sp_") (kge_model.py:652-659,
    lookup_embedder.py:91-107, distmult.py:19-20)."""
    s_emb, p_emb = _gather(ent, s), _gather(rel, p)
    o_emb = _gather(ent, torch.arange(ent.shape[0]))
    return (s_emb * p_emb).mm(o_emb.transpose(0, 1))


def distmult_score_po(ent, rel, p, o):
    """KgeModel.score_po -> DistMultScorer.score_emb(..., "_po") (kge_model.py:675-682,
    distmult.py:21-22)."""
    s_emb = _gather(ent, torch.arange(ent.shape[0]))
    o_emb, p_emb = _gather(ent, o), _gather(rel, p)
    return (o_emb * p_emb).mm(s_emb.transpose(0, 1))


def train_step_kvsall(ent: torch.nn.Parameter, rel: torch.nn.Parameter, optimizer, queries: torch.Tensor,
                      query_type_indexes: torch.Tensor, label_coords: torch.Tensor, label_smoothing: float = 0.0,
                      query_types=("sp_", "_po")) -> float:
    """One TrainingJobKvsAll batch of a DistMult model as the reference runs it on the CPU
    (train.py:314-375, 679-756, job/util.py:41-57, loss.py:209-213): zero_grad; the label
    coordinates densified into a [B, max(E, R)] matrix through a sparse tensor; per query type
    the examples' label rows (smoothed as (1 - ls) * L + 1 / E), score_sp / score_po on the
    examples' queries, KLDivLoss(sum)(log_softmax(scores), normalize(labels, p=1)) / B,
    .item(), backward; optimizer.step().  Returns what the reference reports as the batch
    loss: the LAST query type's (train.py:747 overwrites instead of summing).  The batch
    itself (queries, query_type_indexes, label_coords) is what the reference's collate
    (train.py:590-677) hands over; (s, ?, o) queries are not replayed here."""
    kl = torch.nn.KLDivLoss(reduction="sum")
    E, R = ent.shape[0], rel.shape[0]
    n = len(queries)
    optimizer.zero_grad()
    examples_for = {qt: (query_type_indexes == qi).nonzero().view(-1) for qi, qt in enumerate(query_types)}
    labels_batch = torch.sparse_coo_tensor(label_coords.long().t(), torch.ones([len(label_coords)], dtype=torch.float)
                                           * 1.0, torch.Size([n, max(E, R)])).to_dense()
    labels_for = {qt: labels_batch[ex, :E] for qt, ex in examples_for.items()}
    if label_smoothing > 0.0:
        for qt, labels in labels_for.items():
            labels_for[qt] = (1.0 - label_smoothing) * labels + 1.0 / labels.size(1)
    loss_value_total = 0.0
    for qt, ex in examples_for.items():
        if len(ex) > 0:
            if qt == "sp_":
                scores = distmult_score_sp(ent, rel, queries[ex, 0], queries[ex, 1])
            elif qt == "_po":
                scores = distmult_score_po(ent, rel, queries[ex, 0], queries[ex, 1])
            else:
                raise NotImplementedError(qt)
            loss_value = kl(torch.nn.functional.log_softmax(scores, dim=1),
                            torch.nn.functional.normalize(labels_for[qt].float(), p=1, dim=1)) / n
            loss_value_total = loss_value.item()
            loss_value.backward()
    optimizer.step()
    return loss_value_total


def rotate_score_spo(ent, rel, s, p, o, l_norm: float = 1.0):
    """KgeModel.score_spo -> RotatEScorer.score_emb(..., "spo") (kge_model.py:620-637,
    rotate.py:18-40, 113-145): chunk, cos / sin of the phases, complex Hadamard product,
    difference, |.| as the norm over a stacked (re, im) tensor, then the l_norm norm over the
    components.  A positive distance (the reference does not negate it)."""
    s_emb, p_emb, o_emb = _gather(ent, s), _gather(rel, p), _gather(ent, o)
    s_re, s_im = torch.chunk(s_emb, 2, dim=1)
    o_re, o_im = torch.chunk(o_emb, 2, dim=1)
    p_re, p_im = torch.cos(p_emb), torch.sin(p_emb)
    sp_re = s_re * p_re - s_im * p_im
    sp_im = s_re * p_im + s_im * p_re
    diff_re, diff_im = sp_re - o_re, sp_im - o_im
    diff_abs = torch.norm(torch.stack((diff_re, diff_im), dim=0), dim=0)
    return torch.norm(diff_abs, dim=1, p=l_norm).view(len(p), -1)


def train_step_ns_triple(ent: torch.nn.Parameter, rel: torch.nn.Parameter, optimizer, triples: torch.Tensor,
                         negatives, l_norm: float = 1.0) -> float:
    """One TrainingJobNegativeSampling batch of a RotatE model with implementation "triple" and
    train.loss kl, as the reference runs it on the CPU (train.py:314-375, 823-893, 982-999,
    loss.py:192-213): zero_grad; per corrupted slot with samples (negatives = {slot: [B, N]},
    slots 0 = S and 2 = O) the triples repeated 1 + N times with the slot overwritten by
    (positive, negatives), score_spo on all B (1 + N) triples, a [B, 1 + N] label matrix with a
    one in column 0, KLDivLoss(sum)(log_softmax(scores), normalize(labels, p=1)) / B, .item(),
    backward; optimizer.step().  Returns the batch loss (summed over the slots)."""
    kl = torch.nn.KLDivLoss(reduction="sum")
    n = len(triples)
    optimizer.zero_grad()
    loss_value = 0.0
    labels = None
    for slot in (0, 1, 2):
        neg = negatives.get(slot)
        if neg is None or neg.shape[1] <= 0:
            continue
        num_samples = neg.shape[1]
        if labels is None or labels.shape != torch.Size([n, 1 + num_samples]):
            labels = torch.zeros((n, 1 + num_samples))
            labels[:, 0] = 1
        triples_to_score = triples.repeat(1, 1 + num_samples).view(-1, 3)
        triples_to_score[:, slot] = torch.cat((triples[:, [slot]], neg), 1).view(-1)
        scores = rotate_score_spo(ent, rel, triples_to_score[:, 0], triples_to_score[:, 1], triples_to_score[:, 2],
                                  l_norm).view(n, -1)
        loss_value_torch = kl(torch.nn.functional.log_softmax(scores, dim=1),
                              torch.nn.functional.normalize(labels.float(), p=1, dim=1)) / n
        loss_value += loss_value_torch.item()
        loss_value_torch.backward()
    optimizer.step()
    return loss_value


class EntityRankingCPU:
    """The reference's EntityRankingJob on the CPU, op for op (entity_ranking.py:53-77 collate,
    112-265 batch loop, 428-551 helpers; job/util.py:5-57; eval.py:125-146 histogram loop):
    per-triple dictionary lookups building the filter coordinates, sparse +inf label tensors
    densified per chunk, the true scores written into the score matrix, scores - labels,
    sum(scores > true) / sum(scores == true), rounded-mean ranks, one histogram increment per
    rank, fp32 metrics from the histograms.  ComplEx scores come from the functions above.
    Pinned rank for rank against the reference-captured fixtures (tests/test_oracle_golden.py)."""

    def __init__(self, ent, rel, splits, eval_split="valid", filter_splits=("train", "valid"),
                 filter_with_test=True, batch_size=100, hits_at_k_s=(1, 3, 10, 50, 100, 200, 300, 400, 500, 1000)):
        self.ent, self.rel = ent, rel
        self.E = ent.shape[0]
        self.triples = torch.as_tensor(splits[eval_split]).long()
        self.filter_splits = list(filter_splits)
        if eval_split not in self.filter_splits:
            self.filter_splits.append(eval_split)
        self.filter_with_test = filter_with_test and "test" not in self.filter_splits
        self.batch_size = batch_size
        self.hits_at_k_s = [k for k in hits_at_k_s if k <= self.E]
        self.index = {}
        for name in set(self.filter_splits) | ({"test"} if self.filter_with_test else set()):
            t = torch.as_tensor(splits[name]).long()
            self.index[name] = (self._group(t, (0, 1), 2), self._group(t, (1, 2), 0))

    @staticmethod
    def _group(t, key_cols, value_col):
        d = {}
        for row in t.tolist():
            d.setdefault((row[key_cols[0]], row[key_cols[1]]), []).append(row[value_col])
        return {k: torch.tensor(v, dtype=torch.long) for k, v in d.items()}

    def _coords(self, batch, sp_index, po_index):
        nothing = torch.zeros([0], dtype=torch.long)
        rows, cols = [], []
        for i, (s, p, o) in enumerate(batch.tolist()):
            objects = sp_index.get((s, p), nothing)
            subjects = po_index.get((p, o), nothing) + self.E
            rows += [torch.full((len(objects) + len(subjects),), i, dtype=torch.long)]
            cols += [objects, subjects]
        if not rows:
            return torch.zeros([0, 2], dtype=torch.long)
        return torch.stack((torch.cat(rows), torch.cat(cols)), 1)

    def _dense_labels(self, coords, n):
        labels = torch.sparse_coo_tensor(coords.t(), torch.ones(len(coords)) * float("inf"), (n, 2 * self.E))
        return labels.to_dense()

    @staticmethod
    def _rank_and_ties(scores, true):
        scores = scores.clone()
        scores[torch.isnan(scores)] = float("-inf")
        true = true.clone()
        true[torch.isnan(true)] = float("-inf")
        return (torch.sum(scores > true.view(-1, 1), dim=1, dtype=torch.long),
                torch.sum(scores == true.view(-1, 1), dim=1, dtype=torch.long))

    @torch.no_grad()
    def run(self):
        E = self.E
        rankings = ["_raw", "_filt"] + (["_filt_test"] if self.filter_with_test else [])
        hists = {r: torch.zeros(E) for r in rankings}
        ranks = {d + r: [] for d in "so" for r in rankings}
        ar = None
        for b0 in range(0, len(self.triples), self.batch_size):
            batch = self.triples[b0:b0 + self.batch_size]
            n = len(batch)
            coords = torch.cat([self._coords(batch, *self.index[sp]) for sp in self.filter_splits])
            labels = {"_raw": None, "_filt": self._dense_labels(coords, n)}
            if self.filter_with_test:
                labels["_filt_test"] = self._dense_labels(self._coords(batch, *self.index["test"]), n)
            s, p, o = batch[:, 0], batch[:, 1], batch[:, 2]
            true = complex_score_spo(self.ent, self.rel, s, p, o)
            scores_sp = complex_score_sp(self.ent, self.rel, s, p)
            scores_po = complex_score_po(self.ent, self.rel, p, o)
            if ar is None or len(ar) != n:
                ar = torch.arange(n)
            scores_sp[ar, o] = true
            scores_po[ar, s] = true
            for r in rankings:
                lab = labels[r]
                if lab is not None:
                    lab[ar, o] = 0
                    lab[ar, s + E] = 0
                    scores_sp = scores_sp - lab[:, :E]
                    scores_po = scores_po - lab[:, E:]
                o_rank, o_ties = self._rank_and_ties(scores_sp, true)
                s_rank, s_ties = self._rank_and_ties(scores_po, true)
                o_r, s_r = o_rank + o_ties // 2, s_rank + s_ties // 2
                ranks["o" + r].append(o_r)
                ranks["s" + r].append(s_r)
                hist = hists[r]
                for v in o_r:
                    hist[v] += 1
                for v in s_r:
                    hist[v] += 1
        metrics = {}
        suffix = {"_raw": "", "_filt": "_filtered", "_filt_test": "_filtered_with_test"}
        pos = torch.arange(1, E + 1).float()
        for r in rankings:
            h = hists[r]
            n = torch.sum(h).item()
            metrics["mean_rank" + suffix[r]] = torch.sum(h * pos).item() / n if n > 0 else 0.0
            metrics["mean_reciprocal_rank" + suffix[r]] = torch.sum(h * (1.0 / pos)).item() / n if n > 0 else 0.0
            hits = (torch.cumsum(h[:max(self.hits_at_k_s)], dim=0) / n).tolist() if n > 0 else None
            for k in self.hits_at_k_s:
                metrics[f"hits_at_{k}{suffix[r]}"] = hits[k - 1] if hits else 0.0
        return {k: torch.cat(v).numpy() for k, v in ranks.items()}, metrics
