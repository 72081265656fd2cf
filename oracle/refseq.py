"""Reference-op-sequence CPU replica of ComplEx score_sp / score_po.  TEST / BASELINE
INFRASTRUCTURE ONLY (bench.py's ``cpu_baseline`` leg and tests/).

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
