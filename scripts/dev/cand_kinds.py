"""The candidate-gather kernels (forward, dq, d_ent) at the C4 shape (512 queries x 1,025 candidates
x 1,024 floats, 14,541-row table) for every score kind: same bytes, different arithmetic."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "kge-1_amd"))
from kge import _lib as L

torch.manual_seed(0)
n, k, d, E = 512, 1025, 1024, 14541
q = torch.randn(n, d, device="cuda") * 0.1
ent = torch.randn(E, d, device="cuda") * 0.1
cand = torch.randint(0, E, (n, k), device="cuda")
if len(sys.argv) > 1 and sys.argv[1] == "xcd":
    # what a split of every list into 8 entity ranges, range x served by XCD x, could reach: here
    # query i (workgroup i, XCD i % 8) draws all its candidates from range i % 8 -- the same reuse
    # of table rows inside an XCD as 512 queries x 128 candidates per range
    r = torch.arange(n, device="cuda") % 8
    cand = (torch.rand(n, k, device="cuda") * (E // 8)).long() + (r * (E // 8))[:, None]
    cand = torch.sort(cand, 1).values
    print("candidates of query i in entity range i % 8, ascending")
if len(sys.argv) > 1 and sys.argv[1] == "sorted":  # ascending candidates per query: rows shared in the XCD's L2
    cand = torch.sort(cand, 1).values
    print("candidates in ascending order per query")
g = torch.randn(n, k, device="cuda")
dq = torch.empty(n, d, device="cuda")
de = torch.zeros(E, d, device="cuda")


def timed(f, reps=20):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, model, ln in (("dot", L.DISTMULT, 1.0), ("transe l1", L.TRANSE, 1.0), ("transe l2", L.TRANSE, 2.0),
                        ("rotate l1", L.ROTATE, 1.0), ("rotate l2", L.ROTATE, 2.0)):
    s = L.score_cand(model, ln, L.DIR_SP, q, ent, cand)
    tf = timed(lambda: L.score_cand(model, ln, L.DIR_SP, q, ent, cand, out=s))
    tq = timed(lambda: L.score_cand_bwd(model, ln, L.DIR_SP, q, ent, cand, s, g, dq, None))
    te = timed(lambda: L.score_cand_bwd_ent(model, ln, L.DIR_SP, q, ent, cand, s, g, de))
    print(f"{name:10s} forward {tf:7.1f} us   dq {tq:7.1f} us   d_ent (with its counting sort) {te:7.1f} us", flush=True)
