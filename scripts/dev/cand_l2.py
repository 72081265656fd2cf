"""kge_score_cand at the C4 shape, candidate rows in random or ascending order per query
(argv[1] = sorted): for a PMC pass over the L2 hit / miss counters."""
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
if len(sys.argv) > 1 and sys.argv[1] == "sorted":
    cand = torch.sort(cand, 1).values
s = L.score_cand(L.DISTMULT, 1.0, L.DIR_SP, q, ent, cand)
for _ in range(5):
    L.score_cand(L.DISTMULT, 1.0, L.DIR_SP, q, ent, cand, out=s)
torch.cuda.synchronize()
print("done", sys.argv[1:])
