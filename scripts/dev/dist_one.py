"""Dev: the all-entities distance kernel alone (kind = argv[1], default L1) at B = 1,024,
E = 14,541, d = 512, a few launches -- the target of PMC passes (scripts/dev/pmc_dist.sh)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'kge-1_amd'))
import torch
from kge import _lib as L
kind = int(sys.argv[1]) if len(sys.argv) > 1 else 0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, d = 1024, 512
E = int(sys.argv[3]) if len(sys.argv) > 3 else 14541
torch.manual_seed(0)
q = (torch.randn(B, d) * 0.1).cuda(); ent = (torch.randn(E, d) * 0.1).cuda()
out = torch.empty(B, E, device='cuda')
for _ in range(3):
    L.score_dist(kind, -1.0, q, ent, None, out=out)
a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(reps):
    L.score_dist(kind, -1.0, q, ent, None, out=out)
b.record(); torch.cuda.synchronize()
us = a.elapsed_time(b) / reps * 1e3
ops = {0: 2, 1: 2, 2: 6, 3: 4}[kind] * B * E * (d // 2 if kind >= 2 else d)
print(f"kind {kind} E {E}: {us:.1f} us per launch, {ops / us / 1e6:.1f} T lane-ops/s = {ops / us / 1e6 / 78.6:.3f} of 78.6")
