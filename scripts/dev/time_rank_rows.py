"""Dev timing: the ranking launch of one evaluation batch (2,048 x 14,541 block of bf16x3
scores of random N(0, 0.1) tables), refined vs not, fixed seed."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import numpy as np, torch
from kge import _lib as L
from kge.job.entity_ranking import refine_band
torch.manual_seed(0)
E, B, d = 14541, 1024, 512
ent = (torch.randn(E, d) * 0.1).cuda(); q = (torch.randn(2 * B, d) * 0.014).cuda()
qh, ql = L.split_rows(q)
buf = torch.empty(2 * B, (E + 3) // 4 * 4, device="cuda"); s = buf[:, :E]
L.score_dot_split(qh, ql, ent, None, d, out=s)
ti = torch.randint(0, E, (2 * B,)).cuda()
ts = s[torch.arange(2 * B), ti].contiguous()
ptr = torch.zeros(B + 1, dtype=torch.int64).cuda(); col = torch.zeros(1, dtype=torch.int64).cuda()
g = torch.empty(4 * B, dtype=torch.int64).cuda(); t = torch.empty_like(g)
tmax = L.row_norm_max(ent)
pa, pb = (ti[:B], ts[:B], ptr, None), (ti[B:], ts[B:], ptr, None)
for name, ref in (("plain", None), ("refined", (q, ent, refine_band(d), tmax))):
    ts_ = []
    for r in range(5):
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        L.rank_rows(s, B, 0, pa, pb, col, None, g, t, accumulate=False, refine=ref)
        a.record()
        for _ in range(10): L.rank_rows(s, B, 0, pa, pb, col, None, g, t, accumulate=False, refine=ref)
        b.record(); torch.cuda.synchronize()
        ts_.append(a.elapsed_time(b) / 10 * 1e3)
    print(f"rank_rows {name:8s} {np.median(ts_):7.1f} us")
