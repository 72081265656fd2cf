"""Dev timing: does the row pitch of the query planes matter?  Forward contraction and dE GEMM at
the stacked C2 shape with the hi / lo planes (a) in separate arrays (pitch 1 KB), (b) packed
[hi | lo] per row (pitch 2 KB), (c) packed with a padded pitch."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import numpy as np, torch
from kge import _lib as L
n, m, d = 2048, 14541, 512
torch.manual_seed(0)
ent = (torch.randn(m, d) * 0.1).cuda(); q = (torch.randn(n, d) * 0.1).cuda()
labels = torch.randint(0, m, (n,)).cuda()
h, l = L.split_rows(q)
n_pad, ld = L.planes_layout(n, m)
S = torch.randn(n_pad, ld, device="cuda"); bufp = S.clone()
_, gp = L.softmax_planes(bufp, n, m, labels, None, 0.0, 1.0 / n)
out = torch.empty(n, ld, device="cuda")[:, :m]
de = torch.empty(m, d, device="cuda")
layouts = {}
layouts["separate arrays, pitch 1024 B"] = (h.contiguous(), l.contiguous())
for pad in (0, 32, 64, 128):
    pk = torch.zeros(n_pad, 2 * d + pad, device="cuda", dtype=torch.bfloat16)
    pk[:n, :d] = h; pk[:n, d:2 * d] = l
    layouts[f"packed [hi|lo], pitch {pk.stride(0) * 2} B"] = (pk[:, :d], pk[:, d:2 * d])
def run(fn, reps=20):
    for _ in range(3): fn()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
res = {}
for rnd in range(5):
    for name, (qh, ql) in layouts.items():
        res.setdefault(name, ([], []))
        res[name][0].append(run(lambda: L.score_dot_split(qh, ql, ent, None, d, out=out)))
        res[name][1].append(run(lambda: L.score_dot_bwd_t_planes(gp, qh, ql, de)))
for name, (f, b) in res.items():
    print(f"{name:40s} forward {np.median(f):6.1f} us   dE {np.median(b):6.1f} us")
