"""Dev: the distance backward alone (kind = argv[1], default L1) at B = 1,024, E = 14,541,
d = 512 (RotatE kinds: d = 1,024): dq and dt passes timed separately and together, against
float64 on a sub-block.  KGE_DIST_BWD_OWN=1 selects the older owner-computes kernel."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'kge-1_amd'))
import torch
from kge import _lib as L
kind = int(sys.argv[1]) if len(sys.argv) > 1 else 0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
E = int(sys.argv[3]) if len(sys.argv) > 3 else 14541
d = int(sys.argv[5]) if len(sys.argv) > 5 else (1024 if kind >= 2 else 512)
torch.manual_seed(0)
q = (torch.randn(B, d) * 0.1).cuda(); ent = (torch.randn(E, d) * 0.1).cuda()
g = (torch.randn(B, E) * 1e-3).cuda()
def run(dq, dt):
    L.score_dist_bwd(kind, -1.0, g, q, ent, None, dq, dt)
def timed(dq, dt):
    for _ in range(2): run(dq, dt)
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): run(dq, dt)
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
dq = torch.zeros(B, d, device='cuda'); dt = torch.zeros(E, d, device='cuda')
kd = d // 2 if kind >= 2 else d
ops1 = {0: 3, 1: 2, 2: 9, 3: 4}[kind] * B * E * kd
for name, a, b in (("dq", dq, None), ("dt", None, dt), ("both", dq, dt)):
    us = timed(a, b)
    n = 2 if name == "both" else 1
    print(f"kind {kind} {name}: {us:.1f} us, {n * ops1 / us / 1e6:.1f} T lane-ops/s = {n * ops1 / us / 1e6 / 78.6:.3f} of 78.6 (counting {ops1 / (B * E * kd):.0f} VALU per pair-component)", flush=True)
# check against float64 autograd on a sub-block
nb, mb = 40, 300
qs = q[:nb].double().clone().requires_grad_(); ts = ent[:mb].double().clone().requires_grad_()
if kind < 2:
    diff = qs[:, None, :] - ts[None, :, :]
    dist = diff.abs().sum(-1) if kind == 0 else diff.pow(2).sum(-1).sqrt()
else:
    h = d // 2
    dr = qs[:, None, :h] - ts[None, :, :h]; di = qs[:, None, h:] - ts[None, :, h:]
    mod = (dr * dr + di * di).sqrt()
    dist = mod.sum(-1) if kind == 2 else (dr * dr + di * di).sum(-1).sqrt()
gs = g[:nb, :mb].contiguous()
(-dist * gs.double()).sum().backward()
dq = torch.zeros(nb, d, device='cuda'); dt = torch.zeros(mb, d, device='cuda')
L.score_dist_bwd(kind, -1.0, gs, q[:nb].contiguous(), ent[:mb].contiguous(), None, dq, dt)
eq = float((dq.double() - qs.grad).abs().max() / qs.grad.abs().max()); et = float((dt.double() - ts.grad).abs().max() / ts.grad.abs().max())
print(f"sub-block vs float64: dq {eq:.2e} dt {et:.2e}")
