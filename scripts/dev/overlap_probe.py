"""Dev: would the two halves of a stacked 1vsAll step overlap usefully?  Contraction (MFMA-bound)
and fused loss (HBM-bound) of two 1,024-query halves at the C2 shape: back to back on one stream
vs the loss of half A on a second stream while half B's contraction runs; likewise the dQ and dE
GEMMs of one half side by side."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'kge-1_amd'))
import torch
from kge import _lib as L
B, E, d = 1024, 14541, 512
torch.manual_seed(0)
ent = (torch.randn(E, d) * 0.1).cuda()
q = (torch.randn(B, d) * 0.1).cuda()
hi, lo = L.split_rows(q)
labels = torch.randint(0, E, (B,), device="cuda")
n_pad, ld = L.planes_layout(B, E)
bufs = [torch.empty(n_pad, ld, device="cuda") for _ in range(2)]
main = torch.cuda.current_stream()
side = torch.cuda.Stream()

def contraction(b):
    L.score_dot_split(hi, lo, ent, None, d, out=bufs[b][:B, :E])

def loss(b):
    return L.softmax_planes(bufs[b], B, E, labels, None, 0.0, 1.0 / B)

def serial():
    contraction(0); loss(0); contraction(1); loss(1)

def overlapped():
    contraction(0)
    ev = torch.cuda.Event(); ev.record(main)
    with torch.cuda.stream(side):
        side.wait_event(ev)
        loss(0)
        ev2 = torch.cuda.Event(); ev2.record(side)
    contraction(1)
    loss(1)
    main.wait_event(ev2)

def timed(fn, reps=50):
    for _ in range(10): fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3

for name, fn in (("serial", serial), ("loss(A) beside contraction(B)", overlapped), ("serial", serial),
                 ("loss(A) beside contraction(B)", overlapped)):
    print(f"{name:34s} {timed(fn):7.1f} us per pair of halves", flush=True)

# backward GEMMs of one stacked block side by side
n2 = 2 * B
q2 = (torch.randn(n2, d) * 0.1).cuda()
hi2, lo2 = L.split_rows(q2)
n_pad2, ld2 = L.planes_layout(n2, E)
buf2 = torch.empty(n_pad2, ld2, device="cuda")
L.score_dot_split(hi2, lo2, ent, None, d, out=buf2[:n2, :E])
lab2 = torch.randint(0, E, (n2,), device="cuda")
_, gp = L.softmax_planes(buf2, n2, E, lab2, None, 0.0, 1.0 / n2)
hi2p = torch.zeros(n_pad2, hi2.shape[1], device="cuda", dtype=torch.bfloat16); hi2p[:n2] = hi2
lo2p = torch.zeros_like(hi2p); lo2p[:n2] = lo2
d_ent = torch.empty(E, d, device="cuda")
gl = torch.ones(1, device="cuda")

def bwd_serial():
    L.score_dot_bwd_q_planes(gp, ent, gscale=gl)
    L.score_dot_bwd_t_planes(gp, hi2p, lo2p, d_ent, gscale=gl, accumulate=False)

def bwd_side():
    ev = torch.cuda.Event(); ev.record(main)
    with torch.cuda.stream(side):
        side.wait_event(ev)
        L.score_dot_bwd_t_planes(gp, hi2p, lo2p, d_ent, gscale=gl, accumulate=False)
        ev2 = torch.cuda.Event(); ev2.record(side)
    L.score_dot_bwd_q_planes(gp, ent, gscale=gl)
    main.wait_event(ev2)

for name, fn in (("dQ then dE", bwd_serial), ("dQ beside dE", bwd_side), ("dQ then dE", bwd_serial), ("dQ beside dE", bwd_side)):
    print(f"{name:34s} {timed(fn):7.1f} us", flush=True)
