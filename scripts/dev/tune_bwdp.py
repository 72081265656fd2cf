"""Dev timing: plane-fed backward GEMMs and loss kernel vs the fp32-G kernels at the stacked
C2 training shape (2,048 queries x 14,541 entities x 512); interleaved rounds in one process."""
import sys
import os as _os; _os.environ.setdefault('KGE_LIBRARY', _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))), 'kge-1_amd', 'csrc', 'build_dev', 'libkgescore_dev.so'))  # `make dev`
import os as _os; _R = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))); sys.path.insert(0, _R); sys.path.insert(0, _os.path.join(_R, 'kge-1_amd'))
import numpy as np, torch
from kge import _lib as L
n, m, d = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (2048, 14541, 512)))
torch.manual_seed(0)
ent = (torch.randn(m, d) * 0.1).cuda()
q = (torch.randn(n, d) * 0.1).cuda()
labels = torch.randint(0, m, (n,)).cuda()
n_pad, ld = L.planes_layout(n, m)
# KGE_S_SCALE: spread of the scores.  1 (default): peaky softmax, most gradient entries ~0;
# 0.01: the near-uniform softmax of an untrained model (every entry ~1/m) -- denser operand bits
S = torch.randn(n_pad, ld, device="cuda") * float(_os.environ.get("KGE_S_SCALE", "1"))
bufp = S.clone()
_, gp = L.softmax_planes(bufp, n, m, labels, None, 0.0, 1.0 / n)
buf4 = torch.empty(n, (m + 3) // 4 * 4, device="cuda"); s4 = buf4[:, :m]; s4.copy_(S[:n, :m])
L.softmax_xent(s4, labels, 1.0 / n, g=s4)
ldp = (d + 31) // 32 * 32
qh = torch.zeros(n_pad, ldp, device="cuda", dtype=torch.bfloat16); ql = torch.zeros_like(qh)
h, l = L.split_rows(q); qh[:n], ql[:n] = h, l
dq = torch.empty(n, d, device="cuda"); de = torch.empty(m, d, device="cuda")
src_p = S.clone(); src_4 = buf4.clone()
def t_loss_planes():
    bufp.copy_(src_p); 
def run(name, fn, reps=20):
    for _ in range(3): fn()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
def plain(fn):  # the same entry point with the kernels' plain (not software-pipelined) loops
    def run_plain():
        L.lib().kge_dev_bwdp_pipe(0)
        fn()
        L.lib().kge_dev_bwdp_pipe(1)
    return run_plain
dq2 = torch.empty_like(dq); de2 = torch.empty_like(de)
L.score_dot_bwd_q_planes(gp, ent, dq=dq); L.score_dot_bwd_t_planes(gp, qh, ql, de)
plain(lambda: L.score_dot_bwd_q_planes(gp, ent, dq=dq2))(); plain(lambda: L.score_dot_bwd_t_planes(gp, qh, ql, de2))()
torch.cuda.synchronize()
print("pipelined == plain bitwise: dQ", bool((dq == dq2).all()), " dE", bool((de == de2).all()), flush=True)
variants = {
    "dQ planes plain loop": plain(lambda: L.score_dot_bwd_q_planes(gp, ent, dq=dq)),
    "dE planes plain loop": plain(lambda: L.score_dot_bwd_t_planes(gp, qh, ql, de)),
    "dQ old (fp32 G, ws)": lambda: L.score_dot_bwd_q(s4, ent, None, L.PREC_BF16X3, dq=dq),
    "dQ planes": lambda: L.score_dot_bwd_q_planes(gp, ent, dq=dq),
    "dE old (fp32 G)": lambda: L.score_dot_bwd_t(s4, q, None, de, L.PREC_BF16X3, accumulate=False),
    "dE planes": lambda: L.score_dot_bwd_t_planes(gp, qh, ql, de),
    "loss old (in place fp32)": lambda: L.softmax_xent(s4, labels, 1.0 / n, g=s4),
    "loss planes": lambda: L.softmax_planes(bufp, n, m, labels, None, 0.0, 1.0 / n),
}
big = torch.empty(96 * 1024 * 1024, device="cuda")  # 384 MB: more than the 256-MB memory-side cache
variants["dQ then dE (pair)"] = lambda: (L.score_dot_bwd_q_planes(gp, ent, dq=dq), L.score_dot_bwd_t_planes(gp, qh, ql, de))
variants["loss planes then dQ then dE"] = lambda: (L.softmax_planes(bufp, n, m, labels, None, 0.0, 1.0 / n), L.score_dot_bwd_q_planes(gp, ent, dq=dq), L.score_dot_bwd_t_planes(gp, qh, ql, de))
def two_stage(fn):
    def run2():
        L.lib().kge_dev_bwdp_stages(2)
        fn()
        L.lib().kge_dev_bwdp_stages(3)
    return run2
de3 = torch.empty_like(de)
two_stage(lambda: L.score_dot_bwd_t_planes(gp, qh, ql, de3))(); L.score_dot_bwd_t_planes(gp, qh, ql, de); torch.cuda.synchronize()
print("dE 3 stage buffers == 2 stage buffers bitwise:", bool((de == de3).all()), flush=True)
variants["dE planes, 2 stage buffers"] = two_stage(lambda: L.score_dot_bwd_t_planes(gp, qh, ql, de))
variants["384-MB fill then dE, 2 stage buffers"] = two_stage(lambda: (big.fill_(1.0), L.score_dot_bwd_t_planes(gp, qh, ql, de)))
qh1, ql1 = L.split_rows(q)
variants["forward"] = lambda: L.score_dot_split(qh1, ql1, ent, None, d, out=bufp[:n, :m])
variants["forward, loss planes, dQ, dE"] = lambda: (L.score_dot_split(qh1, ql1, ent, None, d, out=bufp[:n, :m]), L.softmax_planes(bufp, n, m, labels, None, 0.0, 1.0 / n), L.score_dot_bwd_q_planes(gp, ent, dq=dq), L.score_dot_bwd_t_planes(gp, qh, ql, de))
state = torch.zeros(m, d, device="cuda"); wts = ent.clone()
variants["forward, loss planes, dQ, dE, adagrad"] = lambda: (L.score_dot_split(qh1, ql1, ent, None, d, out=bufp[:n, :m]), L.softmax_planes(bufp, n, m, labels, None, 0.0, 1.0 / n), L.score_dot_bwd_q_planes(gp, ent, dq=dq), L.score_dot_bwd_t_planes(gp, qh, ql, de), L.adagrad_step(wts, de, state, -0.0, 1e-10, 0.0, False))
variants["adagrad"] = lambda: L.adagrad_step(wts, de, state, -0.0, 1e-10, 0.0, False)
variants["384-MB fill"] = lambda: big.fill_(1.0)
variants["384-MB fill then dE"] = lambda: (big.fill_(1.0), L.score_dot_bwd_t_planes(gp, qh, ql, de))
variants["384-MB fill then dQ"] = lambda: (big.fill_(1.0), L.score_dot_bwd_q_planes(gp, ent, dq=dq))
res = {k: [] for k in variants}
for r in range(5):
    for k, fn in variants.items():
        res[k].append(run(k, fn))
for k, v in res.items():
    print(f"{k:28s} {np.median(v):8.1f} us  (min {min(v):.1f})")
flops = 2.0 * n * m * d
for k in ("dQ planes", "dE planes", "dQ old (fp32 G, ws)", "dE old (fp32 G)"):
    print(f"{k:28s} {flops / np.median(res[k]) / 1e6:6.1f} TF/s = {flops / np.median(res[k]) / 1e6 / 833.3:.3f} of the bf16x3 peak")
