"""Sweep score_dot variants at the C2 shape on one GPU (interleaved rounds, one process)."""
import ctypes, sys, time
import os as _os; _os.environ.setdefault('KGE_LIBRARY', _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))), 'kge-1_amd', 'csrc', 'build_dev', 'libkgescore_dev.so')); _R = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))); sys.path.insert(0, _R); sys.path.insert(0, _os.path.join(_R, 'kge-1_amd'))
import numpy as np, torch
from kge import _lib as L
lib = L.lib()
lib.kge_dev_score_dot_persist.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
E, R, B, d = 14541, 237, 1024, 512
if len(sys.argv) > 1: B = int(sys.argv[1])
import os
E = int(os.environ.get('KGE_E', E))
torch.manual_seed(0)
ent = (torch.randn(E, d) * 0.1).cuda(); rel = (torch.randn(R, d) * 0.1).cuda()
s = torch.randint(0, E, (B,)).cuda(); p = torch.randint(0, R, (B,)).cuda()
q = L.prep_query(0, 0, ent, s, rel, p, B, d, d)
ldo = ((d + 31) // 32) * 32
qh = torch.empty(B, ldo, dtype=torch.bfloat16, device='cuda'); ql = torch.empty_like(qh)
st = L.stream()
assert lib.kge_split_rows(q.data_ptr(), d, B, d, qh.data_ptr(), ql.data_ptr(), ldo, st) == 0
ref = (q.double() @ ent.double().T)
out = torch.empty(B, E, device='cuda')
LDA = (E + 31) // 32 * 32  # 128-B aligned score rows ('a' suffix)
outa_buf = torch.empty(B, LDA, device='cuda')
outa = outa_buf[:, :E]
def run(v):
    global out
    if v == 'fill':
        out.fill_(1.0); return
    if v == 'filla':
        outa.fill_(1.0); return
    if isinstance(v, str) and v.endswith('a'):
        o = out
        out = outa
        try:
            assert lib.kge_dev_score_dot_persist(int(v[1:-1]), qh.data_ptr(), ql.data_ptr(), ldo, ent.data_ptr(), d, None,
                                                 B, E, d, outa_buf.data_ptr(), LDA, st) == 0
        finally:
            out = o
        return
    if v == 'split': L.score_dot_split(qh, ql, ent, None, d, out=out)  # the production entry point (picks the tile height)
    elif v == 'old': L.score_dot(q, ent, None, 1, out=out)
    elif v == 'old32': L.score_dot(q, ent, None, 0, out=out)
    elif isinstance(v, str) and v.startswith('p'):
        assert lib.kge_dev_score_dot_persist(int(v[1:]), qh.data_ptr(), ql.data_ptr(), ldo, ent.data_ptr(), d, None, B, E, d,
                                        out.data_ptr(), E, st) == 0
    else:
        raise ValueError(v)
variants = sys.argv[2].split(',') if len(sys.argv) > 2 else ['p0', 'p1']
res = {v: [] for v in variants}
for v in variants:
    if v.startswith('fill'):
        continue
    o = outa if v.endswith('a') else out
    o.zero_(); run(v); torch.cuda.synchronize()
    err = ((o.double() - ref).abs().amax(1) / ref.abs().amax(1)).max().item()
    if v == variants[0]:
        first = o.clone()
    same = bool((o == first).all().item()) if o.shape == first.shape else None
    print(f"variant {v}: max rel err {err:.2e}  bit-identical to {variants[0]}: {same}", flush=True)
for rnd in range(5):
    for v in variants:
        for _ in range(3): run(v)
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20): run(v)
        b.record(); torch.cuda.synchronize()
        res[v].append(a.elapsed_time(b) / 20 * 1e3)
for v in variants:
    t = np.median(res[v])
    print(f"variant {v}: median {t:.1f} us  min {min(res[v]):.1f}  -> {2*B*E*d/t/1e6:.0f} TF alg, {3*2*B*E*d/t/1e6:.0f} TF bf16")
