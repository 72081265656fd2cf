"""Do two contraction launches on two streams share the CUs?  Variants of the C2 contraction
(dev library) timed back to back on one stream and alternating over two streams."""
import ctypes, os, sys
_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('KGE_LIBRARY', os.path.join(_R, 'kge-1_amd', 'csrc', 'build_dev', 'libkgescore_dev.so'))
sys.path.insert(0, _R); sys.path.insert(0, os.path.join(_R, 'kge-1_amd'))
import numpy as np, torch
from kge import _lib as L
lib = L.lib()
lib.kge_dev_score_dot_persist.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
E, R, B, d = 14541, 237, int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 512
torch.manual_seed(0)
ent = (torch.randn(E, d) * 0.1).cuda(); rel = (torch.randn(R, d) * 0.1).cuda()
s = torch.randint(0, E, (B,)).cuda(); p = torch.randint(0, R, (B,)).cuda()
q = L.prep_query(0, 0, ent, s, rel, p, B, d, d)
ldo = ((d + 31) // 32) * 32
qh = torch.empty(B, ldo, dtype=torch.bfloat16, device='cuda'); ql = torch.empty_like(qh)
assert lib.kge_split_rows(q.data_ptr(), d, B, d, qh.data_ptr(), ql.data_ptr(), ldo, L.stream()) == 0
ref = (q.double() @ ent.double().T)
outs = [torch.empty(B, E, device='cuda') for _ in range(2)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
torch.cuda.synchronize()


def launch(v, which, st):
    assert lib.kge_dev_score_dot_persist(v, qh.data_ptr(), ql.data_ptr(), ldo, ent.data_ptr(), d, None, B, E, d,
                                         outs[which].data_ptr(), E, st.cuda_stream) == 0


def timed(v, nstreams, n=60):
    for rep in range(2):
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        e = [torch.cuda.Event() for _ in streams]
        a.record(streams[0])
        if nstreams == 2:
            streams[1].wait_event(a)
        for i in range(n):
            launch(v, i % nstreams, streams[i % nstreams])
        if nstreams == 2:
            e[1].record(streams[1]); streams[0].wait_event(e[1])
        b.record(streams[0]); torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for v in [int(x) for x in (sys.argv[2].split(',') if len(sys.argv) > 2 else ['30', '31', '60', '61'])]:
    outs[0].zero_(); launch(v, 0, streams[0]); torch.cuda.synchronize()
    err = ((outs[0].double() - ref).abs().amax(1) / ref.abs().amax(1)).max().item()
    rows = []
    for rnd in range(3):
        rows.append((timed(v, 1), timed(v, 2)))
    one, two = np.median([r[0] for r in rows]), np.median([r[1] for r in rows])
    print(f"variant {v}: max rel err {err:.1e}; per launch: one stream {one:.1f} us, alternating over two streams {two:.1f} us", flush=True)
