"""Run one score_dot variant a few times at the C2 shape (for rocprofv3 PMC passes)."""
import ctypes, sys
import os; ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'kge-1_amd'))
import torch
from kge import _lib as L
lib = L.lib()
lib.kge_dev_score_dot_x3.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
lib.kge_dev_split_rows.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
v = sys.argv[1]
E, R, B, d = 14541, 237, 1024, 512
torch.manual_seed(0)
ent = (torch.randn(E, d) * 0.1).cuda(); rel = (torch.randn(R, d) * 0.1).cuda()
s = torch.randint(0, E, (B,)).cuda(); p = torch.randint(0, R, (B,)).cuda()
q = L.prep_query(0, 0, ent, s, rel, p, B, d, d)
qh = torch.empty(B, d, dtype=torch.bfloat16, device='cuda'); ql = torch.empty_like(qh)
st = L.stream()
lib.kge_dev_split_rows(q.data_ptr(), d, B, d, qh.data_ptr(), ql.data_ptr(), d, st)
out = torch.empty(B, E, device='cuda')
for _ in range(10):
    if v == 'old':
        L.score_dot(q, ent, None, 1, out=out)
    else:
        lib.kge_dev_score_dot_x3(int(v), qh.data_ptr(), ql.data_ptr(), d, ent.data_ptr(), d, None, B, E, d, out.data_ptr(), E, st)
torch.cuda.synchronize()
