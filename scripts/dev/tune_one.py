"""Run one contraction variant a few times at the C2 shape (for rocprofv3 PMC passes):
python scripts/dev/tune_one.py <variant of kge_dev_score_dot_persist>."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'kge-1_amd'))
import torch
from kge import _lib as L
lib = L.lib()
lib.kge_dev_score_dot_persist.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
v = int(sys.argv[1])
E, R, B, d = 14541, 237, 1024, 512
torch.manual_seed(0)
ent = (torch.randn(E, d) * 0.1).cuda(); q = (torch.randn(B, d) * 0.1).cuda()
qh = torch.empty(B, d, dtype=torch.bfloat16, device='cuda'); ql = torch.empty_like(qh)
st = L.stream()
assert lib.kge_split_rows(q.data_ptr(), d, B, d, qh.data_ptr(), ql.data_ptr(), d, st) == 0
out = torch.empty(B, E, device='cuda')
for _ in range(10):
    assert lib.kge_dev_score_dot_persist(v, qh.data_ptr(), ql.data_ptr(), d, ent.data_ptr(), d, None, B, E, d,
                                         out.data_ptr(), E, st) == 0
torch.cuda.synchronize()
