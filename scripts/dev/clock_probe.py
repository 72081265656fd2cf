"""Dev probe: per-workgroup shader clocks vs 100-MHz real-time ticks inside the contraction kernel."""
import ctypes, sys
sys.path.insert(0, '.'); sys.path.insert(0, 'kge-1_amd')  # run from the repository root
import os; os.environ.setdefault('KGE_LIBRARY', 'kge-1_amd/csrc/build_dev/libkgescore_dev.so')  # `make dev`: has the kge_dev_* probes
import numpy as np, torch
from kge import _lib as L
lib = L.lib()
lib.kge_dev_score_dot_persist.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
E, R, B, d = 14541, 237, 1024, 512
torch.manual_seed(0)
ent = (torch.randn(E, d) * 0.1).cuda()
q = (torch.randn(B, d) * 0.1).cuda()
qh = torch.empty(B, d, dtype=torch.bfloat16, device='cuda'); ql = torch.empty_like(qh)
st = L.stream()
assert lib.kge_split_rows(q.data_ptr(), d, B, d, qh.data_ptr(), ql.data_ptr(), d, st) == 0
out = torch.zeros(B + 2, E, device='cuda')
for v in [int(x) for x in sys.argv[1].split(',')]:
    for _ in range(30):
        assert lib.kge_dev_score_dot_persist(v, qh.data_ptr(), ql.data_ptr(), d, ent.data_ptr(), d, None, B, E, d,
                                             out.data_ptr(), E, st) == 0
    torch.cuda.synchronize()
    r = out[B, :512].cpu().numpy().reshape(-1, 2)
    r = r[r[:, 1] > 0]
    ghz = r[:, 0] / r[:, 1] / 10.0  # memrealtime is 100 MHz
    r2 = out[B + 1, :512].cpu().numpy().reshape(-1, 2)[:len(r)]
    print(f"variant {v}: cycles to K loop entry {np.median(r2[:, 0]):.0f}, in the K loop {np.median(r2[:, 1] - r2[:, 0]):.0f}, "
          f"after it {np.median(r[:, 0] - r2[:, 1]):.0f} (medians over workgroups)")
    print(f"variant {v}: blocks {len(r)}  block time {np.median(r[:,1])/100:.1f} us (max {r[:,1].max()/100:.1f})  "
          f"clock median {np.median(ghz):.3f} GHz  min {ghz.min():.3f}  max {ghz.max():.3f}")
