"""Dev timing: the N > 1 bench's row-sharded step at world size 1 (RCCL, one GPU) next to the
plain score_sp contraction of the same shape -- the overhead the exchange path adds per step."""
import os, socket, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch, torch.distributed as dist
from kge import _lib as L
from kge.sharded import EngineOps, RowShardedScorer
with socket.socket() as s_:
    s_.bind(("127.0.0.1", 0)); port = s_.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("nccl", rank=0, world_size=1)
E, R, B, d = 14541, 237, 1024, 512
torch.manual_seed(0)
ent = (torch.randn(E, d) * 0.1).cuda(); rel = (torch.randn(R, d) * 0.1).cuda()
sh = RowShardedScorer(ent, 0, E, E, rel, EngineOps(L.COMPLEX, L.PREC_BF16X3))
s = torch.randint(0, E, (64, B)).cuda(); p = torch.randint(0, R, (64, B)).cuda()
def loop(fn, n=40, w=10):
    for i in range(w): fn(i)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(n): fn(w + i)
    t1 = time.perf_counter()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e6, (t1 - t0) / n * 1e6
tickets = []
def pipelined(i):
    if not tickets: tickets.append(sh.submit_queries_local(s[i % 64], p[i % 64]))
    tickets.append(sh.submit_queries_local(s[(i + 1) % 64], p[(i + 1) % 64]))
    return sh.score_submitted(tickets.pop(0))
def serial(i):
    return sh.score_submitted(sh.submit_queries_local(s[i % 64], p[i % 64]))
groups = {}
KX = 4
def grouped(i):  # one preparation + one all_gather per KX steps, issued one group ahead
    g0 = i - i % KX
    def sub(a):
        a %= 64 - KX
        return sh.submit_queries_local(s[a:a + KX].reshape(-1), p[a:a + KX].reshape(-1))
    if g0 not in groups: groups[g0] = sub(g0)
    if i % KX == 0 and g0 + KX not in groups: groups[g0 + KX] = sub(g0 + KX)
    out = sh.score_submitted(groups[g0], (i % KX, KX))
    if i % KX == KX - 1: del groups[g0]
    return out
from kge import engine
def plain(i):
    return engine.score_all(L.COMPLEX, L.DIR_SP, L.PREC_BF16X3, 1.0, ent, s[i % 64], rel, p[i % 64], ent, None)
with torch.no_grad():
    for name, fn in (("plain score_all", plain), ("sharded serial", serial), ("sharded pipelined", pipelined),
                     ("sharded grouped x4", grouped)):
        total, issue = loop(fn)
        print(f"{name:20s} {total:7.1f} us/step (host issue {issue:.1f})")
dist.destroy_process_group()

# host-side cost of each piece of the pipelined step (issue time, no sync inside)
dist.init_process_group("nccl", rank=0, world_size=1) if not dist.is_initialized() else None
from kge.sharded import all_gather_into_tensor
sh = RowShardedScorer(ent, 0, E, E, rel, EngineOps(L.COMPLEX, L.PREC_BF16X3))
acc = {"sub": 0.0, "prep": 0.0, "empty": 0.0, "gather": 0.0, "wait": 0.0, "score": 0.0}
with torch.no_grad():
    for i in range(220):
        t0 = time.perf_counter(); local = s[i % 64] - 0
        t1 = time.perf_counter(); q = sh.ops.prep_planes(0, ent, local, rel, p[i % 64])
        t2 = time.perf_counter(); out = torch.empty((q.shape[0], q.shape[1]), dtype=q.dtype, device=q.device)
        t3 = time.perf_counter(); w = all_gather_into_tensor(out, q, async_op=True)
        t4 = time.perf_counter(); w.wait()
        t5 = time.perf_counter(); sc = sh.ops.score_planes(out, ent)
        t6 = time.perf_counter()
        if i >= 20:
            for k, v in zip(acc, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
                acc[k] += v
        if i % 8 == 7:
            torch.cuda.synchronize()
print({k: round(v / 200 * 1e6, 1) for k, v in acc.items()}, "us host time per call")
dist.destroy_process_group()
