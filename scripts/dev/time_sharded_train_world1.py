"""Row-sharded 1vsAll training step (RowShardedScorer.train_1vsall_global) at world size 1 over
RCCL on one GPU, next to the single-GPU fused step: C2 shape and one rank's Wikidata5M shard.

    python scripts/dev/time_sharded_train_world1.py [rows ...]     (default: 14541 574311)

KGE_SHARDED_LOSS=bce times the step with train.loss bce (offset 0) instead of kl.
"""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kge import _lib as L  # noqa: E402
from kge.sharded import EngineOps, RowShardedScorer  # noqa: E402

with socket.socket() as s_:
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("nccl", rank=0, world_size=1)
R, B, d = 237, 1024, 512
LOSS = (os.environ.get("KGE_SHARDED_LOSS", "kl"), 0.0)
for E in ([int(a) for a in sys.argv[1:]] or [14541, 574311]):
    torch.manual_seed(0)
    ent = (torch.randn(E, d, device="cuda") * 0.1)
    rel = (torch.randn(R, d, device="cuda") * 0.1)
    sh = RowShardedScorer(ent, 0, E, E, rel, EngineOps(L.COMPLEX, L.PREC_BF16X3))
    host = torch.stack([torch.randint(0, E, (16, B)), torch.randint(0, R, (16, B)), torch.randint(0, E, (16, B))], 2)
    tr = host.cuda()
    for i in range(3):
        sh.train_1vsall_global(tr[i], host_triples=host[i], loss=LOSS)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 10
    issue = 0.0
    for i in range(n):
        t1 = time.perf_counter()
        loss, d_ent, d_rel = sh.train_1vsall_global(tr[3 + i], host_triples=host[3 + i], loss=LOSS)
        issue += time.perf_counter() - t1  # host time to issue the step (no device sync inside)
    torch.cuda.synchronize()
    print(f"E {E} loss {LOSS[0]}: sharded training gradients {(time.perf_counter() - t0) / n * 1e3:.3f} ms per step, host issue "
          f"{issue / n * 1e3:.3f} ms per step, {sh.collectives_last_step} collectives per step "
          f"(loss {float(loss):.4f})", flush=True)
    del sh, ent, d_ent
    torch.cuda.empty_cache()
dist.destroy_process_group()
