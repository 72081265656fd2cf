"""Dev: the row-sharded EntityRankingJob at world size 1 over RCCL on one GPU (the collectives
degenerate to copies: this is the fixed cost of the sharded evaluation path) beside the unsharded
job -- ComplEx-512, FB15K-237 shape, 20,466 test triples, batch 1,024."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import numpy as np
import torch
import torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1)
torch.cuda.set_device(0)
from kge import Config, Dataset, KgeModel
from kge.job import EntityRankingJob
for mode in ("off", "on"):
    c = Config(); c.set("model", "complex"); c._import("complex"); c.set("job.device", "cuda:0")
    c.set("lookup_embedder.dim", 512); c.set("lookup_embedder.initialize", "normal_")
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("engine.row_sharded", mode); c.set("verbose", False); c.set("eval.split", "test"); c.set("eval.batch_size", 1024)
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    torch.manual_seed(0)
    model = KgeModel.create(c, ds); model.eval()
    ej = EntityRankingJob(c, ds, model=model); ej._prepare()
    ej._run()
    ts = []
    for _ in range(5):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        tr = ej._run(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    print(f"engine.row_sharded {mode}: {np.median(ts) * 1e3:.2f} ms, MRR {tr['mean_reciprocal_rank_filtered']:.10f}", flush=True)
dist.destroy_process_group()
