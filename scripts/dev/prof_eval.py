"""Dev probe: filtered entity-ranking eval of the synthetic FB15K-237 test split (C2 model)."""
import os, sys, time, cProfile, pstats
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch
from kge import Config, Dataset, KgeModel
from kge.job import EntityRankingJob

c = Config()
c.set("model", "complex"); c._import("complex")
c.set("job.device", "cuda")
c.set("lookup_embedder.dim", 512)
c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
c.set("eval.split", "test"); c.set("eval.batch_size", 1024)
c.set("engine.eval_streams", 1)  # per-kernel durations: launches overlapping on two streams stretch each other
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
model = KgeModel.create(c, ds)
model.eval()
ej = EntityRankingJob(c, ds, model=model)
ej._prepare()
for i in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    tr = ej._run()
    torch.cuda.synchronize(); print("eval s", round(time.perf_counter() - t0, 4), tr["mean_reciprocal_rank_filtered"])
pr = cProfile.Profile(); pr.enable()
ej._run(); torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
