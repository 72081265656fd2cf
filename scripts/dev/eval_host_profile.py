"""Dev: cProfile of the host side of EntityRankingJob._run (ComplEx-512, FB15K-237 shape, batch
1,024): where the ~0.1 ms of host time per evaluation batch goes."""
import cProfile
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import Config, Dataset, KgeModel  # noqa: E402
from kge.job import EntityRankingJob  # noqa: E402

c = Config()
c.set("model", "complex")
c._import("complex")
c.set("job.device", "cuda:0")
c.set("lookup_embedder.dim", 512)
c.set("lookup_embedder.initialize", "normal_")
c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
c.set("engine.row_sharded", "off")
c.set("verbose", False)
c.set("eval.split", "test")
c.set("eval.batch_size", 1024)
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
torch.manual_seed(0)
model = KgeModel.create(c, ds)
model.eval()
ej = EntityRankingJob(c, ds, model=model)
ej._prepare()
for _ in range(3):
    ej._run()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    ej._run()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
