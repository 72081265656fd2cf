"""A few recorded C2 1vsAll steps with the options tuned LibKGE configurations carry (embedder
dropout 0.2, frequency-weighted Lp penalties) for rocprofv3; KIND=plain drops the options."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch  # noqa: E402

from kge import Config, Dataset  # noqa: E402
from kge.job import TrainingJob  # noqa: E402

B = 1024
c = Config()
c.set("model", "complex")
c._import("complex")
c.set("job.device", "cuda")
c.set("lookup_embedder.dim", 512)
c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
c.set("train.type", "1vsAll")
c.set("train.optimizer", "Adagrad")
c.set("train.optimizer_args", {"lr": 0.2})
c.set("train.batch_size", B)
c.set("engine.row_sharded", "off")
c.set("verbose", False)
if os.environ.get("KIND", "opts") == "opts":
    c.set("lookup_embedder.dropout", 0.2)
    c.set("lookup_embedder.regularize_args.weighted", True)
    c.set("complex.entity_embedder.regularize_weight", 1e-6)
    c.set("complex.relation_embedder.regularize_weight", 1e-6)
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
torch.manual_seed(0)
job = TrainingJob.create(c, ds)
job._prepare()
train = ds.split("train")
perm = torch.randperm(len(train), generator=torch.Generator().manual_seed(0))
for i in range(6):
    job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(6, 26):
    job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
torch.cuda.synchronize()
gs = job._graph_step
print(f"step {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms, recorded {gs is not None and gs.graph is not None}", flush=True)
