"""A few 1vsAll training steps (ComplEx-512, FB15K-237 shape, B=1024) for rocprofv3."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch  # noqa: E402

from kge import Config, Dataset  # noqa: E402
from kge.job import TrainingJob  # noqa: E402

model_name = sys.argv[1] if len(sys.argv) > 1 else "complex"
train_type = sys.argv[2] if len(sys.argv) > 2 else "1vsAll"
c = Config()
c.set("model", model_name)
c._import(model_name)
c.set("job.device", "cuda")
c.set("lookup_embedder.dim", 512)
c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
c.set("train.type", train_type)
c.set("train.optimizer", "Adagrad")
c.set("train.optimizer_args", {"lr": 0.2})
c.set("train.batch_size", 1024 if train_type == "1vsAll" else 512)
c.set("verbose", False)
if os.environ.get("KGE_PROF_OPTIONS") == "dropout":
    c.set("lookup_embedder.dropout", 0.2)
if os.environ.get("KGE_PROF_OPTIONS") == "dropout_penalties":  # what tuned LibKGE configurations carry
    c.set("lookup_embedder.dropout", 0.2)
    c.set("lookup_embedder.regularize_args.weighted", True)
    c.set(f"{model_name}.entity_embedder.regularize_weight", 1e-6)
    c.set(f"{model_name}.relation_embedder.regularize_weight", 1e-6)
if os.environ.get("KGE_NO_GRAPH") == "1":  # per-kernel times of the eager step, for comparison
    c.set("engine.graph_step", False)
ds = Dataset.synthetic(c, "fb15k-237" if train_type == "1vsAll" else "wn18rr", seed=0)
job = TrainingJob.create(c, ds)
job._prepare()
B = c.get("train.batch_size")
perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))
WARM, STEPS = int(os.environ.get("PROF_WARM", "8")), int(os.environ.get("PROF_STEPS", "10"))
nb = job.num_examples // B


def ids(i):  # (epochs of the same permutation when the run is longer than one)
    return perm[(i % nb) * B:(i % nb + 1) * B]


for i in range(WARM):
    job.train_step(i, job._collate(ids(i)))
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(WARM, WARM + STEPS):
    job.train_step(i, job._collate(ids(i)))
torch.cuda.synchronize()
print(f"{model_name} {train_type} step {(time.perf_counter() - t0) / STEPS * 1e3:.3f} ms")
gs = getattr(job, "_graph_step", None)
print("graph step:", None if gs is None else ("recorded" if gs.graph is not None else f"not recorded: {gs.error}"),
      f"({len(gs.graphs)} split points)" if hasattr(gs, "graphs") else "")
