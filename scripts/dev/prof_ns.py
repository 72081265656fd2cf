"""A few negative-sampling steps of BASELINE config C4 (RotatE-1024, 1,024 negatives per corrupted
slot, FB15K-237 shape, B=512) for rocprofv3.  argv[1]: implementation (triple | batch)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch  # noqa: E402

from kge import Config, Dataset  # noqa: E402
from kge.job import TrainingJob  # noqa: E402

impl = sys.argv[1] if len(sys.argv) > 1 else "triple"
model = sys.argv[2] if len(sys.argv) > 2 else "rotate"
torch.manual_seed(0)
c = Config()
c.set("model", model)
c._import(model)
c.set("job.device", "cuda")
c.set("lookup_embedder.dim", int(os.environ.get("NS_DIM", "1024")))
c.set("train.type", "negative_sampling")
c.set("train.loss", "kl")
c.set("negative_sampling.num_samples.s", int(os.environ.get("NS_NEG", "1024")))
if os.environ.get("KGE_NO_GRAPH") == "1":
    c.set("engine.graph_step", False)
c.set("negative_sampling.implementation", impl)
c.set("train.optimizer", "Adagrad")
c.set("train.optimizer_args", {"lr": 0.1})
c.set("train.batch_size", 512)
c.set("engine.row_sharded", "off")
c.set("verbose", False)
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
job = TrainingJob.create(c, ds)
job._prepare()
if os.environ.get("SORT_NEG") == "1":  # what would rows of ascending candidates buy?
    _sample = job._sampler.sample
    job._sampler.sample = lambda triples, slot: torch.sort(_sample(triples, slot), 1).values
B = 512
perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))
for i in range(5):
    job.train_step(i, job._collate(perm[i * B:(i + 1) * B]))
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(5, 5 + int(os.environ.get("NS_STEPS", "10"))):
    job.train_step(i, job._collate(perm[i * B:(i + 1) * B]))
torch.cuda.synchronize()
print(f"{model} negative_sampling {impl} step {(time.perf_counter() - t0) / int(os.environ.get('NS_STEPS', '10')) * 1e3:.3f} ms")
gs = getattr(job, "_graph_step", None)
print("graph step:", None if gs is None else ("recorded" if gs.graph is not None else f"not recorded: {gs.error}"))
