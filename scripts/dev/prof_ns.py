"""C4: RotatE-1024 negative sampling (1024 negatives per slot, s and o), FB15K-237 shape,
B=512 -- step timing (and a target for rocprofv3)."""
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
c = Config()
c.set("model", "rotate")
c._import("rotate")
c.set("job.device", "cuda")
c.set("lookup_embedder.dim", 1024)
c.set("train.type", "negative_sampling")
c.set("train.loss", "kl")
c.set("negative_sampling.num_samples.s", 1024)
c.set("negative_sampling.implementation", impl)
c.set("train.optimizer", "Adagrad")
c.set("train.optimizer_args", {"lr": 0.1})
c.set("train.batch_size", 512)
c.set("verbose", False)
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
job = TrainingJob.create(c, ds)
job._prepare()
B = 512
perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))


def step(i):
    return job.train_step(i, job._collate(perm[i * B:(i + 1) * B]))[0]


for i in range(5):
    step(i)
torch.cuda.synchronize()
t0 = time.perf_counter()
n = 20
for i in range(5, 5 + n):
    r = step(i)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n
print(f"rotate-1024 NS({impl}) B={B} N=1024: step {dt * 1e3:.3f} ms  "
      f"{2 * B * 1025 / dt / 1e6:.1f} M scored triples/s  loss {r.avg_loss:.4f}")
