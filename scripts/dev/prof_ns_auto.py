"""C4 (RotatE-1024, 1,024 negatives per slot, B = 512) under negative_sampling.implementation
auto / batch: a few steps for a kernel trace (rocprofv3 --kernel-trace --stats -- python3 this)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import Config, Dataset  # noqa: E402
from kge.job import TrainingJob  # noqa: E402

impl = sys.argv[1] if len(sys.argv) > 1 else "auto"
c = Config()
c.set("model", "rotate")
c._import("rotate")
c.set("job.device", "cuda:0")
c.set("lookup_embedder.dim", 1024)
c.set("train.type", "negative_sampling")
c.set("train.loss", "kl")
c.set("negative_sampling.num_samples.s", 1024)
c.set("negative_sampling.implementation", impl)
c.set("train.optimizer", "Adagrad")
c.set("train.optimizer_args", {"lr": 0.1})
c.set("train.batch_size", 512)
c.set("engine.row_sharded", "off")
c.set("verbose", False)
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
torch.manual_seed(0)
job = TrainingJob.create(c, ds)
job._prepare()
perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))
for i in range(6):
    job.train_step(i, job._collate(perm[i * 512:(i + 1) * 512]))
torch.cuda.synchronize()
print("done", job._implementation)
