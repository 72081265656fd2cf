"""1vsAll training step of the distance models at the C2 shape (FB15K-237, B = 1,024, dim 512):
forward all-entities distance kernel, fused CE, distance backward, Adagrad.

    python scripts/dev/dist_train_step.py [model[:dim[:precision]] ...]   (default: transe rotate, dim 512)
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import Config, Dataset  # noqa: E402
from kge.job import TrainingJob  # noqa: E402

B = 1024
for spec in (sys.argv[1:] or ["transe", "rotate"]):
    name, _, dim = spec.partition(":")
    dim, _, prec = dim.partition(":")
    c = Config()
    c.set("model", name)
    c._import(name)
    c.set("job.device", "cuda:0")
    c.set("lookup_embedder.dim", int(dim or 512))
    c.set("lookup_embedder.initialize", "normal_")
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("engine.row_sharded", "off")
    c.set("engine.precision", prec or "bf16x3")
    c.set("train.type", "1vsAll")
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.2})
    c.set("train.batch_size", B)
    c.set("verbose", False)
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    torch.manual_seed(0)
    job = TrainingJob.create(c, ds)
    job._prepare()
    train = ds.split("train")
    perm = torch.randperm(len(train), generator=torch.Generator().manual_seed(0))
    for i in range(4):
        job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 10
    for i in range(4, 4 + n):
        job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
    torch.cuda.synchronize()
    rec = job._graph_step is not None and job._graph_step.graph is not None
    print(f"{spec}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms/step (recorded {rec})", flush=True)
