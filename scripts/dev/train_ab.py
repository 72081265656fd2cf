"""Dev A/B: the bench's 1vsAll training step (C2 shape, job.train_step), eager vs recorded
HIP graph, in one process."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch
from kge import Config, Dataset
from kge.job import TrainingJob

def run(graph, steps=20, warmup=4):
    c = Config()
    c.set("model", "complex"); c._import("complex")
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 512)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", "1vsAll"); c.set("train.optimizer", "Adagrad"); c.set("train.optimizer_args", {"lr": 0.2})
    B = 1024
    c.set("train.batch_size", B); c.set("verbose", False); c.set("engine.graph_step", graph)
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    job = TrainingJob.create(c, ds); job._prepare()
    train = ds.split("train")
    perm = torch.randperm(len(train), generator=torch.Generator().manual_seed(0))
    def tstep(i):
        job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
    for i in range(warmup):
        tstep(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tstep(warmup + i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    gs = job._graph_step
    print(f"graph={graph}: issue {(t1 - t0) / steps * 1e3:.3f} ms total {(t2 - t0) / steps * 1e3:.3f} ms/step "
          f"recorded={gs is not None and gs.graph is not None} err={None if gs is None else gs.error}", flush=True)

for g in (False, True, False, True):
    run(g)
