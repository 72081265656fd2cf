"""Dev probe: the recorded 1vsAll step (C2 shape) -- replay alone, pinned copy + replay, and
job.train_step, each 50x without host syncs."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch
from kge import Config, Dataset
from kge.job import TrainingJob

c = Config()
c.set("model", "complex"); c._import("complex")
c.set("job.device", "cuda")
c.set("lookup_embedder.dim", 512)
c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
c.set("train.type", "1vsAll"); c.set("train.optimizer", "Adagrad"); c.set("train.optimizer_args", {"lr": 0.2})
B = 1024
c.set("train.batch_size", B); c.set("verbose", False)
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
job = TrainingJob.create(c, ds); job._prepare()
train = ds.split("train")
perm = torch.randperm(len(train), generator=torch.Generator().manual_seed(0))
batches = [{"triples": train[perm[i * B:(i + 1) * B]].long()} for i in range(120)]
for i in range(6):
    job.train_step(i, batches[i])
gs = job._graph_step
torch.cuda.synchronize()

def timeit(name, fn, n=50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name}: issue {(t1 - t0) / n * 1e3:.3f} ms, total {(t2 - t0) / n * 1e3:.3f} ms per step", flush=True)

timeit("replay only", lambda i: gs.graph.replay())
timeit("dma copy(pinned)+replay", lambda i: (gs.static.copy_(gs.pinned[0][0], non_blocking=True), gs.graph.replay()))
from kge import _lib
timeit("kernel stage(pinned)+replay", lambda i: (_lib.stage_i64(gs.pinned[0][0], gs.static), gs.graph.replay()))
timeit("train_step", lambda i: job.train_step(10 + i, batches[10 + i]))
timeit("train_step", lambda i: job.train_step(60 + i, batches[60 + i]))
timeit("replay only", lambda i: gs.graph.replay())
