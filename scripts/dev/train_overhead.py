"""Dev probe: host (issue) time vs device time of the 1vsAll training step (C2 shape)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch
from kge import Config, Dataset
from kge.job import TrainingJob

model_name = sys.argv[1] if len(sys.argv) > 1 else "complex"
train_type = sys.argv[2] if len(sys.argv) > 2 else "1vsAll"
c = Config()
c.set("model", model_name); c._import(model_name)
c.set("job.device", "cuda")
c.set("lookup_embedder.dim", 512)
c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
c.set("train.type", train_type); c.set("train.optimizer", "Adagrad"); c.set("train.optimizer_args", {"lr": 0.2})
B = 1024 if train_type == "1vsAll" else 512
c.set("train.batch_size", B); c.set("verbose", False)
ds = Dataset.synthetic(c, "fb15k-237" if train_type == "1vsAll" else "wn18rr", seed=0)
job = TrainingJob.create(c, ds); job._prepare()
perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))
batches = [job._collate(perm[i * B:(i + 1) * B]) for i in range(60)]

def step(i, sync):
    r, _, _ = job.train_step(i, batches[i])
    if sync:
        float(r.avg_loss)

for sync in (False, True):
    for i in range(5): step(i, sync)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(5, 55): step(i, sync)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"sync={sync}: issue {(t1 - t0) / 50 * 1e3:.3f} ms/step, total {(t2 - t0) / 50 * 1e3:.3f} ms/step")
# host-side breakdown of one step
import cProfile, pstats
torch.cuda.synchronize()
pr = cProfile.Profile(); pr.enable()
for i in range(5, 25): step(i, False)
pr.disable(); torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
