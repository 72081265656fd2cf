"""Dev probe: C2 (ComplEx-512, 1vsAll, FB15K-237 shape, synthetic) through TrainingJob.run() with
validation every epoch -- the public job loop end to end with the default engine options."""
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
c.set("train.type", "1vsAll"); c.set("train.batch_size", 1024)
c.set("train.optimizer", "Adagrad"); c.set("train.optimizer_args", {"lr": 0.2})
c.set("train.max_epochs", int(sys.argv[1]) if len(sys.argv) > 1 else 3)
c.set("valid.every", 1); c.set("eval.batch_size", 1024)
c.set("verbose", False)
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
torch.manual_seed(0)
job = TrainingJob.create(c, ds)
t0 = time.perf_counter()
traces = job.run()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
for tr, v in zip(traces, job.valid_trace):
    print(f"epoch {tr['epoch']}: avg_loss {tr['avg_loss']:.4f} epoch_time {tr['epoch_time']:.3f}s "
          f"valid mrr_filt {v['mean_reciprocal_rank_filtered']:.5f} eval_time {v['epoch_time']:.3f}s")
print(f"total {dt:.2f}s; graph recorded: {job._graph_step is not None and job._graph_step.graph is not None}")
