"""End-to-end run of the jobs as a LibKGE user would configure them: ComplEx-512 1vsAll on the
synthetic FB15K-237 shape with embedder dropout, frequency-weighted Lp penalties,
ReduceLROnPlateau on the validation MRR and validation after every epoch.

    python scripts/dev/e2e_train.py [epochs] [eager]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import Config, Dataset  # noqa: E402
from kge.job import TrainingJob  # noqa: E402

epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
c = Config()
c.set("model", "complex")
c._import("complex")
c.set("job.device", "cuda:0")
c.set("lookup_embedder.dim", 512)
c.set("lookup_embedder.initialize", "normal_")
c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
c.set("lookup_embedder.dropout", 0.2)
c.set("lookup_embedder.regularize_args.weighted", True)
c.set("complex.entity_embedder.regularize_weight", 1e-6)
c.set("complex.relation_embedder.regularize_weight", 1e-6)
c.set("train.type", "1vsAll")
c.set("train.optimizer", "Adagrad")
c.set("train.optimizer_args", {"lr": 0.2})
c.set("train.lr_scheduler", "ReduceLROnPlateau")
c.set("train.lr_scheduler_args", {"mode": "max", "patience": 0, "factor": 0.5})
c.set("train.batch_size", 1024)
c.set("train.max_epochs", epochs)
c.set("valid.every", 1)
c.set("eval.batch_size", 1024)
c.set("engine.row_sharded", "off")
if len(sys.argv) > 2 and sys.argv[2] == "eager":
    c.set("engine.graph_step", False)
c.set("verbose", False)
ds = Dataset.synthetic(c, "fb15k-237", seed=0)
torch.manual_seed(0)
job = TrainingJob.create(c, ds)
t0 = time.perf_counter()
traces = job.run()
torch.cuda.synchronize()
total = time.perf_counter() - t0
for t, v in zip(traces, job.valid_trace):
    print(f"epoch {t['epoch']}: avg_loss {t['avg_loss']:.4f} avg_penalty {t['avg_penalty']:.3e} lr {t['lr'][0]:.4f} "
          f"epoch_time {t['epoch_time']:.3f}s ({t['batches']} batches, {t['epoch_time'] / t['batches'] * 1e3:.3f} ms each) "
          f"valid mrr_filt {v['mean_reciprocal_rank_filtered']:.5f} eval_time {v['epoch_time']:.3f}s", flush=True)
rec = job._graph_step is not None and job._graph_step.graph is not None
print(f"total {total:.2f}s, recorded step {rec}, peak memory {torch.cuda.max_memory_allocated() / 2**30:.2f} GiB", flush=True)
