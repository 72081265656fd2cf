"""C2 1vsAll training step (ComplEx-512, FB15K-237 shape, B = 1,024) WITH frequency-weighted Lp
penalties on both embedders: the recorded step against the eager one.

    python scripts/dev/penalty_step.py
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import Config, Dataset  # noqa: E402
from kge.job import TrainingJob  # noqa: E402


def main():
    B = 1024
    for weighted in (True, False):
        for graph in (True, False):
            c = Config()
            c.set("model", "complex")
            c._import("complex")
            c.set("job.device", "cuda:0")
            c.set("lookup_embedder.dim", 512)
            c.set("lookup_embedder.initialize", "normal_")
            c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
            c.set("lookup_embedder.regularize_args.weighted", weighted)
            c.set("complex.entity_embedder.regularize_weight", 1e-5)
            c.set("complex.relation_embedder.regularize_weight", 1e-5)
            c.set("complex.entity_embedder.regularize_args.p", 3)
            c.set("engine.graph_step", graph)
            c.set("engine.row_sharded", "off")
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
            for i in range(6):
                job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 40
            for i in range(6, 6 + n):
                _, pen, _ = job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / n * 1e3
            rec = job._graph_step is not None and job._graph_step.graph is not None
            print(f"weighted {weighted!s:5} graph_step {graph!s:5} (recorded {rec!s:5}): {ms:.3f} ms/step, "
                  f"penalty {float(pen):.4e}", flush=True)


if __name__ == "__main__":
    main()
