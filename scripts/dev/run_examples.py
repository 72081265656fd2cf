"""The reference's runnable training examples (examples/toy-complex-train.yaml,
toy-complex-train-sampling.yaml, toy-transe-train.yaml) with this package's jobs on the small
dataset the reference's tests ship (tests/golden/dataset_test), a few epochs each.

    python scripts/dev/run_examples.py [epochs]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import Config, Dataset  # noqa: E402
from kge.job import TrainingJob  # noqa: E402

EXAMPLES = {
    "toy-complex-train": {
        "model": "complex", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.2},
        "train.lr_scheduler": "ReduceLROnPlateau", "train.lr_scheduler_args": {"mode": "max", "patience": 4},
        "lookup_embedder.dim": 100, "lookup_embedder.regularize_weight": 0.8e-7,
        "lookup_embedder.initialize": "normal_", "lookup_embedder.initialize_args": {"normal_": {"mean": 0.0, "std": 0.1}},
    },
    "toy-complex-train-sampling": {
        "model": "complex", "train.type": "negative_sampling", "train.optimizer": "Adagrad",
        "train.optimizer_args": {"lr": 0.6, "weight_decay": 0.4e-7}, "train.loss": "margin_ranking",
        "train.loss_arg": 2.0, "train.batch_size": 512, "lookup_embedder.dim": 100,
        "negative_sampling.num_samples.s": 30, "negative_sampling.num_samples.p": 30,
        "negative_sampling.num_samples.o": -1, "negative_sampling.filtering.s": True,
        "negative_sampling.filtering.o": True, "negative_sampling.filtering.p": True,
    },
    "toy-transe-train": {
        "model": "transe", "train.batch_size": 256, "train.loss": "margin_ranking", "train.loss_arg": 4.0,
        "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.1}, "train.type": "negative_sampling",
    },
}


def main():
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    folder = os.path.join(ROOT, "tests", "golden", "dataset_test")
    for name, opts in EXAMPLES.items():
        c = Config()
        c.set("model", opts["model"])
        c._import(opts["model"])
        c.set("job.device", "cuda:0")
        c.set("verbose", False)
        c.set("train.max_epochs", epochs)
        c.set("valid.every", 1)
        for k, v in opts.items():
            if k != "model":
                c.set(k, v)
        ds = Dataset.create(c, folder=folder)
        torch.manual_seed(0)
        job = TrainingJob.create(c, ds)
        t0 = time.perf_counter()
        traces = job.run()
        torch.cuda.synchronize()
        print(f"{name}: {len(traces)} epochs in {time.perf_counter() - t0:.2f}s; avg_cost "
              + " -> ".join(f"{t['avg_cost']:.4f}" for t in traces) + "; valid mrr_filt "
              + " -> ".join(f"{v['mean_reciprocal_rank_filtered']:.4f}" for v in job.valid_trace), flush=True)
        assert all(t["avg_cost"] == t["avg_cost"] for t in traces)


if __name__ == "__main__":
    main()
