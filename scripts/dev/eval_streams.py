"""EntityRankingJob over the synthetic FB15K-237 test split (20,466 triples, batch 1,024) with
engine.eval_streams = 1, 2, 3: wall time per run and identical metrics.

    python scripts/dev/eval_streams.py [streams ...]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import Config, Dataset, KgeModel  # noqa: E402
from kge.job import EntityRankingJob  # noqa: E402


def main():
    counts = [int(a) for a in sys.argv[1:]] or [1, 2, 3]
    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda:0")
    c.set("lookup_embedder.dim", 512)
    c.set("lookup_embedder.initialize", "normal_")
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("engine.row_sharded", "off")
    c.set("verbose", False)
    c.set("eval.split", "test")
    c.set("eval.batch_size", 1024)
    c.set("entity_ranking.metrics_per.head_and_tail", True)
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    torch.manual_seed(0)
    model = KgeModel.create(c, ds)
    model.eval()
    first = None
    for ns in counts:
        c2 = c.clone()
        c2.set("engine.eval_streams", ns)
        ej = EntityRankingJob(c2, ds, model=model)
        ej._prepare()
        ej._run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            tr = ej._run()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        metrics = {k: v for k, v in tr.items() if k.startswith(("mean_", "hits_"))}
        if first is None:
            first = metrics
        print(f"streams {ns}: median {np.median(ts) * 1e3:.3f} ms  min {min(ts) * 1e3:.3f} ms  "
              f"metrics identical to the first: {metrics == first}  mrr_filt {tr['mean_reciprocal_rank_filtered']:.6f}",
              flush=True)


if __name__ == "__main__":
    main()
