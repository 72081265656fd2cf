"""Where an EntityRankingJob run spends its wall time: issuing the batch loop (host), the
device finishing it, and the metric arithmetic after it.

    python scripts/dev/eval_phases.py [streams] [head_and_tail 0|1] [fused_rank 0|1]

KGE_GRAPH_EVAL=1: the runs with engine.graph_eval (recorded device pass) timed as a whole -- the
phase marks synchronise inside the loop, which a recording cannot contain.
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
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    hat = bool(int(sys.argv[2])) if len(sys.argv) > 2 else False
    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda:0")
    c.set("lookup_embedder.dim", 512)
    c.set("lookup_embedder.initialize", "normal_")
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("engine.row_sharded", "off")
    c.set("engine.eval_streams", ns)
    c.set("verbose", False)
    c.set("eval.split", "test")
    c.set("eval.batch_size", int(os.environ.get("EVAL_BATCH", "1024")))
    if "ENGINE_EVAL_BATCH" in os.environ:
        c.set("engine.eval_batch_size", int(os.environ["ENGINE_EVAL_BATCH"]))
    c.set("entity_ranking.metrics_per.head_and_tail", hat)
    if len(sys.argv) > 3:
        c.set("engine.fused_rank", bool(int(sys.argv[3])))
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    torch.manual_seed(0)
    model = KgeModel.create(c, ds)
    model.eval()
    graph = os.environ.get("KGE_GRAPH_EVAL", "0") == "1"
    c.set("engine.graph_eval", graph)
    ej = EntityRankingJob(c, ds, model=model)
    ej._prepare()
    if graph:
        ts = []
        for _ in range(10):
            torch.cuda.synchronize()
            a = time.perf_counter()
            ej._run()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - a) * 1e3)
        print(f"group {ej._bs} graph_eval: runs {' '.join(f'{t:.3f}' for t in ts)} ms (first eager, second records); "
              f"median of the replays {np.median(ts[2:]):.3f} ms, recorded: {'graph' in ej._graph_state}", flush=True)
        return
    inner = ej._rank_batches
    marks = {}

    def timed(*a, **k):
        torch.cuda.synchronize()
        marks["t0"] = time.perf_counter()
        inner(*a, **k)
        marks["issued"] = time.perf_counter()
        torch.cuda.synchronize()
        marks["done"] = time.perf_counter()

    ej._rank_batches = timed
    inner_m = ej._compute_metrics_stacked

    def timed_m(*a, **k):
        t = time.perf_counter()
        r = inner_m(*a, **k)
        marks["metrics_fn"] = time.perf_counter() - t
        return r

    ej._compute_metrics_stacked = timed_m
    rows = []
    for _ in range(8):
        a = time.perf_counter()
        ej._run()
        torch.cuda.synchronize()
        b = time.perf_counter()
        rows.append(((marks["t0"] - a) * 1e3, (marks["issued"] - marks["t0"]) * 1e3,
                     (marks["done"] - marks["issued"]) * 1e3, (b - marks["done"]) * 1e3, marks["metrics_fn"] * 1e3))
    med = np.median(np.array(rows[1:]), axis=0)
    print(f"group {ej._bs} total {med[:4].sum():.3f} ms; streams {ns} head_and_tail {hat}: before loop {med[0]:.3f} ms, loop issued in {med[1]:.3f} ms, device "
          f"done {med[2]:.3f} ms later, metrics {med[3]:.3f} ms (of which the metric sums + copy {med[4]:.3f} ms)", flush=True)


if __name__ == "__main__":
    main()
