"""Does alternating consecutive score_sp batches between HIP streams raise throughput?

The C2 contraction runs 456 tiles on 256 workgroup slots: its second round leaves 56 CUs idle,
and the 5-us query preparation of the next batch waits behind it.  Batches are independent, so
a second stream lets the next batch's preparation and first tiles start on the idle CUs.

    python scripts/dev/two_stream.py [streams ...]      (default: 1 2 3)
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import Config, Dataset, KgeModel  # noqa: E402


def main():
    counts = [int(a) for a in sys.argv[1:]] or [1, 2, 3]
    E, R, B, d = 14541, 237, 1024, 512
    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cuda:0")
    c.set("lookup_embedder.dim", d)
    c.set("lookup_embedder.initialize", "normal_")
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("engine.row_sharded", "off")
    c.set("verbose", False)
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    torch.manual_seed(0)
    model = KgeModel.create(c, Dataset(c, None))
    model.eval()
    steps, warm = 200, 30
    s = torch.randint(0, E, (steps + warm, B), device="cuda:0")
    p = torch.randint(0, R, (steps + warm, B), device="cuda:0")
    with torch.no_grad():
        ref = [model.score_sp(s[i], p[i]).clone() for i in range(3)]
    for ns in counts:
        streams = [torch.cuda.Stream() for _ in range(ns)] if ns > 1 else [torch.cuda.current_stream()]
        for st in streams:
            st.wait_stream(torch.cuda.current_stream())

        def step(i):
            with torch.cuda.stream(streams[i % ns]), torch.no_grad():
                return model.score_sp(s[i], p[i])

        outs = [step(i) for i in range(3)]
        torch.cuda.synchronize()
        same = all(torch.equal(a, b) for a, b in zip(outs, ref))
        for rep in range(3):
            for i in range(warm):
                step(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                step(warm + i)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / steps * 1e6
            print(f"streams {ns} rep {rep}: {us:7.2f} us/step  {B * E / us * 1e6:.3e} triples/s  identical {same}",
                  flush=True)


if __name__ == "__main__":
    main()
