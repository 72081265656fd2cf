"""Dev A/B in one process: the recorded 1vsAll training step (C2 shape) with the software-pipelined
K loops of the forward / dQ kernels on and off (libkgescore_dev.so switches)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("KGE_LIBRARY", os.path.join(ROOT, "kge-1_amd", "csrc", "build_dev", "libkgescore_dev.so"))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch
from kge import Config, Dataset, _lib
from kge.job import TrainingJob

model = sys.argv[1] if len(sys.argv) > 1 else "complex"
ttype = sys.argv[2] if len(sys.argv) > 2 else "1vsAll"


_multi = _lib.adagrad_step_multi


def _single(items, eps, wd, maximize):  # one launch per tensor, as before the multi-tensor launch
    for p, g, s, c in items:
        _lib.adagrad_step(p, g, s, c, eps, wd, maximize)


def run(fwd, dq, stages=3, steps=30, warmup=6, multi=True):
    _lib.adagrad_step_multi = _multi if multi else _single
    _lib.lib().kge_dev_dot3_pipe(fwd)
    _lib.lib().kge_dev_bwdp_pipe(dq)
    _lib.lib().kge_dev_bwdp_stages(stages)
    c = Config()
    c.set("model", model); c._import(model)
    c.set("job.device", "cuda")
    c.set("lookup_embedder.dim", 512)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", ttype); c.set("train.optimizer", "Adagrad"); c.set("train.optimizer_args", {"lr": 0.2})
    B = 1024 if ttype == "1vsAll" else 512
    c.set("train.batch_size", B); c.set("verbose", False)
    ds = Dataset.synthetic(c, "fb15k-237" if ttype == "1vsAll" else "wn18rr", seed=0)
    job = TrainingJob.create(c, ds); job._prepare()
    perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))
    for i in range(warmup):
        job.train_step(i, job._collate(perm[i * B:(i + 1) * B]))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        job.train_step(i, job._collate(perm[i * B:(i + 1) * B]))
    torch.cuda.synchronize()
    print(f"{model} {ttype} forward pipe {fwd} dQ pipe {dq} dE stage buffers {stages} adagrad multi {multi}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/step", flush=True)


for _ in range(3):
    # forward: 0 = plain K loop, 1 = production, 2 = production loop with the XCD-after-XCD last round
    for fwd, dq, stages, multi in ((0, 0, 2, False), (2, 1, 3, True), (1, 1, 3, True)):
        run(fwd, dq, stages, multi=multi)
