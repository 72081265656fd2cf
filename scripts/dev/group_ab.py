"""Dev A/B in one process (libkgescore_dev.so; kge_dev_dot3_pipe 3 / kge_dev_bwdp_group 0 select the
in-turn order, the production kernels are the grouped ones): the three MFMAs of a band issued as three runs over
the accumulators with one fragment held per run ("grouped") against three per accumulator in turn,
for the forward contraction, the dQ and the dE GEMM at the stacked C2 training shape, and the
recorded 1vsAll job step with all three switched."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("KGE_LIBRARY", os.path.join(ROOT, "kge-1_amd", "csrc", "build_dev", "libkgescore_dev.so"))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import numpy as np, torch
from kge import Config, Dataset, _lib as L
from kge.job import TrainingJob

lib = L.lib()
n, m, d = 2048, 14541, 512
torch.manual_seed(0)
ent = (torch.randn(m, d) * 0.1).cuda(); q = (torch.randn(n, d) * 0.1).cuda()
labels = torch.randint(0, m, (n,)).cuda()
n_pad, ld = L.planes_layout(n, m)
S = torch.randn(n_pad, ld, device="cuda") * 0.01
bufp = S.clone()
_, gp = L.softmax_planes(bufp, n, m, labels, None, 0.0, 1.0 / n)
ldp = (d + 31) // 32 * 32
qh = torch.zeros(n_pad, ldp, device="cuda", dtype=torch.bfloat16); ql = torch.zeros_like(qh)
h, l = L.split_rows(q); qh[:n], ql[:n] = h, l
out = torch.empty(n, m, device="cuda"); dq = torch.empty(n, d, device="cuda"); de = torch.empty(m, d, device="cuda")


def sw(fwd, bwd):
    lib.kge_dev_dot3_pipe(fwd); lib.kge_dev_bwdp_group(bwd)


kern = {"forward": lambda: L.score_dot_split(h, l, ent, None, d, out=out),
        "dQ": lambda: L.score_dot_bwd_q_planes(gp, ent, dq=dq),
        "dE": lambda: L.score_dot_bwd_t_planes(gp, qh, ql, de)}
refs = {}
for name, fn in kern.items():
    sw(3, 0); fn(); torch.cuda.synchronize()
    a = {"forward": out, "dQ": dq, "dE": de}[name].clone()
    sw(1, 3); fn(); torch.cuda.synchronize()
    b = {"forward": out, "dQ": dq, "dE": de}[name]
    print(f"{name}: grouped == in-turn bitwise: {bool((a == b).all())}", flush=True)


def timeit(fn, reps=20):
    for _ in range(3): fn()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


res = {}
for r in range(5):
    for name, fn in kern.items():
        for tag, (f, b) in (("in turn", (3, 0)), ("grouped", (1, 3))):
            sw(f, b)
            res.setdefault((name, tag), []).append(timeit(fn))
for k, v in res.items():
    print(f"{k[0]:8s} {k[1]:8s} {np.median(v):7.1f} us (min {min(v):.1f})", flush=True)


def job_step(fwd, bwd, steps=40, warmup=6):
    sw(fwd, bwd)
    c = Config()
    c.set("model", "complex"); c._import("complex")
    c.set("job.device", "cuda"); c.set("lookup_embedder.dim", 512)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", "1vsAll"); c.set("train.optimizer", "Adagrad"); c.set("train.optimizer_args", {"lr": 0.2})
    c.set("train.batch_size", 1024); c.set("verbose", False)
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    job = TrainingJob.create(c, ds); job._prepare()
    perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))
    B = 1024
    for i in range(warmup):
        job.train_step(i, job._collate(perm[i * B:(i + 1) * B]))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        job.train_step(i, job._collate(perm[i * B:(i + 1) * B]))
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


for r in range(3):
    for tag, (f, b) in (("in turn", (3, 0)), ("grouped", (1, 3)), ("grouped fwd+dQ", (1, 1)), ("grouped fwd", (1, 0))):
        print(f"job step {tag}: {job_step(f, b):.4f} ms", flush=True)
