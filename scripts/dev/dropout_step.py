import os, sys, time, torch
sys.path.insert(0, "/root/repo/kge-1_amd")
from kge import Config, Dataset
from kge.job import TrainingJob
B = 1024
for drop in ([float(a) for a in sys.argv[1:]] or [0.0, 0.2]):
    c = Config(); c.set("model", "complex"); c._import("complex")
    c.set("job.device", "cuda:0"); c.set("lookup_embedder.dim", 512)
    c.set("lookup_embedder.initialize", "normal_"); c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("lookup_embedder.dropout", drop)
    c.set("engine.row_sharded", "off"); c.set("train.type", "1vsAll"); c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.2}); c.set("train.batch_size", B); c.set("verbose", False)
    ds = Dataset.synthetic(c, "fb15k-237", seed=0)
    torch.manual_seed(0)
    job = TrainingJob.create(c, ds); job._prepare()
    train = ds.split("train"); perm = torch.randperm(len(train), generator=torch.Generator().manual_seed(0))
    for i in range(6): job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(6, 36): job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
    torch.cuda.synchronize()
    print(f"dropout {drop}: {(time.perf_counter() - t0) / 30 * 1e3:.3f} ms/step, graph {job._graph_step is not None and job._graph_step.graph is not None}", flush=True)
