"""Golden-vector generator for the scoring hot path.  BUILD-CONTAINER ONLY.

This script is test infrastructure: it imports the *reference* LibKGE from the
read-only checkout at /root/reference (never shipped, never present on the GPU box),
runs the reference's own code on small seeded inputs, and writes the inputs and the
reference's outputs as ``.npz`` fixtures next to this file.  Only data is written; no
reference source text is copied.  The committed fixtures are what ``tests/`` and the
oracle are pinned against.

Import shims.  The reference imports four things this image lacks
or that changed in Python 3.10; none of them is on the scoring path:

* ``numba`` -- ``njit`` becomes the identity (used by kge/indexing.py:304-317 and
  kge/util/sampler.py:289-315 only);
* ``path`` -- ``Path`` becomes a chdir context manager (kge/misc.py:22,38, git hash);
* ``ax*`` -- empty modules (kge/job/ax_search.py:3-9 only);
* ``collections.Mapping`` -- aliased to ``collections.abc.Mapping`` (kge/config.py:56).

Fixtures written (see tests/golden/README.md for the schema):

* ``scorer_<model>_<regime>.npz`` -- F1: embedding tables, index vectors and the
  outputs of score_spo / score_sp / score_po / score_sp_po (all and subset) for
  ComplEx, DistMult, RESCAL, TransE (L1, L2), RotatE (L1, L2), CP and SimplE, in the N(0, 0.1) and
  the dyadic (k/8, |k| <= 16) value regimes, plus F2 gradients of a weighted sum of
  the outputs w.r.t. both tables;
* ``eval_<regime>.npz`` -- F3: a synthetic dataset, a ComplEx model and the per-query
  ranks (raw / filtered / filtered-with-test) and all metrics of the reference
  EntityRankingJob, unchunked and with entity_ranking.chunk_size = ceil(E / 8);
* ``train1vsall_complex.npz`` -- F4: three 1vsAll batches (sp + po, KL/CE, Adagrad)
  with per-batch losses and the final tables;
* ``shapes.npz`` -- F5: config-derived relation dims (RotatE d/2, RESCAL d^2).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [case,case,...]
"""
import collections
import collections.abc
import contextlib
import json
import math
import os
import shutil
import sys
import tempfile
import types

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
import torch  # noqa: E402  (must be imported before the shims)

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_shims():
    nb = types.ModuleType("numba")
    nb.njit = lambda *a, **k: a[0] if a and callable(a[0]) else (lambda f: f)
    sys.modules["numba"] = nb

    pm = types.ModuleType("path")

    @contextlib.contextmanager
    def _path(p):
        old = os.getcwd()
        os.chdir(p)
        try:
            yield
        finally:
            os.chdir(old)

    pm.Path = _path
    sys.modules["path"] = pm

    class _Dummy:
        def __getattr__(self, n):
            if n.startswith("__"):
                raise AttributeError(n)
            return _Dummy()

        def __call__(self, *a, **k):
            return _Dummy()

    for name in [
        "ax",
        "ax.core",
        "ax.modelbridge",
        "ax.modelbridge.generation_strategy",
        "ax.service",
        "ax.service.ax_client",
    ]:
        m = types.ModuleType(name)

        def _ga(n):
            if n.startswith("__"):
                raise AttributeError(n)
            return _Dummy()

        m.__getattr__ = _ga
        sys.modules[name] = m
    collections.Mapping = collections.abc.Mapping
    sys.path.insert(0, REF)


_install_shims()
import kge  # noqa: E402
from kge import Config, Dataset  # noqa: E402
from kge.model import KgeModel  # noqa: E402

TMP = tempfile.mkdtemp(prefix="kge-golden-")


def make_config(model, dim, num_entities, num_relations, extra=None):
    config = Config()
    config.folder = TMP
    config.set("verbose", False)
    config.set("model", model)
    config._import(model)
    config.set("job.device", "cpu")
    config.set("dataset.name", "synthetic")
    config.set("dataset.num_entities", num_entities)
    config.set("dataset.num_relations", num_relations)
    config.set("dataset.pickle", False)
    config.set("lookup_embedder.dim", dim)
    for k, v in (extra or {}).items():
        config.set(k, v)
    return config


def dyadic(gen, shape):
    """Values k/8, k in [-16, 16]: every fp32 product and sum below is exact."""
    k = torch.randint(-16, 17, shape, generator=gen)
    return k.float() / 8.0


def set_tables(model, ent, rel):
    with torch.no_grad():
        model._entity_embedder._embeddings.weight.copy_(ent)
        model._relation_embedder._embeddings.weight.copy_(rel)


SCORER_CASES = [
    # name, model key, entity dim, extra config
    ("complex", "complex", 64, {}),
    ("complex512", "complex", 512, {}),
    ("distmult", "distmult", 64, {}),
    ("rescal", "rescal", 16, {}),
    ("transe_l1", "transe", 64, {"transe.l_norm": 1.0}),
    ("transe_l2", "transe", 64, {"transe.l_norm": 2.0}),
    ("rotate_l1", "rotate", 64, {"rotate.l_norm": 1.0}),
    ("rotate_l2", "rotate", 64, {"rotate.l_norm": 2.0}),
    ("cp", "cp", 64, {}),
    ("simple", "simple", 64, {}),
]


def gen_scorer_fixture(name, model_key, dim, extra, regime, seed):
    E, R, n, m = (128, 16, 32, 40) if name == "complex512" else (64, 8, 16, 20)
    config = make_config(model_key, dim, E, R, extra)
    ds = Dataset(config, None)
    model = KgeModel.create(config, ds)
    d_e = model._entity_embedder.dim
    d_r = model._relation_embedder.dim
    gen = torch.Generator().manual_seed(seed)
    if regime == "normal":
        ent = torch.randn(E, d_e, generator=gen) * 0.1
        rel = torch.randn(R, d_r, generator=gen) * 0.1
    else:
        ent = dyadic(gen, (E, d_e))
        rel = dyadic(gen, (R, d_r))
    if model_key == "rotate":  # relations are phases: U(-pi, pi) (rotate.yaml:20-24)
        rel = (torch.rand(R, d_r, generator=gen) * 2 - 1) * math.pi
    set_tables(model, ent, rel)
    s = torch.randint(0, E, (n,), generator=gen)
    p = torch.randint(0, R, (n,), generator=gen)
    o = torch.randint(0, E, (n,), generator=gen)
    subset = torch.randperm(E, generator=gen)[:m]
    w_sp = torch.randn(n, E, generator=gen)
    w_po = torch.randn(n, E, generator=gen)
    w_spo = torch.randn(n, generator=gen)

    model.train()
    spo = model.score_spo(s, p, o)
    sp_all = model.score_sp(s, p)
    po_all = model.score_po(p, o)
    loss = (w_sp * sp_all).sum() + (w_po * po_all).sum() + (w_spo * spo).sum()
    model.zero_grad()
    loss.backward()
    g_ent = model._entity_embedder._embeddings.weight.grad.clone()
    g_rel = model._relation_embedder._embeddings.weight.grad.clone()
    with torch.no_grad():
        sp_sub = model.score_sp(s, p, subset)
        po_sub = model.score_po(p, o, subset)
        sppo_sub = model.score_sp_po(s, p, o, subset)
        sppo_all = model.score_sp_po(s, p, o)
    arrays = dict(
        ent=ent.numpy(), rel=rel.numpy(),
        s=s.numpy(), p=p.numpy(), o=o.numpy(), subset=subset.numpy(),
        spo=spo.detach().numpy(), sp_all=sp_all.detach().numpy(),
        po_all=po_all.detach().numpy(), sp_sub=sp_sub.numpy(), po_sub=po_sub.numpy(),
        sppo_sub=sppo_sub.numpy(), sppo_all=sppo_all.numpy(),
        w_sp=w_sp.numpy(), w_po=w_po.numpy(), w_spo=w_spo.numpy(),
        g_ent=g_ent.numpy(), g_rel=g_rel.numpy(),
        meta=np.array(json.dumps(dict(
            model=model_key, name=name, regime=regime, seed=seed, d_e=d_e, d_r=d_r,
            l_norm=extra.get("transe.l_norm", extra.get("rotate.l_norm")),
            torch=torch.__version__))),
    )
    fn = os.path.join(OUT, f"scorer_{name}_{regime}.npz")
    np.savez_compressed(fn, **arrays)
    return fn


# -- synthetic dataset for eval / training fixtures ---------------------------------


def synth_triples(rng, E, R, n):
    """Unique random triples with a skewed entity distribution (so filters matter)."""
    seen = set()
    out = []
    w = 1.0 / np.arange(1, E + 1) ** 0.6
    w /= w.sum()
    while len(out) < n:
        s = int(rng.choice(E, p=w))
        o = int(rng.choice(E, p=w))
        p = int(rng.integers(R))
        if (s, p, o) not in seen:
            seen.add((s, p, o))
            out.append((s, p, o))
    return np.array(out, dtype=np.int64)


def write_dataset(folder, E, R, splits):
    os.makedirs(folder, exist_ok=True)
    for name, t in splits.items():
        np.savetxt(os.path.join(folder, f"{name}.del"), t, fmt="%d", delimiter="\t")
    with open(os.path.join(folder, "entity_ids.del"), "w") as f:
        for i in range(E):
            f.write(f"{i}\te{i}\n")
    with open(os.path.join(folder, "relation_ids.del"), "w") as f:
        for i in range(R):
            f.write(f"{i}\tr{i}\n")


def make_dataset_splits(seed=0, E=300, R=12, n_train=3000, n_valid=150, n_test=150):
    rng = np.random.default_rng(seed)
    allt = synth_triples(rng, E, R, n_train + n_valid + n_test)
    return E, R, dict(
        train=allt[:n_train],
        valid=allt[n_train:n_train + n_valid],
        test=allt[n_train + n_valid:],
    )


def ds_config(model, dim, folder, E, R, extra=None):
    config = make_config(model, dim, E, R, extra)
    config.set("dataset.num_entities", -1)
    config.set("dataset.num_relations", -1)
    return config


def run_eval(config, folder, ent, rel, chunk_size):
    from kge.job import EvaluationJob
    from kge.job.eval import hist_all

    config.set("entity_ranking.chunk_size", chunk_size)
    config.set("eval.batch_size", 64)
    config.set("eval.split", "valid")
    config.set("entity_ranking.filter_splits", ["train", "valid"])
    config.set("entity_ranking.filter_with_test", True)
    ds = Dataset.create(config, folder=folder)
    model = KgeModel.create(config, ds)
    set_tables(model, ent, rel)
    job = EvaluationJob.create(config, ds, model=model)
    captured = []

    def capture(hists, s, p, o, s_ranks, o_ranks, job, **kwargs):
        captured.append((s_ranks.clone().numpy(), o_ranks.clone().numpy()))
        return hist_all(hists, s, p, o, s_ranks, o_ranks, job, **kwargs)

    job.hist_hooks = [capture]
    trace = job.run()
    # per batch the hook runs for _raw, _filt, _filt_test in that order
    raw_s, raw_o, f_s, f_o, ft_s, ft_o = [], [], [], [], [], []
    for i in range(0, len(captured), 3):
        raw_s.append(captured[i][0]); raw_o.append(captured[i][1])
        f_s.append(captured[i + 1][0]); f_o.append(captured[i + 1][1])
        ft_s.append(captured[i + 2][0]); ft_o.append(captured[i + 2][1])
    ranks = dict(
        s_raw=np.concatenate(raw_s), o_raw=np.concatenate(raw_o),
        s_filt=np.concatenate(f_s), o_filt=np.concatenate(f_o),
        s_filt_test=np.concatenate(ft_s), o_filt_test=np.concatenate(ft_o),
    )
    metrics = {k: v for k, v in trace.items() if isinstance(v, (int, float))
               and ("rank" in k or "hits" in k)}
    return ranks, metrics


def gen_eval_fixture(regime):
    E, R, splits = make_dataset_splits()
    folder = os.path.join(TMP, f"ds_eval_{regime}")
    write_dataset(folder, E, R, splits)
    dim = 32
    gen = torch.Generator().manual_seed(7)
    if regime == "dyadic":
        ent = dyadic(gen, (E, dim)) / 4  # small range -> many exact ties
        rel = dyadic(gen, (R, dim)) / 4
    else:
        ent = torch.randn(E, dim, generator=gen) * 0.1
        rel = torch.randn(R, dim, generator=gen) * 0.1
    out = dict(ent=ent.numpy(), rel=rel.numpy(), **{f"tri_{k}": v for k, v in splits.items()})
    metrics_all = {}
    for tag, chunk in [("full", -1), ("chunk8", math.ceil(E / 8))]:
        config = ds_config("complex", dim, folder, E, R)
        ranks, metrics = run_eval(config, folder, ent, rel, chunk)
        for k, v in ranks.items():
            out[f"{tag}_{k}"] = v
        metrics_all[tag] = metrics
    out["metrics"] = np.array(json.dumps(metrics_all))
    out["meta"] = np.array(json.dumps(dict(
        E=E, R=R, dim=dim, model="complex", eval_split="valid",
        filter_splits=["train", "valid"], filter_with_test=True, batch_size=64,
        tie_handling="rounded_mean_rank", chunk8=math.ceil(E / 8),
        torch=torch.__version__)))
    fn = os.path.join(OUT, f"eval_{regime}.npz")
    np.savez_compressed(fn, **out)
    return fn


def gen_train_fixture():
    from kge.job import TrainingJob

    E, R, splits = make_dataset_splits()
    folder = os.path.join(TMP, "ds_train")
    write_dataset(folder, E, R, splits)
    dim = 32
    config = ds_config("complex", dim, folder, E, R, {
        "train.type": "1vsAll", "train.optimizer": "Adagrad",
        "train.optimizer_args": {"lr": 0.2}, "train.loss": "kl",
        "train.batch_size": 128,
    })
    ds = Dataset.create(config, folder=folder)
    gen = torch.Generator().manual_seed(11)
    ent = torch.randn(E, dim, generator=gen) * 0.1
    rel = torch.randn(R, dim, generator=gen) * 0.1
    job = TrainingJob.create(config, ds)
    set_tables(job.model, ent, rel)
    job._prepare()
    perm = torch.randperm(len(splits["train"]), generator=gen)[:3 * 128]
    train = torch.from_numpy(splits["train"])
    losses, batches = [], []
    for b in range(3):
        batch = train[perm[b * 128:(b + 1) * 128]].long()
        batches.append(batch.numpy())
        job.optimizer.zero_grad()
        res = job._process_batch(b, {"triples": batch})
        job.optimizer.step()
        losses.append(res.avg_loss)
    fn = os.path.join(OUT, "train1vsall_complex.npz")
    np.savez_compressed(
        fn, ent0=ent.numpy(), rel0=rel.numpy(), batches=np.stack(batches),
        losses=np.array(losses, dtype=np.float64),
        ent1=job.model._entity_embedder._embeddings.weight.detach().numpy(),
        rel1=job.model._relation_embedder._embeddings.weight.detach().numpy(),
        meta=np.array(json.dumps(dict(E=E, R=R, dim=dim, lr=0.2, optimizer="Adagrad",
                                      loss="kl", batch_size=128,
                                      torch=torch.__version__))))
    return fn


def gen_shapes():
    rows = []
    for model, d in [("rotate", 64), ("rotate", 1024), ("rescal", 16), ("rescal", 32),
                     ("complex", 512), ("distmult", 512), ("transe", 128)]:
        config = make_config(model, d, 10, 3)
        m = KgeModel.create(config, Dataset(config, None))
        rows.append((model, d, m._entity_embedder.dim, m._relation_embedder.dim))
    fn = os.path.join(OUT, "shapes.npz")
    np.savez(fn, table=np.array(json.dumps(rows)))
    return fn


def main():
    # optional argv: names of the scorer cases to (re)generate; nothing else is rewritten
    only = set(sys.argv[1].split(",")) if len(sys.argv) > 1 else None
    torch.set_num_threads(4)
    written = []
    seed = 1000
    for name, key, dim, extra in SCORER_CASES:
        for regime in ("normal", "dyadic"):
            seed += 1
            if only is None or name in only:
                written.append(gen_scorer_fixture(name, key, dim, extra, regime, seed))
    if only is None:
        for regime in ("dyadic", "normal"):
            written.append(gen_eval_fixture(regime))
        written.append(gen_train_fixture())
        written.append(gen_shapes())
    shutil.rmtree(TMP, ignore_errors=True)
    for fn in written:
        print(os.path.relpath(fn, OUT), os.path.getsize(fn))


if __name__ == "__main__":
    main()
