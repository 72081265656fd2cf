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

Fixtures written:

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
* ``shapes.npz`` -- F5: config-derived relation dims (RotatE d/2, RESCAL d^2);
* ``eval_fullsize_normal.npz`` -- F6: the reference EntityRankingJob at the FB15K-237 entity
  count (E = 14,541, R = 237, ComplEx-512, N(0, 0.1) tables regenerated from a recorded numpy
  seed -- the 30 MB tables themselves are not stored, a checksum is), 512 evaluation triples
  filtered against 30,000 training triples, with test filtering;
* ``train_kvsall_so_distmult.npz`` -- the same with (s, ?, o) relation queries enabled as well
  (three query types; label smoothing on entity targets only).
* ``train_kvsall_distmult.npz`` -- F7: three KvsAll batches (DistMult, sp_ and _po queries,
  label smoothing, KL, Adagrad) with the queries / labels of each batch, the per-batch loss
  the reference reports and the final tables;
* ``train_ns_<model>.npz`` -- F8: two negative-sampling batches (implementation "triple",
  KL) with the reference sampler's negatives recorded, so they can be injected;
* ``train_toy_complex.npz`` -- F9: the options of examples/toy-complex-train.yaml as the
  BASELINE config words them (1vsAll, dim 128, Adagrad 0.2, ReduceLROnPlateau, lp penalty
  0.8e-7, N(0, 0.1)) run through the reference's TrainingJob._run on a small synthetic
  dataset with the batch order recorded: per-epoch loss / penalty / lr and every validation;
* ``score_so.npz`` -- the "s_o" combine (KgeModel.score_so, all relations and a subset);
* ``eval_metrics_per.npz`` -- the reference EntityRankingJob with every entity_ranking.metrics_per
  option on (head_and_tail, relation_type, argument_frequency) over a synthetic dataset whose
  relations cover all four cardinality classes: every metric of the epoch trace, and the
  reference's relation_types / frequency_percentiles indexes.

* ``scorer_{rescal128,distmult512,transe_l1_512,rotate_l1_512}_<regime>.npz`` -- F1 / F2 at larger
  shapes (RESCAL d = 128; d = 512 over 640 entities: three 256-wide entity panels): tables from a
  recorded numpy seed, the reference's outputs and gradients stored;
* ``eval_rescal128_normal.npz`` -- the reference EntityRankingJob with RESCAL at d = 128;
* ``train1vsall_complex_large.npz`` -- three 1vsAll batches over 1,600 entities at d = 128, B = 300;
* ``train_toy_complex_epochs.npz`` -- written with the toy fixture: after every epoch of that run the
  tables and the validation ranks computed from them (teacher-forced validation checks).

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


# Larger shapes: tables regenerated by the tests from a recorded numpy seed (only the reference's
# OUTPUTS are stored).  d = 512 with E = 640 crosses the 256-wide tiles of the production kernels
# (three entity panels, a ragged last one); RESCAL at d = 128 has 16,384-wide relation rows.
LARGE_SCORER_CASES = [
    # name, model key, entity dim, extra config, E, R, n, m
    ("rescal128", "rescal", 128, {}, 200, 4, 16, 40),
    ("distmult512", "distmult", 512, {}, 640, 8, 24, 300),
    ("transe_l1_512", "transe", 512, {"transe.l_norm": 1.0}, 640, 8, 24, 300),
    ("rotate_l1_512", "rotate", 512, {"rotate.l_norm": 1.0}, 640, 8, 24, 300),
]


def seeded_scorer_tables(seed, regime, model_key, E, R, d_e, d_r):
    """Tables of a large scorer fixture from numpy's PCG64 stream: N(0, 0.1), or dyadic k / 8 with
    |k| <= 16; RotatE relations are phases U(-pi, pi) in both regimes."""
    rng = np.random.default_rng(seed)
    if regime == "normal":
        ent = (rng.standard_normal((E, d_e), dtype=np.float32) * np.float32(0.1)).astype(np.float32)
        rel = (rng.standard_normal((R, d_r), dtype=np.float32) * np.float32(0.1)).astype(np.float32)
    else:
        ent = (rng.integers(-16, 17, (E, d_e)) / 8.0).astype(np.float32)
        rel = (rng.integers(-16, 17, (R, d_r)) / 8.0).astype(np.float32)
    if model_key == "rotate":
        rel = ((rng.random((R, d_r)) * 2 - 1) * math.pi).astype(np.float32)
    return ent, rel


def gen_scorer_large(name, model_key, dim, extra, E, R, n, m, regime, seed):
    config = make_config(model_key, dim, E, R, extra)
    ds = Dataset(config, None)
    model = KgeModel.create(config, ds)
    d_e = model._entity_embedder.dim
    d_r = model._relation_embedder.dim
    ent, rel = seeded_scorer_tables(seed, regime, model_key, E, R, d_e, d_r)
    set_tables(model, torch.from_numpy(ent), torch.from_numpy(rel))
    gen = torch.Generator().manual_seed(seed)
    s = torch.randint(0, E, (n,), generator=gen)
    p = torch.randint(0, R, (n,), generator=gen)
    o = torch.randint(0, E, (n,), generator=gen)
    subset = torch.randperm(E, generator=gen)[:m]
    # dyadic weights keep the dyadic regime's gradients exact sums
    w_sp = dyadic(gen, (n, E)) if regime == "dyadic" else torch.randn(n, E, generator=gen)
    w_po = dyadic(gen, (n, E)) if regime == "dyadic" else torch.randn(n, E, generator=gen)
    w_spo = dyadic(gen, (n,)) if regime == "dyadic" else torch.randn(n, generator=gen)
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
    arrays = dict(
        s=s.numpy(), p=p.numpy(), o=o.numpy(), subset=subset.numpy(),
        spo=spo.detach().numpy(), sp_all=sp_all.detach().numpy(), po_all=po_all.detach().numpy(),
        sp_sub=sp_sub.numpy(), po_sub=po_sub.numpy(), sppo_sub=sppo_sub.numpy(),
        w_sp=w_sp.numpy(), w_po=w_po.numpy(), w_spo=w_spo.numpy(), g_ent=g_ent.numpy(), g_rel=g_rel.numpy(),
        meta=np.array(json.dumps(dict(
            model=model_key, name=name, regime=regime, seed=seed, table_seed=seed, E=E, R=R, d_e=d_e, d_r=d_r,
            l_norm=extra.get("transe.l_norm", extra.get("rotate.l_norm")),
            ent_checksum=table_checksum(ent), rel_checksum=table_checksum(rel),
            torch=torch.__version__, numpy=np.__version__))))
    fn = os.path.join(OUT, f"scorer_{name}_{regime}.npz")
    np.savez_compressed(fn, **arrays)
    return fn


def gen_eval_rescal128():
    """The reference's EntityRankingJob with RESCAL at d = 128 (relation rows of 16,384 floats)."""
    E, R, splits = make_dataset_splits(seed=21, E=200, R=4, n_train=1500, n_valid=100, n_test=100)
    folder = os.path.join(TMP, "ds_eval_rescal128")
    write_dataset(folder, E, R, splits)
    dim, seed = 128, 4100
    ent, rel = seeded_scorer_tables(seed, "normal", "rescal", E, R, dim, dim * dim)
    config = ds_config("rescal", dim, folder, E, R)
    ranks, metrics = run_eval(config, folder, torch.from_numpy(ent), torch.from_numpy(rel), -1, batch_size=32)
    out = {f"tri_{k}": v.astype(np.int32) for k, v in splits.items()}
    out.update({f"full_{k}": v for k, v in ranks.items()})
    out["metrics"] = np.array(json.dumps({"full": metrics}))
    out["meta"] = np.array(json.dumps(dict(
        E=E, R=R, dim=dim, model="rescal", eval_split="valid", filter_splits=["train", "valid"],
        filter_with_test=True, batch_size=32, tie_handling="rounded_mean_rank", table_seed=seed,
        ent_checksum=table_checksum(ent), rel_checksum=table_checksum(rel), torch=torch.__version__,
        numpy=np.__version__)))
    fn = os.path.join(OUT, "eval_rescal128_normal.npz")
    np.savez_compressed(fn, **out)
    return fn


def gen_train_fixture_large():
    """Three 1vsAll batches (ComplEx-128, Adagrad, kl) over 1,600 entities with batches of 300
    triples: the production kernels' tiles are multi-panel in every dimension (7 entity panels,
    two query tiles).  Tables from a recorded numpy seed; per-batch losses, the first batch's
    gradients and the final tables are stored."""
    from kge.job import TrainingJob

    E, R, dim, bs, nb = 1600, 12, 128, 300, 3
    rng = np.random.default_rng(31)
    allt = synth_triples_fast(rng, E, R, 6000)
    splits = dict(train=allt[:5000], valid=allt[5000:5500], test=allt[5500:])
    folder = os.path.join(TMP, "ds_train_large")
    write_dataset(folder, E, R, splits)
    config = ds_config("complex", dim, folder, E, R, {
        "train.type": "1vsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.2},
        "train.loss": "kl", "train.batch_size": bs})
    ds = Dataset.create(config, folder=folder)
    seed = 4200
    ent, rel = seeded_scorer_tables(seed, "normal", "complex", E, R, dim, dim)
    job = TrainingJob.create(config, ds)
    set_tables(job.model, torch.from_numpy(ent), torch.from_numpy(rel))
    job._prepare()
    gen = torch.Generator().manual_seed(32)
    perm = torch.randperm(len(splits["train"]), generator=gen)[:nb * bs]
    train = torch.from_numpy(splits["train"])
    losses, batches, g0 = [], [], None
    for b in range(nb):
        batch = train[perm[b * bs:(b + 1) * bs]].long()
        batches.append(batch.numpy())
        job.optimizer.zero_grad()
        res = job._process_batch(b, {"triples": batch})
        if b == 0:
            g0 = (job.model._entity_embedder._embeddings.weight.grad.clone().numpy(),
                  job.model._relation_embedder._embeddings.weight.grad.clone().numpy())
        job.optimizer.step()
        losses.append(res.avg_loss)
    fn = os.path.join(OUT, "train1vsall_complex_large.npz")
    np.savez_compressed(
        fn, batches=np.stack(batches).astype(np.int32), losses=np.array(losses, dtype=np.float64),
        g_ent_0=g0[0], g_rel_0=g0[1],
        ent1=job.model._entity_embedder._embeddings.weight.detach().numpy(),
        rel1=job.model._relation_embedder._embeddings.weight.detach().numpy(),
        meta=np.array(json.dumps(dict(E=E, R=R, dim=dim, lr=0.2, optimizer="Adagrad", loss="kl", batch_size=bs,
                                      table_seed=seed, ent_checksum=table_checksum(ent),
                                      rel_checksum=table_checksum(rel), torch=torch.__version__,
                                      numpy=np.__version__))))
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


def run_eval(config, folder, ent, rel, chunk_size, batch_size=64):
    from kge.job import EvaluationJob
    from kge.job.eval import hist_all

    config.set("entity_ranking.chunk_size", chunk_size)
    config.set("eval.batch_size", batch_size)
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


def gen_1vsall_bce_fixture():
    """Three 1vsAll batches with train.loss bce (BCEWithLogitsLoss(sum) against the one-hot label
    matrix the index labels turn into, loss.py:109-117, 137-158): ComplEx-32, Adagrad."""
    from kge.job import TrainingJob

    E, R, splits = make_dataset_splits()
    folder = os.path.join(TMP, "ds_train_bce")
    write_dataset(folder, E, R, splits)
    dim, bs, nb = 32, 128, 3
    config = ds_config("complex", dim, folder, E, R, {
        "train.type": "1vsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.2},
        "train.loss": "bce", "train.batch_size": bs})
    ds = Dataset.create(config, folder=folder)
    gen = torch.Generator().manual_seed(15)
    ent = torch.randn(E, dim, generator=gen) * 0.1
    rel = torch.randn(R, dim, generator=gen) * 0.1
    job = TrainingJob.create(config, ds)
    set_tables(job.model, ent, rel)
    job._prepare()
    perm = torch.randperm(len(splits["train"]), generator=gen)[:nb * bs]
    train = torch.from_numpy(splits["train"])
    losses, batches, g0 = [], [], None
    for b in range(nb):
        batch = train[perm[b * bs:(b + 1) * bs]].long()
        batches.append(batch.numpy())
        job.optimizer.zero_grad()
        res = job._process_batch(b, {"triples": batch})
        if b == 0:
            g0 = (job.model._entity_embedder._embeddings.weight.grad.clone().numpy(),
                  job.model._relation_embedder._embeddings.weight.grad.clone().numpy())
        job.optimizer.step()
        losses.append(res.avg_loss)
    fn = os.path.join(OUT, "train1vsall_bce_complex.npz")
    np.savez_compressed(
        fn, ent0=ent.numpy(), rel0=rel.numpy(), batches=np.stack(batches), losses=np.array(losses, dtype=np.float64),
        g_ent_0=g0[0], g_rel_0=g0[1],
        ent1=job.model._entity_embedder._embeddings.weight.detach().numpy(),
        rel1=job.model._relation_embedder._embeddings.weight.detach().numpy(),
        meta=np.array(json.dumps(dict(E=E, R=R, dim=dim, lr=0.2, optimizer="Adagrad", loss="bce", batch_size=bs,
                                      torch=torch.__version__))))
    return fn


def synth_triples_fast(rng, E, R, n):
    """Unique random triples, skewed entity distribution, vectorised (large E)."""
    w = 1.0 / np.arange(1, E + 1) ** 0.6
    cdf = np.cumsum(w / w.sum())
    uniq = np.zeros(0, np.int64)
    while len(uniq) < n:
        k = int((n - len(uniq)) * 1.3) + 1024
        s = np.minimum(np.searchsorted(cdf, rng.random(k)), E - 1)
        o = np.minimum(np.searchsorted(cdf, rng.random(k)), E - 1)
        p = rng.integers(0, R, k)
        code = (s * R + p) * E + o
        allc = np.concatenate([uniq, code])
        _, first = np.unique(allc, return_index=True)
        uniq = allc[np.sort(first)]
    uniq = uniq[:n]
    o = uniq % E
    sp = uniq // E
    return np.stack([sp // R, sp % R, o], 1).astype(np.int64)


def seeded_tables(seed, E, R, d_e, d_r, std=0.1):
    """N(0, std) tables from numpy's PCG64 stream (regenerated, not stored, by the tests)."""
    rng = np.random.default_rng(seed)
    ent = (rng.standard_normal((E, d_e), dtype=np.float32) * np.float32(std)).astype(np.float32)
    rel = (rng.standard_normal((R, d_r), dtype=np.float32) * np.float32(std)).astype(np.float32)
    return ent, rel


def table_checksum(x):
    return [float(x.astype(np.float64).sum()), float(np.abs(x.astype(np.float64)).sum()),
            float(x[0, 0]), float(x[-1, -1])]


def gen_eval_fullsize():
    E, R, dim = 14541, 237, 512
    n_train, n_valid, n_test = 30000, 512, 512
    rng = np.random.default_rng(3)
    allt = synth_triples_fast(rng, E, R, n_train + n_valid + n_test)
    splits = dict(train=allt[:n_train], valid=allt[n_train:n_train + n_valid], test=allt[n_train + n_valid:])
    folder = os.path.join(TMP, "ds_eval_fullsize")
    write_dataset(folder, E, R, splits)
    seed = 2024
    ent, rel = seeded_tables(seed, E, R, dim, dim)
    config = ds_config("complex", dim, folder, E, R)
    ranks, metrics = run_eval(config, folder, torch.from_numpy(ent), torch.from_numpy(rel), -1, batch_size=128)
    out = {f"tri_{k}": v.astype(np.int32) for k, v in splits.items()}
    out.update({f"full_{k}": v for k, v in ranks.items()})
    out["metrics"] = np.array(json.dumps({"full": metrics}))
    out["meta"] = np.array(json.dumps(dict(
        E=E, R=R, dim=dim, model="complex", eval_split="valid", filter_splits=["train", "valid"],
        filter_with_test=True, batch_size=128, tie_handling="rounded_mean_rank", table_seed=seed, std=0.1,
        ent_checksum=table_checksum(ent), rel_checksum=table_checksum(rel), torch=torch.__version__,
        numpy=np.__version__)))
    fn = os.path.join(OUT, "eval_fullsize_normal.npz")
    np.savez_compressed(fn, **out)
    return fn


def gen_kvsall_fixture(with_so=False, loss="kl", loss_arg=float("nan")):
    from kge.job import TrainingJob

    E, R, splits = make_dataset_splits()
    folder = os.path.join(TMP, "ds_kvsall")
    write_dataset(folder, E, R, splits)
    dim, bs, nb = 32, 64, 3
    config = ds_config("distmult", dim, folder, E, R, {
        "train.type": "KvsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.2},
        "train.loss": loss, "train.loss_arg": loss_arg, "train.batch_size": bs, "KvsAll.label_smoothing": 0.1,
        "KvsAll.query_types.s_o": with_so,
    })
    ds = Dataset.create(config, folder=folder)
    gen = torch.Generator().manual_seed(12)
    ent = torch.randn(E, dim, generator=gen) * 0.1
    rel = torch.randn(R, dim, generator=gen) * 0.1
    job = TrainingJob.create(config, ds)
    set_tables(job.model, ent, rel)
    job._prepare()
    collate = job._get_collate_fun()
    perm = torch.randperm(job.num_examples, generator=gen)[:nb * bs].tolist()
    out = dict(ent0=ent.numpy(), rel0=rel.numpy(), tri_train=splits["train"].astype(np.int32))
    losses = []
    for b in range(nb):
        batch = collate(perm[b * bs:(b + 1) * bs])
        out[f"queries_{b}"] = batch["queries"].numpy()
        out[f"qtype_{b}"] = batch["query_type_indexes"].numpy()
        out[f"label_coords_{b}"] = batch["label_coords"].numpy()
        out[f"triples_{b}"] = batch["triples"].numpy()  # what weighted penalties count on
        # tables before the batch and the gradients its backward leaves (before the step)
        out[f"ent_before_{b}"] = job.model._entity_embedder._embeddings.weight.detach().clone().numpy()
        out[f"rel_before_{b}"] = job.model._relation_embedder._embeddings.weight.detach().clone().numpy()
        job.optimizer.zero_grad()
        res = job._process_batch(b, batch)
        out[f"g_ent_{b}"] = job.model._entity_embedder._embeddings.weight.grad.detach().clone().numpy()
        out[f"g_rel_{b}"] = job.model._relation_embedder._embeddings.weight.grad.detach().clone().numpy()
        job.optimizer.step()
        losses.append(res.avg_loss)
    out["losses"] = np.array(losses, dtype=np.float64)
    out["ent1"] = job.model._entity_embedder._embeddings.weight.detach().numpy()
    out["rel1"] = job.model._relation_embedder._embeddings.weight.detach().numpy()
    out["meta"] = np.array(json.dumps(dict(
        E=E, R=R, dim=dim, model="distmult", lr=0.2, optimizer="Adagrad", loss=loss,
        loss_arg=None if math.isnan(loss_arg) else loss_arg, batch_size=bs,
        label_smoothing=0.1, query_types=job.query_types, num_batches=nb, torch=torch.__version__)))
    tag = "" if loss == "kl" else "_" + loss
    fn = os.path.join(OUT, f"train_kvsall{'_so' if with_so else ''}{tag}_distmult.npz")
    np.savez_compressed(fn, **out)
    return fn


def gen_ns_fixture(model_key, loss="kl", loss_arg=float("nan"), extra=None, tag="", nneg=8):
    from kge.job import TrainingJob

    E, R, splits = make_dataset_splits()
    folder = os.path.join(TMP, f"ds_ns_{model_key}")
    write_dataset(folder, E, R, splits)
    dim, bs, nb = 32, 64, 2
    config = ds_config(model_key, dim, folder, E, R, {
        "train.type": "negative_sampling", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.1},
        "train.loss": loss, "train.loss_arg": loss_arg, "train.batch_size": bs,
        "negative_sampling.num_samples.s": nneg,
        "negative_sampling.num_samples.o": -1, "negative_sampling.num_samples.p": 0,
        "negative_sampling.implementation": "triple", "negative_sampling.filtering.implementation": "standard",
    })
    for k, v in (extra or {}).items():
        config.set(k, v, create=True)
    ds = Dataset.create(config, folder=folder)
    gen = torch.Generator().manual_seed(13)
    job = TrainingJob.create(config, ds)
    d_e, d_r = job.model._entity_embedder.dim, job.model._relation_embedder.dim
    ent = torch.randn(E, d_e, generator=gen) * 0.1
    rel = torch.randn(R, d_r, generator=gen) * 0.1
    if model_key == "rotate":
        rel = (torch.rand(R, d_r, generator=gen) * 2 - 1) * math.pi
    set_tables(job.model, ent, rel)
    job._prepare()
    collate = job._get_collate_fun()
    torch.manual_seed(99)  # the reference sampler draws from torch's global stream
    perm = torch.randperm(job.num_examples, generator=gen)[:nb * bs].tolist()
    out = dict(ent0=ent.numpy(), rel0=rel.numpy(), tri_train=splits["train"].astype(np.int32))
    losses = []
    for b in range(nb):
        batch = collate(perm[b * bs:(b + 1) * bs])
        out[f"triples_{b}"] = batch["triples"].numpy()
        out[f"neg_s_{b}"] = batch["negative_samples"][0].numpy()
        out[f"neg_o_{b}"] = batch["negative_samples"][2].numpy()
        # tables before the batch and the gradients its backward leaves (before the step)
        out[f"ent_before_{b}"] = job.model._entity_embedder._embeddings.weight.detach().clone().numpy()
        out[f"rel_before_{b}"] = job.model._relation_embedder._embeddings.weight.detach().clone().numpy()
        job.optimizer.zero_grad()
        res = job._process_batch(b, batch)
        for key, emb in (("g_ent", job.model._entity_embedder), ("g_rel", job.model._relation_embedder)):
            g = emb._embeddings.weight.grad.detach()
            out[f"{key}_{b}"] = (g.to_dense() if g.is_sparse else g).clone().numpy()  # lookup_embedder.sparse
        job.optimizer.step()
        losses.append(res.avg_loss)
    out["losses"] = np.array(losses, dtype=np.float64)
    out["ent1"] = job.model._entity_embedder._embeddings.weight.detach().numpy()
    out["rel1"] = job.model._relation_embedder._embeddings.weight.detach().numpy()
    out["meta"] = np.array(json.dumps(dict(
        E=E, R=R, dim=dim, d_e=d_e, d_r=d_r, model=model_key, lr=0.1, optimizer="Adagrad", loss=loss,
        loss_arg=None if math.isnan(loss_arg) else loss_arg, batch_size=bs, num_negatives=nneg, implementation="triple", num_batches=nb,
        l_norm=config.get(model_key + ".l_norm") if model_key in ("rotate", "transe") else None,
        extra=extra or {}, torch=torch.__version__)))
    fn = os.path.join(OUT, f"train_ns_{model_key}{'' if loss == 'kl' else '_' + loss}{tag}.npz")
    np.savez_compressed(fn, **out)
    return fn


class _FixedLoader:
    """Stands in for the reference job's shuffling DataLoader: yields the batches of one
    recorded permutation per epoch (the reference iterates `self.loader` and calls len())."""

    def __init__(self, triples, perms, batch_size):
        self.triples, self.perms, self.bs, self.epoch = triples, perms, batch_size, 0

    def __len__(self):
        return math.ceil(self.perms.shape[1] / self.bs)

    def __iter__(self):
        perm = self.perms[self.epoch]
        self.epoch += 1
        for b in range(0, len(perm), self.bs):
            yield {"triples": self.triples[perm[b:b + self.bs], :].long()}


def gen_toy_fixture():
    from kge.job import TrainingJob

    E, R, splits = make_dataset_splits(seed=5, E=400, R=10, n_train=2000, n_valid=200, n_test=200)
    folder = os.path.join(TMP, "ds_toy")
    write_dataset(folder, E, R, splits)
    dim, bs, epochs = 128, 100, 6
    config = ds_config("complex", dim, folder, E, R, {
        # examples/toy-complex-train.yaml, with train.type / dim as BASELINE configs[0] words them
        "train.type": "1vsAll", "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.2},
        "train.lr_scheduler": "ReduceLROnPlateau",
        "train.lr_scheduler_args": {"mode": "max", "patience": 0, "factor": 0.5},
        "lookup_embedder.regularize_weight": 0.8e-7,
        "lookup_embedder.initialize": "normal_",
        "train.batch_size": bs, "train.max_epochs": epochs, "valid.every": 1,
        "train.checkpoint.every": 0, "valid.early_stopping.patience": 0,
    })
    config.set("lookup_embedder.initialize_args.normal_.mean", 0.0)
    config.set("lookup_embedder.initialize_args.normal_.std", 0.1)
    ds = Dataset.create(config, folder=folder)
    gen = torch.Generator().manual_seed(14)
    ent = torch.randn(E, dim, generator=gen) * 0.1
    rel = torch.randn(R, dim, generator=gen) * 0.1
    job = TrainingJob.create(config, ds)
    set_tables(job.model, ent, rel)
    job._prepare()
    job._is_prepared = True
    n = job.num_examples
    perms = np.stack([torch.randperm(n, generator=gen).numpy() for _ in range(epochs)])
    job.loader = _FixedLoader(ds.split("train"), perms, bs)
    epoch_traces, valid_traces = [], []
    job.post_epoch_hooks.append(lambda j, t: epoch_traces.append(dict(t)))
    job.post_valid_hooks.append(lambda j, t: valid_traces.append(dict(t)))
    # per epoch: the tables the validation ranks were computed from, and those ranks
    epoch_tables, epoch_ranks = [], []

    def keep_tables(j, t):
        epoch_tables.append((j.model._entity_embedder._embeddings.weight.detach().clone().numpy(),
                             j.model._relation_embedder._embeddings.weight.detach().clone().numpy()))

    job.post_epoch_hooks.append(keep_tables)
    from kge.job.eval import hist_all

    def keep_ranks(hists, s, p, o, s_ranks, o_ranks, job, **kwargs):
        epoch_ranks.append((s_ranks.clone().numpy(), o_ranks.clone().numpy()))
        return hist_all(hists, s, p, o, s_ranks, o_ranks, job, **kwargs)

    job.valid_job.hist_hooks = [keep_ranks]
    job.run()
    # the hook runs per validation batch for every ranking in turn (raw, filt, filt_test)
    nrk = 3 if job.valid_job.filter_with_test else 2
    per_epoch = len(epoch_ranks) // epochs
    assert per_epoch * epochs == len(epoch_ranks) and per_epoch % nrk == 0
    extra = {}
    for e in range(epochs):
        chunk = epoch_ranks[e * per_epoch:(e + 1) * per_epoch]
        for ri, rname in enumerate(("raw", "filt", "filt_test")[:nrk]):
            extra[f"s_{rname}_{e}"] = np.concatenate([c[0] for c in chunk[ri::nrk]])
            extra[f"o_{rname}_{e}"] = np.concatenate([c[1] for c in chunk[ri::nrk]])
        extra[f"ent_{e}"], extra[f"rel_{e}"] = epoch_tables[e]
    np.savez_compressed(os.path.join(OUT, "train_toy_complex_epochs.npz"), **extra,
                        meta=np.array(json.dumps(dict(epochs=epochs, rankings=nrk, torch=torch.__version__))))
    keep_e = ("epoch", "avg_loss", "avg_penalty", "avg_cost", "lr", "batches", "size")
    ep = [{k: t[k] for k in keep_e} for t in epoch_traces]
    va = [{k: v for k, v in t.items() if isinstance(v, (int, float)) and ("rank" in k or "hits" in k or k == "epoch")}
          for t in valid_traces]
    fn = os.path.join(OUT, "train_toy_complex.npz")
    np.savez_compressed(
        fn, ent0=ent.numpy(), rel0=rel.numpy(), perms=perms.astype(np.int32),
        **{f"tri_{k}": v.astype(np.int32) for k, v in splits.items()},
        ent1=job.model._entity_embedder._embeddings.weight.detach().numpy(),
        rel1=job.model._relation_embedder._embeddings.weight.detach().numpy(),
        epochs=np.array(json.dumps(ep)), valids=np.array(json.dumps(va)),
        final_lr=np.array([g["lr"] for g in job.optimizer.param_groups]),
        meta=np.array(json.dumps(dict(
            E=E, R=R, dim=dim, model="complex", train_type="1vsAll", lr=0.2, optimizer="Adagrad",
            lr_scheduler="ReduceLROnPlateau", lr_scheduler_args={"mode": "max", "patience": 0, "factor": 0.5},
            regularize_weight=0.8e-7, batch_size=bs, max_epochs=epochs, valid_every=1,
            valid_metric=config.get("valid.metric"), eval_batch_size=config.get("eval.batch_size"),
            torch=torch.__version__))))
    return fn


def gen_score_so_fixture():
    out = {}
    names = []
    for name, key, dim, extra in [("complex", "complex", 32, {}), ("distmult", "distmult", 32, {}),
                                  ("transe_l1", "transe", 32, {"transe.l_norm": 1.0}),
                                  ("rotate_l1", "rotate", 32, {"rotate.l_norm": 1.0})]:
        E, R, n, m = 40, 9, 12, 5
        config = make_config(key, dim, E, R, extra)
        model = KgeModel.create(config, Dataset(config, None))
        d_e, d_r = model._entity_embedder.dim, model._relation_embedder.dim
        gen = torch.Generator().manual_seed(31 + len(names))
        ent = torch.randn(E, d_e, generator=gen) * 0.1
        rel = torch.randn(R, d_r, generator=gen) * 0.1
        if key == "rotate":
            rel = (torch.rand(R, d_r, generator=gen) * 2 - 1) * math.pi
        set_tables(model, ent, rel)
        s = torch.randint(0, E, (n,), generator=gen)
        o = torch.randint(0, E, (n,), generator=gen)
        psub = torch.randperm(R, generator=gen)[:m]
        with torch.no_grad():
            so_all = model.score_so(s, o)
            so_sub = model.score_so(s, o, psub)
        for k, v in dict(ent=ent, rel=rel, s=s, o=o, psub=psub, so_all=so_all, so_sub=so_sub).items():
            out[f"{name}_{k}"] = v.numpy()
        names.append(dict(name=name, model=key, d_e=d_e, d_r=d_r,
                          l_norm=extra.get("transe.l_norm", extra.get("rotate.l_norm"))))
    out["meta"] = np.array(json.dumps(dict(cases=names, torch=torch.__version__)))
    fn = os.path.join(OUT, "score_so.npz")
    np.savez_compressed(fn, **out)
    return fn


def typed_triples(rng, E, R, n):
    """Unique triples whose relations differ in cardinality: relation r draws its subjects from
    the first ns[r % 4] entities and its objects from the first no[r % 4] (few subjects and many
    objects gives 1-N, and so on), and relation ids are skewed so that frequencies differ."""
    ns = (12, E, 40, E)
    no = (E, 12, 40, E)
    wr = 1.0 / np.arange(1, R + 1) ** 0.8
    wr /= wr.sum()
    seen, out = set(), []
    while len(out) < n:
        p = int(rng.choice(R, p=wr))
        s = int(rng.integers(ns[p % 4]))
        o = int(rng.integers(no[p % 4]))
        if (s, p, o) not in seen:
            seen.add((s, p, o))
            out.append((s, p, o))
    return np.array(out, dtype=np.int64)


def gen_eval_metrics_per():
    from kge.job import EvaluationJob

    E, R, dim = 300, 12, 32
    rng = np.random.default_rng(11)
    allt = typed_triples(rng, E, R, 3300)
    splits = dict(train=allt[:3000], valid=allt[3000:3150], test=allt[3150:])
    folder = os.path.join(TMP, "ds_eval_metrics_per")
    write_dataset(folder, E, R, splits)
    gen = torch.Generator().manual_seed(13)
    ent = torch.randn(E, dim, generator=gen) * 0.1
    rel = torch.randn(R, dim, generator=gen) * 0.1
    config = ds_config("complex", dim, folder, E, R)
    config.set("eval.batch_size", 64)
    config.set("eval.split", "valid")
    config.set("entity_ranking.filter_splits", ["train", "valid"])
    config.set("entity_ranking.filter_with_test", True)
    for k in ("head_and_tail", "relation_type", "argument_frequency"):
        config.set("entity_ranking.metrics_per." + k, True)
    ds = Dataset.create(config, folder=folder)
    model = KgeModel.create(config, ds)
    set_tables(model, ent, rel)
    job = EvaluationJob.create(config, ds, model=model)
    trace = job.run()
    metrics = {k: v for k, v in trace.items() if isinstance(v, (int, float)) and ("rank" in k or "hits" in k)}
    ds.index("frequency_percentiles")
    percs = {arg: {perc: sorted(int(i) for i in ids) for perc, ids in d.items()}
             for arg, d in ds._indexes["frequency_percentiles"].items()}
    out = dict(ent=ent.numpy(), rel=rel.numpy(), **{f"tri_{k}": v for k, v in splits.items()},
               metrics=np.array(json.dumps(metrics)), metric_order=np.array(json.dumps(list(metrics))),
               relation_types=np.array(json.dumps(list(ds.index("relation_types")))),
               frequency_percentiles=np.array(json.dumps(percs)),
               meta=np.array(json.dumps(dict(
                   E=E, R=R, dim=dim, model="complex", eval_split="valid", filter_splits=["train", "valid"],
                   filter_with_test=True, batch_size=64, tie_handling="rounded_mean_rank",
                   torch=torch.__version__))))
    fn = os.path.join(OUT, "eval_metrics_per.npz")
    np.savez_compressed(fn, **out)
    return fn


def gen_penalty_fixture():
    """Three batch steps of the reference's batch loop (train.py:309-429) WITH embedding
    penalties: weighted L3 on the entities and weighted L2 on the relations (lookup_embedder.py:
    112-158 -- the weights come from the batch's triples, which KvsAll builds per label,
    train.py:625-674), for 1vsAll (ComplEx) and KvsAll (DistMult); plus an unweighted L2 run of
    1vsAll.  Per batch: the loss, every penalty term, and the tables after the steps."""
    from kge.job import TrainingJob

    E, R, splits = make_dataset_splits()
    out = dict(tri_train=splits["train"].astype(np.int32))
    cases = [("1vsall_w", "complex", "1vsAll", True, 128), ("kvsall_w", "distmult", "KvsAll", True, 64),
             ("1vsall_u", "complex", "1vsAll", False, 128)]
    dim, nb = 32, 3
    meta = dict(E=E, R=R, dim=dim, num_batches=nb, lr=0.2, cases={}, torch=torch.__version__)
    for tag, model, ttype, weighted, bs in cases:
        folder = os.path.join(TMP, "ds_pen_" + tag)
        write_dataset(folder, E, R, splits)
        extra = {"train.type": ttype, "train.optimizer": "Adagrad", "train.optimizer_args": {"lr": 0.2},
                 "train.loss": "kl", "train.batch_size": bs,
                 "lookup_embedder.regularize": "lp", "lookup_embedder.regularize_args.weighted": weighted,
                 f"{model}.entity_embedder.regularize_weight": 0.05,
                 f"{model}.relation_embedder.regularize_weight": 0.02,
                 f"{model}.entity_embedder.regularize_args.p": 3,
                 f"{model}.relation_embedder.regularize_args.p": 2}
        config = ds_config(model, dim, folder, E, R, extra)
        ds = Dataset.create(config, folder=folder)
        gen = torch.Generator().manual_seed(21)
        ent = torch.randn(E, dim, generator=gen) * 0.1
        rel = torch.randn(R, dim, generator=gen) * 0.1
        job = TrainingJob.create(config, ds)
        set_tables(job.model, ent, rel)
        job._prepare()
        out[f"{tag}_ent0"], out[f"{tag}_rel0"] = ent.numpy(), rel.numpy()
        losses, pens = [], []
        if ttype == "1vsAll":
            perm = torch.randperm(len(splits["train"]), generator=gen)[:nb * bs]
            train = torch.from_numpy(splits["train"])
            batches = [{"triples": train[perm[b * bs:(b + 1) * bs]].long()} for b in range(nb)]
            out[f"{tag}_batches"] = np.stack([b["triples"].numpy() for b in batches])
        else:
            collate = job._get_collate_fun()
            perm = torch.randperm(job.num_examples, generator=gen)[:nb * bs].tolist()
            batches = [collate(perm[b * bs:(b + 1) * bs]) for b in range(nb)]
            out[f"{tag}_examples"] = np.array(perm, dtype=np.int64).reshape(nb, bs)
            for b, batch in enumerate(batches):
                out[f"{tag}_triples_{b}"] = batch["triples"].numpy()
        keys = None
        for b, batch in enumerate(batches):
            job.optimizer.zero_grad()
            res = job._process_batch(b, batch)
            terms = job.model.penalty(epoch=1, batch_index=b, num_batches=nb, batch=batch)
            for _, t in terms:
                t.backward()
            keys = [k for k, _ in terms]
            pens.append([t.item() for _, t in terms])
            out[f"{tag}_g_ent_{b}"] = job.model._entity_embedder._embeddings.weight.grad.detach().clone().numpy()
            out[f"{tag}_g_rel_{b}"] = job.model._relation_embedder._embeddings.weight.grad.detach().clone().numpy()
            job.optimizer.step()
            losses.append(res.avg_loss)
        out[f"{tag}_losses"] = np.array(losses, dtype=np.float64)
        out[f"{tag}_penalties"] = np.array(pens, dtype=np.float64)
        out[f"{tag}_ent1"] = job.model._entity_embedder._embeddings.weight.detach().numpy()
        out[f"{tag}_rel1"] = job.model._relation_embedder._embeddings.weight.detach().numpy()
        meta["cases"][tag] = dict(model=model, train_type=ttype, weighted=weighted, batch_size=bs,
                                  penalty_keys=keys, extra={k: v for k, v in extra.items() if "regular" in k})
    out["meta"] = np.array(json.dumps(meta))
    fn = os.path.join(OUT, "train_penalties.npz")
    np.savez_compressed(fn, **out)
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
    extra = {"eval_fullsize": gen_eval_fullsize, "kvsall": gen_kvsall_fixture,
             "kvsall_so": lambda: gen_kvsall_fixture(with_so=True),
             "ns_rotate": lambda: gen_ns_fixture("rotate"), "ns_complex": lambda: gen_ns_fixture("complex"),
             "toy": gen_toy_fixture, "score_so": gen_score_so_fixture, "eval_metrics_per": gen_eval_metrics_per,
             "kvsall_bce": lambda: gen_kvsall_fixture(loss="bce", loss_arg=0.5),
             "ns_complex_margin": lambda: gen_ns_fixture("complex", "margin_ranking", 2.0),
             "ns_rotate_bce": lambda: gen_ns_fixture("rotate", "bce", -3.0),
             "ns_transe_bce_self_adv": lambda: gen_ns_fixture("transe", "bce_self_adversarial", 6.0,
                                                              {"user.bce_self_adversarial_temperature": 0.5}),
             "ns_distmult_bce_mean": lambda: gen_ns_fixture("distmult", "bce_mean", 0.5),
             "ns_complex_soft_margin": lambda: gen_ns_fixture("complex", "soft_margin"),
             "ns_simple_se": lambda: gen_ns_fixture("simple", "se"),
             "ns_complex_sparse": lambda: gen_ns_fixture("complex", extra={"lookup_embedder.sparse": True},
                                                         tag="_sparse"),
             # 128 negatives per slot: candidate lists long enough for the engine to order them
             "ns_rotate_n128": lambda: gen_ns_fixture("rotate", tag="_n128", nneg=128),
             "ns_complex_n128": lambda: gen_ns_fixture("complex", tag="_n128", nneg=128),
             "ns_transe_n128": lambda: gen_ns_fixture("transe", tag="_n128", nneg=128),
             "onevsall_bce": gen_1vsall_bce_fixture,
             "penalties": gen_penalty_fixture, "eval_rescal128": gen_eval_rescal128,
             "train_large": gen_train_fixture_large}
    seed = 3000
    for name, key, dim, cfg, E, R, n, m in LARGE_SCORER_CASES:
        for regime in ("normal", "dyadic"):
            seed += 1
            if key == "rotate" and regime == "dyadic":
                continue  # cos / sin of the phases leave nothing exact: the normal regime says it all
            if only is None or name in only:
                written.append(gen_scorer_large(name, key, dim, cfg, E, R, n, m, regime, seed))
    for name, fn in extra.items():
        if only is None or name in only:
            written.append(fn())
    shutil.rmtree(TMP, ignore_errors=True)
    for fn in written:
        print(os.path.relpath(fn, OUT), os.path.getsize(fn))


if __name__ == "__main__":
    main()
