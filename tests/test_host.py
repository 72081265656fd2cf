"""CPU tests of the host side: the C-ABI library loads and exports every declared symbol,
config / dataset / index logic, model construction, and the no-fallback contract."""
import json
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT


def test_library_exports_every_header_symbol():
    from kge import _lib

    header = open(os.path.join(ROOT, "include", "kgescore.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(kge_\w+)\s*\(", header, re.M))
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    lib = _lib.lib()
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.kge_version() >= 100
    # development probes (kge_dev_*, `make dev`) are not part of the product library
    import subprocess
    syms = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "kge_dev_" not in syms
    exported = {ln.split()[-1] for ln in syms.splitlines() if " T kge_" in ln}
    assert exported == declared, exported ^ declared
    assert lib.kge_error_string(1001).decode().startswith("kgescore: invalid argument")


def test_config_defaults_and_imports():
    from kge import Config

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    assert c.get_default("complex.entity_embedder.dim") == 100  # via lookup_embedder.dim
    c.set("lookup_embedder.dim", 512)
    assert c.get_default("complex.relation_embedder.dim") == 512
    c._import("rotate")
    assert c.get_default("rotate.relation_embedder.dim") == -1
    assert c.get_default("rotate.relation_embedder.initialize") == "uniform_"
    assert c.get("engine.precision") == "bf16x3"
    with pytest.raises(KeyError):
        c.get("no.such.key")
    with pytest.raises(ValueError):
        c.check("entity_ranking.tie_handling", ["best_rank"])


def test_config_set_rejects_unknown_keys_and_wrong_types():
    """Config.set with the reference's checks (config.py:144-236): a misspelt key raises
    instead of being stored and ignored; a value of another type raises."""
    from kge import Config

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    with pytest.raises(KeyError):
        c.set("trian.batch_size", 64)            # unknown at root level
    with pytest.raises(KeyError):
        c.set("train.batchsize", 64)             # unknown under an existing key
    with pytest.raises(ValueError):
        c.set("train.batch_size", "many")        # int expected
    with pytest.raises(ValueError):
        c.set("engine.fused_loss", 1)            # bool expected
    assert c.set("train.batch_size", "64") == 64  # numeric strings convert (CLI values)
    assert c.set("lookup_embedder.regularize_weight", 1) == 1.0  # int accepted for a float
    c.set("train.optimizer_args.lr", 0.5)        # "+++" dictionaries take new keys
    c.set("brand_new.key", 3, create=True)
    assert c.get("train.optimizer_args.lr") == 0.5 and c.get("brand_new.key") == 3
    assert c.get("engine.eval_precision") == "bf16x3_refined"


def test_model_dims_match_reference_shapes():
    from kge import Config, Dataset, KgeModel

    rows = json.loads(str(np.load(os.path.join(GOLDEN, "shapes.npz"))["table"]))
    for model, d, d_e, d_r in rows:
        c = Config()
        c.set("model", model)
        c._import(model)
        c.set("job.device", "cpu")
        c.set("dataset.num_entities", 10)
        c.set("dataset.num_relations", 3)
        c.set("lookup_embedder.dim", d)
        m = KgeModel.create(c, Dataset(c, None))
        assert m._entity_embedder.dim == d_e and m._relation_embedder.dim == d_r, model
        assert list(m.state_dict()) == ["_entity_embedder._embeddings.weight",
                                        "_relation_embedder._embeddings.weight"]


def test_scoring_on_cpu_raises_no_fallback():
    from kge import Config, Dataset, KgeModel
    from kge._lib import EngineError

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", "cpu")
    c.set("dataset.num_entities", 10)
    c.set("dataset.num_relations", 3)
    c.set("lookup_embedder.dim", 8)
    m = KgeModel.create(c, Dataset(c, None))
    with pytest.raises(EngineError):
        m.score_sp(torch.tensor([0, 1]), torch.tensor([0, 2]))


def test_dataset_loads_reference_fixture():
    from kge import Config, Dataset

    c = Config()
    ds = Dataset.create(c, folder=os.path.join(GOLDEN, "dataset_test"))
    assert ds.num_entities() == 4 and ds.num_relations() == 3
    assert ds.split("train").dtype == torch.int32
    assert [len(ds.split(s)) for s in ("train", "valid", "test")] == [4, 2, 2]
    idx = ds.index("train_sp_to_o")
    assert idx.get((0, 0)).tolist() == [1]
    assert idx.get((3, 3)).numel() == 0


def test_synthetic_fb15k237_shape_exact_and_unique():
    from kge import Config, Dataset

    ds = Dataset.synthetic(Config(), "fb15k-237", seed=0)
    sizes = [len(ds.split(s)) for s in ("train", "valid", "test")]
    assert sizes == [272115, 17535, 20466]
    allt = torch.cat([ds.split(s) for s in ("train", "valid", "test")]).long().numpy()
    code = (allt[:, 0] * 237 + allt[:, 1]) * 14541 + allt[:, 2]
    assert len(np.unique(code)) == len(code)
    assert allt[:, 0].max() < 14541 and allt[:, 1].max() < 237
    again = Dataset.synthetic(Config(), "fb15k-237", seed=0)
    assert torch.equal(again.split("test"), ds.split("test"))


def test_kvsall_index_csr_matches_dict():
    from kge.dataset import KvsAllIndex

    rng = np.random.default_rng(0)
    t = np.stack([rng.integers(0, 30, 500), rng.integers(0, 4, 500), rng.integers(0, 30, 500)], 1)
    idx = KvsAllIndex(t, (0, 1), 2)
    ref = {}
    for s, p, o in t.tolist():
        ref.setdefault((s, p), set()).add(o)
    q = np.stack([rng.integers(0, 32, 200), rng.integers(0, 5, 200)], 1)
    ptr, col = idx.csr_for(q)
    for i, (a, b) in enumerate(q.tolist()):
        assert sorted(col[ptr[i]:ptr[i + 1]].tolist()) == sorted(ref.get((a, b), set()))
        assert idx.get((a, b)).tolist() == sorted(ref.get((a, b), set()))


def test_csr_minus():
    from kge.job.entity_ranking import _csr_minus

    pa, ca = np.array([0, 3, 3, 5]), np.array([1, 2, 3, 7, 8])
    pb, cb = np.array([0, 1, 2, 3]), np.array([2, 9, 8])
    p, c = _csr_minus(pa, ca, pb, cb, 10)
    assert p.tolist() == [0, 2, 2, 3] and c.tolist() == [1, 3, 7]


def test_kvsall_batch_queries_host_csr():
    """TrainingJobKvsAll._queries (the batch's query pairs and label CSR, built on the host
    and shipped in one copy) against the answers of each query read from the triples."""
    from kge import Config, Dataset
    from kge.job import TrainingJob

    c = Config()
    c.set("model", "distmult")
    c._import("distmult")
    c.set("job.device", "cpu")
    c.set("lookup_embedder.dim", 8)
    c.set("train.type", "KvsAll")
    c.set("dataset.num_entities", 40)
    c.set("dataset.num_relations", 5)
    c.set("verbose", False)
    rng = np.random.default_rng(3)
    t = np.stack([rng.integers(0, 40, 400), rng.integers(0, 5, 400), rng.integers(0, 40, 400)], 1).astype(np.int32)
    ds = Dataset(c, None)
    ds._triples = {"train": torch.from_numpy(t)}
    job = TrainingJob.create(c, ds)
    job._prepare()
    answers = [{}, {}]
    for s, p, o in t.tolist():
        answers[0].setdefault((s, p), set()).add(o)
        answers[1].setdefault((p, o), set()).add(s)
    for qi in range(2):
        n_q = len(job.query_indexes[qi])
        sel = rng.choice(n_q, size=min(n_q, 37), replace=False)
        q, l_ptr, l_col = job._queries(qi, sel)
        assert q.shape == (len(sel), 2) and l_ptr.shape == (len(sel) + 1,) and int(l_ptr[0]) == 0
        for i in range(len(sel)):
            key = tuple(q[i].tolist())
            got = sorted(l_col[int(l_ptr[i]):int(l_ptr[i + 1])].tolist())
            assert got == sorted(answers[qi][key]), (qi, key)


def test_kvsall_batch_triples_and_weighted_penalty_vs_reference():
    """TrainingJobKvsAll._collate under a frequency-weighted penalty: the batch's true triples
    (one per query and label, train.py:625-674) equal the reference collate's, and the penalty
    terms of the first batch (lookup_embedder.py:112-158; plain torch, no engine) equal the
    reference's values -- in the unique-index form and in the per-occurrence form a recorded
    step uses."""
    import json
    import os

    from kge import Config, Dataset
    from kge.job import TrainingJob

    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "train_penalties.npz"))
    meta = json.loads(str(f["meta"]))
    case = meta["cases"]["kvsall_w"]
    c = Config()
    c.set("model", case["model"])
    c._import(case["model"])
    c.set("job.device", "cpu")
    c.set("lookup_embedder.dim", meta["dim"])
    c.set("train.type", "KvsAll")
    c.set("train.batch_size", case["batch_size"])
    c.set("dataset.num_entities", meta["E"])
    c.set("dataset.num_relations", meta["R"])
    c.set("verbose", False)
    for k, v in case["extra"].items():
        c.set(k, v)
    ds = Dataset(c, None)
    ds._triples = {"train": torch.from_numpy(f["tri_train"].astype(np.int32))}
    job = TrainingJob.create(c, ds)
    job._prepare()
    assert job._weighted_penalty()
    with torch.no_grad():
        job.model._entity_embedder._embeddings.weight.copy_(torch.from_numpy(f["kvsall_w_ent0"]))
        job.model._relation_embedder._embeddings.weight.copy_(torch.from_numpy(f["kvsall_w_rel0"]))
    for b in range(meta["num_batches"]):
        batch = job._collate(torch.from_numpy(f["kvsall_w_examples"][b]))
        np.testing.assert_array_equal(batch["triples"].numpy(), f[f"kvsall_w_triples_{b}"])
    batch = job._collate(torch.from_numpy(f["kvsall_w_examples"][0]))
    terms = job.model.penalty(epoch=1, batch_index=0, batch=batch)
    assert [k for k, _ in terms] == case["penalty_keys"]
    np.testing.assert_allclose([t.item() for _, t in terms], f["kvsall_w_penalties"][0], rtol=1e-6)
    # the per-occurrence form of the weighted term: the same sum without torch.unique
    emb = job.model._entity_embedder
    idx = batch["triples"][:, 0]
    occ = (0.05 / 3 * emb._embeddings.weight.index_select(0, idx).abs() ** 3).sum() / len(idx)
    assert occ.item() == pytest.approx(f["kvsall_w_penalties"][0][0], rel=1e-6)
    # no weighted penalty: the batch carries no triples (nothing reads them)
    c2 = c.clone()
    c2.set("lookup_embedder.regularize_args.weighted", False)
    job2 = TrainingJob.create(c2, ds)
    job2._prepare()
    assert "triples" not in job2._collate(torch.arange(5))


def test_dataset_relation_types_and_frequency_percentiles():
    """Dataset.index("relation_types" / "relations_per_type" / "frequency_percentiles") against the
    reference's own indexes (captured in eval_metrics_per.npz) and against the oracle's loops on a
    set with duplicate triples, an unused relation and unused entities."""
    import json

    from kge import Config, Dataset
    from oracle import kge_oracle as K

    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "eval_metrics_per.npz"))
    meta = json.loads(str(f["meta"]))

    def dataset(train, E, R):
        c = Config()
        c.set("dataset.num_entities", E)
        c.set("dataset.num_relations", R)
        ds = Dataset(c, None)
        ds._triples = {"train": torch.from_numpy(train.astype(np.int32))}
        return ds

    ds = dataset(f["tri_train"], meta["E"], meta["R"])
    assert ds.index("relation_types") == json.loads(str(f["relation_types"]))
    got = {a: {q: sorted(v) for q, v in d.items()} for a, d in ds.index("frequency_percentiles").items()}
    assert got == json.loads(str(f["frequency_percentiles"]))
    assert list(ds.index("relations_per_type")) == ["M-N", "1-N", "M-1", "1-1"]

    rng = np.random.default_rng(3)
    E, R = 57, 7
    t = np.stack([rng.integers(0, 50, 400), rng.integers(0, R - 1, 400), rng.integers(0, 9, 400)], 1)
    t = np.concatenate([t, t[:60]])  # duplicates count in both indexes
    ds = dataset(t, E, R)
    types = K.relation_types(t, R)
    assert ds.index("relation_types") == types and types[R - 1] == "1-1"
    assert ds.index("relations_per_type") == K.relations_per_type(types)
    assert ds.index("frequency_percentiles") == K.frequency_percentiles(t, E, R)


def test_bce_losses_on_cpu_vs_numpy():
    """bce / bce_mean / bce_self_adversarial (kge/util/loss.py:137-189) on a small score block with
    the positive in column 0, against the formulas written out in float64 numpy; the temperature
    comes from the user section of the configuration."""
    import numpy as np
    import torch

    from kge import Config
    from kge.util.loss import KgeLoss

    rng = np.random.default_rng(3)
    sc = rng.standard_normal((5, 7)).astype(np.float32) * 2
    labels = np.zeros((5, 7), np.float32)
    labels[:, 0] = 1.0
    x = sc.astype(np.float64) + 0.75
    bce = np.maximum(x, 0) - x * labels + np.log1p(np.exp(-np.abs(x)))
    pos, neg = bce[:, 0], bce[:, 1:]
    w = np.exp(x[:, 1:] * 0.5)
    w /= w.sum(1, keepdims=True)
    want = {"bce": bce.sum(), "bce_mean": (pos.sum() + neg.sum() / 6) / 2,
            "bce_self_adversarial": (pos.sum() + (w * neg).sum()) / 2}
    for name, ref in want.items():
        c = Config()
        c.set("train.type", "negative_sampling")
        c.set("train.loss", name)
        c.set("train.loss_arg", 0.75)
        c.set("user.bce_self_adversarial_temperature", 0.5)
        s = torch.from_numpy(sc).requires_grad_()
        got = KgeLoss.create(c)(s, torch.from_numpy(labels), num_negatives=6)
        assert float(got.detach()) == pytest.approx(float(ref), rel=1e-5), name
        got.backward()
        if name == "bce_self_adversarial":
            # the adversarial weights are constants of the backward pass
            sig = 1 / (1 + np.exp(-x))
            g = np.concatenate([(sig[:, :1] - 1), w * sig[:, 1:]], 1) / 2
            np.testing.assert_allclose(s.grad.numpy(), g, rtol=2e-5, atol=1e-7)
    # without the user option the temperature is 1
    c = Config()
    c.set("train.loss", "bce_self_adversarial")
    assert KgeLoss.create(c)._temperature == 1.0
