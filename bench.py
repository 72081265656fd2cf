#!/usr/bin/env python
"""Headline benchmark: 1vsAll scoring throughput, ComplEx-512 on FB15K-237 (synthetic,
published shape), batch 1024 -- BASELINE.json configs[1] at N=1.

A step is one pass of the hot path over one batch of 1024 fresh (s, p) queries:
KgeModel.score_sp(s, p) -> fused LookupEmbedder gather + ComplEx query prep + the
all-entities contraction against the 14,541-row entity table (libkgescore, gfx950).
value = scored triples / s = (queries x entities) / step time, all ranks.

N > 1 (torchrun, one process per GPU): the scored triples are partitioned by query -- every
rank scores its own 1024 queries against the entity table, replicated at setup -- so the
step has no data-path collective and per-GPU work is constant (weak scaling).  The
entity-row-sharded exchange over RCCL (kge.sharded: query rows all_gathered, global batch
scored against each rank's shard) is timed after the headline loop and reported as
"row_sharded", together with the cost of its all_gather alone.

Also reported (rank 0): the contraction kernel's roofline from HIP events on the launch stream
(100 back-to-back launches after the timed region), score_po, a full 1vsAll training step
(sp + po forward/backward + CE + Adagrad), the filtered eval MRR on the synthetic test
split, and the reference CPU path (oracle/refseq.py: the reference's exact ATen op
sequence, verified bit-exact against it) timed on this host's cores.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
BF16_DENSE_TFLOPS = 2500.0  # dense bf16 MFMA (spec, no sparsity)
FP32_MFMA_TFLOPS = 157.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--dataset", default="fb15k-237")
    ap.add_argument("--precision", default="bf16x3", choices=["bf16x3", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--c5", action="store_true", help="also time one rank's Wikidata5M shard (configs[4])")
    return ap.parse_args()


def make_config(args, device):
    from kge import Config

    c = Config()
    c.set("model", "complex")
    c._import("complex")
    c.set("job.device", device)
    c.set("lookup_embedder.dim", args.dim)
    c.set("lookup_embedder.initialize", "normal_")
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})  # examples/toy-complex-train.yaml
    c.set("engine.precision", args.precision)
    c.set("verbose", False)
    return c


def timed_loop(fn, steps, warmup, world):
    for i in range(warmup):
        fn(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return (time.perf_counter() - t0) / steps


def cpu_baseline(args, E, R, seconds):
    """Reference CPU path: refseq replica of KgeModel.score_sp (ComplEx) on host cores."""
    from oracle import refseq

    torch.set_num_threads(max(1, min(os.cpu_count() or 1, 16)))
    g = torch.Generator().manual_seed(0)
    ent = torch.randn(E, args.dim, generator=g) * 0.1
    rel = torch.randn(R, args.dim, generator=g) * 0.1
    times = []
    t_end = time.perf_counter() + seconds
    i = 0
    while (time.perf_counter() < t_end or len(times) < 3) and len(times) < 200:
        s = torch.randint(0, E, (args.batch,), generator=g)
        p = torch.randint(0, R, (args.batch,), generator=g)
        t0 = time.perf_counter()
        refseq.complex_score_sp(ent, rel, s, p)
        times.append(time.perf_counter() - t0)
        i += 1
    med = float(np.median(times))
    return {"value": args.batch * E / med, "unit": "scored triples/s", "cores": torch.get_num_threads(),
            "kind": "port", "ms_per_step": med * 1e3,
            "sample": f"{len(times)} x score_sp (B={args.batch}, E={E}, d={args.dim}, N(0,0.1)), "
                      f"reference ATen op sequence (oracle/refseq.py) on CPU, median"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    dev_index = local_rank % ndev  # == local_rank on a node with one GPU per rank
    if world > 1:
        torch.cuda.set_device(dev_index)
        # "nccl" is RCCL on ROCm; KGE_DIST_BACKEND=gloo only to rehearse >1 rank on one GPU
        dist.init_process_group(os.environ.get("KGE_DIST_BACKEND", "nccl"))
    device = f"cuda:{dev_index}"

    from kge import Dataset, KgeModel, _lib, engine
    from kge.dataset import SHAPES

    E, R, _ = SHAPES[args.dataset]
    B, d = args.batch, args.dim
    c = make_config(args, device)
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    torch.manual_seed(0)
    model = KgeModel.create(c, Dataset(c, None))
    model.eval()
    ent = model._entity_embedder._embeddings.weight
    rel = model._relation_embedder._embeddings.weight
    steps, warmup = args.steps, args.warmup
    g = torch.Generator(device=device).manual_seed(1 + rank)
    s_all = torch.randint(0, E, (steps + warmup, B), device=device, generator=g)
    p_all = torch.randint(0, R, (steps + warmup, B), device=device, generator=g)
    prec = _lib.PRECISIONS[args.precision]

    # Every rank scores its own 1024 queries against the entity table (30 MB, replicated at
    # setup): the scored triples are partitioned by query and the step has no data-path
    # collective.  The entity-row-sharded exchange (kge.sharded: the design for eval top-k,
    # vocab-parallel training and tables too large to replicate) is timed after the headline
    # loop and reported in "row_sharded".
    def step(i):
        with torch.no_grad():
            return model.score_sp(s_all[i], p_all[i])
    scored_per_step = world * B * E

    # timed region: K steps bracketed by barrier + synchronize, nothing else inside
    sec = timed_loop(step, steps, warmup, world)
    # instrumented re-run of the same steps: HIP events around every contraction launch
    engine.KERNEL_EVENTS = []
    for i in range(min(steps, 20)):
        step(warmup + i)
    torch.cuda.synchronize()
    events = engine.KERNEL_EVENTS
    engine.KERNEL_EVENTS = None
    row_sharded = None
    if world > 1:
        from kge.sharded import EngineOps, RowShardedScorer, shard_bounds

        lo, hi = shard_bounds(E, world, rank)
        sharded = RowShardedScorer(ent.detach()[lo:hi].contiguous(), lo, hi, E, rel.detach(),
                                   EngineOps(_lib.COMPLEX, prec))
        # shard-affine loader: rank k's queries have their subject in shard k
        s_aff = torch.randint(lo, hi, (steps + warmup, B), device=device, generator=g)

        def step_sharded(i):
            with torch.no_grad():
                return sharded.score_sp_local(s_aff[i], p_all[i])

        sec_sh = timed_loop(step_sharded, steps, warmup, world)
        q_loc = torch.randn(B, d, device=device)

        def gather_only(i):
            out = torch.empty(world * B, d, device=device)
            dist.all_gather_into_tensor(out, q_loc)
        sec_ag = timed_loop(gather_only, steps, warmup, world)
        t = torch.tensor([sec_sh, sec_ag], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sec_sh, sec_ag = float(t[0]), float(t[1])
        row_sharded = {"ms_per_step": sec_sh * 1e3, "value": world * B * E / sec_sh,
                       "q_all_gather_ms": sec_ag * 1e3,
                       "what": f"entity table row-sharded x{world}; each rank's 1024 queries (subjects in its "
                               f"shard) -> query rows all_gathered ({world * B * d * 4 / 1e6:.0f} MB) -> global "
                               f"batch scored against every shard (kge.sharded.score_sp_local)"}
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in events])) if events else float("nan")
    # back-to-back launches of the same contraction between two HIP events on the launch
    # stream: the kernel's average duration without per-launch event overhead (this is the
    # figure the rocprofv3 kernel-trace average is compared with)
    with torch.no_grad():
        q = _lib.prep_query(_lib.COMPLEX, _lib.DIR_SP, ent.detach(), s_all[0], rel.detach(), p_all[0], B, d, d)
        tab = ent.detach()
        out_buf = torch.empty(q.shape[0], tab.shape[0], device=device)
        if prec == _lib.PREC_BF16X3:  # the production path: pre-split Q planes + persistent kernel
            qh, ql = _lib.split_rows(q)
            kern = lambda: _lib.score_dot_split(qh, ql, tab, None, d, out=out_buf)  # noqa: E731
        else:
            kern = lambda: _lib.score_dot(q, tab, None, prec, out=out_buf)  # noqa: E731
        for _ in range(20):  # the clock settles under sustained MFMA load
            kern()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        reps = 100
        a.record()
        for _ in range(reps):
            kern()
        b.record()
        torch.cuda.synchronize()
        kern_ms = a.elapsed_time(b) / reps
        del out_buf
    if world > 1:
        t = torch.tensor([sec, kern_ms, launch_ms], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sec, kern_ms, launch_ms = float(t[0]), float(t[1]), float(t[2])

    # roofline of the dominant kernel (the contraction) -- per launch, per GPU
    rows_q = B
    cols = E
    alg_flops = 2.0 * rows_q * cols * d
    alg_bytes = 4.0 * (rows_q * d + cols * d + rows_q * cols)
    k_s = kern_ms / 1e3
    if args.precision == "bf16x3":
        peak = BF16_DENSE_TFLOPS / 3.0
        note = "bf16x3 split MFMA: 3 bf16 passes per fp32 product; peak = 2.5 PF dense bf16 / 3"
    else:
        peak = FP32_MFMA_TFLOPS
        note = "fp32-input MFMA (v_mfma_f32_32x32x2_f32); peak = 157.3 TF"
    achieved = alg_flops / k_s / 1e12
    # HBM bytes per launch from the PMC passes of scripts/pmc_traffic.sh (same kernel, same
    # shape at N=1), committed under profiles/; null when absent or for another shape.
    traffic, traffic_src = None, None
    pmc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01", "pmc_traffic.json")
    if args.precision == "bf16x3" and os.path.exists(pmc):  # same per-GPU launch at every N
        with open(pmc) as f:
            t = json.load(f)
        traffic = int(t["traffic_bytes"])
        traffic_src = ("profiles/r01/pmc_traffic.json: 2 x FETCH_SIZE + WRITE_SIZE per dispatch "
                       f"(read {t['read_bytes'] / 1e6:.1f} MB, write {t['write_bytes'] / 1e6:.1f} MB)")
    roofline = {"bound": "mfma", "achieved": round(achieved, 1), "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": "score_dot_persist16_kernel" if args.precision == "bf16x3" else "score_dot_kernel", "kernel_us": round(kern_ms * 1e3, 2),
                "kernel_us_per_launch_events": round(launch_ms * 1e3, 2),
                "hbm_achieved_GBs": round(alg_bytes / k_s / 1e9, 1),
                "hbm_frac": round(alg_bytes / k_s / 1e9 / HBM_PEAK_GBS, 4),
                "alg_bytes_per_launch": int(alg_bytes), "alg_flops_per_launch": int(alg_flops), "note": note}

    value = scored_per_step / sec
    out = {"metric": "1vsAll scored triples/sec (score_sp, ComplEx-512, FB15K-237 shape, B=1024)",
           "value": value, "unit": "scored triples/s", "n_gpus": world, "steps": steps, "warmup": warmup,
           "ms_per_step": sec * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32 (bf16x3 MFMA)" if args.precision == "bf16x3" else "f32",
           "data": "synthetic (FB15K-237 shape: 14,541 entities / 237 relations), N(0,0.1) random-init tables",
           "config": {"workload": "configs[1]: ComplEx dim=512 1vsAll FB15K-237, batch 1024, score_sp per step",
                      "model": "complex", "dim": d, "global_batch": B * world, "entities": E,
                      "parallelism": "single GPU" if world == 1 else
                      f"dp{world}: queries partitioned over ranks (1024 each), entity table replicated, "
                      f"no collective in the step",
                      "precision": args.precision},
           "roofline": roofline}
    if row_sharded is not None:
        out["row_sharded"] = row_sharded

    if rank == 0 and world == 1 and not args.no_extras:
        out["extras"] = extras(args, model, c, E, R, device)
    if rank == 0 and world == 1 and not args.no_cpu:
        cb = cpu_baseline(args, E, R, args.cpu_seconds)
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu"] = round(value / cb["value"], 1)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def extras(args, model, c, E, R, device):
    """Secondary numbers: score_po, 1vsAll train step, eval MRR (synthetic test split)."""
    from kge import Dataset
    from kge.job import EntityRankingJob, TrainingJob

    B = args.batch
    res = {}
    g = torch.Generator(device=device).manual_seed(7)
    p = torch.randint(0, R, (40, B), device=device, generator=g)
    o = torch.randint(0, E, (40, B), device=device, generator=g)
    with torch.no_grad():
        sec = timed_loop(lambda i: model.score_po(p[i], o[i]), 30, 10, 1)
    res["score_po_ms"] = round(sec * 1e3, 4)
    # 1vsAll training step (sp + po, fwd + bwd + CE + Adagrad), train_step_ms
    c2 = c.clone()
    c2.set("train.type", "1vsAll")
    c2.set("train.optimizer", "Adagrad")
    c2.set("train.optimizer_args", {"lr": 0.2})
    c2.set("train.batch_size", B)
    ds = Dataset.synthetic(c2, args.dataset, seed=0)
    job = TrainingJob.create(c2, ds, model=model)
    job._prepare()
    job.model.train()
    train = ds.split("train")
    perm = torch.randperm(len(train), generator=torch.Generator().manual_seed(0))

    def tstep(i):  # the job's batch step: recorded as a HIP graph after two eager batches
        job.train_step(i, {"triples": train[perm[i * B:(i + 1) * B]].long()})
    sec = timed_loop(tstep, 30, 6, 1)
    res["train_step_ms"] = round(sec * 1e3, 3)
    res["train_scored_triples_per_s"] = 2 * B * E / sec
    res["train_triples_per_s"] = B / sec
    # filtered eval (test split, batch 1024)
    c3 = c.clone()
    c3.set("eval.split", "test")
    c3.set("eval.batch_size", B)
    job.model.eval()
    ej = EntityRankingJob(c3, ds, model=job.model)
    ej._prepare()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ej._run()  # first run: lazily built filter indexes and allocator warm-up
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    tr = ej._run()
    torch.cuda.synchronize()
    res["eval_test_triples"] = int(len(ds.split("test")))
    res["eval_seconds"] = round(time.perf_counter() - t1, 4)
    res["eval_first_run_seconds"] = round(t1 - t0, 4)
    res["eval_mrr_filtered"] = tr["mean_reciprocal_rank_filtered"]
    res["eval_hits_at_10_filtered"] = tr["hits_at_10_filtered"]
    res["eval_note"] = ("synthetic triples are drawn at random (no learnable structure), so the model trained "
                        "for the timing steps ranks near chance; rank / MRR parity with the reference is pinned "
                        "by the reference-captured eval fixtures (tests/test_gpu_api.py, tests/golden/eval_*.npz)")
    res.update(other_configs(device))
    if args.c5:
        res.update(c5_shard(args, device))
    return res


def c5_shard(args, device):
    """BASELINE configs[4] per GPU: ComplEx-512 1vsAll on Wikidata5M with the entity table
    row-sharded over 8 GPUs -- one rank's shard of ceil(4,594,485 / 8) = 574,311 rows scored
    by a batch of 1024 queries (score_sp through the model API; 2.35 GB of scores per step),
    plus the contraction kernel alone (HIP events around back-to-back launches)."""
    from kge import Dataset, KgeModel, _lib

    E_full, R, _ = __import__("kge.dataset", fromlist=["SHAPES"]).SHAPES["wikidata5m"]
    E = (E_full + 7) // 8
    B, d = args.batch, args.dim
    c = make_config(args, device)
    c.set("dataset.num_entities", E)
    c.set("dataset.num_relations", R)
    torch.manual_seed(0)
    model = KgeModel.create(c, Dataset(c, None))
    model.eval()
    g = torch.Generator(device=device).manual_seed(3)
    s = torch.randint(0, E, (8, B), device=device, generator=g)
    p = torch.randint(0, R, (8, B), device=device, generator=g)
    out = {}

    def step(i):
        with torch.no_grad():
            return model.score_sp(s[i % 8], p[i % 8])
    sec = timed_loop(step, 8, 3, 1)
    out["c5_shard_rows"] = E
    out["c5_shard_score_sp_ms"] = round(sec * 1e3, 3)
    out["c5_shard_scored_triples_per_s"] = B * E / sec
    ent = model._entity_embedder._embeddings.weight.detach()
    rel = model._relation_embedder._embeddings.weight.detach()
    with torch.no_grad():
        q = _lib.prep_query(_lib.COMPLEX, _lib.DIR_SP, ent, s[0], rel, p[0], B, d, d)
        qh, ql = _lib.split_rows(q)
        buf = torch.empty(B, E, device=device)
        for _ in range(3):
            _lib.score_dot_split(qh, ql, ent, None, d, out=buf)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            _lib.score_dot_split(qh, ql, ent, None, d, out=buf)
        b.record()
        torch.cuda.synchronize()
    k_s = a.elapsed_time(b) / 10 / 1e3
    flops = 2.0 * B * E * d
    nbytes = 4.0 * (B * d + E * d + B * E)
    out["c5_shard_kernel_us"] = round(k_s * 1e6, 1)
    out["c5_shard_kernel_tflops"] = round(flops / k_s / 1e12, 1)
    out["c5_shard_kernel_mfma_frac"] = round(flops / k_s / 1e12 / (BF16_DENSE_TFLOPS / 3.0), 4)
    out["c5_shard_kernel_hbm_frac"] = round(nbytes / k_s / 1e9 / HBM_PEAK_GBS, 4)
    del model, buf
    torch.cuda.empty_cache()
    return out


def _job_step_time(cfg, dataset, batch, steps=10, warmup=3):
    from kge import Dataset
    from kge.job import TrainingJob

    ds = Dataset.synthetic(cfg, dataset, seed=0)
    job = TrainingJob.create(cfg, ds)
    job._prepare()
    perm = torch.randperm(job.num_examples, generator=torch.Generator().manual_seed(0))

    def step(i):
        job.train_step(i, job._collate(perm[i * batch:(i + 1) * batch]))
    return timed_loop(step, steps, warmup, 1), ds


def other_configs(device):
    """BASELINE configs C3 (DistMult-512 KvsAll WN18RR, B=512) and C4 (RotatE-1024 negative
    sampling, 1024 negatives per corrupted slot, FB15K-237, B=512): full training steps
    (fwd + bwd + loss + Adagrad) on synthetic data of the dataset shape."""
    from kge import Config

    res = {}
    c = Config()
    c.set("model", "distmult")
    c._import("distmult")
    c.set("job.device", str(device))
    c.set("lookup_embedder.dim", 512)
    c.set("lookup_embedder.initialize_args", {"mean": 0.0, "std": 0.1})
    c.set("train.type", "KvsAll")
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.2})
    c.set("train.batch_size", 512)
    c.set("verbose", False)
    sec, ds = _job_step_time(c, "wn18rr", 512)
    E = ds.num_entities()
    res["c3_kvsall_distmult512_wn18rr_b512_step_ms"] = round(sec * 1e3, 3)
    res["c3_scored_triples_per_s"] = 512 * E / sec  # one query type per batch slice; B queries x E
    torch.manual_seed(0)
    c = Config()
    c.set("model", "rotate")
    c._import("rotate")
    c.set("job.device", str(device))
    c.set("lookup_embedder.dim", 1024)
    c.set("train.type", "negative_sampling")
    c.set("train.loss", "kl")
    c.set("negative_sampling.num_samples.s", 1024)
    c.set("negative_sampling.implementation", "triple")
    c.set("train.optimizer", "Adagrad")
    c.set("train.optimizer_args", {"lr": 0.1})
    c.set("train.batch_size", 512)
    c.set("verbose", False)
    sec, _ = _job_step_time(c, "fb15k-237", 512)
    res["c4_ns_rotate1024_fb15k237_b512_n1024_step_ms"] = round(sec * 1e3, 3)
    res["c4_scored_triples_per_s"] = 2 * 512 * 1025 / sec  # s and o slots, positive + 1024 negatives
    return res


if __name__ == "__main__":
    main()
