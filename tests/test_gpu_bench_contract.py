"""The benchmark's output contract: `python bench.py` prints ONE JSON line on stdout with the
driver's keys, BASELINE.json's metric, and the `roofline` / `cpu_baseline` objects.  Run here
with few steps and a short CPU leg (the numbers themselves are not asserted)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_prints_one_json_line_with_the_contract_keys():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2",
                          "--no-extras", "--cpu-seconds", "1"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["warmup"] == 2
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert "workload" in d["config"] and "model" not in d["config"]
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # the value is whole-job throughput: scored triples per step / step time
    assert d["value"] == pytest.approx(d["config"]["global_batch"] * d["config"]["entities"] / (d["ms_per_step"] / 1e3),
                                       rel=1e-6)
    if isinstance(baseline.get("metric"), str):
        assert "scored triples" in d["metric"] or baseline["metric"].split()[0] in d["metric"]
    r = d["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in r, key
    assert r["bound"] in ("hbm", "mfma") and r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    assert r["achieved"] == pytest.approx(r["alg_flops_per_launch"] / (r["kernel_us"] * 1e-6) / 1e12, rel=2e-3)
    c = d["cpu_baseline"]
    for key in ("value", "unit", "cores", "kind", "sample"):
        assert key in c, key
    assert c["kind"] in ("reference", "port") and c["cores"] >= 1 and c["value"] > 0


def test_bench_gpus_2_launches_its_own_ranks():
    """`python bench.py --gpus 2` (no torchrun around it) starts two ranks itself and reports
    n_gpus = 2.  A one-GPU box cannot run RCCL between two ranks, so the two share the card and
    exchange over gloo through host memory (KGE_DIST_BACKEND, the rehearsal switch): the numbers say
    nothing about RCCL, the launch path and the output contract are what is checked."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["KGE_DIST_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup",
                          "2", "--no-c5"], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 4
    assert d["config"]["global_batch"] == 2 * 1024
    assert d["value"] == pytest.approx(2 * 1024 * d["config"]["entities"] / (d["ms_per_step"] / 1e3), rel=1e-6)
    assert "row_sharded" in d and d["row_sharded"]["headline_schedule"] in ("pipelined", "serial", "grouped")
    # the metric's second half at N ranks: filtered MRR of the row-sharded evaluation job, equal to
    # the unsharded job's on the same tables
    ev = d["eval_row_sharded"]
    assert "error" not in ev, ev
    assert ev["metrics_equal"] is True, ev
    assert ev["row_sharded"]["eval_test_triples"] == 20466 and ev["row_sharded"]["mrr_filtered"] > 0
