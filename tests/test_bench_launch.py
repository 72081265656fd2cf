"""`python bench.py --gpus N` outside torchrun starts its own N ranks (a child torchrun job) and
relays rank 0's single JSON line; under torchrun it insists that WORLD_SIZE equals --gpus.  Checked
here without a GPU through --launch-check (the ranks only meet over gloo and count themselves)."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    return env


def test_gpus_2_launches_two_ranks_and_prints_one_json_line():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                         timeout=300, env=_env())
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d == {"launch_check": True, "n_gpus": 2, "ranks_counted": 2}


def test_world_size_must_equal_gpus():
    env = _env()
    env["WORLD_SIZE"] = "1"
    out = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-check"], capture_output=True, text=True,
                         timeout=120, env=env)
    assert out.returncode != 0
    assert "--gpus 3" in out.stderr and out.stdout.strip() == ""


def test_failing_ranks_give_a_nonzero_status():
    # an option the ranks reject: the launcher must hand their failure on, and print no JSON line
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check", "--precision", "nope"],
                         capture_output=True, text=True, timeout=300, env=_env())
    assert out.returncode != 0 and out.stdout.strip() == ""
