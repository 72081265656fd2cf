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


_LEGS_SCRIPT = """
import sys, time
sys.path.insert(0, {root!r})
import bench
out = {{"metric": "m", "value": 1.0}}
legs = bench.OptionalLegs(out, rank={rank}, seconds={seconds})
legs.run("quick", lambda: {{"ok": True}})
legs.run("broken", lambda: 1 / 0)
legs.run("slow", lambda: time.sleep({sleep}) or {{"ok": True}})
if legs.done():
    import json
    print(json.dumps(out), flush=True)
else:
    time.sleep(30)
sys.exit({status})
"""


def _legs(rank, seconds, sleep, status=0):
    code = _LEGS_SCRIPT.format(root=ROOT, rank=rank, seconds=seconds, sleep=sleep, status=status)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=_env())


def test_optional_legs_in_time_change_nothing():
    out = _legs(rank=0, seconds=60.0, sleep=0.0, status=3)
    assert out.returncode == 3
    d = json.loads(out.stdout.strip())
    assert d["quick"] == {"ok": True} and d["slow"] == {"ok": True} and "optional_legs_timed_out" not in d
    assert d["broken"]["error"].startswith("ZeroDivisionError")


def test_optional_legs_deadline_prints_the_headline_and_leaves_with_status_0():
    # a leg that never comes back (a collective that hangs): rank 0 prints the line it has, naming
    # the unfinished leg; every rank leaves with status 0, the other ranks without printing
    out = _legs(rank=0, seconds=1.0, sleep=60.0, status=3)
    assert out.returncode == 0, out.stderr[-1000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and d["quick"] == {"ok": True} and "slow" not in d
    assert d["optional_legs_timed_out"] == {"legs": ["slow"], "after_seconds": 1.0}
    other = _legs(rank=1, seconds=1.0, sleep=60.0, status=3)
    assert other.returncode == 0 and other.stdout.strip() == ""
