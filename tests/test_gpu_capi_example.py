"""examples/capi_score_sp.c: the C ABI of libkgescore.so driven from plain C -- hipMalloc'd buffers,
no Python objects, no torch -- for ComplEx and TransE score_sp on dyadic tables, compared for
equality with host loops inside the program.  Built by kge-1_amd/csrc/Makefile next to the library."""
import os
import subprocess

import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "kge-1_amd", "kge", "capi_score_sp")


def test_c_example_is_built_against_the_in_tree_library():
    assert os.access(EXE, os.X_OK), "run `make -C kge-1_amd/csrc` (or __graft_entry__.build())"
    out = subprocess.run(["ldd", EXE], capture_output=True, text=True, timeout=60).stdout
    lib = [ln for ln in out.splitlines() if "libkgescore.so" in ln]
    assert lib and os.path.join("kge-1_amd", "kge", "libkgescore.so") in lib[0], out


@pytest.mark.gpu
def test_c_example_scores_equal_the_host_loops():
    out = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "complex score_sp [37 x 777]: 0 of 28749 scores differ" in out.stdout
    assert "transe score_sp [37 x 777]: 0 of 28749 scores differ" in out.stdout
    assert "null output pointer -> status 1001" in out.stdout and "capi example ok" in out.stdout
