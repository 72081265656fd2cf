"""Build-time guard for the kernels whose K loop issues its memory operations from inline asm
with hand-counted `s_waitcnt vmcnt` (score_dot3.hip): the generated device assembly is audited
so that no path reaches a use of an asm load's registers before a wait that retires the load
(scripts/audit_asm_loads.py).  hipcc cross-compiles without a GPU, so this runs in the CPU
suite; the audit itself is also checked to catch a planted violation."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import audit_asm_loads as A  # noqa: E402

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-Xclang", "-target-feature",
         "-Xclang", "-packed-fp32-ops", "--cuda-device-only", "-S"]


@pytest.mark.parametrize("src,kernel,dev", [("score_dot3.hip", "score_dot_persist16_kernel", False),
                                            ("score_dot3.hip", "score_dot_persist16_kernel", True),
                                            ("gemm_bwd3p.hip", "bwd3p_q_kernel", False)])
def test_inline_asm_loads_are_retired_before_use(tmp_path, src, kernel, dev):
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    out = tmp_path / (src + ".s")
    cmd = [HIPCC] + FLAGS + (["-DKGE_DEV_BUILD"] if dev else []) + [os.path.join(ROOT, "kge-1_amd", "csrc", src),
                                                                   "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    report = A.audit_file(str(out), kernel)
    with_loads = {k: v for k, v in report.items() if v[1] > 0}
    assert with_loads, f"no {kernel} instantiation with inline-asm loads found in the assembly"
    bad = {k: v[0] for k, v in with_loads.items() if v[0]}
    assert not bad, bad


def test_audit_flags_a_use_before_the_wait():
    body = """\t.type\tk,@function
k:
\t;;#ASMSTART
\tglobal_load_dwordx4 v[4:7], v[0:1], off
\t;;#ASMEND
\tv_add_f32 v8, v4, v4
\ts_waitcnt vmcnt(0)
\ts_endpgm
.Lfunc_end0:
"""
    lines = body.split("\n")
    (sym, a, b), = A.functions(lines)
    findings, loads = A.audit(lines, a, b)
    assert loads == 1 and len(findings) == 1
    ok = body.replace("\tv_add_f32 v8, v4, v4\n\ts_waitcnt vmcnt(0)\n", "\ts_waitcnt vmcnt(0)\n\tv_add_f32 v8, v4, v4\n")
    lines = ok.split("\n")
    (sym, a, b), = A.functions(lines)
    assert A.audit(lines, a, b) == ([], 1)


def test_no_kernel_uses_scratch_flat_or_packed_fp32(tmp_path):
    """Every HIP source of the library, compiled as the Makefile compiles it: no kernel may spill
    to or index scratch memory (register pressure, pointer-select loads), address through flat
    instructions, or contain packed fp32 VALU instructions (the build switches them off)."""
    import glob
    import re
    from concurrent.futures import ThreadPoolExecutor

    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    srcs = sorted(glob.glob(os.path.join(ROOT, "kge-1_amd", "csrc", "*.hip")))
    assert len(srcs) >= 10

    def build(src):
        out = tmp_path / (os.path.basename(src) + ".s")
        subprocess.run([HIPCC] + FLAGS + [src, "-o", str(out)], check=True, capture_output=True)
        return out

    with ThreadPoolExecutor(max_workers=4) as pool:
        outs = list(pool.map(build, srcs))
    bad = {}
    pat = re.compile(r"^\s*(scratch_\w+|flat_(load|store|atomic)\w*|v_pk_(add|mul|fma)_f32)\b")
    for out in outs:
        hits = [ln.strip() for ln in open(out) if pat.match(ln)]
        if hits:
            bad[os.path.basename(str(out))] = hits[:5]
    assert not bad, bad
