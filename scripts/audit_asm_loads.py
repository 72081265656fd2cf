"""Audit of hipcc's device assembly for kernels that issue register loads from inline asm
(`global_load_dwordx4` with hand-counted `s_waitcnt vmcnt`): on every control-flow path from
such a load to a use of its destination registers there must be an `s_waitcnt vmcnt(N)` that
retires it (N <= the number of VMEM operations issued after the load on that path).  A use
before that is hipcc reusing or copying the registers while the data is still in flight
(an asm statement's outputs count as written when the statement ends) -- the cause of a rare
memory fault this code once had.  Used by tests/test_asm_audit.py on every build, and by hand:

    python scripts/audit_asm_loads.py <file.s> [kernel symbol prefix]
"""
import re
import sys

VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")


def _regs(s):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", s):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", s):
        out.add(int(m.group(1)))
    return out


def functions(lines):
    """(symbol, first line, end line) of every function in a device .s listing."""
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"^([A-Za-z_][\w$.]*):\s*(;.*)?$", l)
        if m and not l.startswith(".L") and i > 0 and ".type" in "".join(lines[max(0, i - 3):i]):
            end = next((j for j in range(i, len(lines)) if lines[j].startswith(".Lfunc_end")), None)
            if end is not None:
                out.append((m.group(1), i, end))
    return out


def audit(lines, start, end):
    """Findings (strings) for the function whose body is lines[start:end]; also returns the
    number of inline-asm register loads examined."""
    body = lines[start:end]
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
    in_asm, flags = False, []
    for l in body:
        t = l.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
        elif t.startswith(";;#ASMEND"):
            in_asm = False
        flags.append(in_asm)

    def succ(i):
        t = body[i].strip()
        m = re.match(r"s_branch (\.LBB\S+)", t)
        if m:
            return [labels[m.group(1)]]
        m = re.match(r"s_cbranch_\w+ (\.LBB\S+)", t)
        if m:
            return [labels[m.group(1)], i + 1]
        if t.startswith("s_endpgm"):
            return []
        return [i + 1]

    findings, loads = [], 0
    for i, l in enumerate(body):
        t = l.strip()
        if not (flags[i] and t.startswith("global_load_dwordx4")):
            continue
        loads += 1
        dest = _regs(t.split(",")[0])
        seen, stack = set(), [(i + 1, 0)]
        while stack:
            j, younger = stack.pop()
            if j >= len(body) or (j, younger) in seen:
                continue
            seen.add((j, younger))
            tj = body[j].strip()
            m = re.match(r"s_waitcnt vmcnt\((\d+)\)", tj)
            if m and younger >= int(m.group(1)):
                continue  # retired on this path
            if VMEM.match(tj):
                younger = min(younger + 1, 64)
            if tj and not tj.startswith(";") and not tj.startswith(".") and not flags[j] and not m:
                if _regs(tj) & dest:
                    findings.append(f"load @{start + i}: {t} -> unretired use @{start + j}: {tj}")
                    continue
            for k in succ(j):
                stack.append((k, younger))
    return findings, loads


def audit_file(path, prefix=""):
    lines = open(path).read().split("\n")
    report = {}
    for sym, a, b in functions(lines):
        if prefix in sym:
            report[sym] = audit(lines, a, b)
    return report


if __name__ == "__main__":
    rep = audit_file(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    total = 0
    for sym, (findings, loads) in rep.items():
        if loads:
            print(f"{sym}: {loads} asm loads, {len(findings)} findings")
        for f in findings:
            print("  ", f)
        total += len(findings)
    print("issues", total)
    sys.exit(1 if total else 0)
