"""Dev audit of hipcc output (-save-temps .s) for the inline-asm register loads of a kernel:
on every control-flow path from an asm `global_load_dwordx4` to a use of its destination
registers there must be an `s_waitcnt vmcnt(N)` that retires it (N <= number of VMEM ops
issued after the load on that path).  A use before that is hipcc reusing or copying the
registers while the data is still in flight (cdna_hip_programming.md §5.7 item 1).
usage: python scripts/audit_asm_loads.py <file.s> <kernel symbol prefix>"""
import re, sys
fn, name = sys.argv[1], sys.argv[2]
lines = open(fn).read().split('\n')
st = [i for i, l in enumerate(lines) if l.startswith(name)][0]
end = [i for i in range(st, len(lines)) if lines[i].startswith('.Lfunc_end')][0]
body = lines[st:end]
labels = {l.split(':')[0]: i for i, l in enumerate(body) if re.match(r'^\.LBB\S+:', l)}
def regs(s):
    out = set()
    for m in re.finditer(r'\bv\[(\d+):(\d+)\]', s):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r'\bv(\d+)\b', s):
        out.add(int(m.group(1)))
    return out
inasm = False; asm_flags = []
for l in body:
    t = l.strip()
    if t.startswith(';;#ASMSTART'): inasm = True
    elif t.startswith(';;#ASMEND'): inasm = False
    asm_flags.append(inasm)
def succ(i):
    t = body[i].strip()
    m = re.match(r's_branch (\.LBB\S+)', t)
    if m: return [labels[m.group(1)]]
    m = re.match(r's_cbranch_\w+ (\.LBB\S+)', t)
    if m: return [labels[m.group(1)], i + 1]
    if t.startswith('s_endpgm'): return []
    return [i + 1]
VMEM = re.compile(r'^(global_|buffer_|flat_|scratch_)')
issues = 0
for i, l in enumerate(body):
    t = l.strip()
    if asm_flags[i] and t.startswith('global_load_dwordx4'):
        D = regs(t.split(',')[0])
        seen = set(); stack = [(i + 1, 0)]
        while stack:
            j, y = stack.pop()
            if j >= len(body) or (j, y) in seen: continue
            seen.add((j, y))
            tj = body[j].strip()
            m = re.match(r's_waitcnt vmcnt\((\d+)\)', tj)
            if m and y >= int(m.group(1)):
                continue  # retired on this path
            if VMEM.match(tj):
                y = min(y + 1, 64)
            if tj and not tj.startswith(';') and not tj.startswith('.') and not asm_flags[j] and not m:
                if regs(tj) & D:
                    print(f"load@{i} {t} -> UNRETIRED use @{j}: {tj}")
                    issues += 1
                    continue
            for k in succ(j): stack.append((k, y))
print("issues", issues)
