import sys, time, torch
sys.path.insert(0, 'kge-1_amd')
from kge import _lib as L
E, R, B, d = 14541, 237, 1024, 512
torch.manual_seed(0)
ent = (torch.randn(E, d) * 0.1).cuda(); rel = (torch.randn(R, d) * 0.1).cuda()
s = torch.randint(0, E, (B,)).cuda(); p = torch.randint(0, R, (B,)).cuda()
q = L.prep_query(0, 0, ent, s, rel, p, B, d, d)
out = torch.empty(B, E, device='cuda')
for name, prec in L.PRECISIONS.items():
    for _ in range(5): L.score_dot(q, ent, None, prec, out=out)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(50): L.score_dot(q, ent, None, prec, out=out)
    en.record(); torch.cuda.synchronize()
    ms = st.elapsed_time(en) / 50
    print(f"score_dot {name}: {ms*1e3:.1f} us  {2*B*E*d/ms/1e9:.1f} TFLOP/s  HBM-frac {93.55e6/(ms*1e-3)/8e12:.3f}")
ref = torch.mm(q, ent.t())
for _ in range(5): torch.mm(q, ent.t(), out=out)
torch.cuda.synchronize()
st.record()
for _ in range(50): torch.mm(q, ent.t(), out=out)
en.record(); torch.cuda.synchronize()
ms = st.elapsed_time(en) / 50
print(f"torch.mm fp32 (hipBLASLt) : {ms*1e3:.1f} us")
torch.backends.cuda.matmul.allow_tf32 = True
for _ in range(5): torch.mm(q, ent.t(), out=out)
torch.cuda.synchronize(); st.record()
for _ in range(50): torch.mm(q, ent.t(), out=out)
en.record(); torch.cuda.synchronize()
print(f"torch.mm tf32-allowed : {st.elapsed_time(en)/50*1e3:.1f} us")
qb, eb = q.bfloat16(), ent.bfloat16()
ob = torch.empty(B, E, device='cuda', dtype=torch.bfloat16)
for _ in range(5): torch.mm(qb, eb.t(), out=ob)
torch.cuda.synchronize(); st.record()
for _ in range(50): torch.mm(qb, eb.t(), out=ob)
en.record(); torch.cuda.synchronize()
print(f"torch.mm bf16 : {st.elapsed_time(en)/50*1e3:.1f} us")
for kind in range(4):
    qq = q if kind < 2 else q
    for _ in range(2): L.score_dist(kind, 1.0, qq, ent, None, out=out)
    torch.cuda.synchronize(); st.record()
    for _ in range(5): L.score_dist(kind, 1.0, qq, ent, None, out=out)
    en.record(); torch.cuda.synchronize()
    print(f"score_dist kind {kind}: {st.elapsed_time(en)/5*1e3:.1f} us")
