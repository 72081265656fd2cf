"""Where the time of the ranking launch on codes goes: the same 2,048 x 14,541 code block ranked
with / without filter lists, rescoring and histograms (HIP events over 200 launches each)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "kge-1_amd"))
from kge import _lib as L

torch.manual_seed(0)
rng = np.random.default_rng(0)
n_a = n_b = 1024
n, m, d = n_a + n_b, 14541, 512
q = torch.randn(n, d, device="cuda") * 0.1
t = torch.randn(m, d, device="cuda") * 0.1
ti = torch.randint(0, m, (n,), device="cuda")
ts = (q * t[ti]).sum(1)
hi, lo = L.split_rows(q)
tmax = L.row_norm_max(t)
band_rel = 2.0 ** -16 + 3 * d * 2.0 ** -25


def csr(k):
    lens = rng.integers(0, k + 1, size=n)
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=ptr[1:])
    col = rng.integers(0, m, size=int(ptr[-1]) + 1)
    return torch.from_numpy(ptr).cuda(), torch.from_numpy(col).cuda()


fp, fc = csr(8)
tp, tc = csr(4)
band = L.rank_band(q, band_rel, tmax)
noband = torch.full((n,), -1.0, device="cuda")


def run(name, refined, filt, hist):
    codes = L.score_dot_split_rank(hi, lo, t, d, n_a, (ti[:n_a], ts[:n_a]), (ti[n_a:], ts[n_a:]),
                                   band if refined else noband, 0)
    nrank = 3 if filt == 2 else (2 if filt == 1 else 1)
    g = torch.empty(nrank * n, dtype=torch.int64, device="cuda")
    tt = torch.empty_like(g)
    rk = torch.empty_like(g)
    hs = torch.zeros(nrank * 2, m, device="cuda") if hist else None
    pa = (ti[:n_a], ts[:n_a], fp[:n_a + 1] if filt else None, tp[:n_a + 1] if filt == 2 else None)
    pb = (ti[n_a:], ts[n_a:], fp[n_a:] if filt else None, tp[n_a:] if filt == 2 else None)
    kw = dict(accumulate=False, codes=codes, m=m, refine=(q, t, band_rel, tmax) if refined else None)
    if hist:
        kw.update(tie_handling="rounded_mean_rank", ranks=rk, hists=hs, rows_per_hist=n_a)

    def once():
        L.rank_rows(None, n_a, 0, pa, pb, fc if filt else None, tc if filt == 2 else None, g, tt, **kw)
    for _ in range(20):
        once()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        once()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:44s} {e0.elapsed_time(e1) / 200 * 1e3:7.1f} us per launch", flush=True)


run("codes only", False, 0, False)
run("codes + ranks/histograms", False, 0, True)
run("codes + rescoring", True, 0, False)
run("codes + one filter list", False, 1, False)
run("codes + two filter lists", False, 2, False)
run("everything (the evaluation's launch)", True, 2, True)
