"""Random shapes through the kernels added last (owner-computes distance backward, gradient planes
of the sharded softmax, Lp penalty rows) against float64 torch; prints the worst relative errors.

    python scripts/dev/fuzz_new_kernels.py [cases]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))

from kge import _lib as L  # noqa: E402


def dist_ref(kind, sign, q, t, G):
    qq = q.double().requires_grad_(True)
    tt = t.double().requires_grad_(True)
    d = q.shape[1]
    if kind < 2:
        diff = qq[:, None, :] - tt[None, :, :]
        dist = diff.abs().sum(-1) if kind == 0 else diff.pow(2).sum(-1).sqrt()
    else:
        h = d // 2
        dr, di = qq[:, None, :h] - tt[None, :, :h], qq[:, None, h:] - tt[None, :, h:]
        sq = dr * dr + di * di
        mod = torch.where(sq > 0, sq.clamp_min(1e-300).sqrt(), torch.zeros_like(sq))
        dist = mod.sum(-1) if kind == 2 else sq.sum(-1).sqrt()
    (sign * dist * G.double()).sum().backward()
    return qq.grad, tt.grad


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    g = torch.Generator().manual_seed(0)
    worst = {"dist": 0.0, "planes": 0.0, "lp": 0.0}
    for c in range(cases):
        n = int(torch.randint(1, 300, (1,), generator=g))
        m = int(torch.randint(1, 700, (1,), generator=g))
        d = 8 * int(torch.randint(1, 40, (1,), generator=g))
        kind = c % 4
        print(f"case {c}: kind {kind} n {n} m {m} d {d}", flush=True)
        q = (torch.randn(n, d, generator=g) * 0.3).cuda()
        t = (torch.randn(m, d, generator=g) * 0.3).cuda()
        G = torch.randn(n, m, generator=g).cuda()
        dq = torch.zeros(n, d, device="cuda")
        dt = torch.zeros(m, d, device="cuda")
        L.score_dist_bwd(kind, -1.0, G, q, t, None, dq, dt)
        rq, rt = dist_ref(kind, -1.0, q, t, G)
        scale = max(rq.abs().max().item(), rt.abs().max().item(), 1e-30)
        err = max((dq.double() - rq).abs().max().item(), (dt.double() - rt).abs().max().item()) / scale
        worst["dist"] = max(worst["dist"], err)
        assert err < 5e-5, (c, kind, n, m, d, err)
        # gradient planes of a softmax slice
        s = torch.randn(n, m, generator=g).cuda()
        lse = torch.logsumexp(s.double(), 1).float() + 0.5
        labels = torch.randint(0, m + 20, (n,), generator=g).cuda() + 7
        gp = L.softmax_grad_planes(s, 7, labels, lse, 0.25)
        ref = 0.25 * torch.exp(s.double() - lse.double()[:, None])
        lab = labels - 7
        ok = (lab >= 0) & (lab < m)
        ref[torch.arange(n, device="cuda")[ok], lab[ok]] -= 0.25
        got = gp.hi[:n, :m].double() + gp.lo[:n, :m].double()
        err = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
        worst["planes"] = max(worst["planes"], err)
        assert err < 3e-5, (c, n, m, err)
        assert float(gp.hi[:, m:].float().abs().sum()) == 0.0 and float(gp.hi[n:].float().abs().sum()) == 0.0
        assert float(gp.lo[:, m:].float().abs().sum()) == 0.0 and float(gp.lo[n:].float().abs().sum()) == 0.0
        # Lp rows
        p = 1 + c % 4
        idx = torch.randint(0, m, (n,), generator=g).cuda()
        sums = L.lp_rows(t, idx, p)
        ref = t[idx].double().abs().pow(p).sum(1)
        err = (sums.double() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
        worst["lp"] = max(worst["lp"], err)
        assert err < 1e-5, (c, p, err)
    print("worst relative errors", worst, flush=True)


if __name__ == "__main__":
    main()
