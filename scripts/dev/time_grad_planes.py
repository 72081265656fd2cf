"""Gradient-plane kernels of the row-sharded losses (kge_softmax_grad_planes, kge_bce_grad_planes):
time per launch and the HBM rate of their algorithmic bytes (scores read once, planes written once).

    python scripts/dev/time_grad_planes.py [rows cols ...]     (default: 2048 14541  2048 574311)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch  # noqa: E402

from kge import _lib as L  # noqa: E402

args = [int(a) for a in sys.argv[1:]] or [2048, 14541, 2048, 574311]
for n, m in zip(args[::2], args[1::2]):
    torch.manual_seed(0)
    s = torch.randn(n, (m + 3) // 4 * 4, device="cuda")[:, :m]
    labels = torch.randint(0, 2 * m, (n,), device="cuda")
    lse = torch.logsumexp(s[:, :4096], 1) + 3.0
    n_pad, ld = L.planes_layout(n, m)
    nbytes = n * m * 4 + n_pad * ld * 4
    for name, fn in (("softmax_grad_planes", lambda: L.softmax_grad_planes(s, 0, labels, lse, 1.0 / n)),
                     ("bce_grad_planes", lambda: L.bce_grad_planes(s, 0, labels, 0.0, 1.0 / n))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 10
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) / reps * 1e3
        print(f"[{n} x {m}] {name}: {us:.1f} us per call (incl. the output allocation), "
              f"{nbytes / us / 1e3:.0f} GB/s of {nbytes / 1e6:.0f} MB algorithmic bytes", flush=True)
    del s
    torch.cuda.empty_cache()
