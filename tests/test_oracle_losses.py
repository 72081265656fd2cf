"""CPU: the oracle's fused-loss restatements (softmax_xent, softmax_kl) against the torch
ops the reference composes them from -- CrossEntropyLoss / KLDivLoss(log_softmax,
normalize(labels, p=1)) with reduction "sum" (kge/util/loss.py:192-213), label smoothing
as in kge/job/train.py:715-721.  torch is the reference's own third-party dependency for
this arithmetic, so this pins the restatement."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import kge_oracle as K


@pytest.mark.parametrize("eps", [0.0, 0.1])
def test_softmax_kl_matches_torch(eps):
    rng = np.random.default_rng(0)
    n, m = 9, 57
    S = rng.standard_normal((n, m)) * 3
    pos = [rng.choice(m, size=k, replace=False) for k in [1, 3, 0, 5, 2, 1, 9, 0, 4]]
    y = torch.zeros(n, m, dtype=torch.float64)
    for i, c in enumerate(pos):
        y[i, torch.from_numpy(c)] = 1.0
    if eps > 0:
        y = (1 - eps) * y + 1.0 / m
    St = torch.tensor(S, requires_grad=True)
    loss = torch.nn.KLDivLoss(reduction="sum")(F.log_softmax(St, 1), F.normalize(y, p=1, dim=1)) * 0.25
    loss.backward()
    lo, G = K.softmax_kl(S, pos, eps, 0.25)
    assert abs(lo.sum() * 0.25 - loss.item()) < 1e-12
    np.testing.assert_allclose(G, St.grad.numpy(), atol=1e-14)


def test_softmax_xent_matches_torch():
    rng = np.random.default_rng(1)
    S = rng.standard_normal((7, 31)) * 4
    lab = rng.integers(0, 31, size=7)
    St = torch.tensor(S, requires_grad=True)
    loss = torch.nn.CrossEntropyLoss(reduction="sum")(St, torch.from_numpy(lab)) / 7
    loss.backward()
    lo, G = K.softmax_xent(S, lab, 1 / 7)
    assert abs(lo.sum() / 7 - loss.item()) < 1e-12
    np.testing.assert_allclose(G, St.grad.numpy(), atol=1e-14)
    lo2, G2 = K.softmax_kl(S, [[x] for x in lab], 0.0, 1 / 7)
    np.testing.assert_allclose(lo2, lo, atol=1e-12)
    np.testing.assert_allclose(G2, G, atol=1e-14)
