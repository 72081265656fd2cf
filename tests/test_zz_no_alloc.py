"""kge_score_dot_bwd_q_noalloc -- the dQ GEMM whose split-K slabs live in the library's static
device scratch -- against kge_score_dot_bwd_q_ws (caller workspace), through the C ABI.

Both run the same kernels in the same order, so the results must agree bit for bit; the ws
entry point itself is checked against float64 in test_gpu_kernels.py.  Two calls in a row
share the scratch, the second with a smaller input (stale slab contents of the first call
must not leak into it); then a gathered call and an accumulating call.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kge import _lib
    _lib.lib()
    return _lib


def _padded_g(n, m, gen):
    """G as the fused loss leaves it: rows padded to a multiple of 4 columns (16-B aligned)."""
    buf = torch.zeros(n, (m + 3) // 4 * 4, device="cuda")
    buf[:, :m] = torch.randn(n, m, device="cuda", generator=gen) * 0.05
    return buf[:, :m]


def _both(L, g, t, tidx, accumulate=False, seed_dq=None):
    n, d = g.shape[0], t.shape[1]
    base = seed_dq if seed_dq is not None else torch.full((n, d), float("nan"), device="cuda")
    ref = base.clone()
    L.score_dot_bwd_q(g, t, tidx, L.PREC_BF16X3, dq=ref, accumulate=accumulate)
    got = base.clone()
    L.score_dot_bwd_q_noalloc(g, t, tidx, got, accumulate=accumulate)
    torch.cuda.synchronize()
    return got, ref


def test_noalloc_matches_workspace_entry_two_calls_in_a_row(L):
    gen = torch.Generator(device="cuda").manual_seed(5)
    # call 1: the stacked C2 training shape (2,048 queries x 14,541 entities, d = 512): 8 K chunks,
    # the full 32 MiB of scratch
    E, d = 14541, 512
    t = torch.randn(E, d, device="cuda", generator=gen) * 0.1
    g1 = _padded_g(2048, E, gen)
    assert L.lib().kge_score_dot_bwd_q_ws_size(2048, E, d, L.PREC_BF16X3) == 8 * 2048 * d
    got1, ref1 = _both(L, g1, t, None)
    assert torch.equal(got1, ref1)
    # float64 anchor for the first call (1e-4 of the max |dq|: the bf16x3 contract)
    ref64 = g1.double() @ t.double()
    assert float((got1.double() - ref64).abs().max() / ref64.abs().max()) < 1e-4
    # call 2, right after: smaller in every dimension (other split count, other slab layout)
    t2 = t[:3001, :256].contiguous()
    g2 = _padded_g(300, 3001, gen)
    got2, ref2 = _both(L, g2, t2, None)
    assert torch.equal(got2, ref2)
    ref64 = g2.double() @ t2.double()
    assert float((got2.double() - ref64).abs().max() / ref64.abs().max()) < 1e-4


def test_noalloc_gather_accumulate_and_empty(L):
    gen = torch.Generator(device="cuda").manual_seed(6)
    t = torch.randn(5000, 128, device="cuda", generator=gen)
    tidx = torch.randint(0, 5000, (1999,), device="cuda", generator=gen)
    g = _padded_g(700, 1999, gen)
    got, ref = _both(L, g, t, tidx)
    assert torch.equal(got, ref)
    seed = torch.randn(700, 128, device="cuda", generator=gen)
    got, ref = _both(L, g, t, tidx, accumulate=True, seed_dq=seed)
    assert torch.equal(got, ref)
    # K not split (few candidates): no scratch involved, dq written by its single owner block
    g3 = _padded_g(64, 40, gen)
    got, ref = _both(L, g3, t[:40].contiguous(), None)
    assert torch.equal(got, ref)
    # empty reduction: dq = 0 (no allocation, a fill kernel)
    dq = torch.full((16, 128), 7.0, device="cuda")
    L.score_dot_bwd_q_noalloc(torch.zeros(16, 4, device="cuda")[:, :0], t, None, dq)
    torch.cuda.synchronize()
    assert float(dq.abs().max()) == 0.0


def test_noalloc_rejects_unaligned(L):
    g = torch.zeros(8, 13, device="cuda")  # odd leading dimension: the vector kernel cannot take it
    t = torch.zeros(13, 64, device="cuda")
    dq = torch.zeros(8, 64, device="cuda")
    with pytest.raises(L.EngineError):
        L.score_dot_bwd_q_noalloc(g, t, None, dq)


@pytest.mark.parametrize("n, m, d", [(512, 14541, 512), (1024, 4100, 512)])
def test_split_count_equals_launched_chunks(L, n, m, d):
    """Shapes at which rounding the K chunk up to whole stages leaves FEWER chunks than the CU
    count asks for (32 -> 31 at 512 x 14,541; 16 -> 15 at 1,024 x 4,100 on 256 CUs): the slab sum
    must add exactly the slabs the GEMM wrote.  The workspace of the ws entry point and the
    library's scratch are poisoned with NaN first, so a slab that is summed without having been
    written shows up in dq."""
    gen = torch.Generator(device="cuda").manual_seed(11)
    t = torch.randn(m, d, device="cuda", generator=gen) * 0.1
    g = _padded_g(n, m, gen)
    ref64 = g.double() @ t.double()
    scale = float(ref64.abs().max())
    # ws entry point with a NaN-filled caller workspace (sized by the library)
    ws_n = L.lib().kge_score_dot_bwd_q_ws_size(n, m, d, L.PREC_BF16X3)
    assert ws_n % (n * d) == 0
    ws = torch.full((max(ws_n, 1),), float("nan"), device="cuda")
    dq = torch.full((n, d), float("nan"), device="cuda")
    L._check(L.lib().kge_score_dot_bwd_q_ws(L.ptr(g), L.rows(g), L.ptr(t), L.rows(t), None, n, m, d, L.ptr(dq),
                                            L.rows(dq), 0, L.PREC_BF16X3, L.ptr(ws), ws_n, L.stream()), "bwd_q_ws")
    torch.cuda.synchronize()
    assert torch.isfinite(dq).all()
    assert float((dq.double() - ref64).abs().max()) / scale < 1e-4
    # poison the static scratch: a call whose chunks fill all of it with NaN slabs (G = NaN)
    gp = torch.full((2048, 14544), float("nan"), device="cuda")[:, :14541]
    tp = torch.zeros(14541, 512, device="cuda")
    L.score_dot_bwd_q_noalloc(gp, tp, None, torch.empty(2048, 512, device="cuda"))
    got = torch.full((n, d), float("nan"), device="cuda")
    L.score_dot_bwd_q_noalloc(g, t, None, got)
    torch.cuda.synchronize()
    assert torch.equal(got, dq)
