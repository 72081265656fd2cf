"""The shapes ONE rank sees at N = 8 on the Wikidata5M configuration -- 8,192 global queries against
a 574,311-row shard: a [8192, 574311] score block of 4.7e9 elements, past 2^32 -- through the
row-sharded scoring and training paths at world size 1, with sampled entries checked in float64.

    python scripts/dev/check_c5_n8_shapes.py
"""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kge import _lib as L  # noqa: E402
from kge.sharded import EngineOps, RowShardedScorer  # noqa: E402


def complex_q(e, r, direction):
    """float64 query rows of ComplEx: (s o r) for sp_, (o o conj r) for _po (complex.py:19-44)."""
    h = e.shape[1] // 2
    er, ei, rr, ri = e[:, :h], e[:, h:], r[:, :h], r[:, h:]
    if direction == 0:
        return torch.cat((er * rr - ei * ri, er * ri + ei * rr), 1)
    return torch.cat((rr * er + ri * ei, rr * ei - ri * er), 1)


def main():
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1)
    E, R, B, d = 574311, 237, 8192, 512
    torch.manual_seed(0)
    ent = torch.randn(E, d, device="cuda") * 0.1
    rel = torch.randn(R, d, device="cuda") * 0.1
    sh = RowShardedScorer(ent, 0, E, E, rel, EngineOps(L.COMPLEX, L.PREC_BF16X3))
    g = torch.Generator().manual_seed(1)
    s = torch.randint(0, E, (B,), generator=g).cuda()
    p = torch.randint(0, R, (B,), generator=g).cuda()
    o = torch.randint(0, E, (B,), generator=g).cuda()
    rows = torch.tensor([0, 1, 4095, 4096, 7000, 8191]).cuda()      # rows on both sides of 2^32 / E
    cols = torch.tensor([0, 5, 300000, 523775, 574310]).cuda()

    # ---- scoring (what bench.py's row_sharded_c5 runs per rank at N = 8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scores = sh.score_submitted(sh.submit_queries_local(s, p))
    torch.cuda.synchronize()
    print(f"scores {tuple(scores.shape)} in {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    q64 = complex_q(ent[s[rows]].double(), rel[p[rows]].double(), 0)
    ref = q64 @ ent[cols].double().T
    got = scores[rows][:, cols].double()
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    print(f"sampled scores: max rel err {err:.2e}", flush=True)
    assert err < 2e-5
    del scores
    torch.cuda.empty_cache()

    # ---- training gradients (vocab-parallel 1vsAll; gradient planes at this size)
    tr = torch.stack([s, p, o], 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss, d_ent, d_rel = sh.train_1vsall_global(tr)
    torch.cuda.synchronize()
    print(f"training gradients in {(time.perf_counter() - t0) * 1e3:.1f} ms, loss {float(loss):.4f}", flush=True)
    # the loss in float64, every row, in column chunks
    total = 0.0
    for direction, e_idx, lab in ((0, s, o), (1, o, s)):
        for b0 in range(0, B, 512):
            sl = slice(b0, b0 + 512)
            q64 = complex_q(ent[e_idx[sl]].double(), rel[p[sl]].double(), direction)
            acc_max = torch.full((512,), -float("inf"), device="cuda", dtype=torch.float64)
            acc_sum = torch.zeros(512, device="cuda", dtype=torch.float64)
            for c0 in range(0, E, 65536):
                lg = q64 @ ent[c0:c0 + 65536].double().T
                m = torch.maximum(acc_max, lg.max(1).values)
                acc_sum = acc_sum * torch.exp(acc_max - m) + torch.exp(lg - m[:, None]).sum(1)
                acc_max = m
            tgt = (q64 * ent[lab[sl]].double()).sum(1)
            total += float((acc_max + torch.log(acc_sum) - tgt).sum())
    ref_loss = total / B
    print(f"float64 loss {ref_loss:.6f} vs {float(loss):.6f}", flush=True)
    assert abs(float(loss) - ref_loss) < 1e-5 * abs(ref_loss)
    # dE rows: sum over both directions of G^T Q restricted to sampled entity rows
    ref_de = torch.zeros(len(cols), d, device="cuda", dtype=torch.float64)
    for direction, e_idx, lab in ((0, s, o), (1, o, s)):
        for b0 in range(0, B, 512):
            sl = slice(b0, b0 + 512)
            q64 = complex_q(ent[e_idx[sl]].double(), rel[p[sl]].double(), direction)
            acc_max = torch.full((512,), -float("inf"), device="cuda", dtype=torch.float64)
            acc_sum = torch.zeros(512, device="cuda", dtype=torch.float64)
            for c0 in range(0, E, 65536):
                lg = q64 @ ent[c0:c0 + 65536].double().T
                m = torch.maximum(acc_max, lg.max(1).values)
                acc_sum = acc_sum * torch.exp(acc_max - m) + torch.exp(lg - m[:, None]).sum(1)
                acc_max = m
            lse = acc_max + torch.log(acc_sum)
            gcols = torch.exp(q64 @ ent[cols].double().T - lse[:, None])          # [512, 5]
            gcols -= (lab[sl][:, None] == cols[None, :]).double()
            ref_de += (gcols / B).T @ q64
    # the query rows' own contribution (prep backward) lands on rows s / o, not on the sampled cols
    # unless they coincide: mask those out of the comparison
    touched = torch.isin(cols, torch.cat((s, o)))
    got = d_ent[cols].double()
    err = ((got - ref_de)[~touched]).abs().max().item() / ref_de.abs().max().item()
    print(f"sampled dE rows: max rel err {err:.2e} ({int((~touched).sum())} rows compared)", flush=True)
    assert err < 1e-4
    dist.destroy_process_group()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
