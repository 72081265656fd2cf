import sys, os, json
sys.path.insert(0, '.'); sys.path.insert(0, 'kge-1_amd'); sys.path.insert(0, 'tests')
import numpy as np, torch
from oracle import kge_oracle as K
from kge import _lib as L
f = np.load('tests/golden/eval_dyadic.npz'); meta = json.loads(str(f['meta']))
ent = torch.from_numpy(f['ent']).cuda(); rel = torch.from_numpy(f['rel']).cuda()
tri = f['tri_valid'][:64]
s, p, o = (torch.from_numpy(tri[:, i]).cuda() for i in range(3))
B, E = len(tri), ent.shape[0]
for prec in (1, 0):
    q_sp = L.prep_query(0, 0, ent, s, rel, p, B, 32, 32)
    q_po = L.prep_query(0, 1, ent, o, rel, p, B, 32, 32)
    S_sp = L.score_dot(q_sp, ent, None, prec); S_po = L.score_dot(q_po, ent, None, prec)
    t = L.score_spo(0, 1.0, ent, s, rel, p, o, 32, 32)
    e64, r64 = f['ent'].astype(np.float64), f['rel'].astype(np.float64)
    ref_sp = K.score_emb('complex', e64[tri[:,0]], r64[tri[:,1]], e64, 'sp_')
    ref_po = K.score_emb('complex', e64, r64[tri[:,1]], e64[tri[:,2]], '_po')
    ref_t = K.score_emb('complex', e64[tri[:,0]], r64[tri[:,1]], e64[tri[:,2]], 'spo')
    print('prec', prec, 'sp exact', np.array_equal(S_sp.cpu().numpy(), ref_sp.astype(np.float32)),
          'po exact', np.array_equal(S_po.cpu().numpy(), ref_po.astype(np.float32)),
          't exact', np.array_equal(t.cpu().numpy(), ref_t.astype(np.float32)))
    for name, S, tgt in (('o', S_sp, o), ('s', S_po, s)):
        g = torch.zeros(3 * B, dtype=torch.int64, device='cuda'); ti = torch.zeros_like(g)
        L.rank_counts(S, 0, tgt, t, None, None, None, None, g, ti)
        Sx = S.double().cpu().numpy().copy(); tt = t.double().cpu().numpy()
        for i in range(B): Sx[i, tgt[i].item()] = tt[i]
        rg, rt = K.rank_and_ties(Sx, tt)
        print(name, 'greater ok', np.array_equal(g[:B].cpu().numpy(), rg), 'ties ok', np.array_equal(ti[:B].cpu().numpy(), rt),
              g[:6].tolist(), rg[:6].tolist(), ti[:6].tolist(), rt[:6].tolist())
        # also compare to fixture ranks
    print('fixture o_raw', f['full_o_raw'][:6], 's_raw', f['full_s_raw'][:6])
