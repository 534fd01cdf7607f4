import sys, json, torch
sys.path.insert(0, '.')
from harp_amd.models.sgd_mf import SGDConfig, run_sgd, synthetic_ratings
from harp_amd.parallel.comm import Communicator
cuda = torch.device('cuda')
nu, ni = 3000, 800
u, i, v = synthetic_ratings(nu, ni, 120000, seed=2)
p = torch.randperm(u.numel(), generator=torch.Generator().manual_seed(0))
k = int(0.9 * u.numel())
train = (u[p[:k]], i[p[:k]], v[p[:k]]); test = (u[p[k:]], i[p[k:]], v[p[k:]])
for name, kw in [("cap", dict(conflict_mode="cap")), ("none128", dict(conflict_mode="none")),
                 ("atom3_b8", dict(conflict_mode="none", atomic=3, blocks_per_xcd=8)),
                 ("atom2_b8", dict(conflict_mode="none", atomic=2, blocks_per_xcd=8)),
                 ("atom1_b8", dict(conflict_mode="none", atomic=1, blocks_per_xcd=8)),
                 ("hot", dict())]:
    cfg = SGDConfig(rank=32, lam=0.05, lr=0.01, epochs=10, test_every=1, **kw)
    g = run_sgd(Communicator(None, cuda), cfg, nu, ni, train, test)
    print(name, json.dumps([(e, round(a, 4), round(b, 4)) for e, a, b in g["rmse"]]), g.get("blocks_per_xcd"), g.get("hot_items"), g.get("atomic"), flush=True)
