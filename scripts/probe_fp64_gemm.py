import time, torch
def t(fn, reps=3):
    fn(); torch.cuda.synchronize(); t0=time.perf_counter()
    for _ in range(reps): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-t0)/reps
for d in (16, 64):
    X = torch.randn(4_000_000, d, dtype=torch.float64, device="cuda")
    Ri = torch.randn(d, d, dtype=torch.float64, device="cuda")
    print(d, "XtX mm", t(lambda: X.t() @ X))
    for c in (250, 1000, 4000):
        Xc = X.view(c, -1, d)
        print(d, "XtX bmm c=%d" % c, t(lambda: torch.bmm(Xc.transpose(1, 2), Xc).sum(0)))
    print(d, "X@Ri", t(lambda: X @ Ri))
    print(d, "X@Ri.T-trick", t(lambda: (Ri.t() @ X.t()).t()))
    print(d, "XtX fp32", t(lambda: X.float().t() @ X.float()))
