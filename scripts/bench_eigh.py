"""Stage times of ops.eig.eigh (PCA step 2) at n (default 1000): the chip-wide reduction
(csrc/eig_ll.hip) and the one-XCD reduction (csrc/eig.hip), D&C tridiagonal eigenvectors,
compact-WY back-transform, whole eigh per variant and rocSOLVER; CUDA events, median of 10
after 3 warm-ups, on the PCA correlation matrix shape (uniform data, spectrum around 1).

    python scripts/bench_eigh.py [n]
"""
import ctypes
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from harp_amd.ops import eig as E  # noqa: E402


def timed(fn, reps=10, warm=3):
    out = []
    for it in range(reps + warm):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if it >= warm:
            out.append(a.elapsed_time(b))
    return round(statistics.median(out), 3)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.rand(20 * n, n, generator=g, device=dev, dtype=torch.float64)
    Xc = X - X.mean(0)
    C = Xc.t() @ Xc
    sd = torch.sqrt(torch.diagonal(C))
    C = (C / torch.outer(sd, sd)).contiguous()
    k = E._lib.kernels()
    rec = {"n": n}
    r = E.sytrd_ll(C)
    assert r is not None, "chip-wide reduction fell back"
    d, e, Vt, tau = r
    rec["sytrd_ll_ms"] = timed(lambda: E.sytrd_ll(C))
    rec["sytrd_ll_values_only_ms"] = timed(lambda: E.sytrd_ll(C, vectors=False))
    st = torch.zeros(6, dtype=torch.int64, device=dev)
    k.harp_sytrd_ll_stamps(st.data_ptr())
    E.sytrd_ll(C)
    torch.cuda.synchronize()
    k.harp_sytrd_ll_stamps(None)
    rec["ll_phase_cycles_per_col"] = [round(v / max(n - 2, 1), 1) for v in st.tolist()[:5]]
    rec["ll_polls_per_col"] = round(st.tolist()[5] / max(n - 2, 1), 2)
    # per-workgroup clock marks (100 MHz) at every 64th column: skew of the p stores across
    # workgroups vs the time from the LAST store to each workgroup's exchange done
    nwg = int(k.harp_sytrd_ll_workgroups(n))
    ns = (n - 2 + 63) // 64
    trc = torch.zeros(ns * nwg * 4, dtype=torch.int64, device=dev)
    k.harp_sytrd_ll_trace(trc.data_ptr())
    E.sytrd_ll(C)
    torch.cuda.synchronize()
    k.harp_sytrd_ll_trace(None)
    trc = trc.view(ns, nwg, 4).cpu().double() * 10.0  # ns
    rows = []
    for si in range(ns):
        kk = si * 64
        live = [b for b in range(nwg) if 8 * b + 7 >= kk + 1 or b == nwg - 1]
        t = trc[si, live]
        if float(t[:, 0].min()) <= 0:
            continue
        st_ = t[:, 1]
        rows.append({"k": kk, "wgs": len(live), "start_skew_ns": round(float(t[:, 0].max() - t[:, 0].min())),
                     "store_skew_ns": round(float(st_.max() - st_.min())),
                     "last_store_to_done_ns": [round(float((t[:, 2] - st_.max()).min())),
                                               round(float((t[:, 2] - st_.max()).median())),
                                               round(float((t[:, 2] - st_.max()).max()))],
                     "s1_ns_median": round(float((t[:, 1] - t[:, 0]).median())),
                     "s4_ns_median": round(float((t[:, 3] - t[:, 2]).median())),
                     "step_ns": round(float(t[:, 3].max() - t[:, 0].min()))})
    rec["ll_trace"] = rows

    def fused():
        nb = int(k.harp_eig_workgroups(n, E.NB_DEFAULT))
        A = C.clone()
        ws = torch.zeros(int(k.harp_eig_ws_ints()), dtype=torch.int32, device=dev)
        wsd = torch.zeros(3 * n + 4, dtype=torch.float64, device=dev)
        dd = torch.empty(n, dtype=torch.float64, device=dev)
        ee = torch.zeros(n, dtype=torch.float64, device=dev)
        V = torch.zeros((n, n), dtype=torch.float64, device=dev)
        t = torch.zeros(n, dtype=torch.float64, device=dev)
        E._lib.check(k.harp_sytrd_fused(A.data_ptr(), n, n, dd.data_ptr(), ee.data_ptr(), V.data_ptr(),
                                        t.data_ptr(), nb, ws.data_ptr(), wsd.data_ptr(), E._lib.stream_ptr(dev)),
                     "sytrd_fused")

    rec["sytrd_fused_ms"] = timed(fused)
    lam, Z = E.eigh_tridiag(d, e[:n - 1])
    rec["dc_ms"] = timed(lambda: E.eigh_tridiag(d, e[:n - 1]))
    st = (ctypes.c_longlong * 9)()
    E._lib.check(k.harp_dc_prep_stamps(ctypes.cast(st, ctypes.c_void_p)), "dc_prep_stamps")
    rec["dc_top_prep_cycles"] = [st[i + 1] - st[i] for i in range(8)]
    sw = (ctypes.c_longlong * 9)()
    E._lib.check(k.harp_dc_wave_stamps(ctypes.cast(sw, ctypes.c_void_p)), "dc_wave_stamps")
    # block 0 of the last one-wave merge level: stage, sort+deflate, scatter, secular, Loewner, U, GEMM
    rec["dc_wave_phase_cycles"] = [sw[i + 1] - sw[i] for i in range(7)]
    rec["dc_wave_secular_max_iters"] = sw[8]
    rec["back_transform_ms"] = timed(lambda: E.back_transform(Vt, tau, Z))
    rec["wy_factor_ms"] = timed(lambda: E.wy_factor(Vt, tau))
    Vm, Mt = E.wy_factor(Vt, tau)
    rec["apply_wy_ms"] = timed(lambda: E.apply_wy(Vm, Mt, Z))
    rec["wy_vs_back_transform"] = float((E.apply_wy(Vm, Mt, Z) - E.back_transform(Vt, tau, Z)).abs().max())
    for var in ("ll", "fused"):
        E.VARIANT = var
        rec[f"eigh_{var}_ms"] = timed(lambda: E.eigh(C))
        rec[f"eigvalsh_{var}_ms"] = timed(lambda: E.eigvalsh(C))
    E.VARIANT = "ll"
    rec["rocsolver_eigh_ms"] = timed(lambda: torch.linalg.eigh(C))
    lam, V = E.eigh(C)
    ref = torch.linalg.eigvalsh(C)
    I = torch.eye(n, dtype=torch.float64, device=dev)
    rec["eigval_err"] = float((lam - ref).abs().max())
    rec["orth_err"] = float((V.t() @ V - I).abs().max())
    rec["residual"] = float((C @ V - V * lam).abs().max()) / float(torch.linalg.matrix_norm(C, 2))
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
