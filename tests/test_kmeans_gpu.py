"""GPU numerics of the K-means HIP kernels vs a plain PyTorch fp32 reference of the same
op on the same (bf16-rounded) operands. Runs only on a MI355X box."""
import pytest
import torch

from harp_amd.ops import kmeans as K

pytestmark = pytest.mark.gpu


def _ref_assign(X, c_bf, d):
    x = X[:, :d].float()
    cn = (c_bf.double() ** 2).sum(1)
    dist = cn[None, :] - 2.0 * (x.double() @ c_bf.double().t())
    lab = dist.argmin(1)
    best = dist.gather(1, lab[:, None])[:, 0]
    return lab, dist, best + (x.double() ** 2).sum(1)


def test_generate_points_layout(cuda):
    X = K.generate_points(1000, 37, 2.0, 5.0, seed=3, device=cuda)
    dp = K.padded_dim(37)
    assert X.shape == (1000, dp) and X.dtype == torch.bfloat16
    assert bool((X[:, 37:41] == 1).all()) and bool((X[:, 41:] == 0).all())
    v = X[:, :37].float()
    assert v.min() >= 2.0 and v.max() <= 5.0 and abs(v.mean().item() - 3.5) < 0.05
    X2 = K.generate_points(1000, 37, 2.0, 5.0, seed=3, device=cuda)
    assert torch.equal(X, X2)  # counter-based generator: deterministic


@pytest.mark.parametrize("accumulate", ["bucket", "atomic"])
@pytest.mark.parametrize("variant", [4, 13, 14, 15])
@pytest.mark.parametrize("n,d,k", [(5000, 100, 300), (777, 10, 10), (4099, 31, 129), (2048, 127, 1000), (1500, 250, 200),
                                   (200000, 100, 2000)])
def test_assign_matches_torch(cuda, variant, n, d, k, accumulate):
    torch.manual_seed(0)
    x = torch.rand(n, d, device=cuda) * 1000
    X = K.pack_points(x, cuda)
    c = torch.rand(k, d, device=cuda) * 1000
    op = K.prepare(c, X.shape[1])
    sums = torch.zeros((K.padded_k(k), X.shape[1]), dtype=torch.float32, device=cuda)
    lab, obj = K.assign(X, op, sums=sums, variant=variant, accumulate=accumulate)
    torch.cuda.synchronize()
    c_bf = c.to(torch.bfloat16).float()
    rlab, dist, rbest = _ref_assign(X, c_bf, d)
    lab = lab.long()
    assert int(lab.min()) >= 0 and int(lab.max()) < k
    # near-ties may resolve differently; the chosen centroid must be (near-)optimal
    chosen = dist.gather(1, lab[:, None])[:, 0]
    best = dist.gather(1, rlab[:, None])[:, 0]
    scale = (X[:, :d].double() ** 2).sum(1) + (c_bf.double() ** 2).sum(1).max()
    assert bool(((chosen - best) <= 1e-5 * scale).all())
    assert (lab == rlab).float().mean() > 0.99
    assert abs(obj.item() - rbest.sum().item()) <= 1e-4 * abs(rbest.sum().item()) + 1e-3
    # accumulated (sum x, count) rows match index_add with the kernel's own labels
    ref = torch.zeros_like(sums, dtype=torch.float64)
    ref[:, : d + 1].index_add_(0, lab, X[:, : d + 1].double())
    # columns d+1.. of X are 1.0 as well; the bucket path sums them (== count), compare (x, count)
    assert torch.allclose(sums[:, : d + 1].double(), ref[:, : d + 1], rtol=1e-5, atol=1e-2)
    assert int(sums[:, d].sum().item()) == n


def test_prepare_and_normalize(cuda):
    k, d = 300, 100
    c = torch.rand(k, d, device=cuda) * 10
    op = K.prepare(c, K.padded_dim(d))
    c_bf = c.to(torch.bfloat16).float()
    assert torch.equal(op.Cm2[:k, :d].float(), -2 * c_bf)
    assert bool((op.Cm2[k:, :d] == 0).all()) and bool((op.cn[k:] > 1e37).all())
    folded = op.Cm2[:k, d + 1:d + 4].double().sum(1)  # hi + mid + lo == ||c||^2 (~24 bits)
    assert torch.allclose(folded, op.cn[:k].double(), rtol=1e-6)
    assert bool((op.Cm2[:, d] == 0).all()) and bool((op.Cm2[:, d + 4:] == 0).all())
    assert torch.allclose(op.cn[:k], (c_bf.double() ** 2).sum(1).float(), rtol=1e-6)
    sums = torch.rand(k, K.padded_dim(d), device=cuda) * 100
    sums[::7, d] = 0  # empty clusters keep their centroid
    sums[1::7, d] = 3.0
    cn = c.clone()
    K.normalize(sums, cn, d)
    ref = c.clone()
    m = sums[:, d] > 0
    ref[m] = sums[m, :d] / sums[m, d:d + 1]
    assert torch.allclose(cn, ref, rtol=1e-6)


def test_kmeans_model_gpu_matches_cpu(cuda):
    from harp_amd.models.kmeans import KMeansConfig, run_kmeans
    from harp_amd.parallel.comm import Communicator

    g = torch.Generator().manual_seed(1)
    x = torch.rand(20000, 20, generator=g) * 10
    c0 = torch.rand(16, 20, generator=g) * 10
    cfg = KMeansConfig(num_points=20000, num_centroids=16, dim=20, iterations=20, strategy="allreduce")
    gpu = run_kmeans(Communicator(None, cuda), cfg, points=x, init_centroids=c0)
    cpu = run_kmeans(Communicator(None, torch.device("cpu")), cfg, points=x, init_centroids=c0)
    md_g = torch.cdist(x, gpu["centroids"]).min(1).values.mean()
    md_c = torch.cdist(x, cpu["centroids"]).min(1).values.mean()
    assert abs(md_g - md_c) / md_c < 5e-3, (md_g, md_c)
    obj = gpu["objective"]
    assert obj[-1] <= obj[0]


def test_bucket_labels_and_rowsum(cuda):
    from harp_amd.ops import segment

    n, K, dp = 300000, 5000, 112
    lab = torch.randint(0, K, (n,), device=cuda, dtype=torch.int32)
    lab[:100000] = 7  # one heavy bucket (skew)
    lab[lab == 11] = 12  # an empty bucket
    perm, start = segment.bucket_labels(lab, K)
    cnt = torch.bincount(lab.long(), minlength=K)
    assert torch.equal((start[1:] - start[:-1]).long(), cnt)
    assert torch.equal(torch.sort(perm.long()).values, torch.arange(n, device=cuda))
    assert torch.equal(lab[perm.long()].long(), torch.repeat_interleave(torch.arange(K, device=cuda), cnt))
    X = (torch.rand(n, dp, device=cuda) * 10).to(torch.bfloat16)
    out = torch.zeros(K, dp, device=cuda)
    segment.bucket_rowsum(X, perm, start, out)
    ref = torch.zeros(K, dp, dtype=torch.float64, device=cuda).index_add_(0, lab.long(), X.double())
    assert torch.allclose(out.double(), ref, rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("dp,slice_", [(264, 1024), (512, 1024), (1000, 1024), (1024, 1024), (2048, 1024), (1000, 256)])
def test_bucket_rowsum_wide_rows(cuda, monkeypatch, dp, slice_):
    """Rows wider than 256 columns: the one-pass wave-per-slot gather-sum (slices of up to
    1024 columns) and the former 256-column slices both equal an fp64 index_add, with a
    heavy bucket, an empty one, and a row stride wider than the row."""
    from harp_amd.ops import segment

    monkeypatch.setattr(segment, "SUM_SLICE", slice_)
    n, K = 40000, 700
    lab = torch.randint(0, K, (n,), device=cuda, dtype=torch.int32)
    lab[:9000] = 3
    lab[lab == 5] = 6
    perm, start = segment.bucket_labels(lab, K)
    X = (torch.rand(n, dp + 8, device=cuda) * 10).to(torch.bfloat16)[:, :dp]
    out = torch.zeros(K, dp, device=cuda)
    segment.bucket_rowsum(X, perm, start, out)
    ref = torch.zeros(K, dp, dtype=torch.float64, device=cuda).index_add_(0, lab.long(), X.double())
    assert torch.allclose(out.double(), ref, rtol=1e-5, atol=1e-2)


def test_kmeans_hip_graph_iterations_match_eager(cuda):
    """Iterations replayed from HIP graphs give the same centroids as eager launches."""
    from harp_amd.models.kmeans import KMeansCollectiveMapper, KMeansConfig
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    out = {}
    for graph in (False, True):
        cfg = KMeansConfig(num_points=50000, num_centroids=300, dim=100, iterations=6, strategy="allreduce",
                           objective_every=0, graph=graph)
        m = KMeansCollectiveMapper(Communicator(None, cuda), cfg)
        m.init_model(KeyValReader([]))
        for it in range(cfg.iterations):
            m.step(it)
        torch.cuda.synchronize()
        out[graph] = m.c[:300].clone()
    assert torch.allclose(out[True], out[False], rtol=1e-5, atol=1e-3), (out[True] - out[False]).abs().max()


@pytest.mark.parametrize("chunks", [2, 3])
def test_chunked_side_stream_pipeline_matches_single_pass(cuda, monkeypatch, chunks):
    """HARP_KMEANS_CHUNKS: assign of chunk i+1 overlaps bucket + gather-sum of chunk i on a
    side stream; labels, objective, min distances and (x, count) sums equal the one-pass run."""
    n, d, k = 1024 * 256 * 3 + 777, 100, 500
    torch.manual_seed(1)
    X = K.pack_points(torch.rand(n, d, device=cuda) * 1000, cuda)
    op = K.prepare(torch.rand(k, d, device=cuda) * 1000, X.shape[1])
    out = {}
    for c in (1, chunks):
        monkeypatch.setenv("HARP_KMEANS_CHUNKS", str(c))
        sums = torch.zeros((K.padded_k(k), X.shape[1]), dtype=torch.float32, device=cuda)
        md = torch.empty(n, dtype=torch.float32, device=cuda)
        lab, obj = K.assign(X, op, sums=sums, min_dist=md)
        torch.cuda.synchronize()
        out[c] = (lab.clone(), obj.item(), md.clone(), sums)
    assert K.pipeline_chunks(n, 1024) == chunks
    a, b = out[1], out[chunks]
    assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2])
    assert b[1] == pytest.approx(a[1], rel=1e-9)
    assert torch.allclose(a[3], b[3], rtol=1e-5, atol=1e-2)
    assert int(b[3][:, d].sum().item()) == n


def test_row_stride_view_matches_contiguous(cuda):
    """GPU points live at a 256-B row stride (ops.kmeans.row_stride) as a [n, dp] view; the
    assign and the bucketed gather-sum read that layout exactly like a dense copy."""
    n, d, k = 50_000, 100, 700
    torch.manual_seed(7)
    X = K.pack_points(torch.rand(n, d, device=cuda) * 1000, cuda)
    assert X.shape[1] == K.padded_dim(d) and X.stride(0) == K.row_stride(X.shape[1]) == 128
    Xd = X.contiguous()
    assert Xd.stride(0) == X.shape[1]
    op = K.prepare(torch.rand(k, d, device=cuda) * 1000, X.shape[1])
    out = []
    for A in (X, Xd):
        sums = torch.zeros((K.padded_k(k), X.shape[1]), dtype=torch.float32, device=cuda)
        lab, obj = K.assign(A, op, sums=sums)
        torch.cuda.synchronize()
        out.append((lab.clone(), obj.item(), sums))
    assert torch.equal(out[0][0], out[1][0]) and out[0][1] == pytest.approx(out[1][1], rel=1e-12)
    assert torch.allclose(out[0][2], out[1][2], rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("n,d,k", [(5000, 300, 300), (3000, 512, 1000), (4099, 1000, 257), (2000, 253, 100),
                                   (1000, 2000, 64), (70000, 1000, 1000)])
def test_assign_wide_rows_matches_torch(cuda, n, d, k):
    """d > 252 (padded rows wider than 256): the feature-staged kernel against a torch fp64
    argmin on the same bf16 operands (the reference has no d limit,
    CenCalcTask.java:67-100)."""
    torch.manual_seed(1)
    x = torch.rand(n, d, device=cuda) * 1000
    X = K.pack_points(x, cuda)
    assert X.shape[1] > 256 and X.shape[1] % 64 == 0
    c = torch.rand(k, d, device=cuda) * 1000
    op = K.prepare(c, X.shape[1])
    sums = torch.zeros((K.padded_k(k), X.shape[1]), dtype=torch.float32, device=cuda)
    md = torch.empty(n, dtype=torch.float32, device=cuda)
    lab, obj = K.assign(X, op, sums=sums, min_dist=md)
    torch.cuda.synchronize()
    c_bf = c.to(torch.bfloat16).float()
    rlab, dist, rbest = _ref_assign(X, c_bf, d)
    lab = lab.long()
    assert int(lab.min()) >= 0 and int(lab.max()) < k
    chosen = dist.gather(1, lab[:, None])[:, 0]
    best = dist.gather(1, rlab[:, None])[:, 0]
    scale = (X[:, :d].double() ** 2).sum(1) + (c_bf.double() ** 2).sum(1).max()
    assert bool(((chosen - best) <= 1e-5 * scale).all())
    assert (lab == rlab).float().mean() > 0.99
    assert abs(obj.item() - rbest.sum().item()) <= 1e-4 * abs(rbest.sum().item()) + 1e-3
    assert torch.allclose(md.double(), chosen + (X[:, :d].double() ** 2).sum(1), rtol=1e-4, atol=1.0)
    ref = torch.zeros_like(sums, dtype=torch.float64)
    ref[:, : d + 1].index_add_(0, lab, X[:, : d + 1].double())
    assert torch.allclose(sums[:, : d + 1].double(), ref[:, : d + 1], rtol=1e-5, atol=1e-1)
    assert int(sums[:, d].sum().item()) == n


def test_kmeans_model_wide_d(cuda):
    """The model runs natively at d = 1000 (no NotImplementedError, objective decreasing)."""
    from harp_amd.models.kmeans import KMeansConfig, run_kmeans
    from harp_amd.parallel.comm import Communicator

    cfg = KMeansConfig(num_points=20000, num_centroids=100, dim=1000, iterations=3, strategy="allreduce")
    res = run_kmeans(Communicator(None, cuda), cfg)
    obj = res["objective"]
    assert len(obj) == 3 and obj[2] <= obj[0]


@pytest.mark.parametrize("strategy", ["allreduce", "regroup_allgather", "bcast_reduce", "push_pull", "rotation"])
def test_kmeans_strategies_wide_d_agree(cuda, strategy):
    """Every sync strategy runs the wide-row path (d = 300 > 256 padded features) and gives
    the allreduce trajectory (one worker: the strategies differ only in their collectives)."""
    from harp_amd.models.kmeans import KMeansConfig, run_kmeans
    from harp_amd.parallel.comm import Communicator

    def obj(st):
        cfg = KMeansConfig(num_points=12000, num_centroids=70, dim=300, iterations=3, strategy=st, seed=5)
        return run_kmeans(Communicator(None, cuda), cfg)["objective"]

    ref, got = obj("allreduce"), obj(strategy)
    assert len(got) == 3 and got[2] <= got[0]
    assert all(abs(a - b) <= 1e-4 * abs(a) for a, b in zip(ref, got)), (ref, got)


@pytest.mark.parametrize("variant", [1, 3, 5, 6])
def test_assign_wide_variants_agree(cuda, variant, monkeypatch):
    """Every wide-row tiling gives the labels of the torch fp64 argmin (near-ties aside)."""
    monkeypatch.setattr(K, "WIDE_VARIANT", variant)
    torch.manual_seed(2)
    n, d, k = 9000, 700, 600
    x = torch.rand(n, d, device=cuda) * 1000
    X = K.pack_points(x, cuda)
    c = torch.rand(k, d, device=cuda) * 1000
    op = K.prepare(c, X.shape[1])
    lab, obj = K.assign(X, op)
    c_bf = c.to(torch.bfloat16).float()
    rlab, dist, rbest = _ref_assign(X, c_bf, d)
    lab = lab.long()
    chosen = dist.gather(1, lab[:, None])[:, 0]
    best = dist.gather(1, rlab[:, None])[:, 0]
    scale = (X[:, :d].double() ** 2).sum(1) + (c_bf.double() ** 2).sum(1).max()
    assert bool(((chosen - best) <= 1e-5 * scale).all())
    assert (lab == rlab).float().mean() > 0.99
    assert abs(obj.item() - rbest.sum().item()) <= 1e-4 * abs(rbest.sum().item()) + 1e-3
