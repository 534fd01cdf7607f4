"""Fused MLP epilogues (csrc/nn.hip) vs the fp64 torch formulation of the same gradient."""
import pytest
import torch

from harp_amd.models.nn import MLP
from harp_amd.ops import nn as NO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("act", ["sigmoid", "tanh", "relu"])
@pytest.mark.parametrize("sizes,b", [([20, 32, 10], 64), ([784, 300, 100, 10], 257), ([5, 7, 3000], 33)])
def test_native_gradient_matches_fp64(cuda, act, sizes, b):
    net = MLP(sizes, activation=act, device=cuda, seed=4)
    ref = MLP(sizes, activation=act, device="cpu", dtype=torch.float64, seed=4)
    ref.flat.copy_(net.flat.double().cpu())
    g = torch.Generator().manual_seed(1)
    X = torch.randn(b, sizes[0], generator=g)
    y = torch.randint(0, sizes[-1], (b,), generator=g)
    Y = torch.nn.functional.one_hot(y, sizes[-1])
    assert net._native(X.to(cuda))
    got = net.gradient(X.to(cuda), Y.to(cuda)).double().cpu()
    want = ref.gradient(X.double(), Y)
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-6), (got - want).abs().max()
    loss_ref = float(-(torch.log_softmax(ref.forward(X.double())[-2] @ ref.params[-2].t() + ref.params[-1], 1)
                       .gather(1, y[:, None])).sum())
    assert float(net.last_loss) == pytest.approx(loss_ref, rel=1e-4)


def test_softmax_xent_kernel(cuda):
    z = torch.randn(100, 37, device=cuda)
    lab = torch.randint(0, 37, (100,), device=cuda, dtype=torch.int32)
    delta = torch.empty_like(z)
    db = torch.zeros(37, device=cuda)
    loss = NO.softmax_xent(z, lab, 0.5, delta, db)
    p = torch.softmax(z.double(), 1)
    want = (p - torch.nn.functional.one_hot(lab.long(), 37)) * 0.5
    assert torch.allclose(delta.double(), want, atol=1e-6)
    assert torch.allclose(db.double(), want.sum(0), atol=1e-5)
    assert float(loss) == pytest.approx(float(-torch.log(p.gather(1, lab.long()[:, None])).sum()), rel=1e-5)
