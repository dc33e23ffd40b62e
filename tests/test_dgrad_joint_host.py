"""dgrad.py's deferred joint data-gradient product on the host (CPU tensors, fp32): three consumers
of one input whose output gradients are column slices of one buffer and whose weight operands are
column slices of one transposed copy (engine.FrozenLinearFn, as the engine wires q/k/v) -> one joint
product, equal to the fp64 sum; separate gradient tensors, a consumer left out of the backward, and
slices at mismatched offsets take the per-consumer products."""
import torch

from sparse_matrix_tuning_amd import dgrad
from sparse_matrix_tuning_amd.engine import FrozenLinearFn

OUTS = (64, 16, 16)
IN = 32


def _setup(seed=0):
    g = torch.Generator().manual_seed(seed)
    ws = [torch.randn(o, IN, generator=g) for o in OUTS]
    wt = torch.cat([w.t() for w in ws], 1).contiguous()               # joint transposed copy [in, C]
    offs = [0, OUTS[0], OUTS[0] + OUTS[1]]
    wts = [wt[:, o:o + w.shape[0]] for o, w in zip(offs, ws)]
    x = torch.randn(3, 8, IN, generator=g)
    J = torch.randn(3, 8, sum(OUTS), generator=g)
    gs = [J[..., o:o + w.shape[0]] for o, w in zip(offs, ws)]
    return ws, wts, x, gs


def _run(ws, wts, x, grads, keep=(0, 1, 2)):
    xi = x.clone().requires_grad_(True)
    outs = [FrozenLinearFn.apply(xi, w, t, None) for w, t in zip(ws, wts)]
    torch.autograd.backward([outs[i] for i in keep], [grads[i] for i in keep])
    return xi.grad


def _truth(ws, gs, keep=(0, 1, 2)):
    return sum(gs[i].double() @ ws[i].double() for i in keep)


def _rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


def test_joint_product_when_slices_tile_both_buffers():
    ws, wts, x, gs = _setup()
    n0 = dgrad.JOINT_PRODUCTS
    got = _run(ws, wts, x, gs)
    assert dgrad.JOINT_PRODUCTS == n0 + 1
    assert _rel(got, _truth(ws, gs)) < 1e-5


def test_per_consumer_products_otherwise():
    ws, wts, x, gs = _setup(1)
    n0 = dgrad.JOINT_PRODUCTS
    assert _rel(_run(ws, wts, x, [g.contiguous() for g in gs]), _truth(ws, gs)) < 1e-5   # separate tensors
    assert _rel(_run(ws, wts, x, gs, keep=(0, 2)), _truth(ws, gs, (0, 2))) < 1e-5       # k left out
    # gradient slices in another column order than the transposed copy's: no joint product
    J2 = torch.cat([gs[1], gs[0], gs[2]], -1)
    swapped = [J2[..., OUTS[1]:OUTS[1] + OUTS[0]], J2[..., :OUTS[1]], J2[..., OUTS[0] + OUTS[1]:]]
    assert _rel(_run(ws, wts, x, swapped), _truth(ws, swapped)) < 1e-5
    assert dgrad.JOINT_PRODUCTS == n0
