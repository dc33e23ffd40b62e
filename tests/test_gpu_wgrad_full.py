"""Tile weight gradient at the bench geometry: T = B*S = 16*2048 = 32768 rows,
the LLaMA-3-8B module shapes, 4-436 tiles per call (the quarter-tile kernel at <= 8 tiles, the
full-tile kernel's slab path S > 1 and direct path S == 1), bf16 and fp32 outputs, accumulation,
and linearZ's packed-column input.

Truth is fp64 on the GPU from the same bf16 operands. The reference's own result (smt.py:397-404:
one bf16 matmul per sample, each ``[256, 256]`` partial rounded to bf16, then ``sum(dim=0)``) is
computed the same way it runs on a GPU (torch bf16 matmul + sum), for the same sampled tiles.
Bar: relative Frobenius error vs truth <= max(1e-3, 1.1 x the reference's own error);
fp32 output <= 1e-5.
"""
import pytest
import torch

from sparse_matrix_tuning_amd import _hip

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
B, S = 16, 2048
T = B * S
SHAPES = {"q_proj": (4096, 4096), "k_proj": (1024, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}
SAMPLES = 6


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def _tiles(out_f, in_f, n, seed):
    rb, cb = out_f // 256, in_f // 256
    g = torch.Generator().manual_seed(seed)
    flat = torch.randperm(rb * cb, generator=g)[:n].tolist()
    return [(f // cb, f % cb) for f in flat]


def _operands(out_f, in_f, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(T, in_f, generator=g, device=DEV).bfloat16()
    go = (torch.randn(T, out_f, generator=g, device=DEV) * 1e-2).bfloat16()
    return go, x


def _truth(go, x, r, c):
    return go[:, r * 256:(r + 1) * 256].double().t() @ x[:, c * 256:(c + 1) * 256].double()


def _reference(go, x, r, c):
    """smt.py:397-404 on the GPU: per-sample bf16 partials, then the batch sum."""
    g3 = go.view(B, S, -1)[:, :, r * 256:(r + 1) * 256]
    x3 = x.view(B, S, -1)[:, :, c * 256:(c + 1) * 256]
    return torch.sum(torch.matmul(g3.permute(0, 2, 1), x3), dim=0)


@pytest.mark.parametrize("module,n", [("k_proj", 4), ("gate_proj", 8),          # quarter-tile kernel
                                      ("q_proj", 27), ("q_proj", 256), ("k_proj", 27), ("k_proj", 64),
                                      ("gate_proj", 67), ("gate_proj", 436), ("down_proj", 67), ("down_proj", 436)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_tile_wgrad_bench_geometry(module, n, out_dtype):
    out_f, in_f = SHAPES[module]
    go, x = _operands(out_f, in_f, seed=n)
    tiles = _tiles(out_f, in_f, n, seed=n)
    table = _hip.tile_table(tiles, DEV)
    order = _hip.order_table(tiles, DEV)
    out = torch.empty(n * 256, 256, dtype=out_dtype, device=DEV)
    _hip.tile_wgrad(go, x, table, out, order=order)
    torch.cuda.synchronize()
    pick = torch.randperm(n, generator=torch.Generator().manual_seed(7))[:SAMPLES].tolist()
    for i in pick:
        r, c = tiles[i]
        truth = _truth(go, x, r, c)
        got = out[i * 256:(i + 1) * 256]
        err = _rel(got, truth)
        if out_dtype == torch.float32:
            assert err < 1e-5, (module, n, i, err)
        else:
            ref_err = _rel(_reference(go, x, r, c), truth)
            assert err <= max(1e-3, 1.1 * ref_err), (module, n, i, err, ref_err)


def test_tile_wgrad_bench_geometry_accumulate():
    out_f, in_f = SHAPES["gate_proj"]
    go, x = _operands(out_f, in_f, seed=3)
    tiles = _tiles(out_f, in_f, 67, seed=3)
    table = _hip.tile_table(tiles, DEV)
    base = torch.randn(67 * 256, 256, device=DEV)
    out = base.clone()
    _hip.tile_wgrad(go, x, table, out, accumulate=True)
    torch.cuda.synchronize()
    for i in (0, 33, 66):
        r, c = tiles[i]
        want = _truth(go, x, r, c) + base[i * 256:(i + 1) * 256].double()
        assert _rel(out[i * 256:(i + 1) * 256], want) < 1e-5


def test_linearz_packed_input_at_bench_geometry():
    """down_proj with 14 tiles over 4 of its 56 column blocks: linearZ saves only those blocks
    (smt_colblock_gather) and the tile gradients equal the kernel over the full input bit for bit."""
    from sparse_matrix_tuning_amd.smt import smt
    out_f, in_f = SHAPES["down_proj"]
    go, x = _operands(out_f, in_f, seed=11)
    cols = [3, 17, 40, 55]
    tiles = [(r, cols[r % 4]) for r in range(14)]
    W = torch.nn.Parameter((torch.randn(out_f, in_f, device=DEV) * 0.02).bfloat16())
    mod = smt.LinearLayer_MatrixSparsity(W, index_list=tiles)
    xi = x.view(B, S, in_f).detach().requires_grad_(False)
    y = mod(xi)
    assert y.grad_fn.packed
    y.backward(go.view(B, S, out_f))
    direct = torch.empty(14 * 256, 256, dtype=torch.bfloat16, device=DEV)
    _hip.tile_wgrad(go, x, _hip.tile_table(tiles, DEV), direct)
    assert torch.equal(mod.selected_weight.grad, direct)
    for i in (0, 7, 13):
        r, c = tiles[i]
        truth = _truth(go, x, r, c)
        ref_err = _rel(_reference(go, x, r, c), truth)
        assert _rel(direct[i * 256:(i + 1) * 256], truth) <= max(1e-3, 1.1 * ref_err)
