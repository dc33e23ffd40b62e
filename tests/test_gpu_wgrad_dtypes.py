"""Tile weight gradients in the reference's other dtypes (fine_tune.py:955-959 --dtype fp16 | fp32;
deepspeed_helpers.py:53-61): linearZ then runs on fp16 or fp32 tensors and smt.py:397-404 rounds each
per-sample partial to that dtype. fp16 goes through the 16-bit kernels with the f16 MFMA, fp32 through
wgrad_f32_kernel (exact f32 products, v_mfma_f32_32x32x2_f32).

Tolerances: against the oracle's restatement in the same dtype, fp32 <= 1e-5 and fp16
(reference rounding) <= 1e-3 relative (Frobenius); single rounding against fp64 truth <= max(1e-3,
1.1 x the restatement's own error)."""
import pytest
import torch
from torch import nn

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import _hip
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _operands(B, S, out_f, in_f, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, S, in_f, generator=g).to(dtype)
    go = (torch.randn(B, S, out_f, generator=g) * 0.5).to(dtype)
    return x, go


def _tiles(out_f, in_f, n, seed):
    g = torch.Generator().manual_seed(seed)
    pool = [(r, c) for r in range(out_f // 256) for c in range(in_f // 256)]
    return [pool[i] for i in torch.randperm(len(pool), generator=g)[:n].tolist()]


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("n_tiles", [3, 20])                      # quarter / full-tile 16-bit kernels
@pytest.mark.parametrize("seq", [None, 512])                       # single / reference rounding
def test_tile_wgrad_dtype_vs_restatement(dtype, n_tiles, seq):
    B, S, out_f, in_f = 4, 512, 2048, 1536
    x, go = _operands(B, S, out_f, in_f, dtype, seed=n_tiles + (seq or 0))
    tiles = _tiles(out_f, in_f, n_tiles, seed=n_tiles)
    table = _hip.tile_table(tiles, DEV)
    out = torch.empty(n_tiles * 256, 256, dtype=dtype, device=DEV)
    _hip.tile_wgrad(go.reshape(-1, out_f).to(DEV), x.reshape(-1, in_f).to(DEV), table, out, seq_len=seq)
    restated = ref.linearz_tile_grads(go, x, tiles)               # per-sample partials in `dtype`
    truth = ref.tile_grads_fp64(go, x, tiles)
    e_ref, e_truth, e_alg = _rel(out, restated), _rel(out, truth), _rel(restated, truth)
    print(f"{dtype} tiles {n_tiles} seq {seq}: vs restatement {e_ref:.2e}, vs fp64 {e_truth:.2e} "
          f"(restatement vs fp64 {e_alg:.2e})")
    if dtype == torch.float32:
        assert e_ref <= 1e-5 and e_truth <= 1e-5
    elif seq:
        assert e_ref <= 1e-3
    else:
        assert e_truth <= max(1e-3, 1.1 * e_alg)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_tile_wgrad_dtype_accumulate_and_fp32_out(dtype):
    B, S, out_f, in_f = 2, 256, 1024, 1024
    x, go = _operands(B, S, out_f, in_f, dtype, seed=7)
    tiles = [(0, 1), (3, 3), (2, 0)]
    table = _hip.tile_table(tiles, DEV)
    g2, x2 = go.reshape(-1, out_f).to(DEV), x.reshape(-1, in_f).to(DEV)
    once = torch.empty(3 * 256, 256, dtype=torch.float32, device=DEV)
    _hip.tile_wgrad(g2, x2, table, once)
    twice = once.clone()
    _hip.tile_wgrad(g2, x2, table, twice, accumulate=True)
    assert torch.equal(twice, 2 * once)
    assert _rel(once, ref.tile_grads_fp64(go, x, tiles)) <= (1e-5 if dtype == torch.float32 else 2e-3)


def test_tile_wgrad_dtype_combinations_refused():
    g2 = torch.zeros(256, 256, dtype=torch.float32, device=DEV)
    table = _hip.tile_table([(0, 0)], DEV)
    with pytest.raises((ValueError, NotImplementedError, RuntimeError)):
        _hip.tile_wgrad(g2, g2, table, torch.empty(256, 256, dtype=torch.bfloat16, device=DEV))
    with pytest.raises((ValueError, NotImplementedError, RuntimeError)):
        _hip.tile_wgrad(g2, g2.half(), table, torch.empty(256, 256, dtype=torch.float32, device=DEV))


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_module_autograd_in_dtype(dtype):
    """The drop-in module with the model in fp16 / fp32 (DeepSpeed drives the step: autograd .grad in
    the model dtype): forward, grad_input and tile gradients against the restatement."""
    B, S, out_f, in_f = 4, 384, 1024, 768
    x, go = _operands(B, S, out_f, in_f, dtype, seed=11)
    W = (torch.randn(out_f, in_f, generator=torch.Generator().manual_seed(3)) * 0.02).to(dtype)
    tiles = [(1, 2), (0, 0), (3, 1)]
    mod = smt.LinearLayer_MatrixSparsity(nn.Parameter(W.to(DEV)), index_list=tiles)
    assert mod.selected_weight.dtype == dtype
    xd = x.to(DEV).requires_grad_(True)
    y = mod(xd)
    y.backward(go.to(DEV))
    gi_ref, gw_ref = ref.linearz_backward(go, x, W, tiles)
    assert _rel(y, ref.linearz_forward(x, W)) <= (1e-5 if dtype == torch.float32 else 2e-3)
    assert _rel(xd.grad, gi_ref) <= (1e-5 if dtype == torch.float32 else 2e-3)
    gw = mod.selected_weight.grad
    assert gw.dtype == dtype
    assert _rel(gw, gw_ref) <= (1e-5 if dtype == torch.float32 else 1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_reference_fwbw_demo_geometry(dtype):
    """smt.py:865-903 (fwbwTest): linearZ.apply(input [16, 2560, 2560], selected_weight, [(0, 0), (0, 1)],
    weight [2560, 2560]) with loss = (y - input).sum(), the demo's fp32 (and the bf16 / fp16 runs).
    Here the tiles and the input require gradients (the demo's don't, so its backward trains nothing):
    y and grad_input against torch on the same operands, the tile gradients against the restatement
    (smt.py:382-404). W itself gets no gradient (linearZ returns None for it), as in the demo."""
    torch.manual_seed(865)
    x = torch.randn(16, 2560, 2560).to(dtype)
    W = torch.randn(2560, 2560).to(dtype)
    tiles = [(0, 0), (0, 1)]
    Wd = W.to(DEV).requires_grad_(True)
    sel = torch.randn(256 * 2, 256).to(dtype).to(DEV).requires_grad_(True)
    xd = x.to(DEV).requires_grad_(True)
    y = smt.linearZ.apply(xd, sel, tiles, Wd)
    (y - xd).sum().backward()
    assert Wd.grad is None
    assert torch.equal(y, torch.matmul(xd.detach(), Wd.detach().t()))
    g = torch.ones(16, 2560, 2560, dtype=dtype)
    # dL/dx = 1 @ W - 1 in every row (the GEMM's own summation order: compared within rounding)
    ones_w = torch.matmul(torch.ones(1, 2560, dtype=torch.float64, device=DEV), Wd.detach().double())
    assert _rel(xd.grad[0, :7], (ones_w - 1).expand(7, 2560)) <= (1e-5 if dtype == torch.float32 else 1e-2)
    assert torch.equal(xd.grad[0], xd.grad[15])
    restated = ref.linearz_tile_grads(g, x, tiles)
    e = _rel(sel.grad, restated)
    print(f"{dtype}: tile grads vs the restatement {e:.2e}")
    assert e <= (1e-5 if dtype == torch.float32 else 1e-3)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_channel_module_in_dtype(dtype):
    """LinearLayer_ChannelSparsity (smt.py:185-296) with the model in fp16 / fp32: the partial input
    gather (an fp32 column is a 16-bit column pair), the channel gradient through the tile kernels of
    that dtype, against the restatement (oracle.linearchannel_*) and fp64."""
    torch.manual_seed(31)
    W = (torch.randn(512, 512) * 0.05).to(dtype)
    idx = [3, 100, 7, 511, 256]
    x = torch.randn(2, 96, 512).to(dtype)
    g = torch.randn(2, 96, 512).to(dtype)
    mod = smt.LinearLayer_ChannelSparsity(nn.Parameter(W.to(DEV)), index_list=idx)
    assert mod.selected_weight.dtype == dtype
    xd = x.to(DEV).requires_grad_(True)
    y = mod(xd)
    y.backward(g.to(DEV))
    y_ref, partial = ref.linearchannel_forward(x, W, idx)
    gi_ref, gw_ref = ref.linearchannel_backward(g, partial, W)
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    assert _rel(y, y_ref) <= tol and _rel(xd.grad, gi_ref) <= tol
    truth = ref.channel_grads_fp64(g, x, idx)
    gw = mod.selected_weight.grad
    assert gw.dtype == dtype and gw.shape == (len(idx), 512)
    assert _rel(gw, truth) <= max(tol, 1.1 * _rel(gw_ref, truth)), (_rel(gw, truth), _rel(gw_ref, truth))
