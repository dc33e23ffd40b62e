"""GPU parity of every HIP kernel against the CPU oracle (through the C ABI, ctypes)."""
import math

import numpy as np
import pytest
import torch

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import _hip

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(1234)


# ---------------------------------------------------------------- wgrad (smt.py:382-404)
WGRAD_CASES = [
    # (B, S, out, in, tiles)
    (2, 128, 512, 768, [(0, 0), (1, 2), (0, 1)]),
    (1, 2048, 1024, 4096, [(3, 15), (0, 0), (2, 7), (3, 0), (1, 8)]),
    (3, 100, 256, 512, [(0, 1)]),                    # ragged T = 300 (not a multiple of 64)
    (4, 512, 768, 512, [(r, c) for r in range(3) for c in range(2)]),   # every tile of the matrix
    (1, 192, 4096, 2048, [(r, c) for r in range(16) for c in range(8)] + [(0, 0), (15, 7)]),  # n >= 128: S == 1
]


@pytest.mark.parametrize("B,S,out_f,in_f,tiles", WGRAD_CASES)
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_tile_wgrad_vs_fp64(B, S, out_f, in_f, tiles, out_dtype):
    x = torch.randn(B, S, in_f).bfloat16()
    g = torch.randn(B, S, out_f).bfloat16()
    truth = ref.tile_grads_fp64(g, x, tiles)
    rc = _hip.tile_table(tiles, torch.device(DEV))
    out = torch.empty(len(tiles) * 256, 256, dtype=out_dtype, device=DEV)
    _hip.tile_wgrad(g.reshape(-1, out_f).to(DEV), x.reshape(-1, in_f).to(DEV), rc, out)
    torch.cuda.synchronize()
    err = _rel(out, truth)
    if out_dtype == torch.float32:
        assert err < 1e-5, err          # fp32 accumulation of exact bf16 products
    else:
        # one bf16 rounding of the output: <= 2^-9 relative per element (RNE), ~1.2e-3 Frobenius
        assert err < 2e-3, err
        # and never worse than the reference's own per-sample-rounded result (smt.py:397-404)
        _gi, ref_gw = ref.linearz_backward(g, x, torch.zeros(out_f, in_f, dtype=torch.bfloat16), tiles)
        assert err <= max(1e-3, 1.1 * _rel(ref_gw, truth))


@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_tile_wgrad_direct_epilogue_accumulate(out_dtype):
    # 130 tiles -> S == 1: the partial kernel writes (and accumulates into) the output itself
    tiles = [(r, c) for r in range(13) for c in range(10)]
    x = torch.randn(2, 48, 2560).bfloat16()
    g = torch.randn(2, 48, 3328).bfloat16()
    out = torch.full((len(tiles) * 256, 256), 0.5, dtype=out_dtype, device=DEV)
    _hip.tile_wgrad(g.reshape(-1, 3328).to(DEV), x.reshape(-1, 2560).to(DEV), _hip.tile_table(tiles, torch.device(DEV)),
                    out, accumulate=True)
    truth = ref.tile_grads_fp64(g, x, tiles) + 0.5
    assert _rel(out, truth) < (1e-5 if out_dtype == torch.float32 else 2e-3)


def test_tile_wgrad_accumulate_and_empty():
    x = torch.randn(2, 64, 512).bfloat16()
    g = torch.randn(2, 64, 256).bfloat16()
    tiles = [(0, 1), (0, 0)]
    rc = _hip.tile_table(tiles, torch.device(DEV))
    out = torch.ones(2 * 256, 256, dtype=torch.float32, device=DEV)
    _hip.tile_wgrad(g.reshape(-1, 256).to(DEV), x.reshape(-1, 512).to(DEV), rc, out, accumulate=True)
    truth = ref.tile_grads_fp64(g, x, tiles) + 1.0
    assert _rel(out, truth) < 1e-5
    # T = 0 -> zeros (an empty batch contributes nothing)
    z = torch.full((2 * 256, 256), 7.0, device=DEV)
    _hip.tile_wgrad(torch.empty(0, 256, dtype=torch.bfloat16, device=DEV),
                    torch.empty(0, 512, dtype=torch.bfloat16, device=DEV), rc, z)
    assert z.abs().max().item() == 0.0


def test_tile_wgrad_mfma_layout_exact():
    # integer-valued operands: every product and partial sum is exact in fp32, so any
    # fragment / C-layout mistake shows as a hard mismatch (asymmetric data, A = shifted identity)
    T = 256
    g = torch.zeros(T, 512)
    x = torch.zeros(T, 256)
    for t in range(T):
        g[t, 256 + (t * 7) % 256] = 1.0 + (t % 3)
        x[t, t % 256] = float((t % 5) - 2)
    tiles = [(1, 0)]
    truth = ref.tile_grads_fp64(g.unsqueeze(0), x.unsqueeze(0), tiles)
    out = torch.empty(256, 256, dtype=torch.float32, device=DEV)
    _hip.tile_wgrad(g.bfloat16().to(DEV), x.bfloat16().to(DEV), _hip.tile_table(tiles, torch.device(DEV)), out)
    assert torch.equal(out.cpu().double(), truth)


# ---------------------------------------------------------------- gather / scatter (smt.py:317-341)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gather_scatter_bit_exact(dtype):
    W = torch.randn(1024, 768).to(dtype)
    tiles = [(3, 2), (0, 0), (1, 1), (3, 0)]
    rc = _hip.tile_table(tiles, torch.device(DEV))
    Wd = W.to(DEV)
    out = torch.empty(len(tiles) * 256, 256, dtype=dtype, device=DEV)
    _hip.tile_gather(Wd, rc, out)
    assert torch.equal(out.cpu(), ref.gather_tiles(W, tiles))
    new = torch.randn_like(out)
    _hip.tile_scatter(Wd, rc, new)
    W2 = W.clone()
    ref.writeback_tiles(W2, new.cpu(), tiles)
    assert torch.equal(Wd.cpu(), W2)


def test_tile_scatter_transposed_bit_exact():
    W = torch.randn(1024, 768).bfloat16()
    tiles = [(3, 2), (0, 0), (1, 1)]
    Wt = W.t().contiguous().to(DEV)
    new = torch.randn(len(tiles) * 256, 256).bfloat16()
    descs = _hip.tile_descs([(Wt, r, c, i * 65536) for i, (r, c) in enumerate(tiles)], torch.device(DEV))
    _hip.tile_scatter_t(descs, len(tiles), new.to(DEV))
    W2 = W.clone()
    ref.writeback_tiles(W2, new, tiles)
    assert torch.equal(Wt.cpu(), W2.t())


# ---------------------------------------------------------------- warm-up accumulation (fine_tune.py:731-741)
def test_grad_accumulate_bit_exact():
    shapes = [(512, 256), (256, 768), (33, 17), (4096,)]
    grads = [torch.randn(s).bfloat16() for s in shapes]
    grads2 = [torch.randn(s).bfloat16() for s in shapes]
    accs = [torch.empty(s, dtype=torch.float32, device=DEV) for s in shapes]
    _hip.grad_accumulate([(a, g.to(DEV)) for a, g in zip(accs, grads)], assign=True)
    _hip.grad_accumulate([(a, g.to(DEV)) for a, g in zip(accs, grads2)], assign=False)
    for a, g1, g2 in zip(accs, grads, grads2):
        want = g1.to(torch.float32)
        want += g2.to(torch.float32)
        assert torch.equal(a.cpu(), want)


# ---------------------------------------------------------------- block scores (smt_helper.py:67-78, 233-251)
@pytest.mark.parametrize("strategy", ["mean_abs", "abs_mean", "L1", "L2"])
def test_block_scores_match_fp64_oracle(strategy):
    from sparse_matrix_tuning_amd.smt import ranking
    from sparse_matrix_tuning_amd.smt.smt_helper import finalize_scores
    g = torch.randn(768, 1024) * torch.rand(768, 1024)
    g[:256, :256] = 0.0                                             # an exact (all-zero) block
    code = _hip.__dict__["SCORE_" + {"mean_abs": "MEAN_ABS", "abs_mean": "ABS_MEAN", "L1": "L1", "L2": "L2"}[strategy]]
    raw = _hip.block_scores([g.to(DEV)], [(3, 4)], code)[0].cpu()
    want = ref.block_raw_fp64(g, 3, 4, strategy)
    # fp64 sums of the same fp32 terms in another order: equal to ~1e-15 relative
    assert torch.allclose(raw, want, rtol=1e-13, atol=0)
    got = finalize_scores(raw.numpy(), strategy).reshape(3, 4)
    assert (got == ref.block_stat_fp64(g, 3, 4, strategy).numpy()).all()
    # the reference's fp32 ATen values lie inside the intervals the ranking uses
    _nom, lo, hi = ranking.block_intervals(raw.numpy(), strategy)
    lit = ref.block_stat(g, 3, 4, strategy).numpy().reshape(-1)
    assert np.all(lo <= lit) and np.all(lit <= hi)
    assert lo[0] == hi[0] == 0.0


# ---------------------------------------------------------------- sq-norm + AdamW (DeepSpeed FusedAdam, external)
def test_sq_norm():
    x = torch.randn(1_000_003)
    out = _hip.sq_norm(x.to(DEV))
    assert math.isclose(out.item(), (x.double() ** 2).sum().item(), rel_tol=1e-12)


@pytest.mark.parametrize("tiled", [False, True])
def test_adamw_matches_oracle(tiled):
    n_tiles = 3
    n = n_tiles * 65536
    p0 = torch.randn(n)
    g = torch.randn(n) * 0.01
    lr, betas, eps, wd = 1e-3, (0.9, 0.95), 1e-8, 0.01
    master = p0.clone().to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    param = p0.bfloat16().to(DEV)
    rp, rm, rv = p0.clone(), torch.zeros(n), torch.zeros(n)
    W = torch.zeros(512, 512, dtype=torch.bfloat16, device=DEV)
    tile_list = [(1, 0), (0, 1), (1, 1)]
    descs = _hip.tile_descs([(W, r, c, i * 65536) for i, (r, c) in enumerate(tile_list)], torch.device(DEV)) if tiled else None
    gd = g.to(DEV)
    norm = _hip.sq_norm(gd)
    max_norm = 1.0
    for step in range(1, 4):
        args = _hip.AdamWArgs(lr=lr, beta1=betas[0], beta2=betas[1], eps=eps, weight_decay=wd,
                              bias_correction1=1 - betas[0] ** step, bias_correction2=1 - betas[1] ** step,
                              max_grad_norm=max_norm, grad_scale=1.0, mode=_hip.ADAM_DEEPSPEED, grad_dtype=0)
        _hip.adamw_step(gd, master, m, v, param, args, tiles=descs, n_tiles=n_tiles, grad_sq_norm=norm)
        coef = ref.clip_coef([g], max_norm)
        ref.fused_adam_step(rp, g * coef, rm, rv, step, lr, betas, eps, wd)
    torch.cuda.synchronize()
    assert _rel(master, rp) < 1e-6
    assert torch.equal(param.cpu(), master.cpu().bfloat16())
    if tiled:
        tiles_now = ref.gather_tiles(W.cpu(), tile_list)
        assert torch.equal(tiles_now.reshape(-1), param.cpu())


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
def test_adamw_multi_equals_per_tensor_steps(gdt):
    """One smt_adamw_multi launch over ragged tensors (tails of 1-2047 elements, a 1-element
    tensor, one spanning many workgroups) equals smt_adamw_step per tensor bit for bit."""
    gen = torch.Generator().manual_seed(4)
    sizes = [1, 7, 2048, 2049, 65536 * 3 + 5, 4096, 13]
    states = []
    for n in sizes:
        p0 = torch.randn(n, generator=gen)
        g = (torch.randn(n, generator=gen) * 0.01).to(gdt).to(DEV)
        a = [p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV), p0.bfloat16().to(DEV)]
        b = [t.clone() for t in a]
        states.append((g, a, b))
    norm = torch.tensor([4.0], dtype=torch.float64, device=DEV)
    for step in range(1, 4):
        args = lambda: _hip.AdamWArgs(lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.01,
                                      bias_correction1=1 - 0.9 ** step, bias_correction2=1 - 0.95 ** step,
                                      max_grad_norm=1.0, grad_scale=0.5, mode=_hip.ADAM_DEEPSPEED, grad_dtype=0)
        _hip.adamw_multi([(g, *a) for g, a, _b in states], args(), grad_sq_norm=norm)
        for g, _a, b in states:
            _hip.adamw_step(g, *b, args(), grad_sq_norm=norm)
    torch.cuda.synchronize()
    for g, a, b in states:
        for x, y in zip(a, b):
            assert torch.equal(x, y)


# ---------------------------------------------------------------- packed input column blocks (smt.py:351-358)
@pytest.mark.parametrize("T,in_f,cbs", [(300, 1024, [3, 0]), (4096, 14336, [55, 7, 8, 30]), (1, 512, [1])])
def test_colblock_gather_bit_exact(T, in_f, cbs):
    x = torch.randn(T, in_f).bfloat16().to(DEV)
    out = _hip.colblock_gather(x, torch.tensor(cbs, dtype=torch.int32, device=DEV))
    want = torch.stack([x[:, c * 256:(c + 1) * 256] for c in cbs])      # block-major [n_cb, T, 256]
    assert out.shape == (len(cbs), T, 256) and torch.equal(out, want)


def test_linearz_packed_input_grads_bit_identical():
    """A module whose tiles touch few column blocks saves only those blocks; its tile gradients are
    bit-identical to the grouped kernel over the full input, and to the unpacked path."""
    from sparse_matrix_tuning_amd.smt import smt
    B, S, out_f, in_f = 2, 160, 512, 2048              # 8 column blocks
    tiles = [(1, 6), (0, 2), (1, 2)]                    # 2 distinct column blocks -> packed
    W = torch.nn.Parameter((torch.randn(out_f, in_f) * 0.02).bfloat16().to(DEV))
    mod = smt.LinearLayer_MatrixSparsity(W, index_list=tiles)
    x = torch.randn(B, S, in_f).bfloat16().to(DEV).requires_grad_(True)
    g = torch.randn(B, S, out_f).bfloat16().to(DEV)
    y = mod(x)
    assert y.grad_fn.packed
    y.backward(g)
    direct = torch.empty(len(tiles) * 256, 256, dtype=torch.bfloat16, device=DEV)
    seq = S if smt.wgrad_rounding() == "reference" else None     # the module's rounding (smt.py:397-404)
    _hip.tile_wgrad(g.reshape(-1, out_f), x.detach().reshape(-1, in_f), _hip.tile_table(tiles, torch.device(DEV)), direct,
                    seq_len=seq)
    assert torch.equal(mod.selected_weight.grad, direct)
    assert torch.equal(x.grad, torch.matmul(g, W.detach()))
    wide = [(0, c) for c in range(5)]                   # 5 of 8 blocks -> the input itself is saved
    mod2 = smt.LinearLayer_MatrixSparsity(W, index_list=wide)
    y2 = mod2(x.detach())
    assert not y2.grad_fn.packed
