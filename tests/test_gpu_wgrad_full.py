"""Tile weight gradient at the bench geometry: T = B*S = 16*2048 = 32768 rows,
the LLaMA-3-8B module shapes, 4-436 tiles per call (the quarter-tile kernel at <= 8 tiles, the
full-tile kernel's slab path S > 1 and direct path S == 1), bf16 and fp32 outputs, accumulation,
and linearZ's packed-column input.

Truth is fp64 on the GPU from the same bf16 operands. The reference's own result (smt.py:397-404:
one bf16 matmul per sample, each ``[256, 256]`` partial rounded to bf16, then ``sum(dim=0)``) is
computed the same way it runs on a GPU (torch bf16 matmul + sum), for the same sampled tiles.
Bar: relative Frobenius error vs truth <= max(1e-3, 1.1 x the reference's own error);
fp32 output <= 1e-5.

Direct parity with the reference algorithm: the CPU restatement
``oracle.linearz_tile_grads`` (smt.py:382-404) on the same operands at B = 16, S = 2048 against
(a) the reference-rounding mode (the default since round 5) (``smt_tile_wgrad_batch_seq``: per-sample partials rounded to
bf16, then the batch sum): <= 1e-3 relative (north_star's bf16 tolerance), and
(b) the opt-in single-rounding mode: the direct difference printed and <= 1.5 x the reference's own
error vs fp64 truth (the two differ by the reference's per-sample rounding, ~2.4e-3 at B = 16).
"""
import os

import pytest
import torch

from oracle import smt_oracle as ref
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
    seq = S if smt.wgrad_rounding() == "reference" else None     # the module's rounding (smt.py:397-404)
    _hip.tile_wgrad(go, x, _hip.tile_table(tiles, DEV), direct, seq_len=seq)
    assert torch.equal(mod.selected_weight.grad, direct)
    for i in (0, 7, 13):
        r, c = tiles[i]
        truth = _truth(go, x, r, c)
        ref_err = _rel(_reference(go, x, r, c), truth)
        assert _rel(direct[i * 256:(i + 1) * 256], truth) <= max(1e-3, 1.1 * ref_err)


def _restatement(go, x, sel):
    """oracle.linearz_tile_grads (CPU, the reference's own arithmetic) and fp64 truth for the tiles
    ``sel`` of [T, *] operands, viewed as linearZ's [B, S, *] input."""
    gs = torch.cat([go[:, r * 256:(r + 1) * 256] for r, _c in sel], 1).view(B, S, -1).cpu()
    xs = torch.cat([x[:, c * 256:(c + 1) * 256] for _r, c in sel], 1).view(B, S, -1).cpu()
    diag = [(k, k) for k in range(len(sel))]
    return ref.linearz_tile_grads(gs, xs, diag), ref.tile_grads_fp64(gs, xs, diag)


@pytest.mark.parametrize("module,n", [("k_proj", 4), ("down_proj", 8), ("q_proj", 27), ("q_proj", 54),
                                      ("gate_proj", 67), ("down_proj", 436)])
def test_reference_rounding_vs_restatement_at_bench_geometry(module, n):
    out_f, in_f = SHAPES[module]
    go, x = _operands(out_f, in_f, seed=100 + n)
    tiles = _tiles(out_f, in_f, n, seed=n)
    table, order = _hip.tile_table(tiles, DEV), _hip.order_table(tiles, DEV)
    rr = {dt: torch.empty(n * 256, 256, dtype=dt, device=DEV) for dt in (torch.bfloat16, torch.float32)}
    for dt, o in rr.items():
        _hip.tile_wgrad(go, x, table, o, order=order, seq_len=S)
    single = torch.empty(n * 256, 256, dtype=torch.bfloat16, device=DEV)
    _hip.tile_wgrad(go, x, table, single, order=order)
    # accumulate: autograd's bf16 add of the reference's bf16 gradient into an existing .grad
    base = (torch.randn(n * 256, 256, device=DEV) * 1e-2).bfloat16()
    acc = base.clone()
    _hip.tile_wgrad(go, x, table, acc, order=order, seq_len=S, accumulate=True)
    torch.cuda.synchronize()
    # the fp32 output holds the same bf16 values exactly
    assert torch.equal(rr[torch.float32], rr[torch.bfloat16].float())
    assert torch.equal(acc, (base.float() + rr[torch.bfloat16].float()).bfloat16())

    pick = torch.randperm(n, generator=torch.Generator().manual_seed(7))[:4].tolist()
    want, truth = _restatement(go, x, [tiles[i] for i in pick])
    for k, i in enumerate(pick):
        w, t = want[k * 256:(k + 1) * 256], truth[k * 256:(k + 1) * 256]
        d_rr = _rel(rr[torch.bfloat16][i * 256:(i + 1) * 256].cpu(), w)
        d_single = _rel(single[i * 256:(i + 1) * 256].cpu(), w)
        ref_err = _rel(w, t)
        print(f"\n{module} n={n} tile {tiles[i]}: vs oracle.linearz_tile_grads: reference-rounding mode "
              f"{d_rr:.2e}, single-rounding mode {d_single:.2e}; reference vs fp64 truth {ref_err:.2e}")
        assert d_rr <= 1e-3, (module, n, i, d_rr)
        assert d_single <= 1.5 * ref_err, (module, n, i, d_single, ref_err)


def _slab_worker(tmp_path, name, **env):
    """tests/wgrad_slab_worker.py in a child process with the given library switches (read once per
    process) -> its {case: tile gradients}."""
    import subprocess
    import sys
    path = str(tmp_path / f"{name}.pt")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "wgrad_slab_worker.py"), path], cwd=root,
                       env=dict(os.environ, PYTHONPATH=root, **env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(path, weights_only=True)


def test_reference_rounding_bf16_slabs_bit_identical(tmp_path):
    """With one workgroup per sample (kps == 1) the kernels round each sample's partial to bf16 in
    their epilogue and write half-size slabs: bit-identical to rounding them in the reduce from fp32
    slabs (SMT_WGRAD_SLAB16=0, a child process: the library reads the switch once)."""
    from tests.wgrad_slab_worker import cases
    mine = cases()
    theirs = _slab_worker(tmp_path, "fp32_slabs", SMT_WGRAD_SLAB16="0")
    assert sorted(mine) == sorted(theirs)
    for k in mine:
        assert torch.equal(mine[k], theirs[k]), k


def test_reference_rounding_batch_vs_restatement():
    """The engine's launch: three modules in one batch with the reference rounding
    (smt_tile_wgrad_batch_seq), 54 tiles (the bench's typical launch: 864 workgroups), one module
    accumulating; sampled tiles against oracle.linearz_tile_grads."""
    items, checks, lists = [], [], []
    for k, (name, n) in enumerate((("q_proj", 18), ("k_proj", 12), ("gate_proj", 24))):
        out_f, in_f = SHAPES[name]
        go, x = _operands(out_f, in_f, seed=40 + k)
        tiles = _tiles(out_f, in_f, n, seed=50 + k)
        acc = k == 1
        base = (torch.randn(n * 256, 256, device=DEV) * 1e-2).bfloat16()
        out = base.clone() if acc else torch.empty(n * 256, 256, dtype=torch.bfloat16, device=DEV)
        items.append((go, x, out, acc))
        lists.append(tiles)
        checks.append((go, x, tiles, out, base, acc))
    tab, order = _hip.wgrad_batch_table(lists, DEV)
    _hip.tile_wgrad_batch(items, tab, order, seq_len=S)
    torch.cuda.synchronize()
    for go, x, tiles, out, base, acc in checks:
        pick = [0, len(tiles) - 1]
        want, _truth_ = _restatement(go, x, [tiles[i] for i in pick])
        for k, i in enumerate(pick):
            w = want[k * 256:(k + 1) * 256]
            if acc:
                w = (base[i * 256:(i + 1) * 256].cpu().float() + w.float()).bfloat16()
            d = _rel(out[i * 256:(i + 1) * 256].cpu(), w)
            assert d <= 1e-3, (tiles[i], acc, d)


@pytest.mark.parametrize("n", [12, 60])
def test_reference_rounding_odd_sample_count(n):
    """Five samples of 640 rows: 12 tiles cut each sample into pieces (kps > 1, fp32 slabs, the
    reduce's per-sample loop), 60 tiles give one workgroup per sample (bf16 slabs, the reduce's
    unrolled sample loop with a remainder); sampled tiles vs oracle.linearz_tile_grads."""
    Bo, So = 5, 640
    out_f, in_f = SHAPES["q_proj"]
    g = torch.Generator(device=DEV).manual_seed(7 + n)
    x = torch.randn(Bo * So, in_f, generator=g, device=DEV).bfloat16()
    go = (torch.randn(Bo * So, out_f, generator=g, device=DEV) * 1e-2).bfloat16()
    tiles = _tiles(out_f, in_f, n, seed=70 + n)
    out = torch.empty(n * 256, 256, dtype=torch.bfloat16, device=DEV)
    _hip.tile_wgrad(go, x, _hip.tile_table(tiles, DEV), out, order=_hip.order_table(tiles, DEV), seq_len=So)
    torch.cuda.synchronize()
    pick = [0, n // 2, n - 1]
    sel = [tiles[i] for i in pick]
    gs = torch.cat([go[:, r * 256:(r + 1) * 256] for r, _c in sel], 1).view(Bo, So, -1).cpu()
    xs = torch.cat([x[:, c * 256:(c + 1) * 256] for _r, c in sel], 1).view(Bo, So, -1).cpu()
    want = ref.linearz_tile_grads(gs, xs, [(k, k) for k in range(len(sel))])
    for k, i in enumerate(pick):
        d = _rel(out[i * 256:(i + 1) * 256].cpu(), want[k * 256:(k + 1) * 256])
        assert d <= 1e-3, (tiles[i], d)


def test_reference_rounding_rejects_partial_samples():
    go, x = _operands(1024, 1024, seed=1)
    table = _hip.tile_table([(0, 0)], DEV)
    out = torch.empty(256, 256, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(ValueError):
        _hip.tile_wgrad(go, x, table, out, seq_len=3000)


@pytest.mark.parametrize("seq,n", [(100, 3), (100, 20), (1377, 3), (1377, 20), (33, 64)])
def test_ragged_sequence_lengths(seq, n):
    """Batches padded to a length that is not a multiple of the 32-row LDS-DMA stage (the collator
    pads to the batch's longest sample, helper.py:194-204): every sample's span starts off a stage
    boundary. Quarter-tile (3 tiles) and full-tile (20, 64) kernels, reference rounding vs
    oracle.linearz_tile_grads (<= 1e-3), and the single rounding (ragged T) vs fp64 truth."""
    Bo = 3
    out_f, in_f = 2048, 2048
    To = Bo * seq
    g = torch.Generator(device=DEV).manual_seed(seq + n)
    x = torch.randn(To, in_f, generator=g, device=DEV).bfloat16()
    go = (torch.randn(To, out_f, generator=g, device=DEV) * 1e-2).bfloat16()
    tiles = _tiles(out_f, in_f, n, seed=seq * 7 + n)
    table = _hip.tile_table(tiles, DEV)
    order = _hip.order_table(tiles, DEV)
    ref_out = torch.empty(n * 256, 256, dtype=torch.bfloat16, device=DEV)
    _hip.tile_wgrad(go, x, table, ref_out, order=order, seq_len=seq)
    single = torch.empty(n * 256, 256, dtype=torch.float32, device=DEV)
    _hip.tile_wgrad(go, x, table, single, order=order)
    torch.cuda.synchronize()
    pick = sorted({0, n // 2, n - 1})
    sel = [tiles[i] for i in pick]
    gs = torch.cat([go[:, r * 256:(r + 1) * 256] for r, _c in sel], 1).view(Bo, seq, -1).cpu()
    xs = torch.cat([x[:, c * 256:(c + 1) * 256] for _r, c in sel], 1).view(Bo, seq, -1).cpu()
    want = ref.linearz_tile_grads(gs, xs, [(k, k) for k in range(len(sel))])
    for k, i in enumerate(pick):
        r, c = tiles[i]
        assert _rel(ref_out[i * 256:(i + 1) * 256].cpu(), want[k * 256:(k + 1) * 256]) <= 1e-3, (tiles[i], "reference")
        assert _rel(single[i * 256:(i + 1) * 256], _truth(go, x, r, c)) <= 1e-5, (tiles[i], "single")


def test_register_staged_kernel_past_32bit_buffer_offsets():
    """A split whose rows span >= 2 GiB of an operand (chunk * ld * 2 >= 2^31: here 80000 rows of
    the 14336-wide down_proj input in one split) cannot use the LDS-DMA kernels' 32-bit buffer
    offsets; the launch takes the register-staged kernel, which addresses with 64 bits. Single
    rounding (fp32 out) vs fp64 truth <= 1e-5, reference rounding (one 80000-row sample, bf16 out)
    vs oracle.linearz_tile_grads <= 1e-3."""
    To, (out_f, in_f), n = 80000, SHAPES["down_proj"], 436
    g = torch.Generator(device=DEV).manual_seed(80)
    x = torch.randn(To, in_f, generator=g, device=DEV).bfloat16()
    go = (torch.randn(To, out_f, generator=g, device=DEV) * 1e-2).bfloat16()
    tiles = _tiles(out_f, in_f, n, seed=81)
    table, order = _hip.tile_table(tiles, DEV), _hip.order_table(tiles, DEV)
    single = torch.empty(n * 256, 256, dtype=torch.float32, device=DEV)
    _hip.tile_wgrad(go, x, table, single, order=order)
    refr = torch.empty(n * 256, 256, dtype=torch.bfloat16, device=DEV)
    _hip.tile_wgrad(go, x, table, refr, order=order, seq_len=To)
    torch.cuda.synchronize()
    pick = [0, n // 2, n - 1]
    sel = [tiles[i] for i in pick]
    gs = torch.cat([go[:, r * 256:(r + 1) * 256] for r, _c in sel], 1).view(1, To, -1).cpu()
    xs = torch.cat([x[:, c * 256:(c + 1) * 256] for _r, c in sel], 1).view(1, To, -1).cpu()
    want = ref.linearz_tile_grads(gs, xs, [(k, k) for k in range(len(sel))])
    for k, i in enumerate(pick):
        r, c = tiles[i]
        assert _rel(single[i * 256:(i + 1) * 256], _truth(go, x, r, c)) <= 1e-5, tiles[i]
        assert _rel(refr[i * 256:(i + 1) * 256].cpu(), want[k * 256:(k + 1) * 256]) <= 1e-3, tiles[i]
