"""MX-fp8 tile weight gradient (config 5) on the GPU.

The reference has no fp8 (fine_tune.py:955-959), so the bar is the build's bf16 tile path:
* smt_mx_quant_cols is bit-identical to the oracle's restatement of the documented format
  (oracle.mx_quant_cols: OCP MX, e4m3 elements, one non-saturating e8m0 exponent per 32 rows);
* smt_tile_wgrad_mx equals the fp64 product of the dequantised operands to the MFMA's accumulation
  precision (relative Frobenius <= ACC_TOL = 1e-4; measured 1.5e-5 at T = 2048: the scaled f8
  MFMA's internal sums are coarser than the bf16 MFMA's, ~1e-6; exact on integer data that MX
  represents exactly);
* against the fp64 truth of the bf16 operands, the MX tile gradients stay within MX_TOL (relative
  Frobenius, per tile), the quantisation error of e4m3 with 32-row groups: about 4-5 % on Gaussian
  operands, where the bf16 path is at ~1e-3.
"""
import pytest
import torch

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import _hip

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
MX_TOL = 6e-2
ACC_TOL = 1e-4


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _blocks(ids):
    return torch.tensor(ids, dtype=torch.int32, device=DEV)


@pytest.mark.parametrize("T", [64, 300, 2048])
def test_mx_quant_bit_identical_to_oracle(T):
    gen = torch.Generator().manual_seed(T)
    x = (torch.randn(T, 1024, generator=gen) * torch.exp(3 * torch.randn(T, 1024, generator=gen))).bfloat16()
    x[:40, 300:310] = 0.0                                           # all-zero groups
    x[5, 700] = 448.0                                               # exponent boundaries
    x[37, 701] = float(torch.tensor(448.0).bfloat16().float() * 1.0078125)
    x[70 % T, 702] = 1e-40                                          # bf16 subnormal
    blocks = [3, 0, 2]
    got = _hip.mx_quant_cols(x.to(DEV), _blocks(blocks))
    q, s = ref.mx_quant_cols(x, blocks)
    assert got.ldq == q.shape[1] * 64 and got.T == T
    assert torch.equal(got.scales.cpu(), s)
    assert torch.equal(got.q.cpu(), q)


def test_mx_wgrad_layout_exact():
    """Small integers are exact in MX e4m3 at any exponent and every partial sum is exact in fp32,
    so a fragment / scale / C-layout mistake shows as a hard mismatch (asymmetric operands)."""
    T = 320
    gen = torch.Generator().manual_seed(2)
    g = torch.randint(-7, 8, (T, 768), generator=gen).float()
    x = torch.randint(-7, 8, (T, 512), generator=gen).float()
    g[:, 256:512] *= 4.0                                            # other exponents per block / group
    x[64:96] *= 0.25
    g, x = g.bfloat16(), x.bfloat16()
    tiles = [(1, 0), (2, 1), (0, 1), (1, 1)]
    rbs, cbs = [0, 1, 2], [0, 1]
    qg = _hip.mx_quant_cols(g.to(DEV), _blocks(rbs))
    qx = _hip.mx_quant_cols(x.to(DEV), _blocks(cbs))
    table = _hip.tile_table([(rbs.index(r), cbs.index(c)) for r, c in tiles], DEV)
    out = torch.empty(len(tiles) * 256, 256, dtype=torch.float32, device=DEV)
    _hip.tile_wgrad_mx(qg, qx, table, out)
    truth = ref.tile_grads_fp64(g.unsqueeze(0), x.unsqueeze(0), tiles)
    assert torch.equal(out.cpu().double(), truth)


@pytest.mark.parametrize("T,n_out,n_in,tiles", [
    (2048, 1024, 4096, [(3, 15), (0, 0), (2, 7), (3, 0), (1, 8)]),     # split-K slabs + reduce
    (300, 512, 768, [(0, 0), (1, 2), (0, 1)]),                        # ragged T
    (192, 4096, 2048, [(r, c) for r in range(16) for c in range(8)]),   # n >= 128: S == 1, direct store
])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_mx_wgrad_vs_dequantised_fp64(T, n_out, n_in, tiles, out_dtype):
    gen = torch.Generator().manual_seed(T + len(tiles))
    g = (torch.randn(T, n_out, generator=gen) * 1e-2).bfloat16()
    x = torch.randn(T, n_in, generator=gen).bfloat16()
    rbs = sorted({r for r, _ in tiles})
    cbs = sorted({c for _, c in tiles})
    qg = _hip.mx_quant_cols(g.to(DEV), _blocks(rbs))
    qx = _hip.mx_quant_cols(x.to(DEV), _blocks(cbs))
    packed = [(rbs.index(r), cbs.index(c)) for r, c in tiles]
    out = torch.empty(len(tiles) * 256, 256, dtype=out_dtype, device=DEV)
    _hip.tile_wgrad_mx(qg, qx, _hip.tile_table(packed, DEV), out, order=_hip.order_table(tiles, DEV))
    want = ref.mx_tile_grads_fp64(qg.q.cpu(), qg.scales.cpu(), qx.q.cpu(), qx.scales.cpu(), packed)
    assert _rel(out, want) < (ACC_TOL if out_dtype == torch.float32 else 2e-3)
    # and the quantisation error against the bf16 operands' truth stays within the stated bound
    truth = ref.tile_grads_fp64(g.unsqueeze(0), x.unsqueeze(0), tiles)
    assert _rel(out, truth) < MX_TOL


def test_mx_wgrad_accumulate_and_empty():
    T = 256
    g = torch.randn(T, 512).bfloat16()
    x = torch.randn(T, 256).bfloat16()
    qg = _hip.mx_quant_cols(g.to(DEV), _blocks([1]))
    qx = _hip.mx_quant_cols(x.to(DEV), _blocks([0]))
    table = _hip.tile_table([(0, 0)], DEV)
    base = torch.randn(256, 256, device=DEV)
    out = base.clone()
    _hip.tile_wgrad_mx(qg, qx, table, out, accumulate=True)
    want = ref.mx_tile_grads_fp64(qg.q.cpu(), qg.scales.cpu(), qx.q.cpu(), qx.scales.cpu(), [(0, 0)]) + base.double().cpu()
    assert _rel(out, want) < ACC_TOL
    e = _hip.mx_quant_cols(torch.empty(0, 256, dtype=torch.bfloat16, device=DEV), _blocks([0]))
    z = torch.full((256, 256), 3.0, device=DEV)
    _hip.tile_wgrad_mx(e, e, table, z)
    assert z.abs().max().item() == 0.0


# LLaMA-3-8B module shapes at the bench's T = B*S = 32768
SHAPES = {"q_proj": (4096, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}


@pytest.mark.parametrize("module,n", [("q_proj", 8), ("gate_proj", 67), ("down_proj", 436)])
def test_mx_wgrad_bench_geometry(module, n):
    out_f, in_f = SHAPES[module]
    T = 32768
    gen = torch.Generator(device=DEV).manual_seed(n)
    x = torch.randn(T, in_f, generator=gen, device=DEV).bfloat16()
    go = (torch.randn(T, out_f, generator=gen, device=DEV) * 1e-2).bfloat16()
    rb, cb = out_f // 256, in_f // 256
    flat = torch.randperm(rb * cb, generator=torch.Generator().manual_seed(n))[:n].tolist()
    tiles = [(f // cb, f % cb) for f in flat]
    rbs = sorted({r for r, _ in tiles})
    cbs = sorted({c for _, c in tiles})
    qg = _hip.mx_quant_cols(go, _blocks(rbs))
    qx = _hip.mx_quant_cols(x, _blocks(cbs))
    packed = [(rbs.index(r), cbs.index(c)) for r, c in tiles]
    out = torch.empty(n * 256, 256, dtype=torch.float32, device=DEV)
    _hip.tile_wgrad_mx(qg, qx, _hip.tile_table(packed, DEV), out, order=_hip.order_table(tiles, DEV))
    torch.cuda.synchronize()
    for i in torch.randperm(n, generator=torch.Generator().manual_seed(3))[:4].tolist():
        r, c = tiles[i]
        truth = go[:, r * 256:(r + 1) * 256].double().t() @ x[:, c * 256:(c + 1) * 256].double()
        a = ref.mx_dequant(qg.q[rbs.index(r):rbs.index(r) + 1].cpu(), qg.scales[rbs.index(r):rbs.index(r) + 1].cpu())[0]
        b = ref.mx_dequant(qx.q[cbs.index(c):cbs.index(c) + 1].cpu(), qx.scales[cbs.index(c):cbs.index(c) + 1].cpu())[0]
        got = out[i * 256:(i + 1) * 256]
        assert _rel(got, a.t() @ b) < ACC_TOL, (module, n, i)
        assert _rel(got, truth) < MX_TOL, (module, n, i)
