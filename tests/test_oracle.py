"""Pin the CPU oracle: KAT-1 / KAT-2, dense-autograd identities, committed goldens."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import smt_oracle as ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_kat1_block_selection():
    """smt_helper.py:310-319 with the current signature."""
    grads = {
        ('gate_proj', 1): torch.zeros(11008, 4096),
        ('up_proj', 1): torch.zeros(11008, 4096),
        ('down_proj', 2): torch.ones(4096, 11008),
    }
    grads[('gate_proj', 1)][0:256, 0:256] = torch.ones(256, 256) * 10
    grads[('gate_proj', 1)][256:512, 0:256] = torch.ones(256, 256) * 10
    grads[('up_proj', 1)][0:2560, 0:256] = torch.ones(2560, 256) * 10
    dims = {'gate_proj': [11008, 4096], 'up_proj': [11008, 4096], 'down_proj': [4096, 11008]}
    out = ref.select_submatrix(grads, dims, n=20, selection_strategy="no_restriction")
    assert list(out.keys()) == [('up_proj', 1), ('gate_proj', 1), ('down_proj', 2)]
    assert out[('up_proj', 1)] == [(i, 0) for i in range(9, -1, -1)]
    assert out[('gate_proj', 1)] == [(1, 0), (0, 0)]
    assert out[('down_proj', 2)] == [(15, j) for j in range(42, 34, -1)]


def test_kat2_channel_selection():
    """smt_helper.py:324-337."""
    act = {
        ('gate_proj', 1): torch.zeros(3, 11008, 4096),
        ('up_proj', 1): torch.zeros(3, 11008, 4096),
        ('down_proj', 2): torch.ones(3, 4096, 11008),
    }
    act[('gate_proj', 1)][:, :, 0:256] = torch.ones(3, 11008, 256) * 1
    act[('gate_proj', 1)][:, :, 0:4] = torch.ones(3, 11008, 4) * 10
    act[('up_proj', 1)][:, :, 3:6] = torch.ones(3, 11008, 3) * 100
    act[('down_proj', 2)][:, :, 3:6] = torch.ones(3, 4096, 3) * 100
    out = ref.select_channel(act, n=100, selection_strategy="no_restriction")
    assert list(out.keys()) == [('up_proj', 1), ('down_proj', 2), ('gate_proj', 1)]
    assert out[('up_proj', 1)] == [5, 4, 3]
    assert out[('down_proj', 2)] == [5, 4, 3]
    assert out[('gate_proj', 1)] == [3, 2, 1, 0] + list(range(255, 165, -1))


def test_selection_error_paths():
    dims = {'q_proj': [256, 512]}
    g = {('q_proj', 0): torch.randn(256, 512)}
    with pytest.raises(UnboundLocalError):
        ref.select_submatrix({}, dims, n=3)
    with pytest.raises(UnboundLocalError):
        ref.select_submatrix(g, dims, n=3, calculate_strategy="bogus")
    with pytest.raises(UnboundLocalError):
        ref.select_submatrix(g, dims, n=0)
    with pytest.raises(RuntimeError):
        ref.select_submatrix({('q_proj', 0): torch.randn(256, 256)}, dims, n=1)


def test_linearz_tile_grads_equal_dense_autograd_fp64():
    """In fp64 the per-tile grads of smt.py:397-404 equal slices of the dense dW of x @ W^T."""
    torch.manual_seed(0)
    B, S, out_f, in_f = 2, 16, 512, 768
    x = torch.randn(B, S, in_f, dtype=torch.float64, requires_grad=True)
    W = torch.randn(out_f, in_f, dtype=torch.float64, requires_grad=True)
    g = torch.randn(B, S, out_f, dtype=torch.float64)
    tiles = [(1, 2), (0, 0), (1, 1)]
    (x @ W.t()).backward(g)
    gi, gw = ref.linearz_backward(g, x.detach(), W.detach(), tiles)
    assert torch.allclose(gi, x.grad, rtol=1e-12, atol=1e-12)
    for i, (r, c) in enumerate(tiles):
        assert torch.allclose(gw[i * 256:(i + 1) * 256], W.grad[r * 256:(r + 1) * 256, c * 256:(c + 1) * 256],
                              rtol=1e-12, atol=1e-12)
    assert torch.allclose(ref.tile_grads_fp64(g, x.detach(), tiles), gw, rtol=1e-12, atol=1e-12)


def test_ref_module_roundtrip_and_writeback():
    torch.manual_seed(1)
    W = torch.nn.Parameter(torch.randn(512, 512))
    mod = ref.RefLinearLayer_MatrixSparsity(W, [(1, 0), (0, 1)])
    with torch.no_grad():
        mod.selected_weight.add_(1.0)
    x = torch.randn(2, 8, 512, requires_grad=True)
    y = mod(x)                           # forward writes the tiles back into W (smt.py:332-341)
    assert torch.equal(W.data[256:512, 0:256], mod.selected_weight.data[0:256])
    assert torch.allclose(y, x @ W.data.t())
    y.sum().backward()
    assert mod.selected_weight.grad.shape == (512, 256)


def test_golden_selection_fixture_reproduces():
    from tests.golden.make_golden import digest, selection_inputs
    spec = json.load(open(os.path.join(GOLDEN, "selection_expected.json")))
    grads = selection_inputs()
    assert digest(grads) == spec["inputs_sha256"], "seeded generator drifted: regenerate goldens"
    att = {k: v for k, v in grads.items() if k[0] in ("q_proj", "k_proj", "v_proj")}
    mlp = {k: v for k, v in grads.items() if k[0] in ("gate_proj", "up_proj", "down_proj")}
    for case in spec["cases"]:
        pool = att if case["pool"] == "attention" else mlp
        out = ref.select_submatrix(pool, spec["dims"], case["n"], selection_strategy=case["selection_strategy"],
                                   calculate_strategy=case["strategy"])
        got = [[k[0], k[1], [list(t) for t in v]] for k, v in out.items()]
        assert got == case["expected"], (case["pool"], case["strategy"], case["n"], case["selection_strategy"])


def test_golden_linearz_fixture_reproduces():
    d = np.load(os.path.join(GOLDEN, "linearz_case.npz"))
    as_bf16 = lambda a: torch.from_numpy(a).view(torch.bfloat16)
    x, g, W = as_bf16(d["x"]), as_bf16(d["g"]), as_bf16(d["W"])
    tiles = [tuple(t) for t in d["tiles"].tolist()]
    y = ref.linearz_forward(x, W)
    gi, gw = ref.linearz_backward(g, x, W, tiles)
    # torch-CPU's bf16 GEMM (oneDNN) picks its fp32 blocking from the host ISA, so the final bf16
    # rounding of the dense products can differ by one ulp between hosts (the fixture was made on an
    # AMD EPYC host; 0.02 % of y / grad_input differ by one ulp on an Intel Xeon host).
    for got, want in ((y, as_bf16(d["y"])), (gi, as_bf16(d["grad_input"]))):
        diff = (got.float() - want.float()).abs()
        assert (diff <= want.float().abs() * 2 ** -7).all()
        assert (diff > 0).float().mean().item() < 1e-3
    assert torch.equal(gw, as_bf16(d["grad_tiles_ref"]))


def test_fused_adam_matches_torch_adamw():
    """The restated DeepSpeed ADAM_MODE_1 rule vs torch.optim.AdamW (mathematically equal)."""
    torch.manual_seed(2)
    p0 = torch.randn(4096)
    p = p0.clone()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([tp], lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, foreach=False, fused=False)
    for step in range(1, 6):
        g = torch.randn(4096) * 0.1
        ref.fused_adam_step(p, g, m, v, step, 1e-3, (0.9, 0.95), 1e-8, 0.1)
        tp.grad = g.clone()
        opt.step()
    assert torch.allclose(p, tp.detach(), rtol=1e-5, atol=1e-6)


def test_harvest_keying_opt_naming_collapses_layers():
    """fine_tune.py:716-767 on OPT names: the layer regex never matches -> one key per module."""
    names = [f"model.decoder.layers.{l}.self_attn.{m}.weight" for l in range(3) for m in ("q_proj", "k_proj", "out_proj")]
    grads = [(n, torch.full((256, 256), float(i + 1))) for i, n in enumerate(names)]
    mlp, att = {}, {}
    ref.harvest(grads, mlp, att, num_mlp_blocks=0, num_attention_blocks=5)
    assert set(att) == {('q_proj', None), ('k_proj', None)}
    assert att[('q_proj', None)][0, 0].item() == 1 + 4 + 7
    assert not mlp


# ------------------------------------------------------------------ channel path (smt.py:185-296, smt_helper.py:149-230)
def test_kat2_exact_fp64_channel_pipeline_agrees():
    """KAT-2 through the build's exact-arithmetic definition (fp64 batch + sequence sums, one
    rounding) selects exactly what the ATen fp32 restatement selects."""
    act = {
        ('gate_proj', 1): torch.zeros(3, 11008, 4096),
        ('up_proj', 1): torch.zeros(3, 11008, 4096),
        ('down_proj', 2): torch.ones(3, 4096, 11008),
    }
    act[('gate_proj', 1)][:, :, 0:256] = torch.ones(3, 11008, 256) * 1
    act[('gate_proj', 1)][:, :, 0:4] = torch.ones(3, 11008, 4) * 10
    act[('up_proj', 1)][:, :, 3:6] = torch.ones(3, 11008, 3) * 100
    act[('down_proj', 2)][:, :, 3:6] = torch.ones(3, 4096, 3) * 100
    stats = {k: ref.channel_stat_fp64(v, "mean_abs") for k, v in act.items()}
    assert dict(ref.rank_channels(stats, 100)) == dict(ref.select_channel(act, n=100))


def test_golden_channel_fixtures_reproduce():
    from tests.golden.make_golden import channel_inputs, digest
    spec = json.load(open(os.path.join(GOLDEN, "channel_selection_expected.json")))
    act = channel_inputs()
    assert digest(act) == spec["inputs_sha256"], "seeded generator drifted: regenerate goldens"
    att = {k: v for k, v in act.items() if k[0] in ("q_proj", "k_proj", "v_proj")}
    mlp = {k: v for k, v in act.items() if k[0] in ("gate_proj", "up_proj", "down_proj")}
    for case in spec["cases"][::5]:
        pool = att if case["pool"] == "attention" else mlp
        out = ref.select_channel(pool, case["n"], selection_strategy=case["selection_strategy"],
                                 calculate_strategy=case["strategy"])
        assert [[k[0], k[1], list(v)] for k, v in out.items()] == case["expected"]
    d = np.load(os.path.join(GOLDEN, "linearchannel_case.npz"))
    bf = lambda a: torch.from_numpy(a).view(torch.bfloat16)
    x, g, W, idx = bf(d["x"]), bf(d["g"]), bf(d["W"]), d["idx"].tolist()
    y, partial = ref.linearchannel_forward(x, W, idx)
    gi, gw = ref.linearchannel_backward(g, partial, W)
    for got, want in ((y, bf(d["y"])), (gi, bf(d["grad_input"])), (gw, bf(d["grad_weight_ref"]))):
        diff = (got.float() - want.float()).abs()      # host-ISA bf16 GEMM rounding, see above
        assert (diff <= want.float().abs() * 2 ** -7).all()
        assert (diff > 0).float().mean().item() < 1e-3


def test_linearchannel_grad_is_the_column_gradient_fp64():
    """The reference's channel gradient (smt.py:285-286) is dL/dW[:, idx]^T, i.e. the gradient of
    the COLUMNS idx of W, stored against the ROWS idx: pinned by dense autograd."""
    torch.manual_seed(1)
    B, S, d = 2, 12, 64
    x = torch.randn(B, S, d, dtype=torch.float64, requires_grad=True)
    W = torch.randn(d, d, dtype=torch.float64, requires_grad=True)
    g = torch.randn(B, S, d, dtype=torch.float64)
    idx = [5, 0, 63, 17]
    (x @ W.t()).backward(g)
    y, partial = ref.linearchannel_forward(x.detach(), W.detach(), idx)
    gi, gw = ref.linearchannel_backward(g, partial, W.detach())
    assert torch.allclose(gi, x.grad, rtol=1e-12, atol=1e-12)
    assert torch.allclose(gw, W.grad[:, idx].t(), rtol=1e-12, atol=1e-12)
    assert torch.allclose(ref.channel_grads_fp64(g, x.detach(), idx), gw, rtol=1e-12, atol=1e-12)


def test_channel_selection_error_paths():
    act = {('q_proj', 0): torch.rand(1, 4, 16)}
    with pytest.raises(UnboundLocalError):
        ref.select_channel({}, n=3)
    with pytest.raises(UnboundLocalError):
        ref.select_channel(act, n=3, calculate_strategy="bogus")
    with pytest.raises(UnboundLocalError):
        ref.select_channel(act, n=0)


# ---------------------------------------------------------------- MX-fp8 format (config 5, no reference counterpart)
def test_mx_exponent_rule():
    amax = torch.tensor([0.0, 448.0, 448.0 * (1 + 2 ** -23), 1.0, 2.0 ** -130, 3.0e38, 449.0, 0.875])
    e = ref.mx_exponent(amax).tolist()
    assert e == [-127, 0, 1, -8, -127, 120, 1, -9]
    # smallest e with amax <= 448 * 2^e (checked in fp64)
    for a, k in zip(amax.double().tolist(), e):
        if a > 2.0 ** -126:
            assert a <= 448.0 * 2.0 ** k and a > 448.0 * 2.0 ** (k - 1)


def test_mx_quant_round_trip_and_no_saturation():
    gen = torch.Generator().manual_seed(0)
    x = (torch.randn(200, 512, generator=gen) * torch.exp(2 * torch.randn(200, 512, generator=gen))).bfloat16()
    q, s = ref.mx_quant_cols(x, [1, 0])
    assert q.shape == (2, 4, 256, 64) and s.shape == (2, 8, 256)
    vals = q.view(torch.float8_e4m3fn).float()
    assert vals.abs().max() <= 448.0 and not torch.isnan(vals).any()
    d = ref.mx_dequant(q, s)
    assert torch.all(d[:, 200:] == 0)                                  # rows past T are zero
    # e4m3 relative rounding of normal values <= 2^-4; every group's max is a normal value
    for i, b in enumerate([1, 0]):
        o = x[:, b * 256:(b + 1) * 256].double()
        dd = d[i, :200]
        big = o.abs() > 0
        rel = ((dd - o).abs() / o.abs().clamp_min(1e-300))[big]
        assert rel.median() < 2 ** -4
    # exactly representable data is reproduced exactly
    ints = torch.randint(-15, 16, (64, 256), generator=gen).bfloat16()
    q2, s2 = ref.mx_quant_cols(ints, [0])
    assert torch.equal(ref.mx_dequant(q2, s2)[0], ints.double())
