"""GPU parity of the channel path (smt.py:185-296, smt_helper.py:149-230,
fine_tune.py:406-709) against the oracle.

Tolerances:
* row / column copies and the harvested fp32 [B, S, in] accumulators: bit-exact vs the reference's
  hook arithmetic (oracle.channel_hook_accumulate); per-channel fp64 sums: bit-exact vs the oracle's
  operation-order restatement (oracle.channel_raw_fp64);
* channel selection: bit-exact (same keys, same order, same channel order) vs the golden fixtures,
  which the ATen fp32 restatement of the reference produced, including the near-tie fixture;
* channel gradient (bf16): relative Frobenius error vs fp64 truth from identical bf16 inputs
  <= max(1e-3, 1.1 x the reference restatement's own error);
* whole-model loss: relative <= 1e-3 vs the reference restatement on the same weights / inputs.
"""
import json
import os
from collections import defaultdict

import numpy as np
import pytest
import torch
from torch import nn

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import _hip, trainer
from sparse_matrix_tuning_amd.smt import smt, smt_helper

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_row_gather_scatter_bit_exact(dtype):
    torch.manual_seed(0)
    W = torch.randn(768, 1536).to(dtype).to(DEV)
    idx = [700, 3, 512, 0, 767]
    tab = _hip.index_table(idx, DEV)
    rows = torch.empty(len(idx), 1536, dtype=dtype, device=DEV)
    _hip.row_gather(W, tab, rows)
    assert torch.equal(rows.cpu(), ref.gather_rows(W.cpu(), idx))
    new = torch.randn(len(idx), 1536).to(dtype).to(DEV)
    W0 = W.clone()
    _hip.row_scatter(W, tab, new)
    expect = W0.cpu()
    expect[idx] = new.cpu()
    assert torch.equal(W.cpu(), expect)


@pytest.mark.parametrize("T,k,in_f", [(80, 37, 512), (1000, 256, 512), (33, 300, 512), (7, 1, 512),
                                      (67, 1713, 5120), (9, 500, 13824), (5, 3, 20000)])   # 4, 2, 1 rows per workgroup
def test_column_gather_bit_exact_and_zero_pad(T, k, in_f):
    torch.manual_seed(1)
    x = torch.randn(T, in_f).bfloat16().to(DEV)
    idx = torch.randperm(in_f)[:k].tolist()
    pad = -(-k // 256) * 256
    out = _hip.column_gather(x, _hip.index_table(idx, DEV), k, pad)
    assert torch.equal(out[:, :k].cpu(), x.cpu()[:, idx])
    assert not out[:, k:].any()


@pytest.mark.parametrize("T,k,in_f", [(37, 100, 517), (6, 2000, 5123)])   # rows end in a partial 16-B chunk
def test_column_gather_ragged_row_width(T, k, in_f):
    torch.manual_seed(3)
    wide = torch.randn(T, in_f + 13).bfloat16().to(DEV)
    ld = (in_f + 13 + 7) // 8 * 8
    buf = torch.zeros(T, ld, dtype=torch.bfloat16, device=DEV)
    buf[:, :in_f + 13] = wide
    x = buf[:, :in_f]                                   # row stride ld, n_in not a multiple of 8
    idx = torch.randperm(in_f)[:k].tolist()
    out = _hip.column_gather(x, _hip.index_table(idx, DEV), k, -(-k // 256) * 256)
    assert torch.equal(out[:, :k].cpu(), x.cpu()[:, idx])
    assert not out[:, k:].any()


@pytest.mark.parametrize("T,k,off,in_f", [(9, 300, 304, 1000), (33, 1713, 8, 5112)])   # 16-B aligned views
def test_column_gather_of_a_column_slice_view(T, k, off, in_f):
    """x = a column slice at an offset of a wider buffer (its last row ends before the buffer does):
    the LDS-DMA staging reads whole 1 KiB pieces, bounded at the last row's n_in-th element."""
    torch.manual_seed(5)
    ld = off + in_f + 8
    buf = torch.randn(T, ld).bfloat16().to(DEV)
    x = buf[:, off:off + in_f]
    idx = torch.randperm(in_f)[:k].tolist()
    out = _hip.column_gather(x, _hip.index_table(idx, DEV), k, -(-k // 256) * 256)
    assert torch.equal(out[:, :k].cpu(), x.cpu()[:, idx])
    assert not out[:, k:].any()


@pytest.mark.parametrize("strategy", ["mean_abs", "abs_mean", "L1", "L2"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_act_accumulate_and_channel_scores_bit_exact(strategy, dtype):
    torch.manual_seed(2)
    steps = [(torch.randn(3, 24, 520) * torch.exp(2 * torch.randn(520))).to(dtype) for _ in range(3)]
    acc = torch.empty(3, 24, 520, dtype=torch.float32, device=DEV)
    feat = {}
    for i, x in enumerate(steps):
        big = torch.zeros(3, 24, 528, dtype=dtype, device=DEV)     # strided input: row stride 528
        big[:, :, :520] = x.to(DEV)
        _hip.act_accumulate(big[:, :, :520], acc, assign=i == 0)
        ref.channel_hook_accumulate(feat, "k", x)                 # fine_tune.py:636-667 at world size 1
    assert torch.equal(acc.cpu(), feat["k"])
    raw = _hip.channel_scores(acc, smt_helper._STRATEGY[strategy])
    assert torch.equal(raw.cpu(), ref.channel_raw_fp64(feat["k"], strategy))
    got = smt_helper.finalize_channel_scores(raw.cpu().numpy(), 24, strategy)
    assert np.array_equal(got, ref.channel_stat_fp64(feat["k"], strategy).numpy())


def test_channel_near_tie_selection_bit_identical():
    """Near-tie fixture: channels holding the same values in another order; the fp64-rounded ranking
    gets some cases wrong (``nominal_ranking_differs``), the product must not."""
    from tests.golden.make_golden import near_tie_channel_inputs
    spec = json.load(open(os.path.join(GOLDEN, "near_tie_expected.json")))["channel"]
    act = near_tie_channel_inputs()
    dev_act = {k: smt_helper.ChannelActivation(v.to(DEV).contiguous(), 1) for k, v in act.items()}
    for case in spec["cases"]:
        st, n, sel = case["strategy"], case["n"], case["selection_strategy"]
        live = ref.select_channel(act, n, selection_strategy=sel, calculate_strategy=st)   # this host's ATen
        for src in (act, dev_act):
            out = smt_helper.select_channel_based_on_activation(src, n, selection_strategy=sel, calculate_strategy=st)
            assert list(out.items()) == list(live.items()), (st, n, sel)
        assert [[k[0], k[1], list(v)] for k, v in live.items()] == case["expected"], (st, n, sel)


def test_channel_selection_bit_exact_vs_golden():
    from tests.golden.make_golden import channel_inputs, digest
    spec = json.load(open(os.path.join(GOLDEN, "channel_selection_expected.json")))
    act = channel_inputs()
    assert digest(act) == spec["inputs_sha256"]
    att = {k: v for k, v in act.items() if k[0] in ("q_proj", "k_proj", "v_proj")}
    mlp = {k: v for k, v in act.items() if k[0] in ("gate_proj", "up_proj", "down_proj")}
    for case in spec["cases"]:
        pool = att if case["pool"] == "attention" else mlp
        out = smt_helper.select_channel_based_on_activation(pool, case["n"], selection_strategy=case["selection_strategy"],
                                                            calculate_strategy=case["strategy"])
        got = [[k[0], k[1], list(v)] for k, v in out.items()]
        assert got == case["expected"], (case["pool"], case["strategy"], case["n"], case["selection_strategy"])


def test_channel_norm_dist_ties_follow_aten_sort_on_gpu():
    """Equal channel statistics under norm_dist come out in the order of ATen's unstable CPU argsort
    (smt_helper.py:191; tests/test_aten_argsort.py), from the GPU scan's intervals and the re-score."""
    from tests.golden.make_golden import digest, tie_channel_inputs
    spec = json.load(open(os.path.join(GOLDEN, "norm_dist_ties_expected.json")))["channel"]
    act = tie_channel_inputs()
    assert digest(act) == spec["inputs_sha256"]
    for case in spec["cases"]:
        out = smt_helper.select_channel_based_on_activation(act, case["n"], selection_strategy="norm_dist",
                                                            calculate_strategy=case["strategy"])
        assert [[k[0], k[1], list(v)] for k, v in out.items()] == case["expected"], (case["strategy"], case["n"])


def test_channel_selection_kat2_on_gpu():
    """SURVEY §4 KAT-2 through the product (reference-format CPU fp32 dict)."""
    act = {
        ('gate_proj', 1): torch.zeros(3, 11008, 4096),
        ('up_proj', 1): torch.zeros(3, 11008, 4096),
        ('down_proj', 2): torch.ones(3, 4096, 11008),
    }
    act[('gate_proj', 1)][:, :, 0:256] = 1.0
    act[('gate_proj', 1)][:, :, 0:4] = 10.0
    act[('up_proj', 1)][:, :, 3:6] = 100.0
    act[('down_proj', 2)][:, :, 3:6] = 100.0
    out = smt_helper.select_channel_based_on_activation(act, n=100)
    assert list(out.keys()) == [('up_proj', 1), ('down_proj', 2), ('gate_proj', 1)]
    assert out[('gate_proj', 1)] == [3, 2, 1, 0] + list(range(255, 165, -1))
    with pytest.raises(UnboundLocalError):
        smt_helper.select_channel_based_on_activation({}, n=3)


def test_linearchannel_matches_golden_fixture():
    d = np.load(os.path.join(GOLDEN, "linearchannel_case.npz"))
    bf = lambda a: torch.from_numpy(a).view(torch.bfloat16)
    x, g, W, idx = bf(d["x"]), bf(d["g"]), bf(d["W"]), d["idx"].tolist()
    mod = smt.LinearLayer_ChannelSparsity(nn.Parameter(W.to(DEV)), index_list=idx)
    assert torch.equal(mod.selected_weight.detach().cpu(), ref.gather_rows(W, idx))
    xd = x.to(DEV).requires_grad_(True)
    y = mod(xd)
    y.backward(g.to(DEV))
    assert _rel(y, bf(d["y"])) < 1e-2 and _rel(xd.grad, bf(d["grad_input"])) < 1e-2   # stock bf16 GEMMs
    truth = torch.from_numpy(d["grad_weight_fp64"])
    err = _rel(mod.selected_weight.grad, truth)
    assert mod.selected_weight.grad.shape == (len(idx), 512)
    assert err <= max(1e-3, 1.1 * _rel(bf(d["grad_weight_ref"]), truth)), err


def test_linearchannel_non_square_raises_and_writeback():
    torch.manual_seed(4)
    W = nn.Parameter((torch.randn(256, 512) * 0.02).bfloat16().to(DEV))
    mod = smt.LinearLayer_ChannelSparsity(W, index_list=[3, 200])
    y = mod(torch.randn(2, 8, 512).bfloat16().to(DEV))
    with pytest.raises(RuntimeError, match="invalid gradient"):
        y.sum().backward()
    # forward write-back (smt.py:208-213): rows of W follow selected_weight
    with torch.no_grad():
        mod.selected_weight.add_(1.0)
    mod(torch.randn(2, 8, 512).bfloat16().to(DEV))
    assert torch.equal(W.detach()[[3, 200]].cpu(), mod.selected_weight.detach().cpu())


# ------------------------------------------------------------------ harvest + selection + training on a mini LLaMA
def _square_mini_llama(layers=2):
    import bench
    cfg = dict(bench.MODELS["mini"])
    cfg["num_hidden_layers"] = layers
    cfg["num_key_value_heads"] = cfg["num_attention_heads"]      # square k/v: the reference path's domain
    bench.MODELS["_tc"] = cfg
    try:
        return bench.build_model("_tc", DEV), cfg
    finally:
        del bench.MODELS["_tc"]


def test_harvester_bit_exact_vs_reference_hook_and_selection():
    model, _cfg = _square_mini_llama(2)
    h = trainer.ActivationHarvester(model, num_mlp_channel=16, num_attention_channel=16)
    seen = defaultdict(list)
    spies = []
    for i, layer in enumerate(model.model.layers):
        for name, lin in smt_helper.get_named_linears(layer).items():
            spies.append(lin.register_forward_hook(
                lambda m, inp, out, key=(name, i): seen[key].append(inp[0].detach().cpu())))
    feat_mlp, feat_att = {}, {}
    for step in range(2):
        ids = torch.randint(0, 4096, (2, 64), generator=torch.Generator().manual_seed(step))
        h.collect({"input_ids": ids.to(DEV)})
    for s in spies:
        s.remove()
    h.finalize()
    for (name, i), xs in seen.items():
        for x in xs:
            if 'mlp' in name:
                ref.channel_hook_accumulate(feat_mlp, (smt._mlp_module_name(name), i), x)
            elif name.split('.')[-1] in ('q_proj', 'k_proj', 'v_proj'):
                ref.channel_hook_accumulate(feat_att, (name.split('.')[-1], i), x)
    assert set(h.activation) == set(feat_mlp) and set(h.attention_activation) == set(feat_att)
    for key, ent in list(h.activation.items()) + list(h.attention_activation.items()):
        assert ent.steps == 2
        want = feat_mlp[key] if key[0] in ('gate_proj', 'up_proj', 'down_proj') else feat_att[key]
        assert torch.equal(ent.acc.cpu(), want)
    # q/k/v (gate/up) read one input: one shared accumulator each
    assert h.attention_activation[('q_proj', 0)] is h.attention_activation[('v_proj', 0)]
    assert h.activation[('gate_proj', 1)] is h.activation[('up_proj', 1)]
    assert h.activation[('down_proj', 1)] is not h.activation[('up_proj', 1)]
    got = smt_helper.select_channel_based_on_activation(h.attention_activation, 16)
    assert dict(got) == dict(ref.select_channel(feat_att, 16))
    got = smt_helper.select_channel_based_on_activation(h.activation, 16, calculate_strategy="L2")
    assert dict(got) == dict(ref.select_channel(feat_mlp, 16, calculate_strategy="L2"))
    h.release()


def test_end_to_end_channel_path_matches_reference_restatement():
    """Harvest -> select -> freeze -> convert -> engine: the converted model's loss and row grads
    vs the CPU restatement of the reference modules on the same weights and batch, then a few
    fused-AdamW steps with the rows written back into W."""
    model, cfg = _square_mini_llama(2)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    h = trainer.ActivationHarvester(model, num_mlp_channel=0, num_attention_channel=24)
    ids = torch.randint(0, 4096, (2, 128), generator=torch.Generator().manual_seed(7))
    h.collect({"input_ids": ids.to(DEV)})
    engine, opt, sched, sel_mlp, sel_att = trainer.select_and_convert_channels(
        model, h, num_attention_channel=24, num_mlp_channel=0, ft_learning_rate=1e-3, num_training_steps=10)
    assert sum(len(v) for v in sel_att.values()) == 24 and not sel_mlp
    mods = {n: m for n, m in model.named_modules() if isinstance(m, smt.LinearLayer_ChannelSparsity)}
    assert mods and all(("q_proj" in n or "k_proj" in n or "v_proj" in n) for n in mods)
    assert opt.param_groups[0]["betas"] == (0.95, 0.999)

    out = engine(input_ids=ids.to(DEV), labels=ids.to(DEV), use_cache=False)
    from transformers import LlamaConfig, LlamaForCausalLM
    cpu_cfg = LlamaConfig(**cfg)
    cpu_cfg._attn_implementation = "sdpa"
    cpu = LlamaForCausalLM(cpu_cfg).to(torch.bfloat16)
    cpu.load_state_dict(sd)
    smt.freeze_unselected_channel_layer(cpu, sel_mlp, sel_att)
    ref.ref_convert_channel(cpu, sel_mlp, sel_att)
    out_ref = cpu(input_ids=ids, labels=ids, use_cache=False)
    out_ref.loss.backward()
    rel = abs(out.loss.item() - out_ref.loss.item()) / abs(out_ref.loss.item())
    assert rel <= 1e-3, (out.loss.item(), out_ref.loss.item())
    engine.backward(out.loss)
    cpu_mods = {n: m for n, m in cpu.named_modules() if isinstance(m, ref.RefLinearLayer_ChannelSparsity)}
    assert sorted(cpu_mods) == sorted(mods)
    for n in mods:
        e = _rel(mods[n].selected_weight.grad, cpu_mods[n].selected_weight.grad)
        assert e < 3e-2, (n, e)
    before = {n: m.selected_weight.detach().clone() for n, m in mods.items()}
    engine.step()
    assert all(not torch.equal(before[n], m.selected_weight.detach()) for n, m in mods.items())
    losses = []
    for _ in range(3):
        o = engine(input_ids=ids.to(DEV), labels=ids.to(DEV), use_cache=False)
        engine.backward(o.loss)
        engine.step()
        losses.append(o.loss.item())
    # (no descent check: the reference's row update uses the column gradient)
    assert all(np.isfinite(losses))
    for n, m in mods.items():
        m(torch.zeros(1, 1, m.weight.shape[1], dtype=torch.bfloat16, device=DEV))     # write-back
        assert torch.equal(m.weight.detach()[m.index_list].cpu(), m.selected_weight.detach().cpu())


# ------------------------------------------------------------------ config 4 geometry (LLaMA-2-13B attention)
def test_channel_path_at_config4_geometry():
    """The channel kernels at the shapes they run at in config 4 (LLaMA-2-13B: hidden 5120, the
    square q/k/v the reference path supports; B = 16, S = 2048): the harvested fp32 [B, S, in]
    accumulator and the per-channel fp64 sums bit-exact vs the reference hook / the oracle, the
    selection of one layer's q/k/v identical to the reference's ATen ranking, and the channel
    gradient over T = 32768 tokens vs fp64 truth."""
    B, S, H = 16, 2048, 5120
    gen = torch.Generator(device=DEV).manual_seed(40)
    col_scale = torch.exp(1.5 * torch.randn(H, generator=gen, device=DEV))
    xs = [(torch.randn(B, S, H, generator=gen, device=DEV) * col_scale).bfloat16() for _ in range(2)]
    acc = torch.empty(B, S, H, dtype=torch.float32, device=DEV)
    feat = {}
    for i, x in enumerate(xs):
        _hip.act_accumulate(x, acc, assign=i == 0)
        ref.channel_hook_accumulate(feat, "q", x.cpu())
    want = feat.pop("q")
    assert torch.equal(acc.cpu(), want)
    for strategy in ("mean_abs", "L2"):
        raw = _hip.channel_scores(acc, smt_helper._STRATEGY[strategy])
        assert torch.equal(raw.cpu(), ref.channel_raw_fp64(want, strategy)), strategy
    # one layer's q/k/v (one shared input in the model; three distinct ones here), config-4 budget scale
    act = {("q_proj", 0): want}
    dev_act = {("q_proj", 0): smt_helper.ChannelActivation(acc, 2)}
    for j, key in enumerate((("k_proj", 0), ("v_proj", 0))):
        a = (acc * (1.0 + 0.25 * j)).contiguous()
        act[key] = a.cpu()
        dev_act[key] = smt_helper.ChannelActivation(a, 2)
    for strategy in ("mean_abs", "L2"):
        got = smt_helper.select_channel_based_on_activation(dev_act, 1713, calculate_strategy=strategy)
        live = ref.select_channel(act, 1713, calculate_strategy=strategy)
        assert list(got.items()) == list(live.items()), strategy
    del act, dev_act, feat
    # the channel gradient x[:, :, idx]^T g over T = 32768 (linearChannel.backward, smt.py:285-286)
    idx = got[("q_proj", 0)][:600] if ("q_proj", 0) in got else list(range(600))
    W = nn.Parameter((torch.randn(H, H, generator=gen, device=DEV) * 0.02).bfloat16())
    mod = smt.LinearLayer_ChannelSparsity(W, index_list=idx)
    x = xs[0].detach()
    g = (torch.randn(B, S, H, generator=gen, device=DEV) * 1e-2).bfloat16()
    mod(x).backward(g)
    gw = mod.selected_weight.grad
    assert gw.shape == (len(idx), H)
    rows = torch.tensor(idx[:64], device=DEV)
    truth = x.view(-1, H)[:, rows].double().t() @ g.view(-1, H).double()          # [64, H]
    assert _rel(gw[:64], truth) < 2e-3


@pytest.mark.parametrize("B,S,C", [(16, 2048, 5120), (4, 2048, 256), (2, 100, 512), (3, 4096, 768), (1, 17, 256)])
def test_channel_mean_aten_bit_identical_to_reference_expression(B, S, C):
    """smt_channel_mean_aten replays ATen's CPU cascade_sum order: every channel's fp32 value equals
    the reference expression (smt_helper.py:167-176: torch.sum(act.abs(), 0) then torch.mean(., 0),
    run here on the host CPU), including S not a multiple of the 16-row chunk and config 4's
    [16, 2048, 5120] state; mean_abs and abs_mean agree on the non-negative harvest."""
    gen = torch.Generator(device=DEV).manual_seed(B * S + C)
    acc = torch.rand(B, S, C, generator=gen, device=DEV) * torch.rand(C, generator=gen, device=DEV) * 3.0
    got = _hip.channel_mean_aten(acc).cpu().numpy()
    for strategy in ("mean_abs", "abs_mean"):
        assert np.array_equal(got, smt_helper.reference_channel_stat(acc, strategy))


def test_exact_channel_scores_skip_the_host_rescore():
    """With the ATen-order means the ranking has nothing undecided: no key is re-scored, and the
    selection equals the oracle's on the same state (near-tie fixture values included)."""
    gen = torch.Generator(device=DEV).manual_seed(5)
    acts = {("q_proj", i): torch.rand(2, 256, 512, generator=gen, device=DEV) for i in range(3)}
    acts[("k_proj", 0)] = acts[("q_proj", 0)] * (1 + 1e-7)          # values a few ulps apart
    from sparse_matrix_tuning_amd.smt import ranking
    got = smt_helper.select_channel_based_on_activation(acts, 40)
    assert ranking.LAST_REPORT["rescored_keys"] == []
    want = ref.select_channel({k: v.cpu() for k, v in acts.items()}, 40)
    assert {k: list(v) for k, v in got.items()} == {k: list(v) for k, v in want.items()}
    assert list(got) == list(want)


def test_channel_modules_share_input_gradient_accumulation():
    """q/k/v channel modules reading one input accumulate their data gradients in one buffer
    (dgrad.py), also when one of them does not reach the loss: the input gradient equals the fp64
    sum over the consumers that ran."""
    torch.manual_seed(21)
    Ws = [nn.Parameter((torch.randn(512, 512) * 0.05).bfloat16().to(DEV), requires_grad=False) for _ in range(3)]
    mods = [smt.LinearLayer_ChannelSparsity(W, index_list=idx) for W, idx in zip(Ws, ([3, 100, 7], [0, 511], [42]))]
    x = torch.randn(2, 96, 512).bfloat16().to(DEV)
    gs = [torch.randn(2, 96, 512).bfloat16().to(DEV) for _ in mods]
    for used in ((0, 1, 2), (0, 2)):
        xi = x.clone().requires_grad_(True)
        outs = [m(xi) for m in mods]
        torch.autograd.backward([outs[i] for i in used], [gs[i] for i in used])
        truth = sum(gs[i].double() @ mods[i].weight.detach().double() for i in used)
        assert ((xi.grad.double() - truth).norm() / truth.norm()).item() < 5e-3, used


def test_channel_engine_transposed_copies_follow_the_rows():
    """Under the engine the channel path's frozen weights get transposed copies (the TN data-gradient
    layout): every row update reaches W^T's columns through sync_weight, the data gradient through
    W^T equals the plain one to GEMM rounding, and the rows' training matches the run without copies."""
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize

    def run(transposed):
        torch.manual_seed(23)
        net = nn.Module()
        W = nn.Parameter((torch.randn(512, 512) * 0.05).bfloat16().to(DEV), requires_grad=False)
        net.q = smt.LinearLayer_ChannelSparsity(W, index_list=[5, 300, 17])
        net.o = nn.Linear(512, 512, bias=False).to(DEV).bfloat16().requires_grad_(False)
        opt = SMTFusedAdam([net.q.selected_weight], lr=1e-2)
        engine, *_ = initialize(model=net, optimizer=opt, config={"transposed_dgrad": transposed})
        assert (getattr(W, "_smt_weight_t", None) is not None) == transposed
        x = torch.randn(2, 64, 512).bfloat16().to(DEV)
        grads = []
        for _ in range(3):
            xi = x.clone().requires_grad_(True)
            loss = net.o(net.q(xi)).float().pow(2).mean()
            engine.backward(loss)
            grads.append(xi.grad.clone())
            engine.step()
            net.q.sync_weight()
            if transposed:
                assert torch.equal(W._smt_weight_t, W.detach().t())
        return grads, net.q.selected_weight.detach().clone()

    g0, r0 = run(False)
    g1, r1 = run(True)
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 1e-2
    assert _rel(r1, r0) < 1e-2


def test_channel_qkv_share_one_column_gather():
    """Under the engine q/k/v_proj channel modules of one attention module gather their partial inputs
    (smt.py:225-233) in ONE column-gather launch into a joint buffer (engine.attach_channel_gather_groups);
    each member's partial is a zero-padded column slice of it. Tile gradients and the trained rows are
    bit-identical to the per-module gathers (shared_channel_gather off)."""
    from sparse_matrix_tuning_amd import _hip
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize

    def run(shared):
        torch.manual_seed(31)
        net = nn.Module()
        net.attn = nn.Module()
        Ws = [nn.Parameter((torch.randn(512, 512) * 0.05).bfloat16().to(DEV), requires_grad=False) for _ in range(3)]
        idx = ([5, 300, 17, 260, 511], list(range(0, 512, 2)) + [1, 3], [42])     # 5, 258 (ragged), 1 channels
        for name, W, ix in zip(("q_proj", "k_proj", "v_proj"), Ws, idx):
            setattr(net.attn, name, smt.LinearLayer_ChannelSparsity(W, index_list=ix))
        mods = [net.attn.q_proj, net.attn.k_proj, net.attn.v_proj]
        opt = SMTFusedAdam([m.selected_weight for m in mods], lr=1e-2)
        engine, *_ = initialize(model=net, optimizer=opt, config={"shared_channel_gather": shared})
        assert engine.channel_gather_groups == (1 if shared else 0)
        calls = []
        real = _hip.column_gather

        def counting(*a, **k):
            calls.append(a[2])
            return real(*a, **k)
        _hip.column_gather = counting
        try:
            x = torch.randn(2, 64, 512).bfloat16().to(DEV)
            grads = []
            for _ in range(2):
                xi = x.clone().requires_grad_(True)
                loss = sum(m(xi).float().pow(2).mean() for m in mods)
                engine.backward(loss)
                grads.append([m.selected_weight.grad.clone() for m in mods])
                engine.step()
        finally:
            _hip.column_gather = real
        return calls, grads, [m.selected_weight.detach().clone() for m in mods]

    calls_s, grads_s, rows_s = run(True)
    calls_p, grads_p, rows_p = run(False)
    assert len(calls_s) == 2 and calls_s[0] == 256 + 512 + 256          # one joint gather per forward
    assert len(calls_p) == 6
    for gs, gp in zip(grads_s, grads_p):
        for a, b in zip(gs, gp):
            assert torch.equal(a, b)
    for a, b in zip(rows_s, rows_p):
        assert torch.equal(a, b)


def test_channel_joint_gather_freed_after_backward_while_input_lives():
    """the joint partial-input buffer of a ChannelGatherGroup is held by weak references
    only, so it is freed with the members' backward even while something else keeps the q/k/v input
    alive (here: the test itself)."""
    import gc
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    torch.manual_seed(37)
    net = nn.Module()
    net.attn = nn.Module()
    for name in ("q_proj", "k_proj", "v_proj"):
        W = nn.Parameter((torch.randn(512, 512) * 0.05).bfloat16().to(DEV), requires_grad=False)
        setattr(net.attn, name, smt.LinearLayer_ChannelSparsity(W, index_list=[3, 77, 400]))
    mods = [net.attn.q_proj, net.attn.k_proj, net.attn.v_proj]
    engine, *_ = initialize(model=net, optimizer=SMTFusedAdam([m.selected_weight for m in mods], lr=1e-2), config={})
    assert engine.channel_gather_groups == 1
    grp = mods[0].weight._smt_cgather[0]
    xi = torch.randn(2, 64, 512).bfloat16().to(DEV).requires_grad_(True)      # kept alive throughout
    loss = sum(m(xi).float().pow(2).mean() for m in mods)
    assert grp._cache is not None and grp._cache[2]() is not None           # alive while backward needs it
    engine.backward(loss)
    del loss
    gc.collect()
    assert grp._cache[0]() is xi and grp._cache[2]() is None               # the input lives, the buffer is gone
    assert "_smt_cgather" not in xi.__dict__
