"""The engine in the reference's other dtypes (--dtype fp16 | fp32: fine_tune.py:955-959,
deepspeed_helpers.py:53-61): the fused AdamW writing fp16 / fp32 tiles into W (ABI v12), fp16 dynamic
loss scaling and fp32 training through SMTEngine, against the oracle's restatement of DeepSpeed's
FusedAdam / clipping / loss scaler (external: parity unpinned by the reference).

Tolerances: fp32 master weights within 1e-5 relative of the restatement over the steps (the same
bar as the bf16 engine test in test_gpu_parity.py); the parameter / W values are the master rounded to
the parameter dtype, bit for bit; the loss scale and the skipped steps identical.
"""
import pytest
import torch
from torch import nn

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import _hip
from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _args(step, max_norm=0.0, grad_scale=1.0, wd=0.01):
    return _hip.AdamWArgs(lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=wd,
                          bias_correction1=1 - 0.9 ** step, bias_correction2=1 - 0.95 ** step,
                          max_grad_norm=max_norm, grad_scale=grad_scale, mode=_hip.ADAM_DEEPSPEED, grad_dtype=0)


@pytest.mark.parametrize("pdt", [torch.float16, torch.float32, torch.bfloat16])
def test_adamw_tiles_write_the_parameter_dtype_into_w(pdt):
    """smt_adamw_step over tiles (fp32 gradients) with the scatter into a W of the parameter dtype:
    master / moments as the restatement, tiles and W = master rounded to that dtype, the rest of W
    untouched; 3 steps, the clip active."""
    torch.manual_seed(1)
    W = (torch.randn(768, 1024) * 0.05).to(pdt).to(DEV)
    W0 = W.clone()
    tiles = [(2, 3), (0, 0), (1, 2)]
    n = len(tiles) * 65536
    master = ref.gather_tiles(W0.cpu(), tiles).float().reshape(-1).to(DEV)
    m, v = torch.zeros_like(master), torch.zeros_like(master)
    param = master.to(pdt)
    descs = _hip.tile_descs([(W, r, c, i * 65536) for i, (r, c) in enumerate(tiles)], DEV, pdt)
    t_ref = master.cpu().clone()
    m_ref, v_ref = torch.zeros_like(t_ref), torch.zeros_like(t_ref)
    for step in range(1, 4):
        g = torch.randn(n, device=DEV) * 0.5
        norm = (g.double() ** 2).sum().reshape(1)
        _hip.adamw_step(g, master, m, v, param, _args(step, 1.0), tiles=descs, n_tiles=len(tiles), grad_sq_norm=norm)
        coef = ref.clip_coef([g.cpu()], 1.0)
        assert coef < 0.5
        ref.fused_adam_step(t_ref, g.cpu() * coef, m_ref, v_ref, step, 1e-3, (0.9, 0.95), 1e-8, 0.01)
    torch.cuda.synchronize()
    assert _rel(master, t_ref) < 1e-6
    assert torch.equal(param.cpu(), master.cpu().to(pdt))
    assert torch.equal(ref.gather_tiles(W.cpu(), tiles).reshape(-1), param.cpu())
    keep = torch.ones(3, 4, dtype=torch.bool)
    for r, c in tiles:
        keep[r, c] = False
    for r in range(3):
        for c in range(4):
            if keep[r, c]:
                assert torch.equal(W[r * 256:(r + 1) * 256, c * 256:(c + 1) * 256], W0[r * 256:(r + 1) * 256, c * 256:(c + 1) * 256])


@pytest.mark.parametrize("pdt", [torch.float16, torch.float32])
def test_adamw_multi_in_the_parameter_dtype(pdt):
    """smt_adamw_multi over ragged tensors with gradients of the parameter dtype (the warm-up's dense
    fp16 / fp32 step): equal to smt_adamw_step per tensor bit for bit, and to the restatement."""
    torch.manual_seed(2)
    sizes = [1, 2047, 4096 + 5, 3 * 2048]
    rows, solo = [], []
    for k in sizes:
        p = (torch.randn(k) * 0.1).to(pdt)
        g = (torch.randn(k) * 0.3).to(pdt).to(DEV)
        st = [p.float().to(DEV), torch.zeros(k, device=DEV), torch.zeros(k, device=DEV), p.to(DEV)]
        rows.append((g, *st))
        solo.append((g, *[t.clone() for t in st]))
    norm = sum((r[0].double() ** 2).sum() for r in rows).reshape(1)
    for step in (1, 2):
        _hip.adamw_multi(rows, _args(step, 1.0), grad_sq_norm=norm)
        for r in solo:
            _hip.adamw_step(*r, _args(step, 1.0), grad_sq_norm=norm)
    torch.cuda.synchronize()
    coef = ref.clip_coef([r[0].float().cpu() for r in rows], 1.0)
    for r, s in zip(rows, solo):
        for a, b in zip(r[1:], s[1:]):
            assert torch.equal(a, b)
        assert torch.equal(r[4].cpu(), r[1].cpu().to(pdt))
    # the restatement, from the same initial values and gradients
    torch.manual_seed(2)
    for (k, r) in zip(sizes, rows):
        p0 = (torch.randn(k) * 0.1).to(pdt).float()
        g = (torch.randn(k) * 0.3).to(pdt).float()
        mm, vv = torch.zeros(k), torch.zeros(k)
        for step in (1, 2):
            ref.fused_adam_step(p0, g * coef, mm, vv, step, 1e-3, (0.9, 0.95), 1e-8, 0.01)
        assert _rel(r[1], p0) < 1e-6


def _tile_net(dtype, seed=8):
    torch.manual_seed(seed)
    W1 = nn.Parameter((torch.randn(512, 512) * 0.05).to(dtype).to(DEV))
    W2 = nn.Parameter((torch.randn(768, 512) * 0.05).to(dtype).to(DEV))
    net = nn.Module()
    net.layers = nn.ModuleList([smt.LinearLayer_MatrixSparsity(W1, index_list=[(1, 1), (0, 0)]),
                                smt.LinearLayer_MatrixSparsity(W2, index_list=[(2, 0)])])
    masters = [ref.gather_tiles(W1.detach().cpu(), [(1, 1), (0, 0)]).float(),
               ref.gather_tiles(W2.detach().cpu(), [(2, 0)]).float()]
    return net, masters


def _sink_grads(net):
    return [m.selected_weight._smt_grad_sink.buffer.clone().cpu() for m in net.layers]


def test_engine_fp32_step_matches_oracle():
    """--dtype fp32 (``"fp16": {"enabled": false}``): fp32 tiles, fp32 W, no loss scale; the clip
    and AdamW as the bf16 engine's, 3 steps."""
    net, masters = _tile_net(torch.float32)
    opt = SMTFusedAdam([{"params": [m.selected_weight for m in net.layers], "weight_decay": 0.01, "lr": 1e-3}],
                       lr=1e-3, betas=(0.9, 0.95))
    engine, _, _, _ = initialize(model=net, optimizer=opt, config={"gradient_clipping": 1.0, "fp16": {"enabled": False}})
    assert engine.loss_scaler is None and engine.tile_groups[0].param.dtype == torch.float32
    ms = [torch.zeros_like(t) for t in masters]
    vs = [torch.zeros_like(t) for t in masters]
    x = torch.randn(2, 32, 512)
    for step in range(1, 4):
        loss = (net.layers[1](net.layers[0](x.to(DEV))) ** 2).mean() * 100.0
        engine.backward(loss)
        grads = _sink_grads(net)
        engine.step()
        coef = ref.clip_coef(grads, 1.0)
        for t, g, m, v in zip(masters, grads, ms, vs):
            ref.fused_adam_step(t, g * coef, m, v, step, 1e-3, (0.9, 0.95), 1e-8, 0.01)
    torch.cuda.synchronize()
    tg = engine.tile_groups[0]
    assert _rel(tg.master, torch.cat([t.reshape(-1) for t in masters])) < 1e-5
    assert torch.equal(tg.param, tg.master)
    for mod in net.layers:
        assert torch.equal(ref.gather_tiles(mod.weight.detach().cpu(), mod.index_list), mod.selected_weight.detach().cpu())


@pytest.mark.parametrize("window", [100, 2])
def test_engine_fp16_loss_scaling_matches_restatement(window):
    """--dtype fp16 (``"fp16": {"enabled": true, "loss_scale_window": ...}``): the loss is scaled
    before backward, fp16 tile gradients overflow at a large scale and skip their steps (no update, no
    optimizer step count, no LR step), the scale follows DeepSpeed's schedule (restated), and the
    applied steps unscale and clip with the scale the scaler holds after its update. Starts at 2**26 so
    the first steps overflow; window 2 also exercises growth between applied steps."""
    net, masters = _tile_net(torch.float16)
    opt = SMTFusedAdam([{"params": [m.selected_weight for m in net.layers], "weight_decay": 0.01, "lr": 1e-3}],
                       lr=1e-3, betas=(0.9, 0.95))
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0)
    engine, _, _, _ = initialize(model=net, optimizer=opt, lr_scheduler=sched, config={
        "gradient_clipping": 1.0, "fp16": {"enabled": True, "loss_scale_window": window, "initial_scale_power": 26}})
    scaler = ref.RefDynamicLossScaler(init_scale=2.0 ** 26, scale_window=window)
    ms = [torch.zeros_like(t) for t in masters]
    vs = [torch.zeros_like(t) for t in masters]
    x = torch.randn(2, 32, 512).half()
    applied, skipped = 0, 0
    for it in range(30):
        loss = (net.layers[1](net.layers[0](x.to(DEV))).float() ** 2).mean() * 100.0
        engine.backward(loss)
        grads = _sink_grads(net)
        engine.step()
        overflow, mult = ref.fp16_step_scales(scaler, grads, 1.0)
        assert engine.loss_scaler.scale == scaler.cur_scale, it
        if overflow:
            skipped += 1
        else:
            applied += 1
            for t, g, m, v in zip(masters, grads, ms, vs):
                ref.fused_adam_step(t, g * mult, m, v, applied, 1e-3, (0.9, 0.95), 1e-8, 0.01)
    torch.cuda.synchronize()
    assert skipped >= 2 and applied >= 3, (skipped, applied)
    assert engine.skipped_steps == skipped and engine.global_steps == 30
    assert engine.tile_groups[0].step == applied and sched.last_epoch == applied
    tg = engine.tile_groups[0]
    assert _rel(tg.master, torch.cat([t.reshape(-1) for t in masters])) < 1e-5
    assert torch.equal(tg.param, tg.master.half())
    for mod in net.layers:
        assert torch.equal(ref.gather_tiles(mod.weight.detach().cpu(), mod.index_list), mod.selected_weight.detach().cpu())


def test_fp16_engine_refuses_single_rounding():
    """under fp16's dynamic loss scale an overflow is detected from inf / nan in the tile
    gradients. The reference rounding overflows exactly where the reference's fp16 per-sample partials
    do; the single fp32 rounding would not, so an fp16 engine refuses it (explicitly or by default)."""
    net, _m = _tile_net(torch.float16)
    opt = SMTFusedAdam([m.selected_weight for m in net.layers], lr=1e-3)
    with pytest.raises(ValueError, match="reference"):
        initialize(model=net, optimizer=opt, config={"fp16": {"enabled": True}, "wgrad_rounding": "single"})
    old = smt.set_wgrad_rounding("single")
    try:
        net, _m = _tile_net(torch.float16, seed=9)
        with pytest.raises(ValueError, match="reference"):
            initialize(model=net, optimizer=SMTFusedAdam([m.selected_weight for m in net.layers], lr=1e-3),
                       config={"fp16": {"enabled": True}})
    finally:
        smt.set_wgrad_rounding(old)
    net, _m = _tile_net(torch.float16, seed=10)
    eng, *_ = initialize(model=net, optimizer=SMTFusedAdam([m.selected_weight for m in net.layers], lr=1e-3),
                         config={"fp16": {"enabled": True}})
    assert eng.wgrad_rounding == "reference"


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_mini_llama_trains_through_the_engine_in_dtype(dtype):
    """A converted 2-layer mini-LLaMA in fp16 / fp32 through SMTEngine (the reference's --dtype with
    DeepSpeed's config for it): 8 steps run with finite losses, at most 5 of them skipped, the loss
    goes down on a repeated batch, and W's tiles follow the tile parameters in the model dtype."""
    import bench
    cfg = dict(bench.MODELS["mini"])
    cfg["num_hidden_layers"] = 2
    bench.MODELS["_t"] = cfg
    try:
        torch.manual_seed(10)
        model = bench.build_model("_t", DEV).to(dtype)
    finally:
        del bench.MODELS["_t"]
    from collections import defaultdict
    sel_mlp = defaultdict(list, {('up_proj', 1): [(2, 1), (0, 0)], ('down_proj', 0): [(1, 0)]})
    sel_att = defaultdict(list, {('v_proj', 1): [(0, 1)], ('q_proj', 0): [(1, 1)]})
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    groups = smt.get_optimizer_sparse_grouped_parameters(model, 0.0, smt_lr=1e-3)
    opt = SMTFusedAdam(groups, lr=1e-3, betas=(0.9, 0.95))
    ds = {"gradient_clipping": 1.0, "fp16": ({"enabled": True, "loss_scale_window": 100} if dtype == torch.float16
                                             else {"enabled": False})}
    engine, _, _, _ = initialize(model=model, optimizer=opt, config=ds)
    ids = torch.randint(0, 4096, (2, 128), generator=torch.Generator().manual_seed(0)).to(DEV)
    losses = []
    for _ in range(8):
        loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
        engine.backward(loss)
        engine.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses))), losses
    applied = 8 - engine.skipped_steps
    assert applied >= 3, engine.skipped_steps
    assert losses[-1] < losses[0], losses
    for mod in model.modules():
        if isinstance(mod, smt.LinearLayer_MatrixSparsity):
            assert mod.selected_weight.dtype == dtype
            assert torch.equal(ref.gather_tiles(mod.weight.detach().cpu(), mod.index_list), mod.selected_weight.detach().cpu())


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_reference_flow_in_dtype(dtype):
    """fine_tune.py's whole flow in the reference's fp16 / fp32: full fine-tuning warm-up steps through
    the engine (dense fused AdamW on fp16 / fp32 parameters; fp16 under the loss scale) with the GPU
    harvest, then selection, freeze, conversion and SMT steps. The harvest equals the restatement's
    CPU accumulation of the same gradients bit for bit (in fp16 these are the LOSS-SCALED gradients,
    what DeepSpeed's safe_get_full_grad returns between backward and step), and the selection the
    restatement's on them. A small initial scale keeps the warm-up free of overflow steps here (an
    overflow step's inf gradients would enter the harvest, as in the reference)."""
    import bench
    cfg = dict(bench.MODELS["mini"])
    cfg["num_hidden_layers"] = 2
    bench.MODELS["_td"] = cfg
    try:
        torch.manual_seed(21)
        model = bench.build_model("_td", DEV).to(dtype)
    finally:
        del bench.MODELS["_td"]
    from sparse_matrix_tuning_amd import trainer
    from sparse_matrix_tuning_amd.engine import safe_get_full_grad
    ds = {"gradient_clipping": 1.0, "fp16": ({"enabled": True, "loss_scale_window": 100, "initial_scale_power": 10}
                                             if dtype == torch.float16 else {"enabled": False})}
    dims = trainer.get_targeted_module_dims(model)
    n_att, n_mlp = trainer.block_budgets(trainer.count_total_blocks(model), 0.1, 0.1)
    opt = SMTFusedAdam(model.parameters(), lr=1e-4, betas=(0.9, 0.95))
    engine, _, _, _ = initialize(model=model, optimizer=opt, config=ds)
    harvester = trainer.GradHarvester(model, n_mlp, n_att)
    mlp_ref, att_ref = {}, {}
    for b in bench.batches(3, 2, 128, bench.MODELS["mini"]["vocab_size"], 0, DEV):
        engine.backward(engine(**b, use_cache=False).loss)
        harvester.harvest()
        named = [(n, safe_get_full_grad(p)) for n, p in model.named_parameters()]
        assert all(g is None or g.dtype == dtype for _n, g in named)
        ref.harvest([(n, g) for n, g in named if g is not None], mlp_ref, att_ref, n_mlp, n_att)
        engine.step()
    assert engine.skipped_steps == 0 and all(p.dtype == dtype for p in model.parameters())
    for k in mlp_ref:
        assert torch.equal(harvester.warmup_grads[k].cpu(), mlp_ref[k])
    for k in att_ref:
        assert torch.equal(harvester.attention_warmup_grads[k].cpu(), att_ref[k])
    want_att = ref.select_submatrix(att_ref, dims, n_att)
    want_mlp = ref.select_submatrix(mlp_ref, dims, n_mlp, calculate_strategy="abs_mean")
    engine, _opt, _sched, sel_mlp, sel_att = trainer.select_and_convert(
        engine, harvester, dims, n_att, n_mlp, calculate_strategy="abs_mean", smt_lr=1e-4,
        num_training_steps=10, ds_config=ds)
    assert list(sel_mlp.items()) == list(want_mlp.items())
    assert list(dict(sel_att).items()) == list(dict(want_att).items())
    assert engine.tile_groups and all(tg.param.dtype == dtype for tg in engine.tile_groups)
    for b in bench.batches(3, 2, 128, bench.MODELS["mini"]["vocab_size"], 0, DEV, offset=7):
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        engine.step()
        assert torch.isfinite(loss).item()
    for mod in model.modules():
        if isinstance(mod, smt.LinearLayer_MatrixSparsity):
            assert torch.equal(ref.gather_tiles(mod.weight.detach().cpu(), mod.index_list), mod.selected_weight.detach().cpu())


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_channel_path_through_the_engine_in_dtype(dtype):
    """The channel (activation-selected rows) path, fine_tune.py:406-709, in the reference's fp16 /
    fp32: harvest -> select -> convert -> engine with DeepSpeed's dtype config. The selected rows are
    dense parameters of the model's dtype for the engine (fp16 under the loss scale); 4 steps run
    with finite losses, and the rows written back into W are the rows' values in that dtype."""
    import bench
    import numpy as np
    from sparse_matrix_tuning_amd import trainer
    cfg = dict(bench.MODELS["mini"])
    cfg["num_hidden_layers"] = 2
    cfg["num_key_value_heads"] = cfg["num_attention_heads"]
    bench.MODELS["_tcd"] = cfg
    try:
        model = bench.build_model("_tcd", DEV).to(dtype)
    finally:
        del bench.MODELS["_tcd"]
    ds = {"gradient_clipping": 1.0, "fp16": ({"enabled": True, "loss_scale_window": 100}
                                             if dtype == torch.float16 else {"enabled": False})}
    h = trainer.ActivationHarvester(model, num_mlp_channel=0, num_attention_channel=24)
    ids = torch.randint(0, 4096, (2, 128), generator=torch.Generator().manual_seed(7)).to(DEV)
    h.collect({"input_ids": ids})
    engine, _opt, _sched, sel_mlp, sel_att = trainer.select_and_convert_channels(
        model, h, num_attention_channel=24, num_mlp_channel=0, ft_learning_rate=1e-3, num_training_steps=10,
        ds_config=ds)
    assert sum(len(v) for v in sel_att.values()) == 24
    assert (engine.loss_scaler is not None) == (dtype == torch.float16)
    mods = {n: m for n, m in model.named_modules() if isinstance(m, smt.LinearLayer_ChannelSparsity)}
    assert mods and all(m.selected_weight.dtype == dtype for m in mods.values())
    before = {n: m.selected_weight.detach().clone() for n, m in mods.items()}
    losses = []
    for _ in range(4):
        o = engine(input_ids=ids, labels=ids, use_cache=False)
        engine.backward(o.loss)
        engine.step()
        losses.append(o.loss.item())
    assert all(np.isfinite(losses)), losses
    assert engine.global_steps - engine.skipped_steps >= 2
    assert any(not torch.equal(before[n], m.selected_weight.detach()) for n, m in mods.items())
    for n, m in mods.items():
        m(torch.zeros(1, 1, m.weight.shape[1], dtype=dtype, device=DEV))     # the per-forward write-back
        assert torch.equal(m.weight.detach()[m.index_list].cpu(), m.selected_weight.detach().cpu())
