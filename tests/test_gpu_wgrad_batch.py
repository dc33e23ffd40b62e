"""Batched tile weight gradient (``smt_tile_wgrad_batch``): the tiles of several SMT modules that
share T in one launch, as the engine's WgradBatcher issues them in backward.

Each module's tiles must equal what ``smt_tile_wgrad`` computes for that module (smt.py:397-404):
- bit-exact where the split is the same (one module in the batch, or modules that are column
  slices of one operand pair, so the batch IS one module's tile list);
- otherwise against fp64 truth at the fp32 sink bar (1e-5), since the split over T follows the
  batch's tile count.
Shapes: LLaMA-3-8B modules at the bench's T = 32768 (q, k, gate, down; packed and row-major inputs;
quarter-tile, slab and direct paths), plus the engine end to end against the unbatched engine.
"""
import pytest
import torch

from sparse_matrix_tuning_amd import _hip

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
T = 32768
SHAPES = {"q_proj": (4096, 4096), "k_proj": (1024, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def _tiles(out_f, in_f, n, seed):
    rb, cb = out_f // 256, in_f // 256
    g = torch.Generator().manual_seed(seed)
    flat = torch.randperm(rb * cb, generator=g)[:n].tolist()
    return [(f // cb, f % cb) for f in flat]


def _operands(out_f, in_f, seed, t=T):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(t, in_f, generator=g, device=DEV).bfloat16()
    go = (torch.randn(t, out_f, generator=g, device=DEV) * 1e-2).bfloat16()
    return go, x


def _truth(go, x, r, c):
    return go[:, r * 256:(r + 1) * 256].double().t() @ x[:, c * 256:(c + 1) * 256].double()


def _packed(x, tiles):
    cbs = []
    for _r, c in tiles:
        if c not in cbs:
            cbs.append(c)
    xp = _hip.colblock_gather(x, torch.tensor(cbs, dtype=torch.int32, device=DEV))
    pos = {c: i for i, c in enumerate(cbs)}
    return xp, [(r, pos[c]) for r, c in tiles]


@pytest.mark.parametrize("n", [5, 27, 300])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_single_module_batch_bit_exact(n, out_dtype):
    """A batch of one module runs the same kernels with the same split as smt_tile_wgrad."""
    out_f, in_f = SHAPES["gate_proj"]
    go, x = _operands(out_f, in_f, seed=n)
    tiles = _tiles(out_f, in_f, n, seed=n)
    ref = torch.empty(n * 256, 256, dtype=out_dtype, device=DEV)
    _hip.tile_wgrad(go, x, _hip.tile_table(tiles, DEV), ref, order=_hip.order_table(tiles, DEV))
    out = torch.empty_like(ref)
    tab, order = _hip.wgrad_batch_table([tiles], DEV)
    _hip.tile_wgrad_batch([(go, x, out, False)], tab, order)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_batch_of_slices_equals_one_module():
    """Modules that read one (g, x) pair: the batch equals smt_tile_wgrad over their concatenated
    tile list bit for bit, whatever the order the schedule visits them in."""
    out_f, in_f = SHAPES["q_proj"]
    go, x = _operands(out_f, in_f, seed=3)
    tiles = _tiles(out_f, in_f, 36, seed=3)
    parts = [tiles[:9], tiles[9:17], tiles[17:30], tiles[30:]]
    ref = torch.empty(36 * 256, 256, dtype=torch.float32, device=DEV)
    _hip.tile_wgrad(go, x, _hip.tile_table(tiles, DEV), ref)
    outs = [torch.empty(len(p) * 256, 256, dtype=torch.float32, device=DEV) for p in parts]
    tab, order = _hip.wgrad_batch_table(parts, DEV)
    _hip.tile_wgrad_batch([(go, x, o, False) for o in outs], tab, order)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), ref)


@pytest.mark.parametrize("total", [8, 24, 48])
def test_mixed_modules_vs_fp64(total):
    """q, k, gate (row-major input) and down (packed block-major input) in one launch, with
    accumulation on two of them, fp32 outputs: every tile within 1e-5 of fp64 truth."""
    per = {"q_proj": total // 4, "k_proj": total // 4, "gate_proj": total // 4, "down_proj": total - 3 * (total // 4)}
    items, tile_lists, checks = [], [], []
    for k, (name, n) in enumerate(per.items()):
        out_f, in_f = SHAPES[name]
        go, x = _operands(out_f, in_f, seed=10 + k)
        tiles = _tiles(out_f, in_f, n, seed=20 + k)
        acc = k % 2 == 1
        out = (torch.randn(n * 256, 256, device=DEV) * 1e-3) if acc else torch.empty(n * 256, 256, device=DEV)
        prior = out.clone()
        if name == "down_proj":
            xk, ktiles = _packed(x, tiles)
        else:
            xk, ktiles = x, tiles
        items.append((go, xk, out, acc))
        tile_lists.append(ktiles)
        checks.append((go, x, tiles, out, prior, acc))
    tab, order = _hip.wgrad_batch_table(tile_lists, DEV)
    _hip.tile_wgrad_batch(items, tab, order)
    torch.cuda.synchronize()
    for go, x, tiles, out, prior, acc in checks:
        for i in (0, len(tiles) // 2, len(tiles) - 1):
            r, c = tiles[i]
            truth = _truth(go, x, r, c) + (prior[i * 256:(i + 1) * 256].double() if acc else 0)
            err = _rel(out[i * 256:(i + 1) * 256], truth)
            assert err < 1e-5, (r, c, acc, err)


def test_batch_rejects_bad_arguments():
    go, x = _operands(1024, 1024, seed=1, t=512)
    out = torch.empty(256, 256, device=DEV)
    tab, order = _hip.wgrad_batch_table([[(0, 0)]], DEV)
    with pytest.raises(ValueError):
        _hip.tile_wgrad_batch([(go, x, out, False)], tab.view(-1)[:2].view(1, 2), None)
    with pytest.raises(ValueError):
        _hip.tile_wgrad_batch([(go, x, out, False)] * (_hip.WGRAD_MAX_MODULES + 1), tab, order)
    go2, _ = _operands(1024, 1024, seed=2, t=256)
    with pytest.raises(ValueError):          # modules with different T
        _hip.tile_wgrad_batch([(go, x, out, False), (go2, x, out, False)], tab, order)


def _mini_engine(batch_tiles, seed=0):
    from sparse_matrix_tuning_amd import engine as eng
    from sparse_matrix_tuning_amd.smt import smt

    torch.manual_seed(seed)
    layers = torch.nn.ModuleList()
    for _ in range(3):
        layers.append(torch.nn.ModuleDict({
            "q_proj": torch.nn.Linear(1024, 1024, bias=False),
            "k_proj": torch.nn.Linear(1024, 512, bias=False),
            "up_proj": torch.nn.Linear(1024, 2048, bias=False),
            "down_proj": torch.nn.Linear(2048, 1024, bias=False)}))
    model = torch.nn.Module()
    model.layers = layers
    model = model.to(DEV).bfloat16()
    sel = {}
    for li, layer in enumerate(model.layers):
        for name, lin in layer.items():
            rb, cb = lin.weight.shape[0] // 256, lin.weight.shape[1] // 256
            sel[f"layers.{li}.{name}"] = _tiles(rb * 256, cb * 256, min(3 + li, rb * cb), seed=li * 7 + len(name))
    for name, tl in sel.items():
        smt._replace(model, name, tl)
    params = [m.selected_weight for m in model.modules() if isinstance(m, smt.LinearLayer_MatrixSparsity)]
    opt = eng.SMTFusedAdam(params, lr=1e-3)
    engine, *_ = eng.initialize(model=model, optimizer=opt,
                                # single rounding: batched and per-module launches split T differently,
                                # which fp32 sums absorb (1e-6) but a per-sample bf16 rounding may not
                                config={"gradient_clipping": 1.0, "wgrad_batch_tiles": batch_tiles,
                                        "wgrad_rounding": "single"})

    def fwd(x):
        for layer in model.layers:
            h = layer["q_proj"](x) + torch.nn.functional.pad(layer["k_proj"](x), (0, 512))
            x = x + layer["down_proj"](torch.nn.functional.silu(layer["up_proj"](h)))
        return x
    return engine, fwd


def test_engine_batched_equals_unbatched():
    """The engine with batched tile launches gives the same tile gradients (fp32, within the sink
    bar) and, through the same AdamW, the same tiles as one launch per module; two steps."""
    x = torch.randn(4, 512, 1024, device=DEV).bfloat16()
    res = {}
    for bt in (0, 10, 48):
        engine, fwd = _mini_engine(bt)
        for _ in range(2):
            loss = fwd(x).float().pow(2).mean()
            engine.backward(loss)
            grads = [tg.grad.clone() for tg in engine.tile_groups]
            engine.step()
        res[bt] = (grads, [tg.master.clone() for tg in engine.tile_groups])
    for bt in (10, 48):
        for a, b in zip(res[bt][0], res[0][0]):
            assert _rel(a, b) < 1e-6
        for a, b in zip(res[bt][1], res[0][1]):
            assert _rel(a, b) < 1e-6
    assert engine.wgrad_batcher is not None and not engine.wgrad_batcher.pending


def test_engine_batcher_module_used_twice():
    """A module whose backward runs twice in one pass accumulates (the batcher launches the first
    use before queueing the second)."""
    x = torch.randn(2, 256, 1024, device=DEV).bfloat16()
    out = {}
    for bt in (0, 48):
        engine, _fwd = _mini_engine(bt, seed=1)
        q = engine.module.layers[0]["q_proj"]
        loss = (q(q(x)).float().pow(2).mean())
        engine.backward(loss)
        out[bt] = engine.tile_groups[0].grad.clone()
    assert _rel(out[48], out[0]) < 1e-6


# ---- MX-fp8 operands (config 5) -----------------------------------------------------------------
def _mx_module(out_f, in_f, n, seed, t=T):
    go, x = _operands(out_f, in_f, seed, t)
    tiles = _tiles(out_f, in_f, n, seed)
    rbs, cbs = [], []
    for r, c in tiles:
        if r not in rbs:
            rbs.append(r)
        if c not in cbs:
            cbs.append(c)
    gq = _hip.mx_quant_cols(go, torch.tensor(rbs, dtype=torch.int32, device=DEV))
    xq = _hip.mx_quant_cols(x, torch.tensor(cbs, dtype=torch.int32, device=DEV))
    ktiles = [(rbs.index(r), cbs.index(c)) for r, c in tiles]
    return gq, xq, ktiles


@pytest.mark.parametrize("n", [6, 40])
def test_mx_single_module_batch_bit_exact(n):
    gq, xq, kt = _mx_module(*SHAPES["gate_proj"], n, seed=n)
    ref = torch.empty(n * 256, 256, device=DEV)
    _hip.tile_wgrad_mx(gq, xq, _hip.tile_table(kt, DEV), ref, order=_hip.order_table(kt, DEV))
    out = torch.empty_like(ref)
    tab, order = _hip.wgrad_batch_table([kt], DEV)
    _hip.tile_wgrad_mx_batch([(gq, xq, out, False)], tab, order)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("total", [8, 44])
def test_mx_mixed_modules_vs_per_module(total):
    """q, k, gate, down MX operands in one launch (two of them accumulating): each module's tiles
    equal its own smt_tile_wgrad_mx launch to fp32 rounding (1e-5; only the split over T differs)."""
    per = {"q_proj": total // 4, "k_proj": total // 4, "gate_proj": total // 4, "down_proj": total - 3 * (total // 4)}
    items, kts, refs = [], [], []
    for k, (name, n) in enumerate(per.items()):
        gq, xq, kt = _mx_module(*SHAPES[name], n, seed=30 + k)
        acc = k % 2 == 0
        prior = torch.randn(n * 256, 256, device=DEV) * 1e-3
        ref = prior.clone()
        _hip.tile_wgrad_mx(gq, xq, _hip.tile_table(kt, DEV), ref, accumulate=acc)
        out = prior.clone()
        items.append((gq, xq, out, acc))
        kts.append(kt)
        refs.append(ref)
    tab, order = _hip.wgrad_batch_table(kts, DEV)
    _hip.tile_wgrad_mx_batch(items, tab, order)
    torch.cuda.synchronize()
    for (_g, _x, out, _a), ref in zip(items, refs):
        assert _rel(out, ref) < 1e-5


def test_engine_fp8_batched_equals_unbatched():
    """The fp8 engine (MX tile wgrad) with batched launches: the same tile gradients as one launch
    per module (fp32 rounding), over two steps of the mini LLaMA."""
    import bench
    from collections import defaultdict
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.smt import smt

    def run(bt):
        cfg = dict(bench.MODELS["mini"], num_hidden_layers=2)
        bench.MODELS["_b"] = cfg
        try:
            model = bench.build_model("_b", DEV)
        finally:
            del bench.MODELS["_b"]
        sel_mlp = defaultdict(list, {("up_proj", 1): [(2, 1), (0, 0)], ("down_proj", 0): [(1, 0), (0, 1)],
                                     ("gate_proj", 1): [(1, 1)]})
        sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)], ("k_proj", 1): [(0, 0)], ("v_proj", 1): [(0, 1)]})
        smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
        smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
        opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3, betas=(0.9, 0.95))
        engine, *_ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0, "fp8_linears": True,
                                                                    "wgrad_batch_tiles": bt})
        ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
        grads = []
        for _ in range(2):
            loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
            engine.backward(loss)
            grads.append([tg.grad.clone() for tg in engine.tile_groups])
            engine.step()
        return grads

    a, b = run(0), run(48)
    for ga, gb in zip(a, b):
        for x, y in zip(ga, gb):
            assert _rel(y, x) < 1e-5


def test_engine_batcher_flushes_on_a_different_T():
    """Modules whose inputs have different row counts in one backward (here two separate inputs
    through different modules) go out in separate launches, each exact."""
    out = {}
    for bt in (0, 48):
        engine, _fwd = _mini_engine(bt, seed=2)
        l0 = engine.module.layers[0]
        xa = torch.randn(2, 256, 1024, device=DEV).bfloat16()
        xb = torch.randn(1, 384, 1024, device=DEV).bfloat16()
        loss = l0["q_proj"](xa).float().pow(2).mean() + l0["up_proj"](xb).float().pow(2).mean()
        engine.backward(loss)
        out[bt] = engine.tile_groups[0].grad.clone()
    assert _rel(out[48], out[0]) < 1e-6


def test_fp8_group_shares_mx_input_blocks():
    """q/k/v (gate/up) of one layer quantise their shared input's MX column blocks once, for the
    union of the blocks their tiles read; the tile gradients equal the per-module quantisation's
    (the MX values of a block do not depend on which other blocks are quantised with it)."""
    import bench
    from collections import defaultdict
    from sparse_matrix_tuning_amd import engine as eng
    from sparse_matrix_tuning_amd.smt import smt

    def run(share):
        cfg = dict(bench.MODELS["mini"], num_hidden_layers=1)
        bench.MODELS["_s"] = cfg
        try:
            model = bench.build_model("_s", DEV)
        finally:
            del bench.MODELS["_s"]
        sel_att = defaultdict(list, {("q_proj", 0): [(1, 1), (0, 0)], ("k_proj", 0): [(0, 1)], ("v_proj", 0): [(0, 0)]})
        sel_mlp = defaultdict(list, {("gate_proj", 0): [(2, 1)], ("up_proj", 0): [(1, 0), (0, 1)]})
        smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
        smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
        opt = eng.SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3)
        engine, *_ = eng.initialize(model=model, optimizer=opt, config={"fp8_linears": True})
        if not share:
            for tg in engine.tile_groups:
                for g, _cb in tg.fp8_groups:
                    g.mx_union = None
        calls = []
        orig = smt._hip.mx_quant_cols
        smt._hip.mx_quant_cols = lambda x, b: (calls.append(b.numel()), orig(x, b))[1]
        try:
            ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
            loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
            engine.backward(loss)
        finally:
            smt._hip.mx_quant_cols = orig
        return [tg.grad.clone() for tg in engine.tile_groups], calls

    shared, c_shared = run(True)
    alone, c_alone = run(False)
    # forward input quantisations: 2 groups once each vs 5 modules (backward: one per module either way)
    assert len(c_shared) == len(c_alone) - 3
    for a, b in zip(shared, alone):
        assert torch.equal(a, b)


def _tensors_in(obj, seen=None) -> int:
    """Count torch tensors reachable through tuples / lists / dicts (not through other objects)."""
    if isinstance(obj, torch.Tensor):
        return 1
    if isinstance(obj, (tuple, list)):
        return sum(_tensors_in(o) for o in obj)
    if isinstance(obj, dict):
        return sum(_tensors_in(o) for o in obj.values())
    return 0


@pytest.mark.parametrize("fp8", [False, True])
def test_engine_batcher_holds_no_operands(fp8):
    """The batcher's launch-table cache keeps the objects its keys name (TileIndex, the column map)
    and the device tables, never an operand: a cached output gradient or saved input stayed allocated
    for the whole run (+50 GB at the 8B point). Memory after a step is the same every step."""
    x = torch.randn(4, 512, 1024, device=DEV).bfloat16()
    engine, fwd = _mini_engine(10)
    if fp8:
        import bench
        from collections import defaultdict
        from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
        from sparse_matrix_tuning_amd.smt import smt
        cfg = dict(bench.MODELS["mini"], num_hidden_layers=2)
        bench.MODELS["_h"] = cfg
        try:
            model = bench.build_model("_h", DEV)
        finally:
            del bench.MODELS["_h"]
        sel_mlp = defaultdict(list, {("up_proj", 1): [(2, 1), (0, 0)], ("gate_proj", 1): [(1, 1)]})
        sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)], ("k_proj", 0): [(0, 0)], ("v_proj", 0): [(0, 1)]})
        smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
        smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
        opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3)
        engine, *_ = initialize(model=model, optimizer=opt, config={"fp8_linears": True, "wgrad_batch_tiles": 2})
        ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
        fwd = lambda _x: engine(input_ids=ids, labels=ids, use_cache=False).loss
    used = []
    for _ in range(3):
        out = fwd(x)
        loss = out if out.dim() == 0 else out.float().pow(2).mean()
        engine.backward(loss)
        engine.step()
        del out, loss
        torch.cuda.synchronize()
        used.append(torch.cuda.memory_allocated(DEV))
    assert engine.wgrad_batcher._tables
    for tab, held in engine.wgrad_batcher._tables.values():
        assert _tensors_in(held) == 0
    assert used[1] == used[2]
