"""fp8 path (config 5): e4m3 quantisation kernels bit-exact vs torch, fp8
linears vs the bf16 path, and the engine keeping the fp8 copies in step with the trained tiles.

The reference has no fp8, so parity is stated against the build's bf16 path (parity unpinned by the
reference). Tolerances: the quantisation bytes and scales are bit-exact against
``scale = amax * (1/448)``, ``(x.float() / scale).to(float8_e4m3fn)``; an fp8 GEMM is within 2e-3 relative of the fp32 product
of its own quantised operands; against the bf16 GEMM it is within 8 % relative (two e4m3 roundings,
3 mantissa bits, per element); a 2-layer model's loss is within 1 % of the bf16 path's."""
import pytest
import torch
from torch import nn

from sparse_matrix_tuning_amd import _hip
from sparse_matrix_tuning_amd import fp8 as f8
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm()).item()


def _ref_rows(x):
    amax = x.float().abs().amax(dim=1)
    scale = torch.where(amax > 0, amax * (1.0 / 448.0), torch.ones_like(amax))     # fp32 reciprocal, as ATen
    return (x.float() / scale[:, None]).to(torch.float8_e4m3fn), scale


@pytest.mark.parametrize("rows,cols", [(64, 4096), (300, 1024), (17, 14336), (9, 16392)])   # register variants + two-pass
def test_quant_rows_bit_exact(rows, cols):
    torch.manual_seed(rows)
    x = (torch.randn(rows, cols, device=DEV) * torch.logspace(-3, 2, rows, device=DEV)[:, None]).bfloat16()
    x[3 % rows] = 0                                          # an all-zero row: scale 1
    q, s = f8.quant_rows(x)
    rq, rs = _ref_rows(x)
    assert torch.equal(s, rs)
    assert torch.equal(q.view(torch.uint8), rq.view(torch.uint8))


def test_quant_rows_selected_blocks_only():
    x = torch.randn(1024, 512, device=DEV).bfloat16()
    q, s = f8.quant_rows(x)
    x2 = x.clone()
    x2[256:512] *= 3
    x2[768:] *= 0.5
    blocks = torch.tensor([1, 3], dtype=torch.int32, device=DEV)
    f8.quant_rows(x2, blocks, out=q, scales=s)
    rq, rs = _ref_rows(x2)
    assert torch.equal(s, rs) and torch.equal(q.view(torch.uint8), rq.view(torch.uint8))


@pytest.mark.parametrize("rows,cols", [(1024, 4096), (4096, 1024), (192, 512), (14400, 768)])   # 256-row segments, ragged last
def test_quant_cols_t_bit_exact(rows, cols):
    torch.manual_seed(cols)
    w = (torch.randn(rows, cols, device=DEV) * torch.logspace(-2, 1, cols, device=DEV)[None, :]).bfloat16()
    qt, s = f8.quant_cols_t(w)
    rq, rs = _ref_rows(w.t().contiguous())
    assert qt.shape == (cols, rows)
    assert torch.equal(s, rs) and torch.equal(qt.view(torch.uint8), rq.view(torch.uint8))
    # a subset of column blocks
    w2 = w.clone()
    w2[:, 256:512] *= 4
    f8.quant_cols_t(w2, torch.tensor([1], dtype=torch.int32, device=DEV), out_t=qt, scales=s)
    rq2, rs2 = _ref_rows(w2.t().contiguous())
    assert torch.equal(s, rs2) and torch.equal(qt.view(torch.uint8), rq2.view(torch.uint8))


def test_fp8_gemm_vs_quantised_fp32_and_bf16():
    torch.manual_seed(5)
    x = torch.randn(512, 1024, device=DEV).bfloat16()
    W = (torch.randn(768, 1024, device=DEV) * 0.05).bfloat16()
    fw = f8.Fp8Weight(W)
    y = f8.fp8_linear_forward(x, fw)
    xq, xs = _ref_rows(x)
    exact = (xq.float() * xs[:, None]) @ (fw.w8.float() * fw.sw[:, None]).t()
    assert _rel(y, exact) < 2e-3
    assert _rel(y, x.float() @ W.float().t()) < 8e-2
    g = torch.randn(512, 768, device=DEV).bfloat16()
    gi = f8.fp8_linear_dgrad(g, fw)
    assert _rel(gi, g.float() @ W.float()) < 8e-2


def test_smt_module_fp8_forward_backward():
    torch.manual_seed(6)
    W = nn.Parameter((torch.randn(512, 768) * 0.05).bfloat16().to(DEV), requires_grad=False)
    mod = smt.LinearLayer_MatrixSparsity(W, index_list=[(1, 2), (0, 0)])
    x = torch.randn(2, 64, 768).bfloat16().to(DEV)
    g = torch.randn(2, 64, 512).bfloat16().to(DEV)
    xb = x.clone().requires_grad_(True)
    mod(xb).backward(g)
    gi_bf16, gw_bf16 = xb.grad.clone(), mod.selected_weight.grad.clone()
    mod.selected_weight.grad = None
    W._smt_fp8 = f8.Fp8Weight(W)
    x8 = x.clone().requires_grad_(True)
    y8 = mod(x8)
    y8.backward(g)
    assert _rel(y8, x.float() @ W.float().t()) < 8e-2
    assert _rel(x8.grad, gi_bf16) < 8e-2
    # tile gradients: the MX-fp8 kernel on the MX column blocks of g and x (bit-identical to calling
    # it directly), within the MX quantisation bound of the bf16 path (tests/test_gpu_mx.py)
    rb, cb, table = mod.tiles.mx_tables(DEV)
    want = torch.empty_like(gw_bf16)
    _hip.tile_wgrad_mx(_hip.mx_quant_cols(g.view(-1, 512), rb), _hip.mx_quant_cols(x.view(-1, 768), cb), table, want)
    assert torch.equal(mod.selected_weight.grad, want)
    assert _rel(mod.selected_weight.grad, gw_bf16) < 6e-2
    # SMT_FP8_TILE_WGRAD=bf16: the bf16 tile kernel, bf16-exact
    mod.selected_weight.grad = None
    W._smt_fp8.mx_wgrad = False
    mod(x.clone().requires_grad_(True)).backward(g)
    assert torch.equal(mod.selected_weight.grad, gw_bf16)
    del W._smt_fp8


def test_engine_fp8_keeps_copies_in_step_and_loss_close_to_bf16():
    import bench
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from collections import defaultdict

    def run(fp8):
        cfg = dict(bench.MODELS["mini"], num_hidden_layers=2)
        bench.MODELS["_f"] = cfg
        try:
            model = bench.build_model("_f", DEV)
        finally:
            del bench.MODELS["_f"]
        sel_mlp = defaultdict(list, {("up_proj", 1): [(2, 1), (0, 0)], ("down_proj", 0): [(1, 0)]})
        sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)]})
        smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
        smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
        opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3, betas=(0.9, 0.95))
        engine, *_ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0, "fp8_linears": fp8})
        ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
        losses = []
        for _ in range(3):
            loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
            engine.backward(loss)
            engine.step()
            losses.append(loss.item())
        return engine, model, losses

    e8, m8, l8 = run(True)
    assert e8.fp8_bytes > 0
    _e, _m, lb = run(False)
    for a, b in zip(l8, lb):
        assert abs(a - b) / abs(b) < 1e-2, (l8, lb)
    # after the steps every fp8 copy equals a fresh quantisation of the (tile-updated) bf16 W
    n, groups = 0, set()
    for mod in m8.modules():
        w = getattr(mod, "weight", None)
        fw = getattr(w, "_smt_fp8", None)
        if fw is None:
            continue
        rq, rs = _ref_rows(w.detach())
        assert torch.equal(fw.sw, rs) and torch.equal(fw.w8.view(torch.uint8), rq.view(torch.uint8))
        if fw.group is None:
            tq, ts = _ref_rows(w.detach().t().contiguous())
            assert torch.equal(fw.swt, ts) and torch.equal(fw.wt8.view(torch.uint8), tq.view(torch.uint8))
        else:                                   # joint transposed copy of [W_q; W_k; W_v] / [W_gate; W_up]
            g = fw.group
            tq, ts = _ref_rows(torch.cat([x.detach() for x in g.weights], 0).t().contiguous())
            assert torch.equal(g.swt, ts) and torch.equal(g.wt8.view(torch.uint8), tq.view(torch.uint8))
            groups.add(id(g))
        n += 1
    assert n == 2 * 7                                                  # every decoder-layer linear
    assert len(groups) == 2 * 2                                        # q/k/v and gate/up per layer
    assert getattr(m8.lm_head.weight, "_smt_fp8", None) is None        # the head stays bf16


def test_quant_rows_cat_matches_quant_of_concatenation():
    torch.manual_seed(5)
    parts = [torch.randn(300, c, device=DEV).bfloat16() * s for c, s in ((4096, 1.0), (1024, 30.0), (1024, 0.01))]
    q, s = f8.quant_rows_cat(parts)
    rq, rs = _ref_rows(torch.cat(parts, 1))
    assert torch.equal(s, rs) and torch.equal(q.view(torch.uint8), rq.view(torch.uint8))
    big = [torch.randn(7, 14336, device=DEV).bfloat16(), torch.randn(7, 20000, device=DEV).bfloat16()[:, :14336]]
    q, s = f8.quant_rows_cat(big)
    rq, rs = _ref_rows(torch.cat(big, 1))
    assert torch.equal(s, rs) and torch.equal(q.view(torch.uint8), rq.view(torch.uint8))


def test_fp8_group_joint_input_grad():
    """q/k/v sharing one input: the joint fp8 data gradient is close to the bf16 sum of the three."""
    torch.manual_seed(6)
    ws = [(torch.randn(o, 512, device=DEV) * 0.02).bfloat16() for o in (512, 256, 256)]
    g = f8.Fp8Group(ws)
    fws = [f8.Fp8Weight(w, g, i) for i, w in enumerate(ws)]
    x = torch.randn(2, 128, 512, device=DEV).bfloat16().requires_grad_()
    ys = [f8.Fp8LinearFn.apply(x, w, fw, None) for w, fw in zip(ws, fws)]
    dys = [torch.randn_like(y) for y in ys]
    torch.autograd.backward(ys, dys)
    ref = sum(dy.float() @ w.float() for dy, w in zip(dys, ws))
    assert _rel(x.grad, ref) < 8e-2
    # a subset of the members (only q and v take part) falls back to per-member GEMMs on the slices
    x2 = x.detach().clone().requires_grad_()
    y0 = f8.Fp8LinearFn.apply(x2, ws[0], fws[0], None)
    y2 = f8.Fp8LinearFn.apply(x2, ws[2], fws[2], None)
    torch.autograd.backward([y0, y2], [dys[0], dys[2]])
    ref2 = dys[0].float() @ ws[0].float() + dys[2].float() @ ws[2].float()
    assert _rel(x2.grad, ref2) < 8e-2


def test_fp8_group_members_alias_one_joint_buffer():
    """The members' W are row slices of the group's joint buffer: the per-step re-quantisation reads
    it in place (no concatenation), sees in-place tile updates, and a replaced member falls back."""
    torch.manual_seed(8)
    ws = [torch.nn.Parameter((torch.randn(o, 512, device=DEV) * 0.02).bfloat16(), requires_grad=False)
          for o in (512, 256, 256)]
    vals = [w.detach().clone() for w in ws]
    g = f8.Fp8Group(ws)
    assert all(torch.equal(w, v) for w, v in zip(ws, vals))
    assert g._cat() is g.joint and g.joint.shape == (1024, 512)
    ws[1].data[0:256, 256:512] += 0.5                  # an AdamW scatter into member 1's tile
    cb = torch.tensor([1], dtype=torch.int32, device=DEV)
    g.refresh(cb)
    ref_q, ref_s = f8.quant_cols_t(torch.cat([w.detach() for w in ws], 0))
    assert torch.equal(g.wt8.view(torch.uint8), ref_q.view(torch.uint8)) and torch.equal(g.swt, ref_s)
    ws[2].data = ws[2].detach().clone()                # no longer a view: concatenated afresh
    assert g._cat() is not g.joint and torch.equal(g._cat(), torch.cat([w.detach() for w in ws], 0))


def test_fp8_rejects_cpu_and_fp32():
    with pytest.raises(RuntimeError):
        f8.quant_rows(torch.randn(4, 16).bfloat16())
    with pytest.raises(RuntimeError):
        f8.quant_rows(torch.randn(4, 16, device=DEV))
    assert "smt_quant_rows_e4m3" in _hip.ABI_FUNCTIONS


@pytest.mark.parametrize("rows,cols", [(300, 14336), (64, 1024), (5, 4104)])
def test_swiglu_bwd_quant_matches_swiglu_bwd_then_cat_quant(rows, cols):
    torch.manual_seed(cols)
    g = (torch.randn(rows, cols, device=DEV) * 3).bfloat16()
    u = torch.randn(rows, cols, device=DEV).bfloat16()
    dh = (torch.randn(rows, cols, device=DEV) * 1e-3).bfloat16()
    dg_ref, du_ref = torch.empty_like(g), torch.empty_like(u)
    rc = _hip.load().smt_swiglu_bwd(g.data_ptr(), u.data_ptr(), dh.data_ptr(), dg_ref.data_ptr(), du_ref.data_ptr(),
                                    g.numel(), _hip.DTYPE_BF16, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    q_ref, s_ref = f8.quant_rows_cat([dg_ref, du_ref])
    q, s, dg, du = f8.swiglu_bwd_quant(g, u, dh, True, True)
    assert torch.equal(s, s_ref) and torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    assert torch.equal(dg, dg_ref) and torch.equal(du, du_ref)
    q2, s2, n1, n2 = f8.swiglu_bwd_quant(g, u, dh, False, False)
    assert n1 is None and n2 is None and torch.equal(q2.view(torch.uint8), q_ref.view(torch.uint8))


@pytest.mark.parametrize("rows,cols", [(300, 14336), (7, 1024)])
def test_swiglu_bwd_quant_packed_row_blocks(rows, cols):
    """smt_swiglu_bwd_quant_e4m3_packed: the bf16 gradients hold only the mapped 256-column blocks,
    in map order (bit-identical to those blocks of the full gradients); the e4m3 rows are unchanged."""
    torch.manual_seed(rows)
    g = (torch.randn(rows, cols, device=DEV) * 3).bfloat16()
    u = torch.randn(rows, cols, device=DEV).bfloat16()
    dh = (torch.randn(rows, cols, device=DEV) * 1e-3).bfloat16()
    q_ref, s_ref, dg_ref, du_ref = f8.swiglu_bwd_quant(g, u, dh, True, True)
    nb = cols // 256
    g_tiles = smt.TileIndex([(nb - 1, 0), (1, 2), (nb - 1, 1)])          # row blocks in first-use order
    u_tiles = smt.TileIndex([(0, 0)])
    q, s, dg, du = f8.swiglu_bwd_quant(g, u, dh, ("mx_rows", g_tiles), ("mx_rows", u_tiles))
    assert dg.shape == (rows, 512) and du.shape == (rows, 256)
    assert torch.equal(dg[:, :256], dg_ref[:, (nb - 1) * 256:]) and torch.equal(dg[:, 256:], dg_ref[:, 256:512])
    assert torch.equal(du, du_ref[:, :256])
    assert torch.equal(s, s_ref) and torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    # one packed, the other not written
    _q, _s, dg2, du2 = f8.swiglu_bwd_quant(g, u, dh, ("mx_rows", u_tiles), False)
    assert du2 is None and torch.equal(dg2, dg_ref[:, :256])
    with pytest.raises(RuntimeError, match="cols % 256"):
        _hip._check(_hip.load().smt_swiglu_bwd_quant_e4m3_packed(
            g.data_ptr(), u.data_ptr(), dh.data_ptr(), rows, 1000, q.data_ptr(), q.stride(0), s.data_ptr(),
            dg.data_ptr(), g_tiles.mx_row_pack(cols, DEV)[1].data_ptr(), 512, None, None, 1000,
            torch.cuda.current_stream().cuda_stream), "smt_swiglu_bwd_quant_e4m3_packed")


def test_fp8_swiglu_packed_grad_tile_grads_bit_identical():
    """fp8 path, SMT gate/up with MX tile gradients: the SwiGLU backward hands each module only its
    tiles' row blocks of the bf16 output gradient, packed (the rest of the [T, 14336]-shaped gradient is
    never read: the group's data gradient uses the joint e4m3 rows). Tile gradients and loss are
    bit-identical to writing the whole gradient, and the MX quantisation reads the packed width."""
    import bench
    from collections import defaultdict
    from sparse_matrix_tuning_amd import engine as eng
    from sparse_matrix_tuning_amd.fused_llama import patch_llama

    def run(pack):
        cfg = dict(bench.MODELS["mini"], num_hidden_layers=1)
        bench.MODELS["_p"] = cfg
        try:
            model = bench.build_model("_p", DEV)
        finally:
            del bench.MODELS["_p"]
        patch_llama(model)
        sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)]})
        sel_mlp = defaultdict(list, {("gate_proj", 0): [(3, 1), (0, 0), (3, 0)], ("up_proj", 0): [(1, 0), (2, 1)]})
        smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
        smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
        opt = eng.SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3)
        engine, *_ = eng.initialize(model=model, optimizer=opt, config={"fp8_linears": True})
        widths, orig, old = [], smt._hip.mx_quant_cols, f8.PACK_SWIGLU_GRAD
        smt._hip.mx_quant_cols = lambda x, b: (widths.append(x.shape[1]), orig(x, b))[1]
        f8.PACK_SWIGLU_GRAD = pack
        try:
            ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
            loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
            engine.backward(loss)
        finally:
            smt._hip.mx_quant_cols, f8.PACK_SWIGLU_GRAD = orig, old
        inter = cfg["intermediate_size"]
        return loss.detach(), [tg.grad.clone() for tg in engine.tile_groups], widths, inter

    l_pack, g_pack, w_pack, inter = run(True)
    l_full, g_full, w_full, _ = run(False)
    assert torch.equal(l_pack, l_full)
    for a, b in zip(g_pack, g_full):
        assert torch.equal(a, b)
    assert w_full.count(inter) == 2 and inter not in w_pack          # gate / up: whole vs packed gradient
    assert len(w_pack) == len(w_full)                                # (2 row blocks each: 512 wide)


@pytest.mark.parametrize("pack,match", [(True, "summed with another consumer"),
                                        (False, "not the tensor its producer quantised")])
def test_fp8_packed_grad_summed_away_raises(pack, match):
    """A gate output with a second consumer: autograd sums what the SwiGLU backward hands over with
    that consumer's gradient. Packed (a zero placeholder): the row blocks never reach gate_proj's
    linearZ, so the tile gradient would miss the SwiGLU's share. Either way the group's data gradient
    would use the SwiGLU's e4m3 rows, which miss the other consumer's share. Both must raise."""
    import bench
    from collections import defaultdict
    from sparse_matrix_tuning_amd import engine as eng
    from sparse_matrix_tuning_amd import fused_llama
    from sparse_matrix_tuning_amd.fused_llama import patch_llama

    cfg = dict(bench.MODELS["mini"], num_hidden_layers=1)
    bench.MODELS["_p"] = cfg
    try:
        model = bench.build_model("_p", DEV)
    finally:
        del bench.MODELS["_p"]
    patch_llama(model)
    # q_proj trainable too: the MLP input then needs a gradient, so gate/up form their fp8 group
    sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)]})
    sel_mlp = defaultdict(list, {("gate_proj", 0): [(3, 1), (0, 0)], ("up_proj", 0): [(1, 0)]})
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    opt = eng.SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3)
    engine, *_ = eng.initialize(model=model, optimizer=opt, config={"fp8_linears": True})
    orig = fused_llama.FusedSwiGLUFn

    class TwoConsumers:
        @staticmethod
        def apply(g, u, *rest):
            return orig.apply(g, u, *rest) + 0 * g          # a second consumer of the gate output

    old = f8.PACK_SWIGLU_GRAD
    fused_llama.FusedSwiGLUFn, f8.PACK_SWIGLU_GRAD = TwoConsumers, pack
    try:
        ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
        loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
        with pytest.raises(RuntimeError, match=match):
            engine.backward(loss)
    finally:
        fused_llama.FusedSwiGLUFn, f8.PACK_SWIGLU_GRAD = orig, old
    torch.cuda.synchronize()


def test_fused_swiglu_group_grad_bit_identical_to_unfused():
    from sparse_matrix_tuning_amd.fused_llama import FusedSwiGLUFn
    torch.manual_seed(7)
    ws = [(torch.randn(1024, 512, device=DEV) * 0.02).bfloat16() for _ in range(2)]
    g = f8.Fp8Group(ws)
    fws = [f8.Fp8Weight(w, g, i) for i, w in enumerate(ws)]
    x0 = torch.randn(2, 128, 512, device=DEV).bfloat16()
    dh = torch.randn(2, 128, 1024, device=DEV).bfloat16()

    def run(fused):
        old = f8.FUSED_SWIGLU_QUANT
        f8.FUSED_SWIGLU_QUANT = fused
        try:
            x = x0.clone().requires_grad_()
            with f8.sole_swiglu_consumer():        # as fused_mlp_forward computes them
                gate = f8.Fp8LinearFn.apply(x, ws[0], fws[0], None)
                up = f8.Fp8LinearFn.apply(x, ws[1], fws[1], None)
            assert (f8.swiglu_group(gate, up) is not None) == fused
            h = FusedSwiGLUFn.apply(gate, up)
            h.backward(dh)
            return x.grad
        finally:
            f8.FUSED_SWIGLU_QUANT = old

    fused, plain = run(True), run(False)
    assert torch.equal(fused, plain)


def test_gate_up_outside_fused_mlp_fall_back_to_full_gradients():
    """packed gate/up row blocks (and the SwiGLU's pre-quantised group rows) are used only
    where fused_mlp_forward makes the SwiGLU their sole consumer. A custom MLP whose gate output has a
    second consumer trains without raising, and its tile and data gradients equal the fused MLP's."""
    import bench
    from collections import defaultdict
    from sparse_matrix_tuning_amd import engine as eng
    from sparse_matrix_tuning_amd import fused_llama
    from sparse_matrix_tuning_amd.fused_llama import FusedSwiGLUFn, patch_llama

    def custom_two(self, x):
        gate, up = self.gate_proj(x), self.up_proj(x)
        return self.down_proj(FusedSwiGLUFn.apply(gate, up) + 0 * gate)

    def custom_one(self, x):
        return self.down_proj(FusedSwiGLUFn.apply(self.gate_proj(x), self.up_proj(x)))

    results = {}
    for label, fwd in (("fused", None), ("one", custom_one), ("two", custom_two)):
        cfg = dict(bench.MODELS["mini"], num_hidden_layers=1)
        bench.MODELS["_p"] = cfg
        try:
            model = bench.build_model("_p", DEV)
        finally:
            del bench.MODELS["_p"]
        patch_llama(model)
        if fwd is not None:
            for layer in model.model.layers:
                layer.mlp.forward = fwd.__get__(layer.mlp, type(layer.mlp))
        sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)]})
        sel_mlp = defaultdict(list, {("gate_proj", 0): [(3, 1), (0, 0)], ("up_proj", 0): [(1, 0)]})
        smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
        smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
        opt = eng.SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3)
        engine, *_ = eng.initialize(model=model, optimizer=opt, config={"fp8_linears": True})
        ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
        loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
        engine.backward(loss)                       # no RuntimeError for the two-consumer graph
        torch.cuda.synchronize()
        results[label] = (loss.item(), torch.cat([tg.grad.clone() for tg in engine.tile_groups]))
        del engine, model, opt
    assert results["one"][0] == results["fused"][0] == results["two"][0]
    assert torch.equal(results["one"][1], results["fused"][1])
    assert torch.equal(results["two"][1], results["fused"][1])


@pytest.mark.parametrize("rows,cols", [(300, 14336), (17, 1024)])
def test_swiglu_fwd_quant_matches_swiglu_then_quant(rows, cols):
    torch.manual_seed(cols + 1)
    g = (torch.randn(rows, cols, device=DEV) * 3).bfloat16()
    u = torch.randn(rows, cols, device=DEV).bfloat16()
    h_ref = torch.empty_like(g)
    assert _hip.load().smt_swiglu_fwd(g.data_ptr(), u.data_ptr(), h_ref.data_ptr(), g.numel(), _hip.DTYPE_BF16,
                                      torch.cuda.current_stream().cuda_stream) == 0
    q_ref, s_ref = f8.quant_rows(h_ref)
    q, s, h = f8.swiglu_fwd_quant(g, u, True)
    assert torch.equal(h, h_ref)
    assert torch.equal(s, s_ref) and torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    q2, s2, none = f8.swiglu_fwd_quant(g, u, False)
    assert none is None and torch.equal(q2.view(torch.uint8), q_ref.view(torch.uint8))


def test_fused_swiglu_into_fp8_down_proj_bit_identical():
    from sparse_matrix_tuning_amd.fused_llama import FusedSwiGLUFn
    torch.manual_seed(8)
    Wd = (torch.randn(512, 1024, device=DEV) * 0.02).bfloat16()
    fwd = f8.Fp8Weight(Wd)
    g0 = torch.randn(2, 64, 1024, device=DEV).bfloat16()
    u0 = torch.randn(2, 64, 1024, device=DEV).bfloat16()
    dy = torch.randn(2, 64, 512, device=DEV).bfloat16()
    outs = []
    for fused in (True, False):
        g, u = g0.clone().requires_grad_(), u0.clone().requires_grad_()
        h = FusedSwiGLUFn.apply(g, u, True, False) if fused else FusedSwiGLUFn.apply(g, u)
        y = f8.Fp8LinearFn.apply(h, Wd, fwd, None)
        y.backward(dy)
        outs.append((y.detach(), g.grad, u.grad))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("H,residual,need_y", [(4096, False, True), (4096, True, False), (1024, True, True)])
def test_rmsnorm_quant_matches_rmsnorm_then_quant(H, residual, need_y):
    torch.manual_seed(H)
    rows = 300
    x = (torch.randn(rows, H, device=DEV) * 2).bfloat16()
    r = torch.randn(rows, H, device=DEV).bfloat16() if residual else None
    w = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    st = torch.cuda.current_stream().cuda_stream
    y_ref = torch.empty_like(x)
    rstd_ref = torch.empty(rows, device=DEV)
    lib = _hip.load()
    if residual:
        h_ref = torch.empty_like(x)
        assert lib.smt_add_rmsnorm_fwd(x.data_ptr(), H, r.data_ptr(), H, w.data_ptr(), h_ref.data_ptr(), H,
                                       y_ref.data_ptr(), H, rstd_ref.data_ptr(), rows, H, 1e-5, _hip.DTYPE_BF16, st) == 0
    else:
        assert lib.smt_rmsnorm_fwd(x.data_ptr(), H, w.data_ptr(), y_ref.data_ptr(), H, rstd_ref.data_ptr(), rows, H,
                                   1e-5, _hip.DTYPE_BF16, st) == 0
    q_ref, s_ref = f8.quant_rows(y_ref)
    h, y, rstd, q, s = f8.rmsnorm_quant(x, r, w, 1e-5, need_y)
    assert torch.equal(rstd, rstd_ref)
    assert torch.equal(s, s_ref) and torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    if need_y:
        assert torch.equal(y, y_ref)
    else:
        assert y is None
    if residual:
        assert torch.equal(h, h_ref)


def test_decoder_with_norm_quant_matches_unfused():
    """A patched 2-layer LLaMA (hidden 1024) on the fp8 path: the RMSNorms emitting their consumers'
    e4m3 input change nothing beyond GEMM run-to-run noise (the kernels themselves are bit-exact, above)."""
    import bench
    from sparse_matrix_tuning_amd.engine import attach_fp8_weights
    from sparse_matrix_tuning_amd.fused_llama import patch_llama
    cfg = dict(bench.MODELS["mini"], hidden_size=1024, intermediate_size=2048, num_attention_heads=8,
               num_key_value_heads=2, num_hidden_layers=2)
    bench.MODELS["_n"] = cfg
    try:
        model = bench.build_model("_n", DEV)
    finally:
        del bench.MODELS["_n"]
    patch_llama(model)
    for p in model.parameters():
        p.requires_grad_(False)
    model.model.embed_tokens.weight.requires_grad_(True)
    assert attach_fp8_weights(model) > 0
    ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(3)).to(DEV)
    out = []
    for fused in (True, False):
        old = f8.FUSED_NORM_QUANT
        f8.FUSED_NORM_QUANT = fused
        try:
            model.model.embed_tokens.weight.grad = None
            loss = model(input_ids=ids, labels=ids, use_cache=False).loss
            loss.backward()
            out.append((loss.item(), model.model.embed_tokens.weight.grad.clone()))
        finally:
            f8.FUSED_NORM_QUANT = old
    (l1, g1), (l2, g2) = out
    assert abs(l1 - l2) <= 1e-4 * abs(l2), (l1, l2)
    assert _rel(g1, g2) < 1e-3


@pytest.mark.parametrize("H", [4096, 1024])
def test_rmsnorm_bwd_add_quant_matches_bwd_then_quant(H):
    torch.manual_seed(H + 1)
    rows = 260
    x = (torch.randn(rows, H, device=DEV) * 2).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    dy = torch.randn(rows, H, device=DEV).bfloat16()
    dres = torch.randn(rows, H, device=DEV).bfloat16()
    rstd = (torch.rand(rows, device=DEV) + 0.5)
    dx_ref = torch.empty_like(x)
    assert _hip.load().smt_rmsnorm_bwd_add(dy.data_ptr(), H, x.data_ptr(), H, w.data_ptr(), rstd.data_ptr(),
                                           dres.data_ptr(), H, dx_ref.data_ptr(), H, rows, H, _hip.DTYPE_BF16,
                                           torch.cuda.current_stream().cuda_stream) == 0
    q_ref, s_ref = f8.quant_rows(dx_ref)
    dx, q, s = f8.rmsnorm_bwd_add_quant(dy, x, w, rstd, dres)
    assert torch.equal(dx, dx_ref)
    assert torch.equal(s, s_ref) and torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))


def test_fp8_layer_tail_fusion_matches_separate_add():
    """The MLP residual add fused with the next layer's input RMSNorm on the fp8 path (the norm also
    emits the next q/k/v's e4m3 rows; its backward the down_proj data gradient's): loss and gradient
    identical to the separate add + norm, and the tail is used (one more fused add+norm per layer)."""
    import bench
    from sparse_matrix_tuning_amd import fused_llama as fl
    from sparse_matrix_tuning_amd.engine import attach_fp8_weights
    cfg = dict(bench.MODELS["mini"], hidden_size=1024, intermediate_size=2048, num_attention_heads=8,
               num_key_value_heads=2, num_hidden_layers=3)
    bench.MODELS["_n"] = cfg
    try:
        model = bench.build_model("_n", DEV)
    finally:
        del bench.MODELS["_n"]
    fl.patch_llama(model)
    for p in model.parameters():
        p.requires_grad_(False)
    model.model.embed_tokens.weight.requires_grad_(True)
    assert attach_fp8_weights(model) > 0
    ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(3)).to(DEV)
    out = []
    real = fl.FusedAddRMSNormFn.apply
    for tail in (False, True):
        old = fl._LAYER_TAIL
        fl._LAYER_TAIL = tail
        calls = [0]

        def counting(*a, **k):
            calls[0] += 1
            return real(*a, **k)
        fl.FusedAddRMSNormFn.apply = counting
        try:
            model.model.embed_tokens.weight.grad = None
            loss = model(input_ids=ids, labels=ids, use_cache=False).loss
            loss.backward()
            out.append((loss.detach().clone(), model.model.embed_tokens.weight.grad.clone(), calls[0]))
        finally:
            fl._LAYER_TAIL = old
            del fl.FusedAddRMSNormFn.apply          # the inherited autograd.Function.apply again
    (l0, g0, c0), (l1, g1, c1) = out
    assert (c0, c1) == (3, 5)
    assert torch.equal(l0, l1), (l0.item(), l1.item())
    assert torch.equal(g0, g1)
