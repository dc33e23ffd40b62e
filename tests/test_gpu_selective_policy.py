"""Activation policy "selective" (VERDICT r02 item 8): SMT linears fed by an RMSNorm or SwiGLU keep no
input blocks between forward and backward; the backward rebuilds the column blocks from the
producer's own saved operands (smt_colblock_recompute). The reference keeps the input's column
slices (deepspeed/smt/smt.py:351-358, ctx.list1); the tile gradients must not change at all."""
from collections import defaultdict

import pytest
import torch

from sparse_matrix_tuning_amd import _hip
from sparse_matrix_tuning_amd import fused_llama as fl
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("T,H,cbs", [(4096, 4096, [0, 3, 15]), (300, 1024, [2]), (1, 512, [1, 0])])
def test_recompute_rmsnorm_blocks_bit_exact(T, H, cbs):
    g = torch.Generator(device=DEV).manual_seed(T + H)
    x = torch.randn(T, H, device=DEV, generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).bfloat16()
    cb = torch.tensor(cbs, dtype=torch.int32, device=DEV)
    xr = x.clone().requires_grad_()
    y = fl.FusedRMSNormFn.apply(xr, w, 1e-5)
    rstd = y.grad_fn.saved_tensors[2]
    got = _hip.colblock_recompute(_hip.RECOMPUTE_RMSNORM, x, cb, weight=w, rstd=rstd)
    want = _hip.colblock_gather(y.detach(), cb)
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


@pytest.mark.parametrize("T,H,cbs", [(2048, 4096, [5, 1]), (64, 8192, [31])])
def test_recompute_add_rmsnorm_blocks_bit_exact(T, H, cbs):
    g = torch.Generator(device=DEV).manual_seed(T)
    x = torch.randn(T, H, device=DEV, generator=g).bfloat16()
    r = torch.randn(T, H, device=DEV, generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).bfloat16()
    cb = torch.tensor(cbs, dtype=torch.int32, device=DEV)
    h, y = fl.FusedAddRMSNormFn.apply(x.requires_grad_(), r, w, 1e-5)
    hs, _w, rstd = y.grad_fn.saved_tensors
    got = _hip.colblock_recompute(_hip.RECOMPUTE_RMSNORM, hs, cb, weight=_w, rstd=rstd)
    want = _hip.colblock_gather(y.detach(), cb)
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


@pytest.mark.parametrize("T,I,cbs", [(4096, 14336, [0, 55, 17]), (100, 512, [1])])
def test_recompute_swiglu_blocks_bit_exact(T, I, cbs):
    g = torch.Generator(device=DEV).manual_seed(I)
    gate = (3 * torch.randn(T, I, device=DEV, generator=g)).bfloat16()
    up = torch.randn(T, I, device=DEV, generator=g).bfloat16()
    cb = torch.tensor(cbs, dtype=torch.int32, device=DEV)
    h = fl.FusedSwiGLUFn.apply(gate, up)
    got = _hip.colblock_recompute(_hip.RECOMPUTE_SWIGLU, gate, cb, b2d=up)
    want = _hip.colblock_gather(h, cb)
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


def test_recompute_validation():
    x = torch.zeros(8, 512, dtype=torch.bfloat16, device=DEV)
    cb = torch.tensor([0], dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError, match="null weight"):
        _hip.colblock_recompute(_hip.RECOMPUTE_RMSNORM, x, cb)
    with pytest.raises(RuntimeError, match="null up"):
        _hip.colblock_recompute(_hip.RECOMPUTE_SWIGLU, x, cb)


CFG = dict(vocab_size=4096, hidden_size=4096, intermediate_size=14336, num_hidden_layers=2,
           num_attention_heads=32, num_key_value_heads=8, rope_theta=500000.0, rms_norm_eps=1e-5,
           tie_word_embeddings=False, max_position_embeddings=4096)


def _model():
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(**CFG)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(5)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(DEV):
            model = LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)
    sel_att = defaultdict(list, {("q_proj", 0): [(15, 3), (0, 0)], ("k_proj", 1): [(3, 15)], ("v_proj", 0): [(2, 2)],
                                 ("o_proj", 1): [(4, 9)]})
    sel_mlp = defaultdict(list, {("gate_proj", 0): [(55, 0)], ("up_proj", 1): [(0, 15), (31, 4)],
                                 ("down_proj", 0): [(15, 55), (0, 1)], ("down_proj", 1): [(3, 3)]})
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    return model


def _step(model, ids, policy):
    """One forward + backward; returns the loss, the tile gradients and the bytes of the distinct
    storages the autograd graph keeps for the backward (saved-tensor hooks)."""
    old = smt.set_activation_policy(policy)
    kept = {}

    def pack(t):
        st = t.untyped_storage()
        kept[st.data_ptr()] = st.nbytes()
        return t

    try:
        model.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated(DEV)
        with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
            out = model(input_ids=ids, labels=ids, use_cache=False)
        torch.cuda.synchronize()
        print(f"\n{policy}: allocated after forward {(torch.cuda.memory_allocated(DEV) - base) / 1e6:.1f} MB")
        held = sum(kept.values())
        out.loss.backward()
        torch.cuda.synchronize()
    finally:
        smt.set_activation_policy(old)
    grads = {n: m.selected_weight.grad.clone() for n, m in model.named_modules()
             if isinstance(m, smt.LinearLayer_MatrixSparsity)}
    return out.loss.detach(), grads, held


def test_selective_policy_same_tile_grads_less_memory():
    model = _model()
    fl.patch_llama(model)
    try:
        gen = torch.Generator().manual_seed(9)
        ids = torch.randint(1, CFG["vocab_size"], (2, 1024), generator=gen).to(DEV)
        loss_r, grads_r, held_r = _step(model, ids, "resident")
        loss_s, grads_s, held_s = _step(model, ids, "selective")
        loss_v, grads_v, held_v = _step(model, ids, "views")
        loss_r2, grads_r2, _ = _step(model, ids, "resident")
    finally:
        fl.unpatch_llama()
    print(f"\nsaved for backward: resident {held_r / 1e6:.1f} MB, selective {held_s / 1e6:.1f} MB, "
          f"views {held_v / 1e6:.1f} MB")
    assert torch.equal(loss_r, loss_r2)               # the step itself is deterministic
    assert torch.equal(loss_r, loss_s) and torch.equal(loss_r, loss_v)
    assert grads_r.keys() == grads_s.keys() == grads_v.keys() and len(grads_r) == 8
    for n in grads_r:
        assert torch.equal(grads_r[n], grads_r2[n]), n
        assert torch.equal(grads_r[n], grads_s[n]), n
        assert torch.equal(grads_r[n], grads_v[n]), n
    assert held_s < held_r < held_v                   # views keep whole inputs (the reference's ctx.list1)


def test_selective_policy_detects_in_place_change():
    x = torch.randn(1, 64, 512, device=DEV).bfloat16().requires_grad_()
    w = torch.ones(512, dtype=torch.bfloat16, device=DEV)
    lin = torch.nn.Linear(512, 512, bias=False, device=DEV, dtype=torch.bfloat16)
    m = smt.LinearLayer_MatrixSparsity(lin.weight, index_list=[(0, 1)])
    old = smt.set_activation_policy("selective")
    try:
        y = fl.FusedRMSNormFn.apply(x, w, 1e-5)
        out = m(y)
        with torch.no_grad():
            y.grad_fn.saved_tensors[0].add_(1)        # the producer's operand changes after the forward
        with pytest.raises(RuntimeError, match="modified in place"):
            out.float().sum().backward()
    finally:
        smt.set_activation_policy(old)


def test_selective_policy_through_the_engine_bit_identical():
    """Under the engine the rebuilt blocks are made on the wgrad stream (beside the data-gradient
    GEMMs, like the forward's block copies): two SMT steps with "activation_policy": "selective" give
    the same loss, tile optimizer state and W as with "resident", bit for bit."""
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize

    def run(policy):
        model = _model()
        fl.patch_llama(model)
        try:
            groups = smt.get_optimizer_sparse_grouped_parameters(model, 0.0, smt_lr=1e-3)
            opt = SMTFusedAdam(groups, lr=1e-3, betas=(0.9, 0.95))
            eng, _, _, _ = initialize(model=model, optimizer=opt,
                                      config={"gradient_clipping": 1.0, "activation_policy": policy})
            assert eng.wgrad_stream is not None
            losses = []
            for i in range(2):
                ids = torch.randint(1, CFG["vocab_size"], (2, 1024), generator=torch.Generator().manual_seed(20 + i)).to(DEV)
                loss = eng(input_ids=ids, labels=ids, use_cache=False).loss
                eng.backward(loss)
                eng.step()
                losses.append(loss.detach())
            torch.cuda.synchronize()
            tg = eng.tile_groups[0]
            W = {n: m.weight.detach().clone() for n, m in model.named_modules()
                 if isinstance(m, smt.LinearLayer_MatrixSparsity)}
            return losses, tg.master.clone(), tg.exp_avg_sq.clone(), W
        finally:
            fl.unpatch_llama(model)

    lr_, mr, vr, Wr = run("resident")
    ls_, ms, vs, Ws = run("selective")
    assert all(torch.equal(a, b) for a, b in zip(lr_, ls_))
    assert torch.equal(mr, ms) and torch.equal(vr, vs)
    assert Wr.keys() == Ws.keys() and all(torch.equal(Wr[n], Ws[n]) for n in Wr)
