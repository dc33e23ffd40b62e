"""Shared packed input blocks (engine.attach_column_block_groups, smt.ColumnBlockGroup): q/k/v_proj
(and gate/up_proj) read one input, so they keep ONE packed copy of the union of the column blocks
their tiles read instead of one copy each. The reference keeps views of each module's column slices
(deepspeed/smt/smt.py:351-358, ctx.list1); only what is kept changes, never an operand value, so the
loss and every tile gradient must be bit-identical with and without the groups."""
from collections import defaultdict

import pytest
import torch

from sparse_matrix_tuning_amd import engine as eng
from sparse_matrix_tuning_amd import fused_llama as fl
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

CFG = dict(vocab_size=4096, hidden_size=4096, intermediate_size=14336, num_hidden_layers=2,
           num_attention_heads=32, num_key_value_heads=8, rope_theta=500000.0, rms_norm_eps=1e-5,
           tie_word_embeddings=False, max_position_embeddings=4096)

# layer 0: q/k/v share column blocks 0, 3, 7 (union {0, 3, 7, 9}); gate/up share 2 (union {0, 2, 4});
# layer 1: one q/k/v member only (no group), gate/up with disjoint blocks
SEL_ATT = {("q_proj", 0): [(15, 3), (0, 0)], ("k_proj", 0): [(1, 3), (2, 7)], ("v_proj", 0): [(0, 0), (3, 7), (1, 9)],
           ("q_proj", 1): [(4, 5)], ("o_proj", 1): [(4, 9)]}
SEL_MLP = {("gate_proj", 0): [(55, 0), (10, 2)], ("up_proj", 0): [(0, 2), (31, 4)], ("down_proj", 0): [(15, 55)],
           ("gate_proj", 1): [(3, 1)], ("up_proj", 1): [(7, 12)]}


def _model(sel_att=SEL_ATT, sel_mlp=SEL_MLP):
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
    sa, sm = defaultdict(list, sel_att), defaultdict(list, sel_mlp)
    smt.freeze_unselected_matrix_layer(model, sm, sa)
    smt.convert_linear_layer_to_matrix_sparsity(model, sm, sa)
    return model


def _step(model, ids):
    """Forward + backward through autograd (bf16 .grad); loss, tile grads, distinct saved bytes and
    the storages the q/k/v and gate/up members of layer 0 saved."""
    kept = {}

    def pack(t):
        st = t.untyped_storage()
        kept[st.data_ptr()] = st.nbytes()
        return t

    model.zero_grad(set_to_none=True)
    with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
        out = model(input_ids=ids, labels=ids, use_cache=False)
    held = sum(kept.values())
    layer = model.model.layers[0]
    saved = {n: getattr(getattr(layer, part), n) for part, names in (("self_attn", ("q_proj", "k_proj", "v_proj")),
                                                                    ("mlp", ("gate_proj", "up_proj")))
             for n in names}
    out.loss.backward()
    torch.cuda.synchronize()
    grads = {n: m.selected_weight.grad.clone() for n, m in model.named_modules()
             if isinstance(m, smt.LinearLayer_MatrixSparsity)}
    return out.loss.detach(), grads, held, saved


def test_shared_blocks_same_tile_grads_less_memory():
    model = _model()
    fl.patch_llama(model)
    try:
        ids = torch.randint(1, CFG["vocab_size"], (2, 1024), generator=torch.Generator().manual_seed(9)).to(DEV)
        loss_a, grads_a, held_a, _ = _step(model, ids)
        groups = eng.attach_column_block_groups(model)
        seen = {}
        orig = smt.ColumnBlockGroup.packed_input

        def spy(self, x, x2d, sink):
            p = orig(self, x, x2d, sink)
            seen.setdefault(id(self), set()).add(p.untyped_storage().data_ptr())
            return p
        smt.ColumnBlockGroup.packed_input = spy
        try:
            loss_b, grads_b, held_b, _ = _step(model, ids)
        finally:
            smt.ColumnBlockGroup.packed_input = orig
        eng.detach_transposed_weights(model)
        loss_c, grads_c, held_c, _ = _step(model, ids)
    finally:
        fl.unpatch_llama()
    print(f"\nsaved for backward: per-member copies {held_a / 1e6:.1f} MB, shared {held_b / 1e6:.1f} MB")
    assert groups == 3                                  # layer 0 q/k/v and gate/up, layer 1 gate/up
    assert all(len(v) == 1 for v in seen.values()) and len(seen) == 3   # one copy per group and forward
    assert torch.equal(loss_a, loss_b) and torch.equal(loss_a, loss_c)
    assert grads_a.keys() == grads_b.keys()
    for n in grads_a:
        assert torch.equal(grads_a[n], grads_b[n]), n
        assert torch.equal(grads_a[n], grads_c[n]), n
    # layer 0: q/k/v 7 blocks -> 4, gate/up 4 -> 3; layer 1 gate/up 2 -> 2 (x 2048 rows x 256 x 2 B)
    assert held_a - held_b == (3 + 1) * 2048 * 256 * 2, (held_a, held_b)


def test_shared_blocks_union_covering_the_input_keeps_it_whole():
    """A union of every column block: the members keep the input itself (one view), no copy."""
    att = {("q_proj", 0): [(c, c) for c in range(0, 16, 2)], ("k_proj", 0): [(c % 4, c) for c in range(1, 16, 2)]}
    model = _model(att, {("down_proj", 0): [(1, 2)]})
    fl.patch_llama(model)
    try:
        ids = torch.randint(1, CFG["vocab_size"], (1, 512), generator=torch.Generator().manual_seed(3)).to(DEV)
        loss_a, grads_a, held_a, _ = _step(model, ids)
        assert eng.attach_column_block_groups(model) == 1
        loss_b, grads_b, held_b, _ = _step(model, ids)
        eng.detach_transposed_weights(model)
    finally:
        fl.unpatch_llama()
    assert torch.equal(loss_a, loss_b)
    for n in grads_a:
        assert torch.equal(grads_a[n], grads_b[n]), n
    # q alone packed 8 of 16 blocks and k 8 (each <= half); together: the input itself (16 blocks, shared)
    assert held_b == held_a


def test_engine_step_bit_identical_with_shared_blocks():
    """The engine (batched wgrad launches keyed by the group's position map, reference rounding, packed
    fp32 gradient buffer, fused AdamW): tiles after two steps equal with and without the groups."""
    ids = torch.randint(1, CFG["vocab_size"], (2, 1024), generator=torch.Generator().manual_seed(4)).to(DEV)

    def run(shared):
        model = _model()
        fl.patch_llama(model)
        try:
            opt = eng.SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3,
                                   betas=(0.9, 0.95))
            engine, *_ = eng.initialize(model=model, optimizer=opt,
                                        config={"gradient_clipping": 1.0, "shared_input_blocks": shared})
            assert engine.column_block_groups == (3 if shared else 0)
            losses = []
            for _ in range(2):
                loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
                engine.backward(loss)
                engine.step()
                losses.append(loss.detach())
            torch.cuda.synchronize()
            tiles = {n: m.selected_weight.detach().clone() for n, m in model.named_modules()
                     if isinstance(m, smt.LinearLayer_MatrixSparsity)}
        finally:
            fl.unpatch_llama()
            eng.detach_transposed_weights(model)
        return losses, tiles

    la, ta = run(False)
    lb, tb = run(True)
    assert all(torch.equal(a, b) for a, b in zip(la, lb))
    for n in ta:
        assert torch.equal(ta[n], tb[n]), n
