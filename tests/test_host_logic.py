"""Host-side logic of the product on CPU: ranking, model surgery, budgets, param groups, harvest order,
error behaviour. No GPU compute here (SMT modules are built on the ``meta`` device)."""
import json
import os
from collections import defaultdict

import numpy as np
import pytest
import torch
from torch import nn

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd.smt import smt, smt_helper
from sparse_matrix_tuning_amd import trainer

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# ------------------------------------------------------------------ ranking (smt_helper.py:81-146)
def _golden_pools():
    from tests.golden.make_golden import selection_inputs
    grads = selection_inputs()
    att = {k: v for k, v in grads.items() if k[0] in ("q_proj", "k_proj", "v_proj")}
    mlp = {k: v for k, v in grads.items() if k[0] in ("gate_proj", "up_proj", "down_proj")}
    return att, mlp


def test_rank_blocks_matches_reference_heap_on_golden_cases():
    spec = json.load(open(os.path.join(GOLDEN, "selection_expected.json")))
    att, mlp = _golden_pools()
    dims = spec["dims"]
    for case in spec["cases"]:
        pool = att if case["pool"] == "attention" else mlp
        scores = {}
        for key, g in pool.items():
            d1, d2 = dims[key[0]][0] // 256, dims[key[0]][1] // 256
            scores[key] = ref.block_stat(g, d1, d2, case["strategy"]).numpy()
        out = smt_helper.rank_blocks(scores, case["n"], case["selection_strategy"])
        got = [[k[0], k[1], [list(t) for t in v]] for k, v in out.items()]
        assert got == case["expected"]


def test_rank_blocks_tie_order_is_tuple_order():
    # all-equal scores: order is by (module name, layer, i, j) descending
    scores = {('q_proj', 0): np.ones((2, 2), np.float32), ('v_proj', 0): np.ones((1, 2), np.float32),
              ('k_proj', 1): np.ones((1, 2), np.float32)}
    out = smt_helper.rank_blocks(scores, 5)
    assert list(out.items()) == [(('v_proj', 0), [(0, 1), (0, 0)]), (('q_proj', 0), [(1, 1), (1, 0), (0, 1)])]
    # -0.0 and 0.0 tie exactly (python float comparison), then the key decides
    z = {('a', 0): np.array([[-0.0]], np.float32), ('b', 0): np.array([[0.0]], np.float32)}
    assert list(smt_helper.rank_blocks(z, 1).keys()) == [('b', 0)]


def test_rank_blocks_n_larger_than_candidates_and_errors():
    s = {('q_proj', 0): np.array([[1.0, 3.0]], np.float32)}
    assert dict(smt_helper.rank_blocks(s, 10)) == {('q_proj', 0): [(0, 1), (0, 0)]}
    with pytest.raises(UnboundLocalError):
        smt_helper.rank_blocks({}, 3)
    with pytest.raises(UnboundLocalError):
        smt_helper.rank_blocks(s, 0)
    assert dict(smt_helper.rank_blocks(s, 0, "norm_dist")) == {}


def test_score_blocks_unknown_strategy_and_bad_dims():
    g = {('q_proj', 0): torch.zeros(256, 512)}
    assert smt_helper.score_blocks(g, {'q_proj': [256, 512]}, "bogus") == {}
    with pytest.raises(RuntimeError):
        smt_helper.score_blocks(g, {'q_proj': [512, 512]}, "mean_abs")
    with pytest.raises(UnboundLocalError):
        smt_helper.select_submatrix_based_on_grads(g, {'q_proj': [256, 512]}, n=1, calculate_strategy="bogus")


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_product_scoring_fails_loudly_without_gpu():
    g = {('q_proj', 0): torch.zeros(256, 512)}
    with pytest.raises(RuntimeError, match="ROCm"):
        smt_helper.select_submatrix_based_on_grads(g, {'q_proj': [256, 512]}, n=1)


def test_finalize_scores_rounding():
    raw = np.array([65536.0 * 3.0, -65536.0 * 0.5, 2.0 ** -30], np.float64)
    assert smt_helper.finalize_scores(raw, "mean_abs").tolist() == [3.0, 0.5, np.float32(2.0 ** -46)]
    assert smt_helper.finalize_scores(np.array([4.0]), "L2").tolist() == [2.0]


# ------------------------------------------------------------------ model surgery on meta tensors
class _Attn(nn.Module):
    def __init__(self, h, kv):
        super().__init__()
        self.q_proj = nn.Linear(h, h, bias=False)
        self.k_proj = nn.Linear(h, kv, bias=False)
        self.v_proj = nn.Linear(h, kv, bias=False)
        self.o_proj = nn.Linear(h, h, bias=False)


class _MLP(nn.Module):
    def __init__(self, h, i):
        super().__init__()
        self.gate_proj = nn.Linear(h, i, bias=False)
        self.up_proj = nn.Linear(h, i, bias=False)
        self.down_proj = nn.Linear(i, h, bias=False)


class _Layer(nn.Module):
    def __init__(self, h, kv, i):
        super().__init__()
        self.self_attn = _Attn(h, kv)
        self.mlp = _MLP(h, i)
        self.input_layernorm = nn.LayerNorm(h)
        self.post_attention_layernorm = nn.LayerNorm(h)


class _Body(nn.Module):
    def __init__(self, n, h, kv, i, vocab):
        super().__init__()
        self.embed_tokens = nn.Embedding(vocab, h)
        self.layers = nn.ModuleList([_Layer(h, kv, i) for _ in range(n)])
        self.norm = nn.LayerNorm(h)


class TinyLlama(nn.Module):
    def __init__(self, n=2, h=512, kv=256, i=768, vocab=1024, device="meta"):
        super().__init__()
        with torch.device(device):
            self.model = _Body(n, h, kv, i, vocab)
            self.lm_head = nn.Linear(h, vocab, bias=False)


def test_targeted_dims_total_blocks_and_budget_llama3_8b_meta():
    from transformers import LlamaConfig, LlamaForCausalLM
    import bench
    cfg = LlamaConfig(**bench.MODELS["llama3-8b"])
    with torch.device("meta"):
        m = LlamaForCausalLM(cfg)
    dims = trainer.get_targeted_module_dims(m)
    assert dims == {'q_proj': [4096, 4096], 'k_proj': [1024, 4096], 'v_proj': [1024, 4096],
                    'gate_proj': [14336, 4096], 'up_proj': [14336, 4096], 'down_proj': [4096, 14336]}
    total = trainer.count_total_blocks(m)
    assert total == 122528.0                        # SURVEY §8 sizing constants
    assert trainer.block_budgets(total, 0.00356, 0.00356) == (436, 436)
    assert 872 * 65536 == 57147392


def test_freeze_and_convert_on_meta():
    m = TinyLlama()
    sel_mlp = defaultdict(list, {('up_proj', 1): [(2, 1), (0, 0)], ('down_proj', 0): [(1, 2)]})
    sel_att = defaultdict(list, {('v_proj', 1): [(0, 1)], ('q_proj', 0): [(1, 1), (0, 0)]})
    smt.freeze_unselected_matrix_layer(m, sel_mlp, sel_att)
    trainable = sorted(n for n, p in m.named_parameters() if p.requires_grad)
    assert trainable == ['model.layers.0.mlp.down_proj.weight', 'model.layers.0.self_attn.q_proj.weight',
                         'model.layers.1.mlp.up_proj.weight', 'model.layers.1.self_attn.v_proj.weight']
    smt.convert_linear_layer_to_matrix_sparsity(m, sel_mlp, sel_att)
    conv = {n: mod for n, mod in m.named_modules() if isinstance(mod, smt.LinearLayer_MatrixSparsity)}
    assert sorted(conv) == ['model.layers.0.mlp.down_proj', 'model.layers.0.self_attn.q_proj',
                            'model.layers.1.mlp.up_proj', 'model.layers.1.self_attn.v_proj']
    up = conv['model.layers.1.mlp.up_proj']
    assert up.index_list == [(2, 1), (0, 0)] and tuple(up.selected_weight.shape) == (512, 256)
    assert up.weight.requires_grad is False and up.selected_weight.requires_grad is True
    assert up.bias is None
    groups = smt.get_optimizer_sparse_grouped_parameters(m, 0.0, 9.865e-6)
    assert len(groups) == 1 and groups[0]["lr"] == 9.865e-6
    assert sum(p.numel() for p in groups[0]["params"]) == (2 + 1 + 1 + 2) * 65536
    # merge back: an nn.Linear sharing W (smt.py:416-457)
    W = up.weight
    smt.convert_matrix_sparsity_to_linear_layer(m)
    assert isinstance(m.model.layers[1].mlp.up_proj, nn.Linear)
    assert m.model.layers[1].mlp.up_proj.weight is W


def test_mixture_freeze_and_qk_groups():
    m = TinyLlama()
    sel = {('gate_proj', 0): [(0, 0)], ('k_proj', 1): [(0, 0)], ('embed_tokens', None): []}
    smt.freeze_unselected_matrix_layer(m, sel, {}, mixture=True, layernorm=True)
    tr = {n for n, p in m.named_parameters() if p.requires_grad}
    assert 'model.embed_tokens.weight' in tr and 'model.layers.0.mlp.gate_proj.weight' in tr
    assert 'model.layers.1.self_attn.k_proj.weight' in tr
    assert 'model.layers.0.input_layernorm.weight' in tr and 'model.norm.weight' not in tr
    for p in m.parameters():
        p.requires_grad = True
    g = smt.get_optimizer_qk_augment_grouped_parameters(m, 0.1, 1e-5, 5e-4)
    assert [grp.get("lr") for grp in g] == [1e-5, 5e-4, None]
    names_qk = sum(p.numel() for p in g[1]["params"])
    assert names_qk == 2 * (512 * 512 + 256 * 512)


def test_smt_module_rejects_cpu_and_bad_tiles():
    with pytest.raises(RuntimeError, match="ROCm"):
        smt.LinearLayer_MatrixSparsity(nn.Parameter(torch.zeros(512, 512)), index_list=[(0, 0)])
    with pytest.raises(RuntimeError):
        smt.LinearLayer_MatrixSparsity(nn.Parameter(torch.zeros(512, 512, device="meta")), index_list=[(2, 0)])
    m = smt.LinearLayer_MatrixSparsity(nn.Parameter(torch.zeros(512, 512, device="meta")), index_list=[])
    assert tuple(m.selected_weight.shape) == (0, 256)


def test_linearz_rejects_non_3d_input():
    w = torch.zeros(512, 512, device="meta")
    with pytest.raises(IndexError):
        smt.linearZ.apply(torch.zeros(4, 512, device="meta"), torch.zeros(256, 256, device="meta"), [(0, 0)], w)


# ------------------------------------------------------------------ warm-up harvest launch order
def test_harvest_rounds_preserve_reference_add_order(monkeypatch):
    """Keys shared by several params in one step (OPT naming) must add in named_parameters() order:
    the harvester splits them over successive launches. The launches are replaced by a CPU stand-in
    here (test-only) to check the schedule against the oracle bit-for-bit."""
    from sparse_matrix_tuning_amd import _hip

    def fake_accumulate(pairs, assign=False):
        for dst, src in pairs:
            if assign:
                dst.copy_(src.float())
            else:
                dst += src.float()
    monkeypatch.setattr(_hip, "grad_accumulate", fake_accumulate)

    class OPTish(nn.Module):
        def __init__(self):
            super().__init__()
            self.model = nn.Module()
            self.model.decoder = nn.Module()
            self.model.decoder.layers = nn.ModuleList()
            for _ in range(3):
                layer = nn.Module()
                layer.self_attn = _Attn(256, 256)
                self.model.decoder.layers.append(layer)
    m = OPTish().to(torch.bfloat16)       # bf16 grads, as the reference's (so .to(float32) copies)
    torch.manual_seed(0)
    for i, p in enumerate(m.parameters()):
        p.grad = (torch.randn(p.shape) * 10.0 ** (i % 4)).bfloat16()   # magnitudes where fp32 add order matters
    h = trainer.GradHarvester(m, num_mlp_blocks=0, num_attention_blocks=1)
    for _ in range(2):
        h.harvest()
    mlp_ref, att_ref = {}, {}
    named = [(n, p.grad) for n, p in m.named_parameters()]
    for _ in range(2):
        ref.harvest(named, mlp_ref, att_ref, 0, 1)
    assert set(h.attention_warmup_grads) == set(att_ref) == {('q_proj', None), ('k_proj', None), ('v_proj', None)}
    for k in att_ref:
        assert torch.equal(h.attention_warmup_grads[k], att_ref[k])


# ------------------------------------------------------------------ channel path host logic
def test_rank_channels_matches_reference_heap_on_golden_cases():
    from tests.golden.make_golden import channel_inputs
    spec = json.load(open(os.path.join(GOLDEN, "channel_selection_expected.json")))
    act = channel_inputs()
    for case in spec["cases"]:
        pool = {k: a for k, a in act.items()
                if (k[0] in ("q_proj", "k_proj", "v_proj")) == (case["pool"] == "attention")}
        stats = {k: ref.channel_stat_fp64(a, case["strategy"]).numpy() for k, a in pool.items()}
        out = smt_helper.rank_channels(stats, case["n"], case["selection_strategy"])
        assert [[k[0], k[1], list(v)] for k, v in out.items()] == case["expected"], case["n"]


def test_rank_channels_ties_and_errors():
    s = {('q_proj', 0): np.array([1.0, 1.0, 2.0], np.float32), ('v_proj', 0): np.array([1.0], np.float32)}
    out = smt_helper.rank_channels(s, 3)
    # (2.0, q/2) first; the 1.0 ties go to the larger key ('v_proj' > 'q_proj'), then the larger index
    assert list(out.items()) == [(('q_proj', 0), [2, 1]), (('v_proj', 0), [0])]
    ref_out = ref.rank_channels({k: torch.from_numpy(v) for k, v in s.items()}, 3)
    assert list(out.items()) == list(ref_out.items())
    with pytest.raises(UnboundLocalError):
        smt_helper.rank_channels({}, 3)
    with pytest.raises(UnboundLocalError):
        smt_helper.rank_channels(s, 0)
    assert dict(smt_helper.rank_channels(s, 2, "norm_dist")) == {('q_proj', 0): [2, 0], ('v_proj', 0): [0]}
    assert smt_helper.score_channels({('q_proj', 0): torch.zeros(1, 2, 8)}, "bogus") == {}


def test_finalize_channel_scores():
    raw = np.array([6.0, 0.0, 2.0 ** -40], np.float64)
    assert smt_helper.finalize_channel_scores(raw, 3, "mean_abs").tolist() == [2.0, 0.0, np.float32(2.0 ** -40 / 3)]
    assert smt_helper.finalize_channel_scores(raw, 3, "abs_mean").tolist() == [2.0, 0.0, np.float32(2.0 ** -40 / 3)]
    assert smt_helper.finalize_channel_scores(raw, 3, "L1").tolist() == [6.0, 0.0, np.float32(2.0 ** -40)]
    assert smt_helper.finalize_channel_scores(np.array([9.0]), 3, "L2").tolist() == [3.0]


def test_channel_freeze_and_convert_on_meta():
    m = TinyLlama(kv=512)                   # square q/k/v/o: the only shapes the reference path trains
    sel_mlp = defaultdict(list)
    sel_att = defaultdict(list, {('q_proj', 0): [5, 300, 1], ('v_proj', 1): [511], ('o_proj', 0): [3]})
    smt.freeze_unselected_channel_layer(m, sel_mlp, sel_att)
    trainable = sorted(n for n, p in m.named_parameters() if p.requires_grad)
    # o_proj has no name on this path (smt.py:796-797): never trainable
    assert trainable == ['model.layers.0.self_attn.q_proj.weight', 'model.layers.1.self_attn.v_proj.weight']
    smt.convert_linear_layer_to_channel_sparsity(m, sel_mlp, sel_att)
    conv = {n: mod for n, mod in m.named_modules() if isinstance(mod, smt.LinearLayer_ChannelSparsity)}
    assert sorted(conv) == ['model.layers.0.self_attn.q_proj', 'model.layers.1.self_attn.v_proj']
    q = conv['model.layers.0.self_attn.q_proj']
    assert q.index_list == [5, 300, 1] and tuple(q.selected_weight.shape) == (3, 512)
    assert q.channels.padded == 256 and q.bias is None and q.weight.requires_grad is False
    groups = smt.get_optimizer_sparse_grouped_parameters(m, 0.0, 1e-5)
    assert sum(p.numel() for p in groups[0]["params"]) == 4 * 512
    # mixture: attention keys are looked up in the MLP selection
    m2 = TinyLlama(kv=512)
    smt.freeze_unselected_channel_layer(m2, {('k_proj', 1): [0], ('gate_proj', 0): [1]}, {}, mixture=True)
    assert sorted(n for n, p in m2.named_parameters() if p.requires_grad) == [
        'model.layers.0.mlp.gate_proj.weight', 'model.layers.1.self_attn.k_proj.weight']


def test_channel_module_errors():
    with pytest.raises(RuntimeError, match="ROCm"):
        smt.LinearLayer_ChannelSparsity(nn.Parameter(torch.zeros(512, 512)), index_list=[0])
    meta = lambda: nn.Parameter(torch.zeros(512, 512, device="meta"))
    with pytest.raises(IndexError):
        smt.LinearLayer_ChannelSparsity(meta(), index_list=[512])
    with pytest.raises(ValueError):
        smt.LinearLayer_ChannelSparsity(meta(), index_list=[3, 3])
    assert smt.LinearLayer_ChannelSparsity(meta(), index_list=[-1]).index_list == [511]
    with pytest.raises(IndexError):
        smt.linearChannel.apply(torch.zeros(4, 512, device="meta"), torch.zeros(1, 512, device="meta"), [0],
                                torch.zeros(512, 512, device="meta"))


def test_activation_harvester_hook_keys_on_meta():
    m = TinyLlama(kv=512)
    h = trainer.ActivationHarvester(m, num_mlp_channel=1, num_attention_channel=1)
    assert len(h._handles) == 2 * 6            # q, k, v, gate, up, down per layer; o_proj skipped
    h.remove()
    h2 = trainer.ActivationHarvester(m, num_mlp_channel=0, num_attention_channel=4)
    assert len(h2._handles) == 2 * 3
    h2.release()
    assert not h2._handles and h2.attention_activation == {}


def test_tile_index_column_blocks_first_use_order():
    from sparse_matrix_tuning_amd.smt.smt import TileIndex
    t = TileIndex([(1, 6), (0, 2), (1, 2), (3, 6), (2, 0)])
    assert t.column_blocks() == [6, 2, 0]


def test_top_level_smt_package_serves_fine_tune_imports():
    """fine_tune.py:39-40 imports, unchanged, resolve to the MI355X implementation."""
    from smt.smt import (convert_linear_layer_to_matrix_sparsity, get_optimizer_sparse_grouped_parameters,  # noqa: F401
                         get_optimizer_qk_augment_grouped_parameters, freeze_unselected_matrix_layer,
                         freeze_unselected_channel_layer, convert_linear_layer_to_channel_sparsity)
    from smt.smt_helper import (select_submatrix_based_on_grads, get_blocks, get_named_linears,  # noqa: F401
                                select_channel_based_on_activation)
    import smt.smt as top
    assert top.LinearLayer_MatrixSparsity is smt.LinearLayer_MatrixSparsity
    assert select_submatrix_based_on_grads is smt_helper.select_submatrix_based_on_grads
    import torch.distributed as dist
    assert not dist.is_initialized()                 # no process group at import (smt.py:20 does one)


def test_resident_layers_policy_host_logic():
    """trainer.checkpointed_layers / set_resident_layers on a meta-device LLaMA with transformers'
    gradient checkpointing: the LAST n decoder layers stop recomputing, n is clamped, 0 restores the
    reference's recompute-everything policy."""
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=5,
                      num_attention_heads=4, num_key_value_heads=2)
    with torch.device("meta"):
        model = LlamaForCausalLM(cfg)
    assert trainer.checkpointed_layers(model) == []          # not checkpointing: nothing to switch
    model.gradient_checkpointing_enable()
    layers = trainer.checkpointed_layers(model)
    assert len(layers) == 5 and all(m.gradient_checkpointing for m in layers)
    assert trainer.set_resident_layers(model, 2) == 2
    assert [m.gradient_checkpointing for m in layers] == [True, True, True, False, False]
    assert trainer.set_resident_layers(model, 99) == 5
    assert not any(m.gradient_checkpointing for m in layers)
    assert trainer.set_resident_layers(model, 0) == 0
    assert all(m.gradient_checkpointing for m in layers)
