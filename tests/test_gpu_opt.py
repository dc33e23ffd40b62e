"""BASELINE config 1 on the HIP path: OPT-125m SMT(1%).

``OPTConfig(vocab 50272, hidden 768, ffn 3072, 12 layers, 12 heads)``, random init, bf16 on the GPU.
``num_total_blocks`` = 1909.15 (tied lm_head counted once), so ``--downsample_attention_blocks_ratio
0.01`` gives ``int(19.09)`` = 19 attention blocks and the MLP ratio stays negative (OPT has fc1/fc2,
no ``mlp`` names: an MLP budget > 0 would end in the reference's UnboundLocalError).

Reference quirks this configuration exercises (SURVEY §8(d) "Config 1 plumbing"):
* the layer regex ``model\\.layers\\.(\\d+)\\.`` (fine_tune.py:716-722, smt.py:90) does not match
  ``model.decoder.layers.N``: every layer's q/k/v gradient lands in ONE key ``(q_proj, None)`` etc.,
  summed over the 12 layers in named_parameters() order;
* the same 19 tiles are therefore applied to every layer's q/k/v (smt.py:83-134);
* q/k/v biases are dropped on conversion (smt.py:113-115).

Checked against the oracle: harvest bit for bit, selection identical, freeze flags and conversion plan
identical, loss of the converted model vs the CPU restatement, per-module tile gradients vs fp64 truth,
then fused AdamW steps.
"""
import pytest
import torch

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import trainer
from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize, safe_get_full_grad
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
OPT_125M = dict(vocab_size=50272, hidden_size=768, ffn_dim=3072, num_hidden_layers=12, num_attention_heads=12,
                word_embed_proj_dim=768, max_position_embeddings=2048)


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def build_opt(device):
    from transformers import OPTConfig, OPTForCausalLM
    cfg = OPTConfig(**OPT_125M)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(1234)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(device):
            return OPTForCausalLM(cfg), cfg
    finally:
        torch.set_default_dtype(prev)


def _batch(step, B=4, S=128):
    g = torch.Generator().manual_seed(4321 + step)
    ids = torch.randint(2, 50272, (B, S), generator=g)
    return {"input_ids": ids, "attention_mask": torch.ones_like(ids), "labels": ids}


def test_opt125m_smt_1pct_matches_reference():
    model, cfg = build_opt(DEV)
    dims = trainer.get_targeted_module_dims(model)
    assert dims == {'k_proj': [768, 768], 'v_proj': [768, 768], 'q_proj': [768, 768]}
    total = trainer.count_total_blocks(model)
    assert abs(total - 1909.1484375) < 1e-9
    n_att, n_mlp = trainer.block_budgets(total, 0.01, -1)
    assert (n_att, n_mlp) == (19, -1909)

    opt = SMTFusedAdam(model.parameters(), lr=1e-5, betas=(0.9, 0.95))
    engine, _, _, _ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0})
    harvester = trainer.GradHarvester(model, n_mlp, n_att)
    mlp_ref, att_ref = {}, {}
    for step in range(2):
        b = {k: v.to(DEV) for k, v in _batch(step).items()}
        engine.backward(engine(**b, use_cache=False).loss)
        harvester.harvest()
        named = [(n, safe_get_full_grad(p)) for n, p in model.named_parameters()]
        ref.harvest([(n, g) for n, g in named if g is not None], mlp_ref, att_ref, n_mlp, n_att)
        engine.step()
    # quirk 1: one key per projection, layer None, summed over the 12 layers in the reference's order
    assert set(att_ref) == {('q_proj', None), ('k_proj', None), ('v_proj', None)} and not mlp_ref
    assert set(harvester.attention_warmup_grads) == set(att_ref) and not harvester.warmup_grads
    for k in att_ref:
        assert torch.equal(harvester.attention_warmup_grads[k].cpu(), att_ref[k])

    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    want_att = ref.select_submatrix(att_ref, dims, n_att)              # attention: mean_abs (fine_tune.py:306-313)
    names = [n for n, _ in model.named_parameters()]
    want_flags = ref.freeze_flags(names, {}, want_att)
    linears = [(n, want_flags.get(n + ".weight", False)) for n, m in model.named_modules()
               if isinstance(m, torch.nn.Linear)]          # lm_head is tied to embed_tokens: not listed
    want_plan = ref.convert_plan(linears, {}, want_att)

    engine, opt, sched, sel_mlp, sel_att = trainer.select_and_convert(
        engine, harvester, dims, n_att, n_mlp, calculate_strategy="abs_mean", smt_lr=1e-4, num_training_steps=10)
    assert not sel_mlp and list(sel_att.items()) == list(want_att.items())
    assert sum(len(v) for v in sel_att.values()) == 19
    conv = {n: m for n, m in model.named_modules() if isinstance(m, smt.LinearLayer_MatrixSparsity)}
    assert {n: m.index_list for n, m in conv.items()} == want_plan
    # quirk 2: the same tiles in every layer; quirk 3: biases dropped
    for key, tiles in sel_att.items():
        mods = [m for n, m in conv.items() if n.endswith(f"self_attn.{key[0]}")]
        assert len(mods) == 12 and all(m.index_list == list(tiles) for m in mods)
    assert all(m.bias is None for m in conv.values())
    for n, flag in want_flags.items():
        mod = n.rsplit(".", 1)[0]
        if mod not in conv:
            assert dict(model.named_parameters())[n].requires_grad == flag, n
    for n, m in conv.items():
        assert torch.equal(m.selected_weight.detach().cpu(), ref.gather_tiles(sd[n + ".weight"], m.index_list))

    # the converted model vs the CPU restatement on the same weights and batch
    seen_x, seen_g = {}, {}

    def capture(name):
        def hook(_m, inp, out):
            seen_x[name] = inp[0].detach().clone()
            out.register_hook(lambda g: seen_g.__setitem__(name, g.detach().clone()))
        return hook
    handles = [m.register_forward_hook(capture(n)) for n, m in conv.items()]
    b = _batch(10)
    out = engine(**{k: v.to(DEV) for k, v in b.items()}, use_cache=False)
    engine.backward(out.loss)
    for h in handles:
        h.remove()
    from transformers import OPTForCausalLM
    cpu = OPTForCausalLM(cfg).to(torch.bfloat16)
    cpu.load_state_dict(sd)
    for n, p in cpu.named_parameters():
        p.requires_grad = want_flags[n]
    ref.ref_convert(cpu, {}, want_att)
    out_ref = cpu(**b, use_cache=False)
    rel = abs(out.loss.item() - out_ref.loss.item()) / abs(out_ref.loss.item())
    assert rel <= 1e-3, (out.loss.item(), out_ref.loss.item())
    for n, m in conv.items():
        x, g = seen_x[n].cpu(), seen_g[n].cpu()
        truth = ref.tile_grads_fp64(g, x, m.index_list)
        _gi, ref_gw = ref.linearz_backward(g, x, m.weight.detach().cpu(), m.index_list)
        err = _rel(engine.tile_grad(m.selected_weight), truth)
        # the engine keeps fp32 tile gradients: compare against the reference's bf16 error bar
        assert err <= max(1e-3, 1.1 * _rel(ref_gw, truth)), (n, err)
    before = {n: m.selected_weight.detach().clone() for n, m in conv.items()}
    engine.step()
    for n, m in conv.items():
        assert not torch.equal(before[n], m.selected_weight.detach())
        assert torch.equal(ref.gather_tiles(m.weight.detach().cpu(), m.index_list), m.selected_weight.detach().cpu())
    for step in range(2):
        b = {k: v.to(DEV) for k, v in _batch(20 + step).items()}
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        engine.step()
        assert torch.isfinite(loss).item()


def test_opt_mlp_budget_crashes_like_the_reference():
    """An MLP budget > 0 on OPT: no parameter name contains 'mlp', the MLP dict stays empty and the
    reference's selection ends in UnboundLocalError (smt_helper.py:141-145)."""
    from sparse_matrix_tuning_amd.smt import smt_helper
    with pytest.raises(UnboundLocalError):
        smt_helper.select_submatrix_based_on_grads({}, {'q_proj': [768, 768]}, 5, calculate_strategy="abs_mean")
