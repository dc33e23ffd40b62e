"""Selection dispatch end to end: warm-up steps through the
engine with the GPU harvest, then ``trainer.select_and_convert``, against the reference's sequence
restated on CPU copies of the same gradients:

* harvest: fine_tune.py:714-767 (``oracle.harvest``), bit for bit;
* selection: fine_tune.py:257-337 (``oracle.select_submatrix``): attention scored with the default
  ``mean_abs`` whatever ``calculate_strategy`` is, MLP with ``calculate_strategy``, ``no_limit_mixture``
  selecting from the MLP gradients only with the summed budget; identical dicts (keys, key order,
  tile order);
* freeze: smt.py:641-745 (``oracle.freeze_flags``): identical ``requires_grad`` for every parameter;
* convert: smt.py:83-179 (``oracle.convert_plan``): the same modules converted with the same tile
  lists, and each module's tiles equal to the gathered blocks of the post-warm-up W.
"""
import pytest
import torch

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import trainer
from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize, safe_get_full_grad
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _mini(layers=2):
    import bench
    cfg = dict(bench.MODELS["mini"])
    cfg["num_hidden_layers"] = layers
    bench.MODELS["_td"] = cfg
    try:
        return bench.build_model("_td", DEV)
    finally:
        del bench.MODELS["_td"]


def _warm_up(model, n_mlp, n_att, steps=3):
    import bench
    opt = SMTFusedAdam(model.parameters(), lr=1e-4, betas=(0.9, 0.95))
    engine, _, _, _ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0})
    harvester = trainer.GradHarvester(model, n_mlp, n_att)
    mlp_ref, att_ref = {}, {}
    for b in bench.batches(steps, 2, 128, bench.MODELS["mini"]["vocab_size"], 0, DEV):
        engine.backward(engine(**b, use_cache=False).loss)
        harvester.harvest()
        named = [(n, safe_get_full_grad(p)) for n, p in model.named_parameters()]
        ref.harvest([(n, g) for n, g in named if g is not None], mlp_ref, att_ref, n_mlp, n_att)
        engine.step()
    return engine, harvester, mlp_ref, att_ref


@pytest.mark.parametrize("no_limit_mixture,selection_strategy,calculate_strategy", [
    (False, "no_restriction", "abs_mean"),      # the README's flags: MLP abs_mean, attention forced mean_abs
    (False, "no_restriction", "L2"),
    (False, "norm_dist", "L1"),
    (True, "no_restriction", "abs_mean"),       # --no_limit_mixture: MLP pool only, summed budget
])
def test_dispatch_matches_reference_sequence(no_limit_mixture, selection_strategy, calculate_strategy):
    torch.manual_seed(21)
    model = _mini(2)
    dims = trainer.get_targeted_module_dims(model)
    total = trainer.count_total_blocks(model)
    ratio = 0.025 if selection_strategy == "norm_dist" else 0.1
    n_att, n_mlp = trainer.block_budgets(total, ratio, ratio)
    assert n_att > 0 and n_mlp > 0
    engine, harvester, mlp_ref, att_ref = _warm_up(model, n_mlp, n_att)
    assert set(harvester.warmup_grads) == set(mlp_ref) and set(harvester.attention_warmup_grads) == set(att_ref)
    for k in mlp_ref:
        assert torch.equal(harvester.warmup_grads[k].cpu(), mlp_ref[k])
    for k in att_ref:
        assert torch.equal(harvester.attention_warmup_grads[k].cpu(), att_ref[k])
    W_after = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}

    # the reference's dispatch (fine_tune.py:257-337) on the CPU copies
    if no_limit_mixture:
        want_mlp = ref.select_submatrix(mlp_ref, dims, n_mlp + n_att, selection_strategy=selection_strategy,
                                        calculate_strategy=calculate_strategy)
        want_att = {}
    else:
        want_att = ref.select_submatrix(att_ref, dims, n_att, selection_strategy=selection_strategy)
        want_mlp = ref.select_submatrix(mlp_ref, dims, n_mlp, selection_strategy=selection_strategy,
                                        calculate_strategy=calculate_strategy)
    names = [n for n, _ in model.named_parameters()]
    want_flags = ref.freeze_flags(names, want_mlp, {} if no_limit_mixture else want_att, mixture=no_limit_mixture)
    linears = [(n, want_flags[n + ".weight"]) for n, m in model.named_modules() if isinstance(m, torch.nn.Linear)]
    want_plan = ref.convert_plan(linears, want_mlp, want_att)

    engine, opt, sched, sel_mlp, sel_att = trainer.select_and_convert(
        engine, harvester, dims, n_att, n_mlp, selection_strategy=selection_strategy,
        calculate_strategy=calculate_strategy, no_limit_mixture=no_limit_mixture, smt_lr=1e-4, num_training_steps=10)
    assert list(sel_mlp.items()) == list(want_mlp.items())
    assert list(dict(sel_att).items()) == list(dict(want_att).items())
    got_flags = {n: p.requires_grad for n, p in model.named_parameters()}
    # converted linears hold `selected_weight` (trainable) and a frozen W: compare the weights' flags
    # before conversion through the plan, and everything that was not converted directly
    conv = {n: m for n, m in model.named_modules() if isinstance(m, smt.LinearLayer_MatrixSparsity)}
    assert {n: m.index_list for n, m in conv.items()} == want_plan
    for n, flag in want_flags.items():
        mod = n.rsplit(".", 1)[0]
        if mod in conv and n.endswith(".weight"):
            assert flag and conv[mod].selected_weight.requires_grad and not conv[mod].weight.requires_grad
        elif mod in conv:
            continue                                   # bias dropped on conversion (smt.py:113-115)
        else:
            assert got_flags[n] == flag, n
    for n, m in conv.items():
        assert torch.equal(m.selected_weight.detach().cpu(), ref.gather_tiles(W_after[n + ".weight"], m.index_list))
    # and the converted model trains
    import bench
    for b in bench.batches(2, 2, 128, bench.MODELS["mini"]["vocab_size"], 0, DEV, offset=7):
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        engine.step()
        assert torch.isfinite(loss).item()
