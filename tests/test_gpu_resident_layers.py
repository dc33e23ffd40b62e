"""The warm-up's memory policy (trainer.set_resident_layers / resident_layers_for): decoder layers
whose activations stay resident skip the per-layer recompute of fine_tune.py:192. Recompute replays
the same kernels on the same inputs, so gradients must be bit-identical to full recompute."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _grads(n_resident):
    import bench
    from sparse_matrix_tuning_amd import trainer
    from sparse_matrix_tuning_amd.fused_llama import patch_llama
    model = bench.build_model("mini", DEV)
    patch_llama(model)
    model.gradient_checkpointing_enable()
    model.train()
    assert trainer.set_resident_layers(model, n_resident) == n_resident
    flags = [m.gradient_checkpointing for m in trainer.checkpointed_layers(model)]
    assert flags == [i < len(flags) - n_resident for i in range(len(flags))]
    b = bench.batches(1, 2, 256, bench.MODELS["mini"]["vocab_size"], 0, DEV)[0]
    model(**b, use_cache=False).loss.backward()
    torch.cuda.synchronize()
    return {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}


def test_resident_layers_bit_identical_to_full_recompute():
    full = _grads(0)
    for n in (1, 4):
        part = _grads(n)
        assert part.keys() == full.keys()
        for k in full:
            assert torch.equal(part[k], full[k]), (n, k)


def test_resident_layers_for_budget():
    import bench
    from sparse_matrix_tuning_amd import trainer
    model = bench.build_model("mini", DEV)
    model.gradient_checkpointing_enable()
    model.train()
    per = trainer.layer_activation_bytes(model, 2, 256)
    hidden = bench.MODELS["mini"]["hidden_size"]
    assert per > 4 * 2 * 256 * hidden * 2                   # more than a few [T, H] bf16 tensors
    total = torch.cuda.get_device_properties(DEV).total_memory
    assert trainer.resident_layers_for(model, 2, 256, peak_bytes=total) == 0      # no room
    n = trainer.resident_layers_for(model, 2, 256, peak_bytes=0)
    assert n == len(trainer.checkpointed_layers(model))                           # room for all
    assert all(m.gradient_checkpointing for m in trainer.checkpointed_layers(model))   # probe restored


def _smt_tile_grads(mode):
    """One SMT-phase backward of the mini LLaMA through the engine, with activations resident
    ("none"), every layer recomputed ("all", fine_tune.py:192) or the last half of the layers
    resident under recompute ("half"): the packed fp32 tile gradients."""
    import bench
    from sparse_matrix_tuning_amd import trainer
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.fused_llama import patch_llama
    from sparse_matrix_tuning_amd.smt import smt
    model = bench.build_model("mini", DEV)
    patch_llama(model)
    sel_mlp = {("gate_proj", 1): [(0, 0), (2, 1)], ("down_proj", 2): [(1, 0)]}
    sel_att = {("q_proj", 0): [(0, 1)], ("v_proj", 3): [(0, 0)]}
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3, betas=(0.9, 0.95))
    eng, _, _, _ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0})
    model.train()
    if mode != "none":
        model.gradient_checkpointing_enable()
        n = len(trainer.checkpointed_layers(model))
        trainer.set_resident_layers(model, n // 2 if mode == "half" else 0)
    b = bench.batches(1, 2, 256, bench.MODELS["mini"]["vocab_size"], 0, DEV)[0]
    eng.backward(eng(**b, use_cache=False).loss)
    torch.cuda.synchronize()
    return [tg.grad.clone() for tg in eng.tile_groups]


def test_smt_phase_tile_grads_identical_across_memory_policies():
    """The bench's memory points (resident, per-layer recompute, half the layers resident under
    recompute) give the same tile gradients bit for bit."""
    ref_grads = _smt_tile_grads("none")
    assert ref_grads and all(g.abs().sum() > 0 for g in ref_grads)
    for mode in ("all", "half"):
        got = _smt_tile_grads(mode)
        assert len(got) == len(ref_grads)
        for a, b in zip(got, ref_grads):
            assert torch.equal(a, b), mode
