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
