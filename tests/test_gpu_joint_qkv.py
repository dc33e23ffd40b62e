"""q/k/v_proj's data gradient as ONE GEMM in the engine's step (engine "joint_qkv_dgrad", default on):
smt_flash hands back [dq | dk | dv] as slices of one buffer, the fused RoPE backward rotates the
q / k slices in place, and dgrad.py sums the three products through the joint transposed copy.
A mini-LLaMA through the product path (fused ops, smt_flash, smt_ce, the engine) with and without
it: the joint GEMM runs once per layer (past the first) per backward, and losses and tile weights agree within bf16
rounding (the joint sum is rounded once instead of once per consumer). Weights after AdamW steps are
not compared: Adam's early updates are ~lr * sign(g), so a gradient element near zero may flip."""
from collections import defaultdict

import pytest
import torch

from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _run(joint, steps=2):
    import bench
    from sparse_matrix_tuning_amd import dgrad
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.fused_llama import patch_llama, unpatch_llama
    model = bench.build_model("mini", DEV)
    sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)], ("k_proj", 1): [(0, 0)], ("v_proj", 2): [(0, 1)]})
    sel_mlp = defaultdict(list, {("up_proj", 1): [(2, 1)], ("down_proj", 3): [(1, 0)]})
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    patch_llama(model)
    try:
        opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3, betas=(0.9, 0.95))
        engine, *_ = initialize(model=model, optimizer=opt,
                                config={"gradient_clipping": 1.0, "joint_qkv_dgrad": joint})
        marked = sum(1 for m in model.modules() if getattr(m, "_smt_joint_qkv_grad", False))
        ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
        n0, losses, grads = dgrad.JOINT_PRODUCTS, [], []
        for _ in range(steps):
            loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
            engine.backward(loss)
            torch.cuda.synchronize()
            grads.append(torch.cat([g.grad.detach().clone() for g in engine.tile_groups]))
            engine.step()
            losses.append(loss.item())
        return losses, dgrad.JOINT_PRODUCTS - n0, marked, grads
    finally:
        unpatch_llama()


def test_engine_joint_qkv_data_gradient():
    l_sep, n_sep, m_sep, t_sep = _run(False)
    l_j, n_j, m_j, t_j = _run(True)
    assert (m_sep, n_sep) == (0, 0)
    # every backward, every layer whose q/k/v input needs a gradient: layer 0 reads the frozen
    # embedding through a frozen norm, so its data gradient is never formed
    assert m_j == 4 and n_j == 2 * 3
    for a, b in zip(l_j, l_sep):
        assert abs(a - b) <= 1e-3 * abs(b), (l_j, l_sep)
    # tile gradients of the first backward (the same weights): the layers below a joint product see
    # an input gradient rounded once instead of three times, ~2^-9 relative per element
    d = ((t_j[0] - t_sep[0]).norm() / t_sep[0].norm()).item()
    assert d <= 1e-2, d
