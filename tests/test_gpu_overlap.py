"""The engine's wgrad stream (overlap_wgrad, default on): the tile weight gradients run on a stream of
their own beside the data-gradient GEMMs. Same kernels, same inputs, same order per buffer, so the
trained state must be bit-identical to the run with everything on one stream."""
from collections import defaultdict

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _run(overlap: bool, max_lag: int = 2):
    import bench
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.smt import smt
    cfg = dict(bench.MODELS["mini"], num_hidden_layers=2)
    bench.MODELS["_ov"] = cfg
    try:
        torch.manual_seed(0)
        model = bench.build_model("_ov", DEV)
    finally:
        del bench.MODELS["_ov"]
    sel_mlp = defaultdict(list, {("up_proj", 1): [(2, 1), (0, 0)], ("down_proj", 0): [(1, 0), (0, 1)],
                                 ("gate_proj", 1): [(1, 1)]})
    sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)], ("k_proj", 1): [(0, 0)], ("v_proj", 1): [(0, 1)]})
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3, betas=(0.9, 0.95))
    engine, *_ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0, "overlap_wgrad": overlap,
                                                                  "wgrad_max_lag": max_lag})
    assert (engine.wgrad_stream is not None) == overlap
    gen = torch.Generator().manual_seed(1)
    losses = []
    for _ in range(3):
        ids = torch.randint(0, 4096, (2, 256), generator=gen).to(DEV)
        loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
        engine.backward(loss)
        engine.step()
        losses.append(loss.item())
    torch.cuda.synchronize()
    return losses, [(tg.master.clone(), tg.grad.clone()) for tg in engine.tile_groups]


@pytest.mark.parametrize("max_lag", [0, 1, 2])
def test_overlapped_wgrad_bit_identical(max_lag):
    """0: the wgrad stream may run arbitrarily far behind; 1, 2: the current stream waits for all
    but the last 1 (2) wgrad launches (the bound on the operands held for the wgrad stream)."""
    l0, s0 = _run(False)
    l1, s1 = _run(True, max_lag)
    assert l0 == l1
    for (m0, g0), (m1, g1) in zip(s0, s1):
        assert torch.equal(m0, m1) and torch.equal(g0, g1)
