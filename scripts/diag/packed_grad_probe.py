"""Diagnostic: what reaches gate_proj's linearZ.backward on the fp8 path when the gate output has a
second consumer (tests/test_gpu_fp8.py::test_fp8_packed_grad_summed_away_raises)."""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from sparse_matrix_tuning_amd import engine as eng  # noqa: E402
from sparse_matrix_tuning_amd import fp8 as f8  # noqa: E402
from sparse_matrix_tuning_amd import fused_llama  # noqa: E402
from sparse_matrix_tuning_amd.fused_llama import patch_llama  # noqa: E402
from sparse_matrix_tuning_amd.smt import smt  # noqa: E402

DEV = torch.device("cuda", 0)
cfg = dict(bench.MODELS["mini"], num_hidden_layers=1)
bench.MODELS["_p"] = cfg
model = bench.build_model("_p", DEV)
patch_llama(model)
sel_mlp = defaultdict(list, {("gate_proj", 0): [(3, 1), (0, 0)], ("up_proj", 0): [(1, 0)]})
sel_att = defaultdict(list, {("q_proj", 0): [(1, 1)]})
smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
opt = eng.SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3)
engine, *_ = eng.initialize(model=model, optimizer=opt, config={"fp8_linears": True})

orig_q = f8.swiglu_bwd_quant


def logged_q(g, u, dh, need_dg, need_du):
    print("swiglu_bwd_quant needs:", type(need_dg).__name__, type(need_du).__name__, flush=True)
    return orig_q(g, u, dh, need_dg, need_du)


f8.swiglu_bwd_quant = logged_q
orig_fn = fused_llama.FusedSwiGLUFn
orig_group = f8.swiglu_group


def logged_group(gate, up):
    r = orig_group(gate, up)
    print("swiglu_group:", None if r is None else (type(r[1]).__name__, type(r[2]).__name__),
          "gate tag:", None if "_smt_gout" not in gate.__dict__ else type(gate._smt_gout[2]).__name__, flush=True)
    return r


f8.swiglu_group = logged_group
orig_bwd = smt.linearZ.backward


def logged_bwd(ctx, grad_output):
    need = getattr(ctx, "mx_need", None)
    print("linearZ.backward: mx", ctx.mx is not None, "need", type(need).__name__,
          None if need is None else dict(need.__dict__), "stride", grad_output.stride(),
          "gpack", "_smt_gpack" in grad_output.__dict__, flush=True)
    return orig_bwd(ctx, grad_output)


smt.linearZ.backward = staticmethod(logged_bwd)


class TwoConsumers:
    @staticmethod
    def apply(g, u, *rest):
        print("TwoConsumers.apply rest", rest, flush=True)
        return orig_fn.apply(g, u, *rest) + 0 * g


for mode in ("plain", "two"):
    print("=== mode", mode, flush=True)
    fused_llama.FusedSwiGLUFn = TwoConsumers if mode == "two" else orig_fn
    ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(0)).to(DEV)
    loss = engine(input_ids=ids, labels=ids, use_cache=False).loss
    try:
        engine.backward(loss)
        print("backward returned", flush=True)
    except RuntimeError as e:
        print("raised:", str(e)[:120], flush=True)
    torch.cuda.synchronize()
fused_llama.FusedSwiGLUFn = orig_fn
print("probe done", flush=True)
