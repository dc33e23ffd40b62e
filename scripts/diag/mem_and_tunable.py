"""Diagnostics (GPU): (1) HBM retained per decoder-layer submodule in the SMT phase without
recompute, and the backward peak; (2) TunableOp on/off for the q/o GEMM in one process."""
import collections
import json
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sparse_matrix_tuning_amd import fused_llama, trainer  # noqa: E402
from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize  # noqa: E402
from sparse_matrix_tuning_amd.smt import smt  # noqa: E402

dev = torch.device("cuda", 0)
out = {}


def timed(fn, iters=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record(); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / iters, 4)


def tunable_check():
    import torch.cuda.tunable as tunable
    x = torch.randn(16, 2048, 4096, device=dev, dtype=torch.bfloat16)
    W = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16) * 0.02
    r = {"off_fwd": timed(lambda: torch.matmul(x, W.t())), "off_dgrad": timed(lambda: torch.matmul(x, W))}
    path = os.path.join(ROOT, "profiles", "tunableop_gfx950.csv")
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    tunable.set_filename("/tmp/tunable_diag.csv")
    r["read_ok"] = bool(tunable.read_file(path))
    r["on_fwd"] = timed(lambda: torch.matmul(x, W.t()))
    r["on_dgrad"] = timed(lambda: torch.matmul(x, W))
    r["results"] = [list(map(str, t)) for t in tunable.get_results()][:8]
    r["validators"] = [list(map(str, t)) for t in tunable.get_validators()]
    tunable.enable(False)
    r["off2_fwd"] = timed(lambda: torch.matmul(x, W.t()))
    return r


def mem_breakdown():
    model = bench.build_model("llama3-8b", dev)
    fused_llama.patch_llama(model)
    model.train()
    rnd = random.Random(0)
    dims = trainer.get_targeted_module_dims(model)
    cand_att, cand_mlp = [], []
    for layer in range(32):
        for m in ("q_proj", "k_proj", "v_proj"):
            r, c = dims[m]
            cand_att += [(m, layer, i, j) for i in range(r // 256) for j in range(c // 256)]
        for m in ("gate_proj", "up_proj", "down_proj"):
            r, c = dims[m]
            cand_mlp += [(m, layer, i, j) for i in range(r // 256) for j in range(c // 256)]
    sel_att, sel_mlp = collections.defaultdict(list), collections.defaultdict(list)
    for m, l, i, j in rnd.sample(cand_att, 436):
        sel_att[(m, l)].append((i, j))
    for m, l, i, j in rnd.sample(cand_mlp, 436):
        sel_mlp[(m, l)].append((i, j))
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    groups = smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-5)
    opt = SMTFusedAdam(groups, lr=1e-5, betas=(0.9, 0.95))
    engine, *_ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0})
    b = bench.batches(1, 16, 2048, 128256, 0, dev)[0]
    loss = engine(**b, use_cache=False).loss
    engine.backward(loss)
    engine.step()
    del loss
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    deltas = collections.defaultdict(float)
    handles = []
    layer0 = model.model.layers[5]
    for name, mod in [("input_layernorm", layer0.input_layernorm), ("self_attn", layer0.self_attn),
                      ("post_attention_layernorm", layer0.post_attention_layernorm), ("mlp", layer0.mlp),
                      ("layer", layer0)] + [(f"mlp.{n}", getattr(layer0.mlp, n)) for n in ("gate_proj", "up_proj", "down_proj")] \
            + [(f"attn.{n}", getattr(layer0.self_attn, n)) for n in ("q_proj", "k_proj", "v_proj", "o_proj")]:
        st = {}
        handles.append(mod.register_forward_pre_hook(lambda m, a, st=st: st.__setitem__("m", torch.cuda.memory_allocated())))
        handles.append(mod.register_forward_hook(lambda m, a, o, st=st, n=name: deltas.__setitem__(n, (torch.cuda.memory_allocated() - st["m"]) / 1e6)))
    torch.cuda.reset_peak_memory_stats()
    loss = engine(**b, use_cache=False).loss
    torch.cuda.synchronize()
    after_fwd = torch.cuda.memory_allocated()
    fwd_peak = torch.cuda.max_memory_allocated()
    engine.backward(loss)
    torch.cuda.synchronize()
    bwd_peak = torch.cuda.max_memory_allocated()
    for h in handles:
        h.remove()
    mods = {n: (type(m).__name__, len(getattr(m, "tiles", []))) for n, m in [(n, getattr(layer0.mlp, n)) for n in ("gate_proj", "up_proj", "down_proj")] + [(n, getattr(layer0.self_attn, n)) for n in ("q_proj", "k_proj", "v_proj", "o_proj")]}
    return {"base_gb": base / 1e9, "after_fwd_gb": after_fwd / 1e9, "retained_gb": (after_fwd - base) / 1e9,
            "fwd_peak_gb": fwd_peak / 1e9, "bwd_peak_gb": bwd_peak / 1e9, "layer5_deltas_mb": dict(deltas),
            "layer5_modules": mods}


out["tunable"] = tunable_check()
print(json.dumps(out), flush=True)
out["mem"] = mem_breakdown()
print(json.dumps(out), flush=True)
