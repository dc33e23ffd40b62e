"""The SMT step of LLaMA-3-8B in the reference's other --dtype (fine_tune.py:955-959): fp16 under
DeepSpeed's dynamic loss scale or fp32, through SMTEngine with DeepSpeed's config for the dtype
(deepspeed_helpers.py:53-61), every layer recomputed (fine_tune.py:192; ``--resident`` keeps them, the
headline's policy). bf16 and fp16 models run the
fused LLaMA kernels, smt_flash and the fused LM head + loss (ABI v13: one template body per 16-bit
format; ``--eager-ops`` keeps transformers' own ops), fp32 models transformers' ops; the SMT modules,
the tile weight gradients, the fused AdamW and the loss scale are this build's. 436 + 436 tiles drawn at random (seeded) over the
attention (q/k/v) and MLP candidate blocks of every layer, as SMT(0.71 %) selects them.

    python scripts/dtype_step_bench.py --dtype fp16 --steps 10

Prints one JSON line (tokens/s, median step, peak HBM, skipped steps, the loss scale, losses)."""
import argparse
import json
import os
import random
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from sparse_matrix_tuning_amd import trainer  # noqa: E402
from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize  # noqa: E402
from sparse_matrix_tuning_amd.smt import smt  # noqa: E402

DTYPES = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}


def random_selection(dims, n_layers, n, modules, seed):
    """n distinct (key, row_block, col_block) over the modules' blocks of every layer, grouped by key."""
    cands = [((m, l), r, c) for m in modules for l in range(n_layers)
             for r in range(dims[m][0] // 256) for c in range(dims[m][1] // 256)]
    pick = random.Random(seed).sample(cands, n)
    sel = defaultdict(list)
    for key, r, c in pick:
        sel[key].append((r, c))
    return sel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16", choices=sorted(DTYPES))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--tiles", type=int, default=436, help="per pool (attention, MLP)")
    ap.add_argument("--eager-ops", action="store_true", help="transformers' own ops even for bf16 / fp16")
    ap.add_argument("--resident", action="store_true",
                    help="keep every layer's activations (the headline's policy) instead of recomputing them")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    dtype = DTYPES[args.dtype]
    model = bench.build_model("llama3-8b", dev).to(dtype)
    fused = dtype != torch.float32 and not args.eager_ops
    if fused:
        from sparse_matrix_tuning_amd.fused_llama import patch_llama
        patch_llama(model)
    dims = trainer.get_targeted_module_dims(model)
    L = bench.MODELS["llama3-8b"]["num_hidden_layers"]
    sel_att = random_selection(dims, L, args.tiles, ("q_proj", "k_proj", "v_proj"), 1)
    sel_mlp = random_selection(dims, L, args.tiles, ("gate_proj", "up_proj", "down_proj"), 2)
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    if not args.resident:
        model.gradient_checkpointing_enable()
        trainer.make_gradient_checkpointing_compatible(model)
    model.train()
    ds = {"gradient_clipping": 1.0, "train_micro_batch_size_per_gpu": args.batch, "train_batch_size": args.batch}
    if args.dtype == "fp16":
        ds["fp16"] = {"enabled": True, "loss_scale_window": 100}       # deepspeed_helpers.py:53-55
    elif args.dtype == "fp32":
        ds["fp16"] = {"enabled": False}                                 # deepspeed_helpers.py:59-61
    else:
        ds["bfloat16"] = {"enabled": True}
    groups = smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 9.865e-6)
    opt = SMTFusedAdam(groups, lr=9.865e-6, betas=(0.9, 0.95))
    engine, _, _, _ = initialize(model=model, optimizer=opt, config=ds)
    n_tiles = sum(tg.n_tiles for tg in engine.tile_groups)
    vocab = bench.MODELS["llama3-8b"]["vocab_size"]
    data = bench.batches(args.warmup + args.steps, args.batch, args.seq, vocab, 0, dev)
    losses = []

    def step(b):
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        engine.step()
        losses.append(loss.detach())
        return loss

    t_w = time.time()
    for b in data[:args.warmup]:
        step(b)
    torch.cuda.synchronize()
    bench.log(f"{args.dtype}: {n_tiles} tiles, {args.warmup} untimed steps in {time.time() - t_w:.1f}s")
    torch.cuda.reset_peak_memory_stats(dev)
    elapsed, per_step, _ = bench.timed_steps(step, data[args.warmup:], 1, dev)
    med = bench._median(per_step)
    tok = args.batch * args.seq
    out = {"metric": f"LLaMA-3-8B SMT(0.71%) training step in the reference's --dtype {args.dtype}",
           "value": round(tok * args.steps / elapsed, 1), "unit": "tokens/s", "steps": args.steps,
           "median_ms_per_step": round(med * 1e3, 2), "median_tokens_per_s": round(tok / med, 1),
           "peak_hbm_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2), "dtype": args.dtype,
           "tiles": n_tiles, "tile_param_dtype": str(engine.tile_groups[0].param.dtype),
           "activations": "resident" if args.resident else "recomputed per layer (fine_tune.py:192)",
           "ops": "fused LLaMA kernels + smt_flash + fused LM head/loss" if fused else "transformers' own ops",
           "transposed_copies_gb": round(engine.transposed_bytes / 1e9, 2),
           "skipped_steps": engine.skipped_steps,
           "loss_scale": engine.loss_scaler.state_dict() if engine.loss_scaler is not None else None,
           "losses": [round(float(x), 4) for x in losses]}
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
