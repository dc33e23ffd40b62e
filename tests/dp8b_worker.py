"""Worker of tests/test_gpu_dp_8b.py (run as a child process, never collected by pytest).

    python tests/dp8b_worker.py --part smt --mode acc --out a.pt
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tests/dp8b_worker.py --part smt --mode dp --out d.pt

BASELINE config 3 (LLaMA-3-8B SMT(0.71%) data-parallel; the reference's exchange is implicit in
``model.backward``, fine_tune.py:712, in ZeRO-2 buckets of ``reduce_bucket_size``,
deepspeed_helpers.py:73) at the real 8B geometry, two ranks sharing cuda:0 over gloo:

* ``--part smt``: the whole 32-layer LLaMA-3-8B (vocabulary 128256, untied head) through the product
  path (fused ops, smt_flash, smt_ce) with SURVEY §8's 872 tiles (a seeded draw over all 32 layers,
  tests/llama8b_tiles.py), the engine at its default ``reduce_bucket_size`` (4 M elements): the
  57.1 M-element packed fp32 tile-gradient buffer (229 MB) cut into buckets of whole modules, issued
  from the comm stream while backward runs; two SMT steps (fused clip + AdamW + scatter into W).
* ``--part warmup``: the 8B width with 2 decoder layers and the full 128256-entry embedding and untied
  LM head (525 M elements each), the reference's DeepSpeed config shape (``zero_optimization``
  ``reduce_bucket_size`` 1e6, bf16, clip 1.0): one full fine-tuning warm-up step with every layer
  recomputed (fine_tune.py:192) through the dense bucketed all-reduce, the gradient harvest,
  the rank-0 selection broadcast + conversion, and one SMT step.

Modes: ``dp`` = 2 ranks, one sample (S = 256) each; ``acc`` = 1 rank, the same two samples as two
gradient-accumulation micro-steps. Rank 0 writes the selection, the exact tile optimizer state, the
exact tiles of every SMT module's W, and bit checksums (tests/llama8b_tiles.bits_hash) of every
multi-GB tensor: each SMT module's whole W, and after the warm-up every parameter and its fp32
master / exp_avg / exp_avg_sq.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

S = 256


def say(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def samples(vocab, offset, dev):
    """Two samples of S tokens (the global batch of 2): row i is rank i's / micro-step i's."""
    gen = torch.Generator().manual_seed(8000 + offset)
    ids = torch.randint(0, vocab, (2, S), generator=gen, dtype=torch.int64).to(dev)
    return [dict(input_ids=ids[i:i + 1], attention_mask=torch.ones_like(ids[i:i + 1]), labels=ids[i:i + 1])
            for i in range(2)]


def mine(parts, mode, rank):
    return [parts[rank]] if mode == "dp" else parts


def tile_state(engine, model):
    from sparse_matrix_tuning_amd.smt.smt import LinearLayer_MatrixSparsity
    from tests.llama8b_tiles import bits_hash
    tg = engine.tile_groups[0]
    mods = {n: m for n, m in model.named_modules() if isinstance(m, LinearLayer_MatrixSparsity) and len(m.tiles)}
    w_tiles = {n: torch.cat([m.weight.detach()[r * 256:(r + 1) * 256, c * 256:(c + 1) * 256] for r, c in m.tiles], 0).cpu()
               for n, m in mods.items()}
    return {"master": tg.master.cpu(), "exp_avg": tg.exp_avg.cpu(), "exp_avg_sq": tg.exp_avg_sq.cpu(),
            "W_tiles": w_tiles, "W_hash": {n: bits_hash(m.weight) for n, m in mods.items()},
            "buckets": [] if tg.buckets is None else [(b[0], b[1], b[2]) for b in tg.buckets.buckets],
            "tile_issued": 0 if tg.buckets is None else tg.buckets.issued,
            "n_modules": len(mods), "n_tiles": tg.n_tiles}


def part_smt(args, rank, dev):
    import bench
    from tests.llama8b_tiles import seeded_selection
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.fused_llama import patch_llama
    from sparse_matrix_tuning_amd.smt import smt

    cfg = bench.MODELS["llama3-8b"]
    model = bench.build_model("llama3-8b", dev)
    patch_llama(model)
    model.train()
    sel_att, sel_mlp = seeded_selection(cfg)
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-3), lr=1e-3, betas=(0.9, 0.95))
    ds = {"gradient_clipping": 1.0, "train_micro_batch_size_per_gpu": 1, "train_batch_size": 2,
          "bf16": {"enabled": True}}                      # reduce_bucket_size: the engine's default
    engine, *_ = initialize(model=model, optimizer=opt, config=ds)
    say(f"8B model converted: {engine.tile_groups[0].n_tiles} tiles, gas {engine.gradient_accumulation_steps}, "
        f"world {engine.world}")
    losses = []
    for step in range(2):
        for b in mine(samples(cfg["vocab_size"], step, dev), args.mode, rank):
            loss = engine(**b, use_cache=False).loss
            engine.backward(loss)
            engine.step()
            losses.append(loss.item())
        say(f"SMT step {step} done")
    torch.cuda.synchronize()
    out = tile_state(engine, model)
    out.update(reduce_bucket_size=engine.reduce_bucket_size, losses=losses,
               sel_att=sorted((k, list(v)) for k, v in sel_att.items()),
               sel_mlp=sorted((k, list(v)) for k, v in sel_mlp.items()))
    return out


def part_warmup(args, rank, dev):
    import bench
    from tests.llama8b_tiles import bits_hash
    from sparse_matrix_tuning_amd import trainer
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.fused_llama import patch_llama
    from sparse_matrix_tuning_amd.smt.smt import _NO_DECAY

    cfg = dict(bench.MODELS["llama3-8b"], num_hidden_layers=2)
    bench.MODELS["_dp8b_w"] = cfg
    model = bench.build_model("_dp8b_w", dev)
    patch_llama(model)
    model.gradient_checkpointing_enable()               # the warm-up recomputes every layer (fine_tune.py:192)
    model.train()
    ds = {"train_batch_size": 2, "train_micro_batch_size_per_gpu": 1, "gradient_clipping": 1.0,
          "bf16": {"enabled": True},
          "zero_optimization": {"stage": 2, "reduce_bucket_size": 1e6}}    # deepspeed_helpers.py:61-73
    groups = [{"params": [p for n, p in model.named_parameters() if not any(nd in n.lower() for nd in _NO_DECAY)],
               "weight_decay": 0.0},
              {"params": [p for n, p in model.named_parameters() if any(nd in n.lower() for nd in _NO_DECAY)],
               "weight_decay": 0.0}]
    opt = SMTFusedAdam(groups, lr=1e-3, betas=(0.9, 0.95))
    engine, *_ = initialize(model=model, optimizer=opt, config=ds)
    dims = trainer.get_targeted_module_dims(model)
    n_att, n_mlp = trainer.block_budgets(trainer.count_total_blocks(model), 0.00356, 0.00356)
    harvester = trainer.GradHarvester(model, n_mlp, n_att)
    dense = engine.dense_buckets
    dense_info = None if dense is None else [sum(p.numel() for p in b) for b in dense.buckets]
    for b in mine(samples(cfg["vocab_size"], 100, dev), args.mode, rank):
        engine.backward(engine(**b, use_cache=False).loss)
        if engine.is_gradient_accumulation_boundary():
            harvester.harvest()                        # the DP-averaged (accumulated) gradients
        engine.step()
    torch.cuda.synchronize()
    say("warm-up step done")
    warm = {}
    if rank == 0:
        for n, p in model.named_parameters():
            st = engine._dense_state[id(p)]
            warm[n] = {"param": bits_hash(p), "master": bits_hash(st["master"]), "exp_avg": bits_hash(st["exp_avg"]),
                       "exp_avg_sq": bits_hash(st["exp_avg_sq"])}
        torch.cuda.empty_cache()
    harvest = {}
    if rank == 0:
        for pool in (harvester.warmup_grads, harvester.attention_warmup_grads):
            for k, t in pool.items():
                harvest[str(k)] = bits_hash(t)
    dense_issued = 0 if dense is None else dense.issued
    engine, opt, _sched, sel_mlp, sel_att = trainer.select_and_convert(
        engine, harvester, dims, n_att, n_mlp, calculate_strategy="abs_mean", smt_lr=1e-3, num_training_steps=10,
        ds_config=ds)
    say(f"selection: {sum(map(len, sel_att.values()))} + {sum(map(len, sel_mlp.values()))} tiles")
    for b in mine(samples(cfg["vocab_size"], 200, dev), args.mode, rank):
        engine.backward(engine(**b, use_cache=False).loss)
        engine.step()
    torch.cuda.synchronize()
    out = tile_state(engine, engine.module)
    out.update(warm=warm, harvest=harvest, dense_buckets=dense_info, dense_issued=dense_issued,
               sel_att=sorted((k, list(v)) for k, v in sel_att.items()),
               sel_mlp=sorted((k, list(v)) for k, v in sel_mlp.items()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", choices=("smt", "warmup"), required=True)
    ap.add_argument("--mode", choices=("dp", "acc"), required=True)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if (args.mode == "dp") != (world == 2):
        raise SystemExit("--mode dp runs as 2 ranks, --mode acc as one process")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if world > 1:
        dist.init_process_group("gloo")
    out = (part_smt if args.part == "smt" else part_warmup)(args, rank, dev)
    out["world"] = world
    out["peak_gb"] = torch.cuda.max_memory_allocated(dev) / 1e9
    if rank == 0:
        torch.save(out, args.out)
        say(f"wrote {args.out} (peak {out['peak_gb']:.1f} GB on rank 0)")
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
