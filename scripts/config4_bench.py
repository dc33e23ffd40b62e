"""BASELINE config 4 on one MI355X: LLaMA-2-13B, activation-based (channel) selection path.

The reference's activation path (fine_tune.py:406-709, smt_helper.py:149-230, smt.py:185-296):
no-grad forwards with a hook on every decoder linear that sums |x| into an fp32 [B, S, in]
accumulator per (module, layer); a per-channel score; the top-n channels over all keys; each
selected channel becomes a trainable ROW of W (LinearLayer_ChannelSparsity / linearChannel). Only the
square attention projections work in the reference (the MLP path fails on non-square weights,
SURVEY §8(f) row 1), so the budget goes to q/k/v, as --num_attention_channel does.

Synthetic data of the config's shape (random init, uniform tokens, B = 16, S = 2048), the model
config LLaMA-2-13B (vocab 32008 after the reference's resize, deepspeed_helpers.py:287-296),
budget 0.86 % of the parameters in 5120-wide rows. Prints one JSON line (tokens/s over the timed
steps, peak HBM, selection time, the channel kernels' times). Per-rank data parallel as the bench.

    python scripts/config4_bench.py [--steps 10 --warmup 3 --act-steps 2 --out gpurun_out/c4.json] [--gpus N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (model builder, batches, timers)

bench.MODELS["llama2-13b"] = dict(
    vocab_size=32008, hidden_size=5120, intermediate_size=13824, num_hidden_layers=40, num_attention_heads=40,
    num_key_value_heads=40, rope_theta=10000.0, rms_norm_eps=1e-5, max_position_embeddings=4096,
    tie_word_embeddings=False, initializer_range=0.02)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-13b", choices=sorted(bench.MODELS))
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--act-steps", type=int, default=2, help="activation-collection forwards (fine_tune.py:586-709)")
    ap.add_argument("--ratio", type=float, default=0.0086, help="trainable fraction, in rows of the attention projections")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--grad-ckpt", action="store_true", help="per-layer recompute (fine_tune.py:192)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one GPU each (WORLD_SIZE unset and N > 1: starts them itself, as bench.py)")
    ap.add_argument("--dist-backend", default="nccl")
    ap.add_argument("--rank-reduction", default="reference", choices=("reference", "fp32_once"),
                    help="how the activation harvest sums ranks (trainer.ActivationHarvester)")
    args = ap.parse_args()

    mode, what = bench.launch_plan(args.gpus, os.environ)
    if mode == "error":
        print(f"config4_bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if mode == "spawn":
        import subprocess
        cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={what}",
               "--master-addr", "127.0.0.1", "--master-port", str(bench._free_port()), os.path.abspath(__file__)]
        sys.exit(subprocess.call(cmd + sys.argv[1:]))
    world = what
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > n_dev:
        raise SystemExit(f"config4_bench.py: {world} RCCL ranks need {world} GPUs; this node has {n_dev}")
    device = torch.device("cuda", local % max(1, n_dev))
    torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.dist_backend)
    from sparse_matrix_tuning_amd import _hip, trainer
    from sparse_matrix_tuning_amd.fused_llama import patch_llama
    _hip.load()

    # HIP events around the channel path's kernels (current stream)
    timers = {}
    for name in ("row_gather", "row_scatter", "column_gather", "tile_wgrad", "act_accumulate"):
        t = bench.LaunchTimer()
        setattr(_hip, name, t.wrap(getattr(_hip, name), lambda *a, **k: 1))
        timers[name] = t

    # wall time (device-synchronised) and band report of the channel selection itself
    from sparse_matrix_tuning_amd.smt import ranking
    sel = {"seconds": 0.0, "reports": []}
    orig_sel = trainer.select_channel_based_on_activation

    def timed_sel(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = orig_sel(*a, **k)
        sel["seconds"] += time.perf_counter() - t
        rep = dict(ranking.LAST_REPORT)
        sel["reports"].append({"flagged": rep.get("flagged"), "rescored_keys": len(rep.get("rescored_keys", [])),
                               "rescored_elements": rep.get("rescored_elements"), "iterations": rep.get("iterations"),
                               "candidates": rep.get("candidates"), "worst_case_bound": rep.get("worst_case_bound"),
                               "ranking_s": round(rep.get("seconds", 0.0), 3)})
        return r
    trainer.select_channel_based_on_activation = timed_sel

    t0 = time.time()
    model = bench.build_model(args.model, device)
    patch_llama(model)
    if args.grad_ckpt:
        model.gradient_checkpointing_enable()
    model.train()
    total = sum(p.numel() for p in model.parameters())
    hidden = bench.MODELS[args.model]["hidden_size"]
    n_att = int(args.ratio * total / hidden)
    vocab = bench.MODELS[args.model]["vocab_size"]
    B, S = args.batch, args.seq
    bench.log(f"{args.model}: {total / 1e9:.3f} B params built in {time.time() - t0:.1f}s; attention channel budget {n_att}")

    # ---- activation collection + selection + conversion ----
    harvester = trainer.ActivationHarvester(model, 0, n_att, rank_reduction=args.rank_reduction)
    torch.cuda.reset_peak_memory_stats(device)
    t_h = time.time()
    for b in bench.batches(args.act_steps, B, S, vocab, rank, device, offset=100000):
        harvester.collect(b)
    torch.cuda.synchronize()
    harvest_s = time.time() - t_h
    harvest_peak = torch.cuda.max_memory_allocated(device) / 1e9
    t_s = time.time()
    engine, _opt, _sched, sel_mlp, sel_att = trainer.select_and_convert_channels(
        model, harvester, n_att, 0, num_training_steps=args.warmup + args.steps + 10,
        ds_config={"gradient_clipping": 1.0, "train_micro_batch_size_per_gpu": B, "train_batch_size": B * world})
    torch.cuda.synchronize()
    select_s = time.time() - t_s
    n_sel = sum(len(v) for v in sel_att.values())
    trainable = sum(p.numel() for p in engine.module.parameters() if p.requires_grad)
    layers = sorted({k[1] for k in sel_att})
    bench.log(f"collection {args.act_steps} x {harvest_s / max(1, args.act_steps):.2f}s, selection+conversion "
              f"{select_s:.2f}s: {n_sel} channels in {len(sel_att)} modules of {len(layers)} layers, trainable "
              f"{trainable} ({100.0 * trainable / total:.3f}%)")

    # ---- training steps ----
    data = bench.batches(args.warmup + args.steps, B, S, vocab, rank, device)
    torch.cuda.reset_peak_memory_stats(device)

    def step(b):
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        engine.step()
        return loss

    for i in range(args.warmup):
        step(data[i])
    for t in timers.values():
        t.records, t.enabled = [], True
    elapsed, per_step, loss = bench.timed_steps(step, data[args.warmup:], world, device)
    for t in timers.values():
        t.enabled = False
    peak = torch.cuda.max_memory_allocated(device) / 1e9
    med = bench._median(per_step)
    if world > 1:
        import torch.distributed as dist
        r = torch.tensor([elapsed, med, peak], dtype=torch.float64, device=device)
        dist.all_reduce(r, op=dist.ReduceOp.MAX)
        elapsed, med, peak = r.tolist()
    kernels = {}
    for name, t in timers.items():
        s = t.summary()
        if s:
            kernels[name] = {"launches_per_step": s["launches"] / args.steps, "ms_per_step": round(s["seconds"] * 1e3 / args.steps, 3)}
    out = {"metric": "config 4: train tokens/s + peak GB HBM, LLaMA-2-13B SMT channel path (activation selection)",
           "value": round(world * B * S * args.steps / elapsed, 1), "unit": "tokens/s", "n_gpus": world,
           "world_size": world, "backend": args.dist_backend if world > 1 else None, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
           "median_ms_per_step": round(med * 1e3, 2), "peak_hbm_gb": round(peak, 2),
           "collection_peak_hbm_gb": round(harvest_peak, 2), "dtype": "bf16",
           "data": "synthetic (uniform token ids, labels=inputs; random-init weights)",
           "config": {"workload": "LLaMA-2-13B channel-sparse fine-tuning step (fwd+bwd+AdamW over selected rows)",
                      "global_batch": B * world, "seq_len": S, "parallelism": f"dp{world}", "channels": n_sel,
                      "rank_reduction": args.rank_reduction,
                      "channel_modules": len(sel_att), "channel_layers": len(layers), "trainable_params": trainable,
                      "trainable_pct": round(100.0 * trainable / total, 3), "grad_ckpt": bool(args.grad_ckpt),
                      "activation_steps": args.act_steps},
           "collection_s_per_step": round(harvest_s / max(1, args.act_steps), 3),
           "selection_and_conversion_s": round(select_s, 3), "selection_s": round(sel["seconds"], 3),
           "selection_band": sel["reports"], "channel_kernels": kernels,
           "final_loss": round(loss.item(), 5)}
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
