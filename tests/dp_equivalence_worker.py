"""Worker of tests/test_gpu_dp_equivalence.py (run as a child process, never collected by pytest).

    python tests/dp_equivalence_worker.py --mode acc --out a.pt
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tests/dp_equivalence_worker.py --mode dp --out d.pt

One full fine-tuning warm-up step with the gradient harvest, selection + conversion, then one SMT
step (fused clip + AdamW), of a 2-layer mini-LLaMA (fused HIP ops, smt_flash attention) on cuda:0:

* ``dp``: 2 ranks (gloo; both on cuda:0), micro-batch 2 each: the engine's bucketed all-reduce of
  the dense warm-up gradients and of the packed tile gradients, the rank-0 selection broadcast;
* ``acc``: 1 rank, the same two micro-batches as 2 gradient-accumulation micro-steps;
* ``big``: 1 rank, the concatenated micro-batch of 4.

``--pg nccl --exchange always`` (with ``big``, under ``torch.distributed.run --nproc-per-node 1``): a
world-1 RCCL process group and the engine's ``"dp_exchange": "always"``, so the bucketed RCCL
all-reduces of the dense warm-up gradients and the tile gradients run (identities at world 1).

``--fp8``: the SMT phase on the fp8 path (e4m3 decoder GEMMs, MX-fp8 tile weight gradients).

``--dtype fp16``: the reference's --dtype fp16 (an fp16 model, transformers' own ops, the engine under
DeepSpeed's dynamic loss scale; the fp16 config of deepspeed_helpers.py:53-55).

Writes the post-warm-up weights, the selection, the tile optimizer state and the SMT modules'
weights after the SMT step (rank 0).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("dp", "acc", "big"), required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--fp8", action="store_true", help="SMT phase on the fp8 path (MX-fp8 tile gradients)")
    ap.add_argument("--pg", default=None, help="process-group backend (default: gloo when WORLD_SIZE > 1)")
    ap.add_argument("--exchange", default="auto", choices=("auto", "always"), help="the engine's dp_exchange")
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp16"))
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if world > 1 or args.pg:
        backend = args.pg or "gloo"
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import bench
    from sparse_matrix_tuning_amd import trainer
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.fused_llama import patch_llama
    from sparse_matrix_tuning_amd.smt.smt import LinearLayer_MatrixSparsity

    cfg = dict(bench.MODELS["mini"])
    cfg["num_hidden_layers"] = 2
    bench.MODELS["_dp"] = cfg
    model = bench.build_model("_dp", dev)
    if args.dtype == "fp16":
        model = model.half()                             # the fused LLaMA ops are bf16-only
    else:
        patch_llama(model)
    model.train()
    vocab = cfg["vocab_size"]

    def halves(offset):
        full = bench.batches(1, 4, 128, vocab, 0, dev, offset=offset)[0]
        parts = [{k: v[2 * i:2 * i + 2] for k, v in full.items()} for i in range(2)]
        if args.mode == "big":
            return [full]
        if args.mode == "dp":
            return [parts[rank]]
        return parts

    micro = 4 if args.mode == "big" else 2
    ds = {"gradient_clipping": 1.0, "train_micro_batch_size_per_gpu": micro, "train_batch_size": 4,
          "reduce_bucket_size": 300000,                 # several buckets on this small model
          "dp_exchange": args.exchange}
    if args.dtype == "fp16":
        ds["fp16"] = {"enabled": True, "loss_scale_window": 100, "initial_scale_power": 12}
    dims = trainer.get_targeted_module_dims(model)
    n_att, n_mlp = trainer.block_budgets(trainer.count_total_blocks(model), 0.05, 0.05)
    opt = SMTFusedAdam(model.parameters(), lr=1e-3, betas=(0.9, 0.95))
    engine, opt, _, _ = initialize(model=model, optimizer=opt, config=ds)
    harvester = trainer.GradHarvester(model, n_mlp, n_att)
    warm_grads = {}
    for b in halves(1000):
        engine.backward(engine(**b, use_cache=False).loss)
        if engine.is_gradient_accumulation_boundary():
            harvester.harvest()                          # the DP-averaged (accumulated) gradients
            warm_grads = {n: p.grad.float().cpu() for n, p in model.named_parameters() if p.grad is not None}
        engine.step()
    warm = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
    dense_issued = engine.dense_buckets.issued if engine.dense_buckets is not None else 0
    engine, opt, sched, sel_mlp, sel_att = trainer.select_and_convert(
        engine, harvester, dims, n_att, n_mlp, calculate_strategy="abs_mean", smt_lr=1e-3, num_training_steps=10,
        ds_config=dict(ds, fp8_linears=args.fp8))
    for b in halves(2000):
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        engine.step()
    torch.cuda.synchronize()
    tg = engine.tile_groups[0]
    out = {"warm": warm, "sel_mlp": [(k, list(v)) for k, v in sel_mlp.items()],
           "sel_att": [(k, list(v)) for k, v in sel_att.items()],
           "master": tg.master.cpu(), "exp_avg": tg.exp_avg.cpu(), "exp_avg_sq": tg.exp_avg_sq.cpu(),
           "W": {n: m.weight.detach().cpu().clone() for n, m in model.named_modules()
                 if isinstance(m, LinearLayer_MatrixSparsity)},
           "buckets": len(tg.buckets.buckets) if tg.buckets is not None else 0,
           "tile_issued": tg.buckets.issued if tg.buckets is not None else 0, "dense_issued": dense_issued,
           "backend": dist.get_backend() if dist.is_initialized() else None,
           "world": dist.get_world_size() if dist.is_initialized() else 1,
           "loss_scale": engine.loss_scaler.state_dict() if engine.loss_scaler is not None else None,
           # the last step's DP-averaged (accumulated) tile gradient, still loss-scaled in fp16
           "grad": tg.grad.cpu() / (dist.get_world_size() if dist.is_initialized() else 1),
           "skipped": engine.skipped_steps,
           "warm_grads": warm_grads if args.dtype == "fp16" else {}}
    if rank == 0:
        torch.save(out, args.out)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
