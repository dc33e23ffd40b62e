"""Worker of tests/test_gpu_channel_dp.py (run as two ranks by torch.distributed.run, gloo, both on
cuda:0; never collected by pytest).

Each rank collects activations of its own batches with ``trainer.ActivationHarvester`` (the
reference's per-hook bf16 all-reduce of ``|x|``, fine_tune.py:651-665) while a second forward hook
keeps every hooked linear's input. Rank 0 replays the reference's arithmetic on those inputs with
``oracle.channel_hook_accumulate_ranks`` and writes what it finds (torch.save, weights only):
accumulators bit-identical on both ranks and to the restatement, and the channel selections of both
pools identical to ``oracle.select_channel`` on the restated accumulators.
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
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")

    import bench
    from oracle import smt_oracle as ref
    from sparse_matrix_tuning_amd import trainer
    from sparse_matrix_tuning_amd.smt.smt_helper import get_named_linears, select_channel_based_on_activation

    cfg = dict(bench.MODELS["mini"], num_hidden_layers=2)
    bench.MODELS["_c"] = cfg
    model = bench.build_model("_c", dev)
    harvester = trainer.ActivationHarvester(model, 64, 64)
    assert harvester.world == world and harvester.rank_reduction == "reference"
    seen = {}                                           # (pool, key) -> [x per step]

    def keep(pool, key):
        def hook(_m, inputs, _out):
            seen.setdefault((pool, key), []).append(inputs[0].detach().cpu().clone())
        return hook
    handles = []
    for i, layer in enumerate(model.model.layers):
        for name, lin in get_named_linears(layer).items():
            if "mlp" in name:
                mod = "gate_proj" if "gate_proj" in name else "up_proj" if "up_proj" in name else "down_proj"
                handles.append(lin.register_forward_hook(keep("mlp", (mod, i))))
            elif "self_attn" in name:
                mod = ("q_proj" if "q_proj" in name else "k_proj" if "k_proj" in name else
                       "v_proj" if "v_proj" in name else None)
                if mod is not None:
                    handles.append(lin.register_forward_hook(keep("att", (mod, i))))
    for b in bench.batches(args.steps, 2, 64, cfg["vocab_size"], rank, dev, offset=300):
        harvester.collect(b)
    torch.cuda.synchronize()
    for h in handles:
        h.remove()
    mine = {("mlp", k): e.acc.cpu() for k, e in harvester.activation.items()}
    mine.update({("att", k): e.acc.cpu() for k, e in harvester.attention_activation.items()})
    gathered_seen = [None] * world
    gathered_acc = [None] * world
    dist.all_gather_object(gathered_seen, seen)
    dist.all_gather_object(gathered_acc, mine)
    sel_att = select_channel_based_on_activation(harvester.attention_activation, 40)
    sel_mlp = select_channel_based_on_activation(harvester.activation, 40, calculate_strategy="abs_mean")
    if rank == 0:
        feats = {"att": {}, "mlp": {}}
        for (pool, key), xs in seen.items():
            for step in range(args.steps):
                ref.channel_hook_accumulate_ranks(feats[pool], key, [gathered_seen[r][(pool, key)][step]
                                                                      for r in range(world)])
        alone = {}
        for (pool, key), xs in seen.items():
            d = {}
            for step in range(args.steps):
                ref.channel_hook_accumulate(d, key, xs[step])
            alone[(pool, key)] = d[key]
        res = {"keys": len(mine),
               "ranks_equal": all(torch.equal(gathered_acc[1][k], v) for k, v in mine.items()),
               "acc_equal_restatement": all(torch.equal(v, feats[k[0]][k[1]]) for k, v in mine.items()),
               "differs_from_rank0_alone": any(not torch.equal(v, alone[k]) for k, v in mine.items()),
               "sel_att": [(k, list(v)) for k, v in sel_att.items()],
               "sel_mlp": [(k, list(v)) for k, v in sel_mlp.items()],
               "ref_att": [(k, list(v)) for k, v in ref.select_channel(feats["att"], 40).items()],
               "ref_mlp": [(k, list(v)) for k, v in ref.select_channel(feats["mlp"], 40,
                                                                        calculate_strategy="abs_mean").items()]}
        torch.save(res, args.out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
